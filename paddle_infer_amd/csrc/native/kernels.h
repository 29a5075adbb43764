// Kernel interface of the native engine: every entry exists as a plain C++ loop (kernels_cpu.cc)
// and as a HIP kernel (gpu.hip); `kern::*` dispatches on the context's device.
#pragma once

#include "engine.h"

namespace pdn {

enum UnaryOp { U_IDENT, U_RELU, U_GELU, U_GELU_TANH, U_TANH, U_SIGMOID, U_SILU, U_EXP, U_SQRT,
               U_RSQRT, U_ABS, U_SCALE, U_SCALE_PRE,
               U_RELU6,      // min(max(x, 0), p0)  (p0 = threshold, 6)
               U_HSWISH,     // x · min(max(x + p1, 0), p0) / p0  (p0 = threshold 6, p1 = offset 3)
               U_HSIGMOID,   // min(max(x · p0 + p1, 0), 1)  (p0 = slope, p1 = offset)
               U_LEAKY };    // x > 0 ? x : p0 · x
enum BinaryOp { B_ADD, B_SUB, B_MUL, B_DIV, B_MAX, B_MIN, B_POW };

constexpr int kMaxDims = 8;
struct Bcast {  // out[i] = a[i·sa] op b[i·sb] over an n-d index space (strides in elements)
  int nd = 0;
  int64_t dims[kMaxDims] = {0};
  int64_t sa[kMaxDims] = {0};
  int64_t sb[kMaxDims] = {0};
  int64_t n = 0;
};
// NCHW convolution / pooling geometry (one group's channels C; top/left padding; outputs OH × OW)
struct ConvG {
  int64_t C, H, W, R, S, OH, OW, sh, sw, ph, pw, dh, dw;
};
struct PoolG {
  int64_t H, W, OH, OW, kh, kw, sh, sw, ph, pw;
  int max, exclusive, adaptive;
};
struct Strided {  // out (contiguous, dims) = src[offset + Σ idx·stride] (elements)
  int nd = 0;
  int64_t dims[kMaxDims] = {0};
  int64_t stride[kMaxDims] = {0};
  int64_t offset = 0;
  int64_t n = 0;
};

#define PDN_KERNELS(NS)                                                                            \
  namespace NS {                                                                                   \
  void unary(Ctx&, int op, const float* x, float* y, int64_t n, float p0, float p1);               \
  void binary(Ctx&, int op, const float* a, const float* b, float* y, const Bcast& bc);            \
  void softmax(Ctx&, const float* x, float* y, int64_t outer, int64_t n, int64_t inner);           \
  void layernorm(Ctx&, const float* x, const float* g, const float* b, float* y, int64_t rows,     \
                 int64_t cols, float eps);                                                         \
  void strided_copy(Ctx&, const void* src, void* dst, int elem, const Strided& s);                 \
  void gather_rows(Ctx&, const float* table, const void* ids, int ids_i64, float* y, int64_t n,    \
                   int64_t width, int64_t rows, int64_t padding_idx);                              \
  void gemm(Ctx&, bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,  \
            int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB, float beta,          \
            float* C, int64_t ldc, int64_t sC, int64_t batch);                                     \
  void cast(Ctx&, const void* x, int dtx, void* y, int dty, int64_t n);                            \
  void fill(Ctx&, void* y, int dt, int64_t n, double v);                                           \
  void reduce(Ctx&, const float* x, float* y, int64_t outer, int64_t n, int64_t inner, bool mean); \
  void copy2d(Ctx&, const void* src, int64_t spitch, void* dst, int64_t dpitch, int64_t rows,      \
              int64_t cols, int elem);                                                             \
  /* col [N][C·R·S][OH·OW] of images x + n·x_img (first channel of the group at x) */              \
  void im2col(Ctx&, const float* x, int64_t x_img, float* col, int64_t N, const ConvG& g);         \
  /* depthwise: y [N][C·m][OH][OW] = conv(x [N][C][H][W], w [C·m][1][R][S]) (+ bias [C·m]) */      \
  void dwconv(Ctx&, const float* x, const float* w, const float* bias, float* y, int64_t N,        \
              int64_t mult, const ConvG& g);                                                       \
  void pool2d(Ctx&, const float* x, float* y, int64_t planes, const PoolG& p);                     \
  /* y[o][c][i] = act(x[o][c][i] · sc[c] + sh[c]) (act: UnaryOp, U_IDENT = none) */                 \
  void channel_affine(Ctx&, const float* x, const float* sc, const float* sh, float* y,            \
                      int64_t outer, int64_t C, int64_t inner, int act, float p0);                 \
  }

PDN_KERNELS(cpu)
PDN_KERNELS(gpu)

namespace gpu {
// bf16 (f16 = 0) / fp16 (f16 = 1) element-wise with f32 math
void unary16(Ctx&, int op, int f16, const void* x, void* y, int64_t n, float p0, float p1);
void binary16(Ctx&, int op, int f16, const void* a, const void* b, void* y, const Bcast& bc);
}  // namespace gpu

inline bool is16(int dt) { return dt == VT_FP16 || dt == VT_BF16; }

// fast_ops.hip: ops on the framework's kernels (libpiamd_kernels.so + the assembly GEMM) for
// bf16 / fp16 tensors on the GPU. fast_run returns false when the op / dtypes are not its own
// (the generic implementation in ops.cc runs instead).
bool fast_run(Ctx& c, const OpDesc& op, Scope& s);
bool fast_knows(const std::string& type);
void fast_release(Ctx& c);

namespace kern {
#define PDN_DISPATCH(name)                                   \
  template <typename... A>                                   \
  inline void name(Ctx& c, A&&... a) {                       \
    if (c.gpu) gpu::name(c, std::forward<A>(a)...);          \
    else cpu::name(c, std::forward<A>(a)...);                \
  }
PDN_DISPATCH(unary)
PDN_DISPATCH(binary)
PDN_DISPATCH(softmax)
PDN_DISPATCH(layernorm)
PDN_DISPATCH(strided_copy)
PDN_DISPATCH(gather_rows)
PDN_DISPATCH(gemm)
PDN_DISPATCH(cast)
PDN_DISPATCH(fill)
PDN_DISPATCH(reduce)
PDN_DISPATCH(copy2d)
PDN_DISPATCH(im2col)
PDN_DISPATCH(dwconv)
PDN_DISPATCH(pool2d)
PDN_DISPATCH(channel_affine)
#undef PDN_DISPATCH
}  // namespace kern

}  // namespace pdn
