// Fused elementwise kernels: bias+activation (fwd/bwd with fused bias-grad column sums),
// dropout, masked softmax — bf16, fp16 and f32 (Paddle's default dtype) element types.
//
// Parity: reference `paddle/fluid/operators/fused/fused_dropout_act_bias.h`
// (fused_bias_act / FusedFeedForward's `dropout(act(x + bias))`), `phi/kernels/gpu/gelu_*`,
// `phi/kernels/fusion/gpu/fused_softmax_mask_kernel.cu` (softmax(x + mask)) and
// `fused_softmax_mask_upper_triangle`.
//
// MI355X design: 16 B/lane vectors everywhere (G13); the activation backward is 2-D (row groups ×
// 2048-column stripes) so each thread also accumulates the bias gradient for its 8 columns in
// registers and adds them with one f32 atomic per column per block — the dbias reduction costs no
// extra pass over the [tokens × 4h] activation.
#include "common.h"

namespace {

enum Act { ACT_NONE = 0, ACT_GELU_TANH = 1, ACT_GELU_ERF = 2, ACT_RELU = 3, ACT_SILU = 4 };

template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if (ACT == ACT_GELU_TANH) return gelu_tanh(x);
  if (ACT == ACT_GELU_ERF) return gelu_erf(x);
  if (ACT == ACT_RELU) return x > 0.f ? x : 0.f;
  if (ACT == ACT_SILU) return x / (1.f + __expf(-x));
  return x;
}
template <int ACT>
__device__ __forceinline__ float act_g(float x) {
  if (ACT == ACT_GELU_TANH) return gelu_tanh_grad(x);
  if (ACT == ACT_GELU_ERF) return gelu_erf_grad(x);
  if (ACT == ACT_RELU) return x > 0.f ? 1.f : 0.f;
  if (ACT == ACT_SILU) { float s = 1.f / (1.f + __expf(-x)); return s * (1.f + x * (1.f - s)); }
  return 1.f;
}

// 8-element vectors of the element type DT (0 bf16, 1 fp16: one 16-B access; 2 f32: two), f32 math
enum { DT_BF16 = 0, DT_F16 = 1, DT_F32 = 2 };
template <int DT>
struct IO8 {
  typedef u16x8 R;
  static __device__ __forceinline__ R ld(const void* p, long long i) { return reinterpret_cast<const u16x8*>(p)[i]; }
  static __device__ __forceinline__ R ldnt(const void* p, long long i) {
    return __builtin_nontemporal_load(&reinterpret_cast<const u16x8*>(p)[i]);
  }
  static __device__ __forceinline__ float get(const R& r, int j) { return h2f<DT == DT_F16>(r[j]); }
  static __device__ __forceinline__ R pack(const float* v) {
    R r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f2h<DT == DT_F16>(v[j]);
    return r;
  }
  static __device__ __forceinline__ void st(void* p, long long i, const float* v) { reinterpret_cast<u16x8*>(p)[i] = pack(v); }
  static __device__ __forceinline__ void stnt(void* p, long long i, const float* v) {
    __builtin_nontemporal_store(pack(v), &reinterpret_cast<u16x8*>(p)[i]);
  }
  static __device__ __forceinline__ float ld1(const void* p, long long i) { return h2f<DT == DT_F16>(reinterpret_cast<const unsigned short*>(p)[i]); }
  static __device__ __forceinline__ void st1(void* p, long long i, float v) { reinterpret_cast<unsigned short*>(p)[i] = f2h<DT == DT_F16>(v); }
};
template <>
struct IO8<DT_F32> {
  struct R { f32x4 a, b; };
  static __device__ __forceinline__ R ld(const void* p, long long i) {
    const f32x4* q = reinterpret_cast<const f32x4*>(p) + 2 * i;
    return R{q[0], q[1]};
  }
  static __device__ __forceinline__ R ldnt(const void* p, long long i) {
    const f32x4* q = reinterpret_cast<const f32x4*>(p) + 2 * i;
    return R{__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1)};
  }
  static __device__ __forceinline__ float get(const R& r, int j) { return j < 4 ? r.a[j] : r.b[j - 4]; }
  static __device__ __forceinline__ void st(void* p, long long i, const float* v) {
    f32x4* q = reinterpret_cast<f32x4*>(p) + 2 * i;
    q[0] = f32x4{v[0], v[1], v[2], v[3]};
    q[1] = f32x4{v[4], v[5], v[6], v[7]};
  }
  static __device__ __forceinline__ void stnt(void* p, long long i, const float* v) {
    f32x4* q = reinterpret_cast<f32x4*>(p) + 2 * i;
    __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, q);
    __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, q + 1);
  }
  static __device__ __forceinline__ float ld1(const void* p, long long i) { return reinterpret_cast<const float*>(p)[i]; }
  static __device__ __forceinline__ void st1(void* p, long long i, float v) { reinterpret_cast<float*>(p)[i] = v; }
};

// y = act(x + bias) (bias optional, broadcast over rows of length N); bf16 / fp16 / f32; N % 8 == 0.
template <int ACT, int DT>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(const void* __restrict__ x,
                                                          const void* __restrict__ bias,
                                                          void* __restrict__ y,
                                                          void* __restrict__ pre, long long n8,
                                                          int N) {
  typedef IO8<DT> io;
  // 4 independent 16-B loads in flight per thread before any math (latency hiding at
  // grid-stride; the memory pipe, not the ALU, bounds this kernel)
  constexpr int U = 4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const int nb8 = N >> 3;
  // bias column of vector i is i % nb8, tracked incrementally (a 64-bit modulo per vector was
  // half of this kernel's VALU instructions and made it VALU-bound)
  const long long first = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int step1 = (int)(stride % nb8), stepU = (int)((U * stride) % nb8);
  int c0 = (int)(first % nb8);
  for (long long i0 = first; i0 < n8; i0 += U * stride) {
    typename io::R r[U], b[U];
    int c = c0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = min(i0 + u * stride, n8 - 1);
      r[u] = io::ldnt(x, i);
      if (bias) b[u] = io::ld(bias, c);
      c += step1;
      c -= c >= nb8 ? nb8 : 0;
    }
    c0 += stepU;
    c0 -= c0 >= nb8 ? nb8 : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      if (i >= n8) break;
      float o[8], pr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = io::get(r[u], j);
        if (bias) v += io::get(b[u], j);
        pr[j] = v;
        o[j] = act_f<ACT>(v);
      }
      if (pre) io::st(pre, i, pr);
      io::stnt(y, i, o);  // streamed: no L2 reuse
    }
  }
}

// dx = dy * act'(h) with h = pre-activation (x + bias); dbias partials. grid = (G, ceil(N/2048)).
template <int ACT, int DT>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(const void* __restrict__ dy,
                                                          const void* __restrict__ h,
                                                          const void* __restrict__ bias,
                                                          void* __restrict__ dx,
                                                          float* __restrict__ part, int rows,
                                                          int N) {
  typedef IO8<DT> io;
  const int c8 = blockIdx.y * 256 + threadIdx.x;  // 8-column group index
  const bool colok = c8 * 8 < N;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  typename io::R b;
  if (bias && colok) b = io::ld(bias, c8);
  constexpr int U = 4;  // rows in flight per thread
  for (int r0 = blockIdx.x; colok && r0 < rows; r0 += U * gridDim.x) {
    typename io::R d[U], hv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(r0 + u * (int)gridDim.x, rows - 1);
      const long long idx = ((long long)r * N >> 3) + c8;
      // nontemporal (streaming) loads / stores: the [tokens x 4h] tensors are read once and never
      // hit in L2 — 5.19 -> 5.50 TB/s backward, 4.28 -> 4.57 forward (profiles/nt_stream_r2.txt)
      d[u] = io::ldnt(dy, idx);
      hv[u] = io::ldnt(h, idx);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = r0 + u * (int)gridDim.x;
      if (r >= rows) break;
      const long long idx = ((long long)r * N >> 3) + c8;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float hh = io::get(hv[u], j);
        if (bias) hh += io::get(b, j);
        const float g = io::get(d[u], j) * act_g<ACT>(hh);
        o[j] = g;
        acc[j] += g;
      }
      io::stnt(dx, idx, o);
    }
  }
  if (part) {
    // transpose the per-thread 8-column sums through LDS so every atomic wave-instruction adds
    // 64 consecutive floats (256 contiguous bytes: the full-rate atomic shape)
    __shared__ float red[2048];
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = acc[j];
    __syncthreads();
    const int col0 = blockIdx.y * 2048;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int cc = threadIdx.x + 256 * j;
      if (col0 + cc < N) atomicAdd(part + col0 + cc, red[cc]);
    }
  }
}

template <int DT>
__global__ __launch_bounds__(256) void colsum16_kernel(const float* __restrict__ part, int G,
                                                         int N, void* __restrict__ out,
                                                         int accumulate) {
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (col < N)
    for (int g = rg; g < G; g += 4) s += part[(size_t)g * N + col];
  __shared__ float red[4][64];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && col < N) {
    float t = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    if (accumulate) t += IO8<DT>::ld1(out, col);
    IO8<DT>::st1(out, col, t);
  }
}

// Row softmax with optional additive mask (broadcast over rows: mask row index = row % mask_rows)
// and optional causal (upper-triangle) masking with query position = row % causal_q. One wave
// per row for N <= 4096 (row in registers), bf16 / fp16 in/out.
template <int NV, int DT>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const void* __restrict__ x,
                                                         const void* __restrict__ mask,
                                                         int mask_rows, int causal_q,
                                                         void* __restrict__ y, int rows, int N,
                                                         float scale) {
  typedef IO8<DT> io;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = N >> 3;
  const size_t base = (size_t)row * N;
  const int qpos = causal_q > 0 ? (row % causal_q) + (N - causal_q) : N;
  float v[NV][8];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * 64 + lane;
    if (vi < nvec) {
      const typename io::R r = io::ld(x, (long long)(base >> 3) + vi);
      typename io::R mk;
      if (mask) mk = io::ld(mask, (long long)(row % mask_rows) * (N >> 3) + vi);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = io::get(r, j) * scale;
        if (mask) t += io::get(mk, j);
        if (vi * 8 + j > qpos) t = -INFINITY;
        v[i][j] = t;
        m = fmaxf(m, t);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = -INFINITY;
    }
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float e = v[i][j] == -INFINITY ? 0.f : __expf(v[i][j] - m);
      v[i][j] = e;
      s += e;
    }
  s = wave_sum(s);
  const float inv = s > 0.f ? 1.f / s : 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * 64 + lane;
    if (vi < nvec) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * inv;
      io::st(y, (long long)(base >> 3) + vi, o);
    }
  }
}

// dx = scale * y * (dy - sum(dy * y))
template <int NV, int DT>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const void* __restrict__ y,
                                                         const void* __restrict__ dy,
                                                         void* __restrict__ dx, int rows, int N,
                                                         float scale) {
  typedef IO8<DT> io;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = N >> 3;
  const size_t base = (size_t)row * N;
  float yv[NV][8], dv[NV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * 64 + lane;
    if (vi < nvec) {
      const typename io::R a = io::ld(y, (long long)(base >> 3) + vi);
      const typename io::R b = io::ld(dy, (long long)(base >> 3) + vi);
#pragma unroll
      for (int j = 0; j < 8; ++j) { yv[i][j] = io::get(a, j); dv[i][j] = io::get(b, j); s += yv[i][j] * dv[i][j]; }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { yv[i][j] = 0.f; dv[i][j] = 0.f; }
    }
  }
  s = wave_sum(s);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * 64 + lane;
    if (vi < nvec) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = scale * yv[i][j] * (dv[i][j] - s);
      io::st(dx, (long long)(base >> 3) + vi, o);
    }
  }
}

// Dropout with stateless hash mask (mask regenerated in backward from seed/offset).
template <int DT>
__global__ __launch_bounds__(256) void dropout_kernel(const void* __restrict__ x,
                                                     void* __restrict__ y, long long n8, float p,
                                                     uint64_t seed, uint64_t offset) {
  typedef IO8<DT> io;
  const float ks = 1.f / (1.f - p);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const typename io::R r = io::ld(x, i);
    float u[8], o[8];
    hash_uniform8(seed, offset, (uint64_t)i * 8, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = u[j] >= p ? io::get(r, j) * ks : 0.f;
    io::st(y, i, o);
  }
}

}  // namespace

// dtype codes of the entry points below: 0 bf16, 1 fp16, 2 f32 (the fp16 flag of older callers)
#define DT_SWITCH(dt, CALL)                                     \
  switch (dt) {                                                 \
    case DT_BF16: { constexpr int D_ = DT_BF16; CALL; } break;  \
    case DT_F16: { constexpr int D_ = DT_F16; CALL; } break;    \
    case DT_F32: { constexpr int D_ = DT_F32; CALL; } break;    \
    default: return (int)hipErrorInvalidValue;                  \
  }

PIAMD_EXPORT int piamd_bias_act_fwd(int dt, int act, const void* x, const void* bias, void* y, void* pre,
                                    long long n, int N, hipStream_t stream) {
  if (n == 0) return 0;
  if (n % 8 || N % 8) return (int)hipErrorInvalidValue;
  const long long n8 = n / 8;
  const int grid = stride_grid(n8, 256);
#define BAF(A)                                                                                     \
  case A:                                                                                          \
    DT_SWITCH(dt, hipLaunchKernelGGL((bias_act_fwd_kernel<A, D_>), dim3(grid), dim3(256), 0, stream, \
                                     x, bias, y, pre, n8, N));                                     \
    break;
  switch (act) { BAF(0) BAF(1) BAF(2) BAF(3) BAF(4) default: return (int)hipErrorInvalidValue; }
#undef BAF
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_bias_act_bwd_grid(int rows) {
  int g = rows < 256 ? rows : 256;
  return g < 1 ? 1 : g;
}

// part: f32 [N] workspace (zeroed here) — needed when dbias != null. dbias in the element type.
PIAMD_EXPORT int piamd_bias_act_bwd(int dt, int act, const void* dy, const void* h, const void* bias,
                                    void* dx, void* dbias, float* part, int rows, int N,
                                    int accumulate, hipStream_t stream) {
  if (rows == 0) return 0;
  if (N % 8) return (int)hipErrorInvalidValue;
  const int G = piamd_bias_act_bwd_grid(rows);
  dim3 grid(G, (N / 8 + 255) / 256);
#define BAB(A)                                                                                   \
  case A:                                                                                        \
    DT_SWITCH(dt, hipLaunchKernelGGL((bias_act_bwd_kernel<A, D_>), grid, dim3(256), 0, stream,  \
                                     dy, h, bias, dx, dbias ? part : nullptr, rows, N));         \
    break;
  if (dbias) (void)hipMemsetAsync(part, 0, sizeof(float) * N, stream);
  switch (act) { BAB(0) BAB(1) BAB(2) BAB(3) BAB(4) default: return (int)hipErrorInvalidValue; }
#undef BAB
  if (dbias)
    DT_SWITCH(dt, hipLaunchKernelGGL((colsum16_kernel<D_>), dim3((N + 63) / 64), dim3(256), 0, stream, part, 1,
                                     N, dbias, accumulate));
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_softmax_fwd(int dt, const void* x, const void* mask, int mask_rows, int causal_q,
                                   void* y, int rows, int N, float scale, hipStream_t stream) {
  if (rows == 0) return 0;
  if (N % 8 || N > 4096) return (int)hipErrorInvalidValue;
  const int nv = (N / 8 + 63) / 64;
  dim3 grid((rows + 3) / 4);
#define SMF(NVV, REAL)                                                                           \
  case REAL:                                                                                     \
    DT_SWITCH(dt, hipLaunchKernelGGL((softmax_fwd_kernel<NVV, D_>), grid, dim3(256), 0, stream, \
                                     x, mask, mask_rows > 0 ? mask_rows : 1, causal_q, y, rows, N, scale)); \
    break;
  switch (nv) { SMF(1, 1) SMF(2, 2) SMF(4, 3) SMF(4, 4) SMF(8, 5) SMF(8, 6) SMF(8, 7) SMF(8, 8)
    default: return (int)hipErrorInvalidValue; }
#undef SMF
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_softmax_bwd(int dt, const void* y, const void* dy, void* dx, int rows, int N,
                                   float scale, hipStream_t stream) {
  if (rows == 0) return 0;
  if (N % 8 || N > 4096) return (int)hipErrorInvalidValue;
  const int nv = (N / 8 + 63) / 64;
  dim3 grid((rows + 3) / 4);
#define SMB(NVV, REAL)                                                                           \
  case REAL:                                                                                     \
    DT_SWITCH(dt, hipLaunchKernelGGL((softmax_bwd_kernel<NVV, D_>), grid, dim3(256), 0, stream, \
                                     y, dy, dx, rows, N, scale));                                \
    break;
  switch (nv) { SMB(1, 1) SMB(2, 2) SMB(4, 3) SMB(4, 4) SMB(8, 5) SMB(8, 6) SMB(8, 7) SMB(8, 8)
    default: return (int)hipErrorInvalidValue; }
#undef SMB
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_dropout(int dt, const void* x, void* y, long long n, float p, uint64_t seed,
                               uint64_t offset, hipStream_t stream) {
  if (n == 0) return 0;
  if (n % 8) return (int)hipErrorInvalidValue;
  const int grid = stride_grid(n / 8, 256);
  DT_SWITCH(dt, hipLaunchKernelGGL((dropout_kernel<D_>), dim3(grid), dim3(256), 0, stream, x, y, n / 8, p, seed,
                                   offset));
  return (int)hipGetLastError();
}
#undef DT_SWITCH

// ---------------------------------------------------------------------------------------------
// 2-D bf16 transpose dst[C][R] = src[R][C] (weight re-layout for the K-contiguous forward GEMM).
// 64x64 tile per 256-thread block: 16-B coalesced row loads → LDS (row stride 66 elements = 33
// dwords, so the column gather of the store phase spreads over distinct banks) → 16-B coalesced
// stores of the transposed rows. Requires R % 8 == 0 and C % 8 == 0 (tails masked per 8-group).
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const bf16_t* __restrict__ src,
                                                             bf16_t* __restrict__ dst, int R,
                                                             int C) {
  __shared__ bf16_t tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64, t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = it * 256 + t, row = idx >> 3, cg = idx & 7;
    const int r = r0 + row, c = c0 + cg * 8;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < R && c < C) v = *(const u16x8*)(src + (size_t)r * C + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[row][cg * 8 + j] = v[j];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = it * 256 + t, orow = idx >> 3, og = idx & 7;
    const int oc = c0 + orow, orr = r0 + og * 8;  // dst row = source column, dst cols = source rows
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tile[og * 8 + j][orow];
    if (oc < C && orr < R) *(u16x8*)(dst + (size_t)oc * R + orr) = v;
  }
}

PIAMD_EXPORT int piamd_transpose_bf16(const void* src, void* dst, int R, int C,
                                      hipStream_t stream) {
  if (R == 0 || C == 0) return 0;
  if (R % 8 || C % 8) return (int)hipErrorInvalidValue;
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, stream, (const bf16_t*)src,
                     (bf16_t*)dst, R, C);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// fp32 GEMM operands as bf16 split products (ops/gemm.py gemm_nt_f32 / wgrad_f32): t = hi + lo
// (hi = bf16(t), lo = bf16(t − hi)), written as THREE segments of one bf16 operand so that
// x·w ≈ x_hi·w_hi + x_lo·w_hi + x_hi·w_lo is ONE bf16 MFMA GEMM with an f32 result ("hlh" on
// the left operand, "hhl" on the right). `lo_mask` bit s: segment s holds lo. axis 0: segments
// side by side along the row (dst[r][s·Cp + c], Cp ≥ C zero-padded: the reduction dim of a
// K-contiguous operand); axis 1: stacked along rows (dst[s·Rp + r][c], rows ≥ R zero: the
// reduction dim of a weight-gradient operand). One pass: 4 B read, 6 B written per element.
__global__ void split3_f32_kernel(const float* __restrict__ src, long long ld, bf16_t* __restrict__ dst, int R,
                                  int C, int Rp, int Cp, int lo_mask, int axis) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // one 8-column group
  const int groups = Cp / 8;
  if (i >= (long long)Rp * groups) return;
  const int r = (int)(i / groups), c0 = (int)(i % groups) * 8;
  u16x8 hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    const float v = (r < R && c < C) ? src[(long long)r * ld + c] : 0.f;
    const bf16_t h = f2bf(v);
    hi[j] = h;
    lo[j] = f2bf(v - bf2f(h));
  }
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const long long o = axis == 0 ? (long long)r * 3 * Cp + (long long)s * Cp + c0
                                  : ((long long)s * Rp + r) * Cp + c0;
    *(u16x8*)(dst + o) = ((lo_mask >> s) & 1) ? lo : hi;
  }
}

PIAMD_EXPORT int piamd_split3_f32(const void* src, long long ld, void* dst, int R, int C, int Rp, int Cp,
                                  int lo_mask, int axis, hipStream_t stream) {
  if (Rp == 0 || Cp == 0) return 0;
  if (Cp % 8 || Rp < R || Cp < C || (axis != 0 && axis != 1)) return (int)hipErrorInvalidValue;
  const long long n = (long long)Rp * (Cp / 8);
  hipLaunchKernelGGL(split3_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const float*)src, ld, (bf16_t*)dst, R, C, Rp, Cp, lo_mask, axis);
  return (int)hipGetLastError();
}
