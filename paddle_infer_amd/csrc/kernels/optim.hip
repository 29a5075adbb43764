// Optimizer kernels over FLAT parameter/gradient buffers.
//
// Parity: reference `paddle/phi/kernels/gpu/adamw_kernel.cu`, `adam_kernel.cu`,
// `merged_adam_kernel.cu`, `sgd_kernel.cu`, `momentum_kernel.cu`, and the global-norm clip in
// `python/paddle/nn/clip.py:ClipGradByGlobalNorm` (squared_l2_norm + sum + clip).
//
// MI355X design: the framework keeps every trainable tensor of a dtype/decay class as a view
// into ONE flat buffer (fp32 master, fp32 m, fp32 v, bf16 model copy, bf16/fp32 grad). The update
// is therefore a single grid-stride streaming kernel per class (no per-tensor launches, no
// multi-tensor-apply chunk tables), 16 B vector accesses, and the bf16 model copy is written in
// the same pass. The clip coefficient is read from device memory so the step needs no host sync
// and can be captured in a hipGraph.
#include "common.h"

namespace {

template <bool GRAD_BF16, bool HAS_MODEL>
__global__ __launch_bounds__(256) void adamw_flat_kernel(
    float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
    const void* __restrict__ grad, bf16_t* __restrict__ model, long long n, float lr,
    const float* __restrict__ lr_ptr, float beta1, float beta2, float eps, float wd, float bc1,
    float bc2_sqrt, const float* __restrict__ grad_scale, float static_grad_scale) {
  const float gs = static_grad_scale * (grad_scale ? *grad_scale : 1.f);
  const float lr_ = lr_ptr ? *lr_ptr : lr;
  const float step = lr_ * bc2_sqrt / bc1;   // lr * sqrt(1-b2^t) / (1-b1^t)
  const float eps_hat = eps * bc2_sqrt;
  const float decay = 1.f - lr_ * wd;
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
    f32x4 mv = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
    float g[4];
    if (GRAD_BF16) {
      u16x4 gr = reinterpret_cast<const u16x4*>(grad)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = bf2f(gr[j]);
    } else {
      f32x4 gr = reinterpret_cast<const f32x4*>(grad)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = gr[j];
    }
    u16x4 mo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = g[j] * gs;
      float pj = pv[j] * decay;
      float mj = beta1 * mv[j] + (1.f - beta1) * gj;
      float vj = beta2 * vv[j] + (1.f - beta2) * gj * gj;
      pj -= step * mj / (sqrtf(vj) + eps_hat);
      pv[j] = pj; mv[j] = mj; vv[j] = vj;
      mo[j] = f2bf(pj);
    }
    reinterpret_cast<f32x4*>(p)[i] = pv;
    reinterpret_cast<f32x4*>(m)[i] = mv;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    if (HAS_MODEL) reinterpret_cast<u16x4*>(model)[i] = mo;
  }
  // tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    long long i = (n4 << 2) + threadIdx.x;
    float gj = (GRAD_BF16 ? bf2f(((const bf16_t*)grad)[i]) : ((const float*)grad)[i]) * gs;
    float pj = p[i] * decay;
    float mj = beta1 * m[i] + (1.f - beta1) * gj;
    float vj = beta2 * v[i] + (1.f - beta2) * gj * gj;
    pj -= step * mj / (sqrtf(vj) + eps_hat);
    p[i] = pj; m[i] = mj; v[i] = vj;
    if (HAS_MODEL) model[i] = f2bf(pj);
  }
}

template <bool GRAD_BF16>
__global__ __launch_bounds__(256) void sumsq_kernel(const void* __restrict__ x, long long n,
                                                   float* __restrict__ partial) {
  float s = 0.f;
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    if (GRAD_BF16) {
      u16x4 g = reinterpret_cast<const u16x4*>(x)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) { float f = bf2f(g[j]); s += f * f; }
    } else {
      f32x4 g = reinterpret_cast<const f32x4*>(x)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) s += g[j] * g[j];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    long long i = (n4 << 2) + threadIdx.x;
    float f = GRAD_BF16 ? bf2f(((const bf16_t*)x)[i]) : ((const float*)x)[i];
    s += f * f;
  }
  __shared__ float red[4];
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ void sum_partials_kernel(const float* __restrict__ partial, int G,
                                    float* __restrict__ out, int accumulate) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < G; i += blockDim.x) s += partial[i];
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) *out = accumulate ? *out + s : s;
}

template <bool GRAD_BF16, bool HAS_MODEL>
__global__ __launch_bounds__(256) void momentum_flat_kernel(
    float* __restrict__ p, float* __restrict__ vel, const void* __restrict__ grad,
    bf16_t* __restrict__ model, long long n, float lr, const float* __restrict__ lr_ptr, float mu,
    float wd, int nesterov, const float* __restrict__ grad_scale) {
  const float gs = grad_scale ? *grad_scale : 1.f;
  const float lr_ = lr_ptr ? *lr_ptr : lr;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float g = (GRAD_BF16 ? bf2f(((const bf16_t*)grad)[i]) : ((const float*)grad)[i]) * gs;
    g += wd * p[i];
    float vv = mu * vel[i] + g;
    vel[i] = vv;
    float pj = p[i] - lr_ * (nesterov ? g + mu * vv : vv);
    p[i] = pj;
    if (HAS_MODEL) model[i] = f2bf(pj);
  }
}

// ---- multi-tensor (merged) optimizer update -----------------------------------------------------
// Parity: reference `phi/kernels/gpu/merged_momentum_kernel.cu`, `merged_adam_kernel.cu` and the
// `use_multi_tensor` path of paddle.optimizer.{Momentum, Adam, AdamW}: every parameter of the
// optimizer updated in ONE launch. Per tensor t the table holds {p, grad, s1, s2, n, grad_dtype}
// (int64) and {wd, lr_mult} (f32); chunk_off[t] = first 2048-element chunk of tensor t. Workgroups
// grid-stride over chunks and find their tensor by binary search over chunk_off (the table lives
// on the device, rebuilt only when a pointer changes).
constexpr int MT_CHUNK = 2048;
enum { MT_SGD = 0, MT_MOMENTUM = 1, MT_ADAM = 2, MT_ADAMW = 3 };

struct MtHyper {
  float lr, mu, beta1, beta2, eps, bc1, bc2_sqrt;
  int nesterov;
};

template <int OP>
__global__ __launch_bounds__(256) void multi_tensor_kernel(const long long* __restrict__ meta,
                                                           const float* __restrict__ fmeta,
                                                           const int* __restrict__ chunk_off,
                                                           int T, MtHyper h,
                                                           const float* __restrict__ grad_scale) {
  const int total = chunk_off[T];
  const float gs = grad_scale ? *grad_scale : 1.f;
  for (int c = blockIdx.x; c < total; c += gridDim.x) {
    int lo = 0, hi = T - 1;
    while (lo < hi) {  // last t with chunk_off[t] <= c
      const int mid = (lo + hi + 1) >> 1;
      if (chunk_off[mid] <= c) lo = mid; else hi = mid - 1;
    }
    const int t = lo;
    float* p = (float*)meta[t * 6 + 0];
    const void* g = (const void*)meta[t * 6 + 1];
    float* s1 = (float*)meta[t * 6 + 2];
    float* s2 = (float*)meta[t * 6 + 3];
    const long long n = meta[t * 6 + 4];
    const int gbf = (int)meta[t * 6 + 5];
    const float wd = fmeta[t * 2 + 0], lr = h.lr * fmeta[t * 2 + 1];
    const long long base = (long long)(c - chunk_off[t]) * MT_CHUNK;
    const long long end = min(base + MT_CHUNK, n);
    for (long long i = base + threadIdx.x; i < end; i += 256) {
      float gi = (gbf ? bf2f(((const bf16_t*)g)[i]) : ((const float*)g)[i]) * gs;
      float pi = p[i];
      if (OP == MT_SGD) {
        pi -= lr * (gi + wd * pi);
      } else if (OP == MT_MOMENTUM) {
        gi += wd * pi;
        const float v = h.mu * s1[i] + gi;
        s1[i] = v;
        pi -= lr * (h.nesterov ? gi + h.mu * v : v);
      } else {
        if (OP == MT_ADAM) gi += wd * pi;
        else pi *= 1.f - lr * wd;
        const float m = h.beta1 * s1[i] + (1.f - h.beta1) * gi;
        const float v = h.beta2 * s2[i] + (1.f - h.beta2) * gi * gi;
        s1[i] = m;
        s2[i] = v;
        pi -= (lr * h.bc2_sqrt / h.bc1) * m / (sqrtf(v) + h.eps * h.bc2_sqrt);
      }
      p[i] = pi;
    }
  }
}

}  // namespace

// AdamW over flat buffers. p/m/v f32 [n]; grad bf16 (grad_dtype=1) or f32 (0); model bf16 copy
// (nullable). bc1 = 1 - beta1^t, bc2_sqrt = sqrt(1 - beta2^t). grad_scale: optional device scalar
// multiplying the grad (global-norm clip coefficient, 1/loss_scale); static_grad_scale: host one.
PIAMD_EXPORT int piamd_adamw_flat(float* p, float* m, float* v, const void* grad, int grad_dtype,
                                  void* model, long long n, float lr, const float* lr_ptr,
                                  float beta1, float beta2, float eps, float wd, float bc1,
                                  float bc2_sqrt, const float* grad_scale,
                                  float static_grad_scale, hipStream_t stream) {
  if (n == 0) return 0;
  if (((uintptr_t)p | (uintptr_t)m | (uintptr_t)v) & 15) return (int)hipErrorInvalidValue;
  const int grid = stride_grid((n + 3) / 4, 256);
#define ADAMW(GB, HM)                                                                            \
  hipLaunchKernelGGL((adamw_flat_kernel<GB, HM>), dim3(grid), dim3(256), 0, stream, p, m, v,    \
                     grad, (bf16_t*)model, n, lr, lr_ptr, beta1, beta2, eps, wd, bc1, bc2_sqrt, \
                     grad_scale, static_grad_scale)
  if (grad_dtype) { if (model) ADAMW(true, true); else ADAMW(true, false); }
  else { if (model) ADAMW(false, true); else ADAMW(false, false); }
#undef ADAMW
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_momentum_flat(float* p, float* vel, const void* grad, int grad_dtype,
                                     void* model, long long n, float lr, const float* lr_ptr,
                                     float mu, float wd, int nesterov, const float* grad_scale,
                                     hipStream_t stream) {
  if (n == 0) return 0;
  const int grid = stride_grid(n, 256);
#define MOM(GB, HM)                                                                               \
  hipLaunchKernelGGL((momentum_flat_kernel<GB, HM>), dim3(grid), dim3(256), 0, stream, p, vel,   \
                     grad, (bf16_t*)model, n, lr, lr_ptr, mu, wd, nesterov, grad_scale)
  if (grad_dtype) { if (model) MOM(true, true); else MOM(true, false); }
  else { if (model) MOM(false, true); else MOM(false, false); }
#undef MOM
  return (int)hipGetLastError();
}

// Sum of squares of a flat buffer → *out (f32 device scalar), optionally accumulated.
// partial: workspace of >= 2048 floats.
PIAMD_EXPORT int piamd_sumsq(const void* x, int dtype, long long n, float* partial, float* out,
                             int accumulate, hipStream_t stream) {
  if (n == 0) {
    if (!accumulate) hipMemsetAsync(out, 0, sizeof(float), stream);
    return (int)hipGetLastError();
  }
  const int grid = stride_grid((n + 3) / 4, 256);
  if (dtype)
    hipLaunchKernelGGL((sumsq_kernel<true>), dim3(grid), dim3(256), 0, stream, x, n, partial);
  else
    hipLaunchKernelGGL((sumsq_kernel<false>), dim3(grid), dim3(256), 0, stream, x, n, partial);
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, stream, partial, grid, out,
                     accumulate);
  return (int)hipGetLastError();
}

// Merged update of T tensors (op: 0 SGD, 1 Momentum, 2 Adam (L2 decay), 3 AdamW (decoupled)).
// meta [T][6] int64 device table {p, grad, s1, s2, n, grad_is_bf16}; fmeta [T][2] f32 {wd,
// lr_mult}; chunk_off [T+1] int32 (2048-element chunks); grad_scale: optional device scalar.
PIAMD_EXPORT int piamd_multi_tensor_update(int op, const long long* meta, const float* fmeta,
                                           const int* chunk_off, int T, int total_chunks, float lr,
                                           float mu, int nesterov, float beta1, float beta2,
                                           float eps, float bc1, float bc2_sqrt,
                                           const float* grad_scale, hipStream_t stream) {
  if (T <= 0 || total_chunks <= 0) return 0;
  MtHyper h{lr, mu, beta1, beta2, eps, bc1, bc2_sqrt, nesterov};
  const int grid = total_chunks < 2048 ? total_chunks : 2048;
#define MT(OP) hipLaunchKernelGGL((multi_tensor_kernel<OP>), dim3(grid), dim3(256), 0, stream, meta, \
                                  fmeta, chunk_off, T, h, grad_scale)
  switch (op) {
    case MT_SGD: MT(MT_SGD); break;
    case MT_MOMENTUM: MT(MT_MOMENTUM); break;
    case MT_ADAM: MT(MT_ADAM); break;
    case MT_ADAMW: MT(MT_ADAMW); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef MT
  return (int)hipGetLastError();
}
