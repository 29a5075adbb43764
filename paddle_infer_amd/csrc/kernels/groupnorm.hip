// Group normalisation (and instance normalisation = one channel per group), NCHW-contiguous
// activations, bf16 / fp16 / f32 I/O with f32 statistics, forward + backward.
//
// Parity: reference `phi/kernels/gpu/group_norm_kernel.cu` / `group_norm_grad_kernel.cu` and
// `instance_norm_kernel.cu` (y = (x − μ_g)·rstd_g·γ_c + β_c over the (C/G)·H·W elements of a
// group; dx = rstd·(dŷ − (Σdŷ + x̂·Σdŷx̂)/L) with dŷ = dy·γ; dγ_c = Σ dy·x̂, dβ_c = Σ dy).
//
// MI355X design: every reduction is per (n, c) PLANE — one workgroup walks a contiguous H·W run
// with 16-B loads — and the group / channel combines are tiny deterministic loops:
//   forward:  plane (count, mean, M2) with a per-plane shift (first element: no E[x²]−E[x]²
//             cancellation), Chan-merged per (n, g) into (mean, rstd); one elementwise apply.
//   backward: plane (Σdy, Σdy·x̂) with the group statistics → per (n, g) the two sums over the
//             group's channels weighted by γ, per channel dγ / dβ summed over n in a fixed order;
//             one elementwise pass for dx. No atomics: bitwise deterministic.
#include "common.h"

namespace {

template <int DT> struct GIO;
template <> struct GIO<0> {  // f32
  typedef float T;
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
};
template <> struct GIO<1> {  // bf16
  typedef bf16_t T;
  static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(bf16_t* p, float v) { *p = f2bf(v); }
};
template <> struct GIO<2> {  // fp16
  typedef unsigned short T;
  static __device__ __forceinline__ float ld(const unsigned short* p) { return h2f<true>(*p); }
  static __device__ __forceinline__ void st(unsigned short* p, float v) { *p = f2h<true>(v); }
};

// 8 consecutive elements from a 16-B (16-bit types) or 2 × 16-B (f32) aligned address.
template <int DT>
__device__ __forceinline__ void ld8(const typename GIO<DT>::T* p, float (&v)[8]) {
  if constexpr (DT == 0) {
    const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  } else {
    const u16x8 u = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = DT == 1 ? bf2f(u[j]) : h2f<true>(u[j]);
  }
}

template <int DT>
__device__ __forceinline__ void st8(typename GIO<DT>::T* p, const float (&v)[8]) {
  if constexpr (DT == 0) {
    f32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[4 + j]; }
    reinterpret_cast<f32x4*>(p)[0] = a;
    reinterpret_cast<f32x4*>(p)[1] = b;
  } else {
    u16x8 u;
#pragma unroll
    for (int j = 0; j < 8; ++j) u[j] = DT == 1 ? f2bf(v[j]) : f2h<true>(v[j]);
    *reinterpret_cast<u16x8*>(p) = u;
  }
}

// Sum of two floats over the 256-thread workgroup.
__device__ __forceinline__ void wg_sum2(float& a, float& b) {
  __shared__ float ra[4], rb[4];
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { ra[w] = a; rb[w] = b; }
  __syncthreads();
  a = ra[0] + ra[1] + ra[2] + ra[3];
  b = rb[0] + rb[1] + rb[2] + rb[3];
  __syncthreads();
}

// ------------------------------------------------------------------------------------ forward
// grid = N·C planes; part[plane] = (count, mean, M2) of the plane's HW elements.
template <int DT>
__global__ __launch_bounds__(256) void gn_plane_stats(const typename GIO<DT>::T* __restrict__ x,
                                                      long long HW, float* __restrict__ part) {
  const typename GIO<DT>::T* p = x + (long long)blockIdx.x * HW;
  const float sh = GIO<DT>::ld(p);
  float s = 0.f, q = 0.f;
  const bool vec = (HW % 8) == 0;
  if (vec) {
    for (long long i = threadIdx.x * 8LL; i < HW; i += 256 * 8) {
      float v[8];
      ld8<DT>(p + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[j] - sh; s += d; q += d * d; }
    }
  } else {
    for (long long i = threadIdx.x; i < HW; i += 256) {
      const float d = GIO<DT>::ld(p + i) - sh;
      s += d;
      q += d * d;
    }
  }
  wg_sum2(s, q);
  if (threadIdx.x == 0) {
    const float n = (float)HW;
    part[3 * blockIdx.x + 0] = n;
    part[3 * blockIdx.x + 1] = sh + s / n;
    part[3 * blockIdx.x + 2] = fmaxf(q - s * s / n, 0.f);
  }
}

// one thread per (n, g): Chan merge of the group's CG planes → mean, rstd.
__global__ __launch_bounds__(256) void gn_group_finalize(const float* __restrict__ part, int NG, int CG,
                                                         float eps, float* __restrict__ mean,
                                                         float* __restrict__ rstd) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= NG) return;
  float n = 0.f, m = 0.f, m2 = 0.f;
  for (int c = 0; c < CG; ++c) {
    const float* e = part + 3LL * ((long long)i * CG + c);
    const float nb = e[0], mb = e[1];
    if (nb == 0.f) continue;
    const float nn = n + nb, d = mb - m;
    m += d * nb / nn;
    m2 += e[2] + d * d * n * nb / nn;
    n = nn;
  }
  mean[i] = m;
  rstd[i] = rsqrtf(m2 / fmaxf(n, 1.f) + eps);
}

// y = (x − μ)·rstd·γ_c + β_c (γ / β f32, nullable); grid-stride over planes × HW.
template <int DT>
__global__ __launch_bounds__(256) void gn_apply(const typename GIO<DT>::T* __restrict__ x,
                                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                                typename GIO<DT>::T* __restrict__ y, long long HW, int C,
                                                int CG, int PB) {
  const long long plane = blockIdx.x / PB;
  const int blk = blockIdx.x % PB;
  const int c = (int)(plane % C);
  const long long g = plane / CG;  // (n·C + c) / CG = n·G + c / CG
  const float mu = mean[g], rs = rstd[g];
  const float a = rs * (gamma ? gamma[c] : 1.f), b = (beta ? beta[c] : 0.f) - mu * a;
  const typename GIO<DT>::T* px = x + plane * HW;
  typename GIO<DT>::T* py = y + plane * HW;
  if ((HW % 8) == 0) {
    for (long long i = (blk * 256LL + threadIdx.x) * 8; i < HW; i += PB * 256LL * 8) {
      float v[8];
      ld8<DT>(px + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] * a + b;
      st8<DT>(py + i, v);
    }
  } else {
    for (long long i = blk * 256LL + threadIdx.x; i < HW; i += PB * 256LL)
      GIO<DT>::st(py + i, GIO<DT>::ld(px + i) * a + b);
  }
}

// ----------------------------------------------------------------------------------- backward
// grid = N·C planes; part[plane] = (Σ dy, Σ dy·x̂) with the group's statistics.
template <int DT>
__global__ __launch_bounds__(256) void gn_bwd_plane(const typename GIO<DT>::T* __restrict__ dy,
                                                    const typename GIO<DT>::T* __restrict__ x,
                                                    const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, long long HW,
                                                    int CG, float* __restrict__ part) {
  const long long plane = blockIdx.x, g = plane / CG;
  const float mu = mean[g], rs = rstd[g];
  const typename GIO<DT>::T* pd = dy + plane * HW;
  const typename GIO<DT>::T* px = x + plane * HW;
  float s1 = 0.f, s2 = 0.f;
  if ((HW % 8) == 0) {
    for (long long i = threadIdx.x * 8LL; i < HW; i += 256 * 8) {
      float d[8], v[8];
      ld8<DT>(pd + i, d);
      ld8<DT>(px + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s1 += d[j]; s2 += d[j] * (v[j] - mu) * rs; }
    }
  } else {
    for (long long i = threadIdx.x; i < HW; i += 256) {
      const float d = GIO<DT>::ld(pd + i);
      s1 += d;
      s2 += d * (GIO<DT>::ld(px + i) - mu) * rs;
    }
  }
  wg_sum2(s1, s2);
  if (threadIdx.x == 0) {
    part[2 * plane] = s1;
    part[2 * plane + 1] = s2;
  }
}

// threads [0, NG): per (n, g) the γ-weighted sums A = Σ_c γ_c Σdy, B = Σ_c γ_c Σdy·x̂ → coef
// (A / L, B / L); threads [NG, NG + C): per channel dγ = Σ_n Σdy·x̂, dβ = Σ_n Σdy (fixed order).
__global__ __launch_bounds__(256) void gn_bwd_finalize(const float* __restrict__ part, int N, int C, int CG,
                                                       float invL, const float* __restrict__ gamma,
                                                       float* __restrict__ coef, float* __restrict__ dgamma,
                                                       float* __restrict__ dbeta) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int G = C / CG, NG = N * G;
  if (i < NG) {
    const int n = i / G, g = i % G;
    float A = 0.f, B = 0.f;
    for (int k = 0; k < CG; ++k) {
      const int c = g * CG + k;
      const float w = gamma ? gamma[c] : 1.f;
      const float* e = part + 2LL * ((long long)n * C + c);
      A += w * e[0];
      B += w * e[1];
    }
    coef[2 * i] = A * invL;
    coef[2 * i + 1] = B * invL;
  } else if (i < NG + C) {
    const int c = i - NG;
    float s1 = 0.f, s2 = 0.f;
    for (int n = 0; n < N; ++n) {
      const float* e = part + 2LL * ((long long)n * C + c);
      s1 += e[0];
      s2 += e[1];
    }
    if (dgamma) dgamma[c] = s2;
    if (dbeta) dbeta[c] = s1;
  }
}

// dx = rstd·(dy·γ_c − A/L − x̂·B/L)
template <int DT>
__global__ __launch_bounds__(256) void gn_bwd_apply(const typename GIO<DT>::T* __restrict__ dy,
                                                    const typename GIO<DT>::T* __restrict__ x,
                                                    const float* __restrict__ mean, const float* __restrict__ rstd,
                                                    const float* __restrict__ gamma, const float* __restrict__ coef,
                                                    typename GIO<DT>::T* __restrict__ dx, long long HW, int C,
                                                    int CG, int PB) {
  const long long plane = blockIdx.x / PB, g = plane / CG;
  const int blk = blockIdx.x % PB;
  const int c = (int)(plane % C);
  const float mu = mean[g], rs = rstd[g], w = gamma ? gamma[c] : 1.f;
  const float cA = coef[2 * g], cB = coef[2 * g + 1];
  const typename GIO<DT>::T* pd = dy + plane * HW;
  const typename GIO<DT>::T* px = x + plane * HW;
  typename GIO<DT>::T* po = dx + plane * HW;
  if ((HW % 8) == 0) {
    for (long long i = (blk * 256LL + threadIdx.x) * 8; i < HW; i += PB * 256LL * 8) {
      float d[8], v[8];
      ld8<DT>(pd + i, d);
      ld8<DT>(px + i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = rs * (d[j] * w - cA - (v[j] - mu) * rs * cB);
      st8<DT>(po + i, d);
    }
  } else {
    for (long long i = blk * 256LL + threadIdx.x; i < HW; i += PB * 256LL) {
      const float v = GIO<DT>::ld(px + i);
      GIO<DT>::st(po + i, rs * (GIO<DT>::ld(pd + i) * w - cA - (v - mu) * rs * cB));
    }
  }
}

// workgroups per plane of the elementwise passes (1-D grid of planes × this)
inline int plane_blocks(long long HW) {
  const long long per = (HW + 2047) / 2048;  // ≈ 2048 elements per workgroup
  return (int)(per < 1 ? 1 : (per > 64 ? 64 : per));
}

template <int DT>
int fwd(const void* x, void* y, const float* gamma, const float* beta, float* mean, float* rstd, float* ws,
        int N, int C, long long HW, int G, float eps, hipStream_t st) {
  typedef typename GIO<DT>::T T;
  const int CG = C / G, NC = N * C, NG = N * G;
  hipLaunchKernelGGL((gn_plane_stats<DT>), dim3(NC), dim3(256), 0, st, (const T*)x, HW, ws);
  hipLaunchKernelGGL(gn_group_finalize, dim3((NG + 255) / 256), dim3(256), 0, st, ws, NG, CG, eps, mean, rstd);
  const int PB = plane_blocks(HW);
  hipLaunchKernelGGL((gn_apply<DT>), dim3((unsigned)NC * PB), dim3(256), 0, st, (const T*)x, mean, rstd,
                     gamma, beta, (T*)y, HW, C, CG, PB);
  return (int)hipGetLastError();
}

template <int DT>
int bwd(const void* dy, const void* x, const float* gamma, const float* mean, const float* rstd, void* dx,
        float* dgamma, float* dbeta, float* ws, int N, int C, long long HW, int G, hipStream_t st) {
  typedef typename GIO<DT>::T T;
  const int CG = C / G, NC = N * C, NG = N * G;
  float* part = ws;              // [NC][2]
  float* coef = ws + 2LL * NC;   // [NG][2]
  hipLaunchKernelGGL((gn_bwd_plane<DT>), dim3(NC), dim3(256), 0, st, (const T*)dy, (const T*)x, mean, rstd,
                     HW, CG, part);
  hipLaunchKernelGGL(gn_bwd_finalize, dim3((NG + C + 255) / 256), dim3(256), 0, st, part, N, C, CG,
                     1.f / (float)((long long)CG * HW), gamma, coef, dgamma, dbeta);
  const int PB = plane_blocks(HW);
  if (dx)
    hipLaunchKernelGGL((gn_bwd_apply<DT>), dim3((unsigned)NC * PB), dim3(256), 0, st, (const T*)dy,
                       (const T*)x, mean, rstd, gamma, coef, (T*)dx, HW, C, CG, PB);
  return (int)hipGetLastError();
}

}  // namespace

// Floats of workspace both entry points need: max(3·N·C, 2·N·C + 2·N·G).
PIAMD_EXPORT long long piamd_group_norm_ws(int N, int C, int G) {
  const long long a = 3LL * N * C, b = 2LL * N * C + 2LL * N * G;
  return a > b ? a : b;
}

// dtype: 0 f32, 1 bf16, 2 fp16. x / y [N][C][HW] contiguous (16-B aligned), C % G == 0; gamma /
// beta f32 [C] (nullable); mean / rstd f32 [N·G] out.
PIAMD_EXPORT int piamd_group_norm_fwd(int dtype, const void* x, void* y, const float* gamma,
                                      const float* beta, float* mean, float* rstd, float* ws, int N,
                                      int C, long long HW, int G, float eps, hipStream_t st) {
  if (N <= 0 || C <= 0 || HW <= 0 || G <= 0 || C % G || dtype < 0 || dtype > 2 ||
      ((uintptr_t)x | (uintptr_t)y) % 16)
    return (int)hipErrorInvalidValue;
  if (dtype == 1) return fwd<1>(x, y, gamma, beta, mean, rstd, ws, N, C, HW, G, eps, st);
  if (dtype == 2) return fwd<2>(x, y, gamma, beta, mean, rstd, ws, N, C, HW, G, eps, st);
  return fwd<0>(x, y, gamma, beta, mean, rstd, ws, N, C, HW, G, eps, st);
}

// dx (nullable) and f32 dgamma / dbeta [C] (nullable) from dy, x and the forward's mean / rstd.
PIAMD_EXPORT int piamd_group_norm_bwd(int dtype, const void* dy, const void* x, const float* gamma,
                                      const float* mean, const float* rstd, void* dx, float* dgamma,
                                      float* dbeta, float* ws, int N, int C, long long HW, int G,
                                      hipStream_t st) {
  if (N <= 0 || C <= 0 || HW <= 0 || G <= 0 || C % G || dtype < 0 || dtype > 2 ||
      ((uintptr_t)dy | (uintptr_t)x | (uintptr_t)dx) % 16)
    return (int)hipErrorInvalidValue;
  if (dtype == 1) return bwd<1>(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, ws, N, C, HW, G, st);
  if (dtype == 2) return bwd<2>(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, ws, N, C, HW, G, st);
  return bwd<0>(dy, x, gamma, mean, rstd, dx, dgamma, dbeta, ws, N, C, HW, G, st);
}

// The elementwise pass alone: y = (x − mean[n·G + c / (C/G)])·rstd[·]·γ_c + β_c (InstanceNorm with
// running statistics passes mean 0 / rstd 1 and the folded per-channel scale / shift as γ / β).
PIAMD_EXPORT int piamd_group_norm_apply(int dtype, const void* x, void* y, const float* gamma,
                                        const float* beta, const float* mean, const float* rstd, int N,
                                        int C, long long HW, int G, hipStream_t st) {
  if (N <= 0 || C <= 0 || HW <= 0 || G <= 0 || C % G || dtype < 0 || dtype > 2 ||
      ((uintptr_t)x | (uintptr_t)y) % 16)
    return (int)hipErrorInvalidValue;
  const int PB = plane_blocks(HW), CG = C / G;
  const dim3 grid((unsigned)(N * C) * PB);
#define APPLY(D)                                                                                   \
  hipLaunchKernelGGL((gn_apply<D>), grid, dim3(256), 0, st, (const typename GIO<D>::T*)x, mean, rstd, \
                     gamma, beta, (typename GIO<D>::T*)y, HW, C, CG, PB)
  if (dtype == 1) APPLY(1);
  else if (dtype == 2) APPLY(2);
  else APPLY(0);
#undef APPLY
  return (int)hipGetLastError();
}
