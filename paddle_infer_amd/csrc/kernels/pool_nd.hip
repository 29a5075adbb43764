// Generic 1-D / 2-D / 3-D pooling (max / avg, fixed or adaptive windows) and linear / nearest
// resampling (interpolate) over N·C planes stored [N, C, D, H, W] (1-D and 2-D as D = H = 1 /
// D = 1), f32 / bf16 / fp16 with f32 arithmetic — forward and backward.
//
// Parity: reference `phi/kernels/funcs/pooling.cu` (Pool3dFunctor / MaxPool3dWithIndex, adaptive
// windows start = ⌊o·I/O⌋, end = ⌈(o+1)·I/O⌉, exclusive / inclusive averaging) and
// `phi/kernels/gpu/interpolate_kernel.cu` (nearest / linear / bilinear / trilinear, align_corners).
// The NHWC max-pool of the conv nets stays on pool.hip; this covers every other pooling layer
// (MaxPool1D/3D, AvgPool1D/2D/3D, AdaptiveAvg/MaxPool1D/2D/3D) and Upsample.
//
// Design: one thread per output element (W fastest: coalesced along rows). Backward passes are
// GATHERS (one thread per input element visits the few output windows that contain it) — no
// atomics, deterministic — except resampling, whose backward scatters bilinear weights with f32
// atomics into an f32 buffer (the weights overlap irregularly between output pixels).
#include "common.h"

namespace {

struct PoolArgs {
  int N, C;
  int I[3], O[3], K[3], S[3], P[3];  // D, H, W
  int mode;                          // 0 max, 1 avg
  int adaptive, exclusive, divisor;  // divisor > 0: divisor_override
};

template <int DT>
__device__ __forceinline__ float ld(const void* p, long long i) {
  if constexpr (DT == 0) return reinterpret_cast<const float*>(p)[i];
  else return h2f<DT == 2>(reinterpret_cast<const unsigned short*>(p)[i]);
}
template <int DT>
__device__ __forceinline__ void st(void* p, long long i, float v) {
  if constexpr (DT == 0) reinterpret_cast<float*>(p)[i] = v;
  else reinterpret_cast<unsigned short*>(p)[i] = f2h<DT == 2>(v);
}

// window of output o along axis a: [lo, hi) clamped to the input, and the unclamped extent used
// by inclusive averaging
__device__ __forceinline__ void window(const PoolArgs& g, int a, int o, int& lo, int& hi, int& span) {
  if (g.adaptive) {
    lo = (int)(((long long)o * g.I[a]) / g.O[a]);
    hi = (int)(((long long)(o + 1) * g.I[a] + g.O[a] - 1) / g.O[a]);
    span = hi - lo;
    return;
  }
  const int s0 = o * g.S[a] - g.P[a];
  const int e0 = min(s0 + g.K[a], g.I[a] + g.P[a]);
  span = e0 - s0;
  lo = max(s0, 0);
  hi = min(e0, g.I[a]);
}

__device__ __forceinline__ float divisor_of(const PoolArgs& g, const int lo[3], const int hi[3], const int sp[3]) {
  if (g.divisor > 0) return (float)g.divisor;
  if (g.exclusive || g.adaptive) return (float)((hi[0] - lo[0]) * (hi[1] - lo[1]) * (hi[2] - lo[2]));
  return (float)(sp[0] * sp[1] * sp[2]);
}

template <int DT>
__global__ __launch_bounds__(256) void pool_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                       int* __restrict__ idx, PoolArgs g, long long total) {
  const long long plane_in = (long long)g.I[0] * g.I[1] * g.I[2];
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    long long r = t;
    const int ow = (int)(r % g.O[2]);
    r /= g.O[2];
    const int oh = (int)(r % g.O[1]);
    r /= g.O[1];
    const int od = (int)(r % g.O[0]);
    const long long nc = r / g.O[0];
    int lo[3], hi[3], sp[3];
    window(g, 0, od, lo[0], hi[0], sp[0]);
    window(g, 1, oh, lo[1], hi[1], sp[1]);
    window(g, 2, ow, lo[2], hi[2], sp[2]);
    const long long base = nc * plane_in;
    if (g.mode == 0) {
      float m = -INFINITY;
      int mi = lo[0] * g.I[1] * g.I[2] + lo[1] * g.I[2] + lo[2];
      bool nan = false;
      for (int d = lo[0]; d < hi[0]; ++d)
        for (int h = lo[1]; h < hi[1]; ++h)
          for (int w = lo[2]; w < hi[2]; ++w) {
            const int fi = (d * g.I[1] + h) * g.I[2] + w;
            const float v = ld<DT>(x, base + fi);
            if (!nan && (v > m || v != v)) {
              m = v;
              mi = fi;
              nan = v != v;
            }
          }
      st<DT>(y, t, m);
      if (idx) idx[t] = mi;
    } else {
      float s = 0.f;
      for (int d = lo[0]; d < hi[0]; ++d)
        for (int h = lo[1]; h < hi[1]; ++h)
          for (int w = lo[2]; w < hi[2]; ++w) s += ld<DT>(x, base + (d * g.I[1] + h) * g.I[2] + w);
      st<DT>(y, t, s / divisor_of(g, lo, hi, sp));
    }
  }
}

// output-index range along axis a whose windows may contain input i
__device__ __forceinline__ void out_range(const PoolArgs& g, int a, int i, int& o0, int& o1) {
  if (g.adaptive) {
    o0 = max(0, (int)(((long long)i * g.O[a]) / g.I[a]) - 1);
    o1 = min(g.O[a] - 1, (int)(((long long)(i + 1) * g.O[a]) / g.I[a]) + 1);
    return;
  }
  const int num = i + g.P[a] - g.K[a] + 1;
  o0 = num <= 0 ? 0 : (num + g.S[a] - 1) / g.S[a];
  o1 = min(g.O[a] - 1, (i + g.P[a]) / g.S[a]);
}

template <int DT>
__global__ __launch_bounds__(256) void pool_bwd_kernel(const void* __restrict__ dy, const int* __restrict__ idx,
                                                       void* __restrict__ dx, PoolArgs g, long long total) {
  const long long plane_out = (long long)g.O[0] * g.O[1] * g.O[2];
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    long long r = t;
    const int w = (int)(r % g.I[2]);
    r /= g.I[2];
    const int h = (int)(r % g.I[1]);
    r /= g.I[1];
    const int d = (int)(r % g.I[0]);
    const long long nc = r / g.I[0];
    const int fi = (d * g.I[1] + h) * g.I[2] + w;
    int a0[3], a1[3];
    out_range(g, 0, d, a0[0], a1[0]);
    out_range(g, 1, h, a0[1], a1[1]);
    out_range(g, 2, w, a0[2], a1[2]);
    const int ii[3] = {d, h, w};
    float acc = 0.f;
    for (int od = a0[0]; od <= a1[0]; ++od)
      for (int oh = a0[1]; oh <= a1[1]; ++oh)
        for (int ow = a0[2]; ow <= a1[2]; ++ow) {
          const int oo[3] = {od, oh, ow};
          int lo[3], hi[3], sp[3];
          bool in = true;
#pragma unroll
          for (int a = 0; a < 3; ++a) {
            window(g, a, oo[a], lo[a], hi[a], sp[a]);
            in = in && ii[a] >= lo[a] && ii[a] < hi[a];
          }
          if (!in) continue;
          const long long o = nc * plane_out + ((long long)od * g.O[1] + oh) * g.O[2] + ow;
          if (g.mode == 0) {
            if (idx[o] == fi) acc += ld<DT>(dy, o);
          } else {
            acc += ld<DT>(dy, o) / divisor_of(g, lo, hi, sp);
          }
        }
    st<DT>(dx, t, acc);
  }
}

// ---------------------------------------------------------------------------------- resampling
struct InterpArgs {
  int N, C;
  int I[3], O[3];
  float scale[3];  // source step per output step: (I-1)/(O-1) with align_corners, else I/O or
                   // 1/scale_factor (computed by the caller in f32, as the reference does)
  int mode;        // 0 nearest, 1 linear (per-axis linear over the active axes)
  int align_corners;
};

// source coordinate of output o along axis a → (i0, i1, w1)
__device__ __forceinline__ void src_of(const InterpArgs& g, int a, int o, int& i0, int& i1, float& w1) {
  if (g.mode == 0) {  // nearest: ⌊o · scale⌋
    i0 = i1 = min((int)floorf((float)o * g.scale[a]), g.I[a] - 1);
    w1 = 0.f;
    return;
  }
  float s;
  if (g.align_corners) s = (float)o * g.scale[a];
  else s = fmaxf(((float)o + 0.5f) * g.scale[a] - 0.5f, 0.f);
  i0 = min((int)s, g.I[a] - 1);
  i1 = min(i0 + 1, g.I[a] - 1);
  w1 = s - (float)i0;
  if (i0 == i1) w1 = 0.f;
}

template <int DT>
__global__ __launch_bounds__(256) void interp_fwd_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                         InterpArgs g, long long total) {
  const long long plane_in = (long long)g.I[0] * g.I[1] * g.I[2];
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    long long r = t;
    const int ow = (int)(r % g.O[2]);
    r /= g.O[2];
    const int oh = (int)(r % g.O[1]);
    r /= g.O[1];
    const int od = (int)(r % g.O[0]);
    const long long nc = r / g.O[0];
    int d0, d1, h0, h1, w0, w1i;
    float fd, fh, fw;
    src_of(g, 0, od, d0, d1, fd);
    src_of(g, 1, oh, h0, h1, fh);
    src_of(g, 2, ow, w0, w1i, fw);
    const long long b = nc * plane_in;
    auto at = [&](int d, int h, int w) { return ld<DT>(x, b + ((long long)d * g.I[1] + h) * g.I[2] + w); };
    const float v = (1.f - fd) * ((1.f - fh) * ((1.f - fw) * at(d0, h0, w0) + fw * at(d0, h0, w1i)) +
                                  fh * ((1.f - fw) * at(d0, h1, w0) + fw * at(d0, h1, w1i))) +
                    fd * ((1.f - fh) * ((1.f - fw) * at(d1, h0, w0) + fw * at(d1, h0, w1i)) +
                          fh * ((1.f - fw) * at(d1, h1, w0) + fw * at(d1, h1, w1i)));
    st<DT>(y, t, v);
  }
}

template <int DT>
__global__ __launch_bounds__(256) void interp_bwd_kernel(const void* __restrict__ dy, float* __restrict__ dx,
                                                         InterpArgs g, long long total) {
  const long long plane_in = (long long)g.I[0] * g.I[1] * g.I[2];
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    long long r = t;
    const int ow = (int)(r % g.O[2]);
    r /= g.O[2];
    const int oh = (int)(r % g.O[1]);
    r /= g.O[1];
    const int od = (int)(r % g.O[0]);
    const long long nc = r / g.O[0];
    int d[2], h[2], w[2];
    float fd, fh, fw;
    src_of(g, 0, od, d[0], d[1], fd);
    src_of(g, 1, oh, h[0], h[1], fh);
    src_of(g, 2, ow, w[0], w[1], fw);
    const float gy = ld<DT>(dy, t);
    const float wd[2] = {1.f - fd, fd}, wh[2] = {1.f - fh, fh}, ww[2] = {1.f - fw, fw};
    const long long b = nc * plane_in;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float wt = wd[a] * wh[c] * ww[e];
          if (wt != 0.f) atomicAdd(dx + b + ((long long)d[a] * g.I[1] + h[c]) * g.I[2] + w[e], gy * wt);
        }
  }
}

// --------------------------------------------------------------------------------- grid_sample
// 2-D bilinear / nearest sampling of x [N, C, IH, IW] at grid [N, OH, OW, 2] (x, y in [-1, 1]),
// padding zeros / border / reflection. Reference `phi/kernels/gpu/grid_sample_kernel.cu` and its
// grad kernel. One thread per output location loops over the channels (the grid gradient is a
// sum over them); dx scatters into an f32 buffer with atomics.
struct GsArgs {
  int N, C, IH, IW, OH, OW;
  int mode;  // 0 bilinear, 1 nearest
  int pad;   // 0 zeros, 1 border, 2 reflection
  int align_corners;
};

__device__ __forceinline__ float gs_clip(float v, int size, float& g) {
  if (v <= 0.f) { g = 0.f; return 0.f; }
  const float mx = (float)(size - 1);
  if (v >= mx) { g = 0.f; return mx; }
  g = 1.f;
  return v;
}

__device__ __forceinline__ float gs_reflect(float v, int tlo, int thi, float& g) {
  if (tlo == thi) { g = 0.f; return 0.f; }
  const float mn = tlo * 0.5f, span = (thi - tlo) * 0.5f;
  v -= mn;
  float sg = 1.f;
  if (v < 0.f) { sg = -1.f; v = -v; }
  const float extra = fmodf(v, span);
  const int flips = (int)floorf(v / span);
  if ((flips & 1) == 0) { g = sg; return extra + mn; }
  g = -sg;
  return span - extra + mn;
}

// grid coordinate → source pixel coordinate and d(source)/d(grid)
__device__ __forceinline__ float gs_source(const GsArgs& g, float c, int size, float& dc) {
  float v, sc;
  if (g.align_corners) { sc = (size - 1) * 0.5f; v = (c + 1.f) * sc; }
  else { sc = size * 0.5f; v = ((c + 1.f) * size - 1.f) * 0.5f; }
  float g1 = 1.f, g2 = 1.f;
  if (g.pad == 1) v = gs_clip(v, size, g1);
  else if (g.pad == 2) {
    v = g.align_corners ? gs_reflect(v, 0, 2 * (size - 1), g1) : gs_reflect(v, -1, 2 * size - 1, g1);
    v = gs_clip(v, size, g2);
  }
  dc = sc * g1 * g2;
  return v;
}

template <int DT>
__global__ __launch_bounds__(256) void grid_sample_fwd_kernel(const void* __restrict__ x, const void* __restrict__ grid,
                                                              void* __restrict__ y, GsArgs g, long long total) {
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int ow = (int)(t % g.OW);
    const int oh = (int)((t / g.OW) % g.OH);
    const long long n = t / ((long long)g.OW * g.OH);
    float d0;
    const float ix = gs_source(g, ld<DT>(grid, 2 * t), g.IW, d0);
    const float iy = gs_source(g, ld<DT>(grid, 2 * t + 1), g.IH, d0);
    const long long plane = (long long)g.IH * g.IW, ostep = (long long)g.OH * g.OW;
    const long long xb = n * g.C * plane, yb = n * g.C * ostep + (long long)oh * g.OW + ow;
    if (g.mode == 1) {
      const int xi = (int)rintf(ix), yi = (int)rintf(iy);
      const bool in = xi >= 0 && xi < g.IW && yi >= 0 && yi < g.IH;
      for (int c = 0; c < g.C; ++c)
        st<DT>(y, yb + c * ostep, in ? ld<DT>(x, xb + c * plane + (long long)yi * g.IW + xi) : 0.f);
      continue;
    }
    const int x0 = (int)floorf(ix), y0 = (int)floorf(iy), x1 = x0 + 1, y1 = y0 + 1;
    const float wx1 = ix - x0, wx0 = 1.f - wx1, wy1 = iy - y0, wy0 = 1.f - wy1;
    const bool vx0 = x0 >= 0 && x0 < g.IW, vx1 = x1 >= 0 && x1 < g.IW;
    const bool vy0 = y0 >= 0 && y0 < g.IH, vy1 = y1 >= 0 && y1 < g.IH;
    for (int c = 0; c < g.C; ++c) {
      const long long b = xb + c * plane;
      float v = 0.f;
      if (vy0 && vx0) v += wy0 * wx0 * ld<DT>(x, b + (long long)y0 * g.IW + x0);
      if (vy0 && vx1) v += wy0 * wx1 * ld<DT>(x, b + (long long)y0 * g.IW + x1);
      if (vy1 && vx0) v += wy1 * wx0 * ld<DT>(x, b + (long long)y1 * g.IW + x0);
      if (vy1 && vx1) v += wy1 * wx1 * ld<DT>(x, b + (long long)y1 * g.IW + x1);
      st<DT>(y, yb + c * ostep, v);
    }
  }
}

template <int DT>
__global__ __launch_bounds__(256) void grid_sample_bwd_kernel(const void* __restrict__ dy, const void* __restrict__ x,
                                                              const void* __restrict__ grid, float* __restrict__ dx,
                                                              float* __restrict__ dgrid, GsArgs g, long long total) {
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int ow = (int)(t % g.OW);
    const int oh = (int)((t / g.OW) % g.OH);
    const long long n = t / ((long long)g.OW * g.OH);
    float dxs, dys;
    const float ix = gs_source(g, ld<DT>(grid, 2 * t), g.IW, dxs);
    const float iy = gs_source(g, ld<DT>(grid, 2 * t + 1), g.IH, dys);
    const long long plane = (long long)g.IH * g.IW, ostep = (long long)g.OH * g.OW;
    const long long xb = n * g.C * plane, yb = n * g.C * ostep + (long long)oh * g.OW + ow;
    if (g.mode == 1) {
      const int xi = (int)rintf(ix), yi = (int)rintf(iy);
      if (xi >= 0 && xi < g.IW && yi >= 0 && yi < g.IH)
        for (int c = 0; c < g.C; ++c)
          atomicAdd(dx + xb + c * plane + (long long)yi * g.IW + xi, ld<DT>(dy, yb + c * ostep));
      dgrid[2 * t] = 0.f;
      dgrid[2 * t + 1] = 0.f;
      continue;
    }
    const int x0 = (int)floorf(ix), y0 = (int)floorf(iy), x1 = x0 + 1, y1 = y0 + 1;
    const float wx1 = ix - x0, wx0 = 1.f - wx1, wy1 = iy - y0, wy0 = 1.f - wy1;
    const bool vx0 = x0 >= 0 && x0 < g.IW, vx1 = x1 >= 0 && x1 < g.IW;
    const bool vy0 = y0 >= 0 && y0 < g.IH, vy1 = y1 >= 0 && y1 < g.IH;
    float gix = 0.f, giy = 0.f;
    for (int c = 0; c < g.C; ++c) {
      const long long b = xb + c * plane;
      const float go = ld<DT>(dy, yb + c * ostep);
      if (vy0 && vx0) {
        const long long o = b + (long long)y0 * g.IW + x0;
        const float v = ld<DT>(x, o);
        atomicAdd(dx + o, wy0 * wx0 * go);
        gix -= v * wy0 * go;
        giy -= v * wx0 * go;
      }
      if (vy0 && vx1) {
        const long long o = b + (long long)y0 * g.IW + x1;
        const float v = ld<DT>(x, o);
        atomicAdd(dx + o, wy0 * wx1 * go);
        gix += v * wy0 * go;
        giy -= v * wx1 * go;
      }
      if (vy1 && vx0) {
        const long long o = b + (long long)y1 * g.IW + x0;
        const float v = ld<DT>(x, o);
        atomicAdd(dx + o, wy1 * wx0 * go);
        gix -= v * wy1 * go;
        giy += v * wx0 * go;
      }
      if (vy1 && vx1) {
        const long long o = b + (long long)y1 * g.IW + x1;
        const float v = ld<DT>(x, o);
        atomicAdd(dx + o, wy1 * wx1 * go);
        gix += v * wy1 * go;
        giy += v * wx1 * go;
      }
    }
    dgrid[2 * t] = gix * dxs;
    dgrid[2 * t + 1] = giy * dys;
  }
}

inline unsigned grid_for(long long n) {
  const long long b = (n + 255) / 256;
  return (unsigned)(b < 65536 * 4 ? (b < 1 ? 1 : b) : 65536 * 4);
}

}  // namespace

#define DISPATCH_DT(dt, KER, ...)                                                                  \
  switch (dt) {                                                                                    \
    case 0: hipLaunchKernelGGL(KER<0>, __VA_ARGS__); break;                                        \
    case 1: hipLaunchKernelGGL(KER<1>, __VA_ARGS__); break;                                        \
    case 2: hipLaunchKernelGGL(KER<2>, __VA_ARGS__); break;                                        \
    default: return (int)hipErrorInvalidValue;                                                     \
  }

// dt: 0 f32, 1 bf16, 2 fp16. dims: [D, H, W] input / output / kernel / stride / padding.
PIAMD_EXPORT int piamd_pool_nd_fwd(int dt, const void* x, void* y, int* idx, int N, int C, const int* I,
                                   const int* O, const int* K, const int* S, const int* P, int mode,
                                   int adaptive, int exclusive, int divisor, hipStream_t st) {
  PoolArgs g{N, C, {I[0], I[1], I[2]}, {O[0], O[1], O[2]}, {K[0], K[1], K[2]}, {S[0], S[1], S[2]},
             {P[0], P[1], P[2]}, mode, adaptive, exclusive, divisor};
  const long long total = (long long)N * C * O[0] * O[1] * O[2];
  if (total == 0) return 0;
  DISPATCH_DT(dt, pool_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, x, y, idx, g, total)
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_pool_nd_bwd(int dt, const void* dy, const int* idx, void* dx, int N, int C, const int* I,
                                   const int* O, const int* K, const int* S, const int* P, int mode,
                                   int adaptive, int exclusive, int divisor, hipStream_t st) {
  PoolArgs g{N, C, {I[0], I[1], I[2]}, {O[0], O[1], O[2]}, {K[0], K[1], K[2]}, {S[0], S[1], S[2]},
             {P[0], P[1], P[2]}, mode, adaptive, exclusive, divisor};
  const long long total = (long long)N * C * I[0] * I[1] * I[2];
  if (total == 0) return 0;
  DISPATCH_DT(dt, pool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, dy, idx, dx, g, total)
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_interp_fwd(int dt, const void* x, void* y, int N, int C, const int* I, const int* O,
                                  const float* scale, int mode, int align_corners, hipStream_t st) {
  InterpArgs g{N, C, {I[0], I[1], I[2]}, {O[0], O[1], O[2]}, {scale[0], scale[1], scale[2]}, mode,
               align_corners};
  const long long total = (long long)N * C * O[0] * O[1] * O[2];
  if (total == 0) return 0;
  DISPATCH_DT(dt, interp_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, x, y, g, total)
  return (int)hipGetLastError();
}

// dx: f32 [N, C, I] zero-filled by the caller (scatter-add of the linear weights)
PIAMD_EXPORT int piamd_interp_bwd(int dt, const void* dy, float* dx, int N, int C, const int* I, const int* O,
                                  const float* scale, int mode, int align_corners, hipStream_t st) {
  InterpArgs g{N, C, {I[0], I[1], I[2]}, {O[0], O[1], O[2]}, {scale[0], scale[1], scale[2]}, mode,
               align_corners};
  const long long total = (long long)N * C * O[0] * O[1] * O[2];
  if (total == 0) return 0;
  DISPATCH_DT(dt, interp_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, dy, dx, g, total)
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_grid_sample_fwd(int dt, const void* x, const void* grid, void* y, int N, int C, int IH,
                                       int IW, int OH, int OW, int mode, int pad, int align_corners, hipStream_t st) {
  GsArgs g{N, C, IH, IW, OH, OW, mode, pad, align_corners};
  const long long total = (long long)N * OH * OW;
  if (total == 0 || C == 0) return 0;
  DISPATCH_DT(dt, grid_sample_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, x, grid, y, g, total)
  return (int)hipGetLastError();
}

// dx: f32 [N, C, IH, IW] zero-filled by the caller; dgrid: f32 [N, OH, OW, 2]
PIAMD_EXPORT int piamd_grid_sample_bwd(int dt, const void* dy, const void* x, const void* grid, float* dx,
                                       float* dgrid, int N, int C, int IH, int IW, int OH, int OW, int mode, int pad,
                                       int align_corners, hipStream_t st) {
  GsArgs g{N, C, IH, IW, OH, OW, mode, pad, align_corners};
  const long long total = (long long)N * OH * OW;
  if (total == 0) return 0;
  DISPATCH_DT(dt, grid_sample_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, dy, x, grid, dx, dgrid, g, total)
  return (int)hipGetLastError();
}
