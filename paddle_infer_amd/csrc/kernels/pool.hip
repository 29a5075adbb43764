// Max pooling over channels-last (NHWC) 16-bit activations, forward + backward.
//
// Parity: reference `phi/kernels/funcs/pooling.cu` (MaxPool2dWithIndex / Pool2dGrad) and the NHWC
// path of `gpudnn/pool_kernel.cu`. ATen's NHWC max-pool backward scattered with atomics and ran at
// ~0.3 ms for the ResNet-50 stem pool (profiles/rocprof_resnet50_r4.txt); here:
//   * forward: a lane owns 8 channels (one 16-B vector) of one output pixel, walks the kh × kw
//     window (padding taps skipped) and stores the max plus the winning tap index (u8 per
//     element, first maximum wins, NaN propagates) — 8 index bytes per 16-B output vector;
//   * backward is a GATHER: a lane owns 8 channels of one INPUT pixel, visits the ≤ ⌈k/s⌉² output
//     windows that contain it and adds dY where the stored tap is this pixel — no atomics, fixed
//     order (deterministic), one 16-B dX store.
#include "common.h"

namespace {

struct PoolGeom {
  int N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw;
};

template <bool F16>
__global__ __launch_bounds__(256) void maxpool_fwd_nhwc8(const unsigned short* __restrict__ x,
                                                        unsigned short* __restrict__ y,
                                                        unsigned char* __restrict__ idx, PoolGeom g,
                                                        long long total) {
  const int CV = g.C / 8;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cv = (int)(i % CV);
    long long p = i / CV;
    const int ow = (int)(p % g.OW);
    p /= g.OW;
    const int oh = (int)(p % g.OH), n = (int)(p / g.OH);
    float m[8];
    unsigned char t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      m[j] = -INFINITY;
      t[j] = 255;
    }
    const int h0 = oh * g.sh - g.ph, w0 = ow * g.sw - g.pw;
    for (int r = 0; r < g.kh; ++r) {
      const int ih = h0 + r;
      if (ih < 0 || ih >= g.H) continue;
      for (int s = 0; s < g.kw; ++s) {
        const int iw = w0 + s;
        if (iw < 0 || iw >= g.W) continue;
        const u16x8 v = *reinterpret_cast<const u16x8*>(x + (((long long)n * g.H + ih) * g.W + iw) * g.C + cv * 8);
        const unsigned char tap = (unsigned char)(r * g.kw + s);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = h2f<F16>(v[j]);
          if (f > m[j] || (f != f && m[j] == m[j]) || t[j] == 255) {
            m[j] = f;
            t[j] = tap;
          }
        }
      }
    }
    u16x8 o;
    unsigned long long tb = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = f2h<F16>(m[j]);
      tb |= (unsigned long long)t[j] << (8 * j);
    }
    *reinterpret_cast<u16x8*>(y + i * 8) = o;
    *reinterpret_cast<unsigned long long*>(idx + i * 8) = tb;
  }
}

template <bool F16>
__global__ __launch_bounds__(256) void maxpool_bwd_nhwc8(const unsigned short* __restrict__ dy,
                                                        const unsigned char* __restrict__ idx,
                                                        unsigned short* __restrict__ dx, PoolGeom g,
                                                        long long total) {
  const int CV = g.C / 8;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cv = (int)(i % CV);
    long long p = i / CV;
    const int iw = (int)(p % g.W);
    p /= g.W;
    const int ih = (int)(p % g.H), n = (int)(p / g.H);
    // output rows oh with oh·sh − ph ≤ ih ≤ oh·sh − ph + kh − 1
    const int oh0 = max(0, (ih + g.ph - g.kh + g.sh) / g.sh), oh1 = min(g.OH - 1, (ih + g.ph) / g.sh);
    const int ow0 = max(0, (iw + g.pw - g.kw + g.sw) / g.sw), ow1 = min(g.OW - 1, (iw + g.pw) / g.sw);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int r = ih - (oh * g.sh - g.ph);
      if (r < 0 || r >= g.kh) continue;
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int s = iw - (ow * g.sw - g.pw);
        if (s < 0 || s >= g.kw) continue;
        const long long o = (((long long)n * g.OH + oh) * g.OW + ow) * g.C + cv * 8;
        const unsigned long long tb = *reinterpret_cast<const unsigned long long*>(idx + o);
        const unsigned char tap = (unsigned char)(r * g.kw + s);
        const u16x8 d = *reinterpret_cast<const u16x8*>(dy + o);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((unsigned char)(tb >> (8 * j)) == tap) acc[j] += h2f<F16>(d[j]);
      }
    }
    u16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = f2h<F16>(acc[j]);
    *reinterpret_cast<u16x8*>(dx + i * 8) = out;
  }
}

bool geom_ok(const PoolGeom& g) {
  return g.N > 0 && g.H > 0 && g.W > 0 && g.C > 0 && g.C % 8 == 0 && g.OH > 0 && g.OW > 0 && g.kh > 0 &&
         g.kw > 0 && g.kh * g.kw <= 255 && g.sh > 0 && g.sw > 0 && g.ph >= 0 && g.pw >= 0 &&
         2 * g.ph <= g.kh && 2 * g.pw <= g.kw;
}

}  // namespace

// y [N][OH][OW][C], idx u8 [N][OH][OW][C] (winning tap r·kw + s) ← max pool of x [N][H][W][C];
// C % 8 == 0, 16-bit (f16 = 1: IEEE half, else bf16). Returns hipError_t.
PIAMD_EXPORT int piamd_maxpool_fwd_nhwc(const void* x, void* y, void* idx, int N, int H, int W, int C,
                                        int OH, int OW, int kh, int kw, int sh, int sw, int ph, int pw,
                                        int f16, hipStream_t st) {
  const PoolGeom g{N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw};
  if (!geom_ok(g) || !x || !y || !idx) return (int)hipErrorInvalidValue;
  const long long total = (long long)N * OH * OW * (C / 8);
  const long long nb = (total + 255) / 256;
  const unsigned grid = (unsigned)(nb < (1 << 20) ? nb : (1 << 20));
  if (f16) hipLaunchKernelGGL(maxpool_fwd_nhwc8<true>, dim3(grid), dim3(256), 0, st, (const unsigned short*)x, (unsigned short*)y, (unsigned char*)idx, g, total);
  else hipLaunchKernelGGL(maxpool_fwd_nhwc8<false>, dim3(grid), dim3(256), 0, st, (const unsigned short*)x, (unsigned short*)y, (unsigned char*)idx, g, total);
  return (int)hipGetLastError();
}

// dx [N][H][W][C] ← gather of dy [N][OH][OW][C] through the forward's tap indices.
PIAMD_EXPORT int piamd_maxpool_bwd_nhwc(const void* dy, const void* idx, void* dx, int N, int H, int W,
                                        int C, int OH, int OW, int kh, int kw, int sh, int sw, int ph,
                                        int pw, int f16, hipStream_t st) {
  const PoolGeom g{N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw};
  if (!geom_ok(g) || !dy || !idx || !dx) return (int)hipErrorInvalidValue;
  const long long total = (long long)N * H * W * (C / 8);
  const long long nb = (total + 255) / 256;
  const unsigned grid = (unsigned)(nb < (1 << 20) ? nb : (1 << 20));
  if (f16) hipLaunchKernelGGL(maxpool_bwd_nhwc8<true>, dim3(grid), dim3(256), 0, st, (const unsigned short*)dy, (const unsigned char*)idx, (unsigned short*)dx, g, total);
  else hipLaunchKernelGGL(maxpool_bwd_nhwc8<false>, dim3(grid), dim3(256), 0, st, (const unsigned short*)dy, (const unsigned char*)idx, (unsigned short*)dx, g, total);
  return (int)hipGetLastError();
}
