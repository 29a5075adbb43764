// Per-step filter preparation of a dense convolution in ONE launch: the fp32 (or 16-bit) master
// filter [K0][C0][R][S] → the forward operand [K4][R][S][Cp] (OHWI, channels zero-padded to the
// implicit GEMM's 64-channel k-steps, output channels to the epilogue's 4) AND the stride-1 data
// gradient's operand [Cp][R][S][Kp] = W[k][c][R-1-r][S-1-s] (flipped, in/out transposed, K zero-
// padded to 64), both 16-bit. Replaces the cast + permute + pad kernels of the forward and the
// flip + permute of the backward (≈3 launches per conv per step, `profiles/rocprof_resnet50_r4b.txt`).
// Parity: the filter transforms of `phi/kernels/gpudnn/conv_grad_kernel.cu` (cuDNN does them
// inside its algorithms).
#include <algorithm>

#include "common.h"

namespace {

template <int SRC, bool F16>
__device__ __forceinline__ float wload(const void* w, long long i) {
  if constexpr (SRC == 0) return reinterpret_cast<const float*>(w)[i];
  else return h2f<SRC == 2>(reinterpret_cast<const unsigned short*>(w)[i]);
}

// grid-stride over max(n_fwd, n_dgr): thread i writes fwd[i] (i < n_fwd) and dgr[i] (i < n_dgr)
template <int SRC, bool F16>
__global__ __launch_bounds__(256) void conv_wprep_kernel(const void* __restrict__ w, unsigned short* __restrict__ fwd,
                                                         unsigned short* __restrict__ dgr, int K0, int C0,
                                                         int R, int S, int K4, int Cp, int Kp) {
  const long long RS = (long long)R * S;
  const long long n_fwd = fwd ? (long long)K4 * RS * Cp : 0;
  const long long n_dgr = dgr ? (long long)Cp * RS * Kp : 0;
  const long long n = n_fwd > n_dgr ? n_fwd : n_dgr;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    if (i < n_fwd) {  // [k][r][s][c]
      const int c = (int)(i % Cp);
      const long long t = i / Cp;
      const int rs = (int)(t % RS), k = (int)(t / RS);
      const float v = (k < K0 && c < C0) ? wload<SRC, F16>(w, ((long long)k * C0 + c) * RS + rs) : 0.f;
      fwd[i] = f2h<F16>(v);
    }
    if (i < n_dgr) {  // [c][r][s][k] = W[k][c][R-1-r][S-1-s]
      const int k = (int)(i % Kp);
      const long long t = i / Kp;
      const int rs = (int)(t % RS), c = (int)(t / RS);
      const int r = rs / S, s = rs % S;
      const long long src = ((long long)k * C0 + c) * RS + (long long)(R - 1 - r) * S + (S - 1 - s);
      const float v = (k < K0 && c < C0) ? wload<SRC, F16>(w, src) : 0.f;
      dgr[i] = f2h<F16>(v);
    }
  }
}

}  // namespace

// src_dt: 0 f32, 1 bf16, 2 fp16 master filter; f16: 16-bit outputs are fp16 (else bf16).
// fwd / dgr nullable. Requires K4 ≥ K0, Cp ≥ C0, Kp ≥ K0.
PIAMD_EXPORT int piamd_conv_wprep(int src_dt, int f16, const void* w, void* fwd, void* dgr, int K0,
                                  int C0, int R, int S, int K4, int Cp, int Kp, hipStream_t st) {
  if (!w || (!fwd && !dgr) || K0 < 1 || C0 < 1 || R < 1 || S < 1 || K4 < K0 || Cp < C0 || Kp < K0 ||
      src_dt < 0 || src_dt > 2)
    return (int)hipErrorInvalidValue;
  const long long n = std::max(fwd ? (long long)K4 * R * S * Cp : 0LL, dgr ? (long long)Cp * R * S * Kp : 0LL);
  const int grid = (int)std::min<long long>((n + 255) / 256, 4096);
#define WP(SD, F)                                                                                  \
  hipLaunchKernelGGL((conv_wprep_kernel<SD, F>), dim3(grid), dim3(256), 0, st, w,                  \
                     (unsigned short*)fwd, (unsigned short*)dgr, K0, C0, R, S, K4, Cp, Kp)
  if (f16) {
    if (src_dt == 0) WP(0, true); else if (src_dt == 1) WP(1, true); else WP(2, true);
  } else {
    if (src_dt == 0) WP(0, false); else if (src_dt == 1) WP(1, false); else WP(2, false);
  }
#undef WP
  return (int)hipGetLastError();
}
