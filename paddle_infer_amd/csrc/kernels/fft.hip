// Batched complex-to-complex FFT of power-of-two length N ≤ 4096 along contiguous rows
// (complex64, interleaved re/im) — the transform kernel behind paddle.fft (fft / ifft / rfft /
// irfft / hfft / fftn ...; other lengths: Bluestein, longer power-of-two rows: four-step, both
// composed in ops/fft.py over this kernel).
//
// Parity: reference `paddle/phi/kernels/funcs/fft.cu` (cuFFT plans behind fft_c2c / fft_r2c /
// fft_c2r). Here a self-sorting Stockham radix-2 transform entirely in LDS:
//   * a 256-thread workgroup (1024 threads for N ≥ 2048) owns R = max(1, 1024 / N) rows (small transforms are batched so every
//     thread has butterflies), rows are loaded with coalesced 8-byte loads into one LDS buffer;
//   * ⌊log4 N⌋ radix-4 stages (+ one radix-2 stage for odd log2 N) ping-pong between two R·N
//     images in LDS: y[(j / Ls)·4Ls + k + q·Ls] = Σ_r x[j + r·N/4]·w^{r·k}·e^{∓2πi·rq/4},
//     k = j mod Ls — natural-order input and output, no bit reversal, half the barriers of
//     radix 2;
//   * twiddles from an N-entry LDS table (one accurate sincospif per entry per workgroup) instead
//     of a sincos per butterfly; scale (1, 1/N or 1/√N) fused in the store.
#include "common.h"

namespace {

constexpr int FFT_MAX_N = 4096;

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

template <int FFT_THREADS>
__global__ __launch_bounds__(FFT_THREADS) void fft_pow2_kernel(const float2* __restrict__ in,
                                                              float2* __restrict__ out, long long rows,
                                                              int N, int logN, int inverse,
                                                              float scale) {
  extern __shared__ float2 buf[];  // [2][R * N] ping-pong images + [N] twiddle table
  const int R = N >= 1024 ? 1 : 1024 / N;
  const int RN = R * N;
  const long long row0 = (long long)blockIdx.x * R;
  const int nrows = (int)min((long long)R, rows - row0);
  const int tid = threadIdx.x;
  float2* x = buf;
  float2* y = buf + RN;
  float2* tw = buf + 2 * RN;  // tw[j] = exp(∓2πi j / N): one accurate sincos per entry per block
  const float sgn = inverse ? 1.f : -1.f;
  for (int j = tid; j < N; j += FFT_THREADS) {
    float sn, cs;
    sincospif(sgn * 2.f * (float)j / (float)N, &sn, &cs);
    tw[j] = make_float2(cs, sn);
  }
  for (int i = tid; i < nrows * N; i += FFT_THREADS) x[i] = in[row0 * N + i];
  __syncthreads();
  int Ls = 1, s = 0;
  // radix-4 Stockham stages: y[(j/Ls)·4Ls + k + q·Ls] = Σ_r x[j + r·N/4]·w^{r·k}·e^{∓2πi·rq/4}
  const int q4 = N >> 2;
  for (; s + 2 <= logN; s += 2) {
    const int tstep = N / (4 * Ls);  // table stride of w = e^{∓2πi/(4Ls)}
    for (int t = tid; t < nrows * q4; t += FFT_THREADS) {
      const int r = t >> (logN - 2), j = t & (q4 - 1);
      const float2* xr = x + r * N;
      float2* yr = y + r * N;
      const int k = j & (Ls - 1);
      const float2 a0 = xr[j];
      const float2 a1 = cmul(xr[j + q4], tw[k * tstep]);
      const float2 a2 = cmul(xr[j + 2 * q4], tw[2 * k * tstep]);
      const float2 a3 = cmul(xr[j + 3 * q4], tw[3 * k * tstep]);
      const float2 s02 = make_float2(a0.x + a2.x, a0.y + a2.y), d02 = make_float2(a0.x - a2.x, a0.y - a2.y);
      const float2 s13 = make_float2(a1.x + a3.x, a1.y + a3.y), d13 = make_float2(a1.x - a3.x, a1.y - a3.y);
      // ∓i·d13 (forward: −i·d13 = (d.y, −d.x); inverse: +i·d13 = (−d.y, d.x))
      const float2 rd = inverse ? make_float2(-d13.y, d13.x) : make_float2(d13.y, -d13.x);
      const int o = ((j >> s) << (s + 2)) + k;
      yr[o] = make_float2(s02.x + s13.x, s02.y + s13.y);
      yr[o + Ls] = make_float2(d02.x + rd.x, d02.y + rd.y);
      yr[o + 2 * Ls] = make_float2(s02.x - s13.x, s02.y - s13.y);
      yr[o + 3 * Ls] = make_float2(d02.x - rd.x, d02.y - rd.y);
    }
    __syncthreads();
    float2* t2 = x;
    x = y;
    y = t2;
    Ls <<= 2;
  }
  if (s < logN) {  // odd log2 N: one radix-2 stage, w = e^{∓iπk/Ls}
    const int half = N >> 1, tstep = N / (2 * Ls);
    for (int t = tid; t < nrows * half; t += FFT_THREADS) {
      const int r = t >> (logN - 1), j = t & (half - 1);
      const float2* xr = x + r * N;
      float2* yr = y + r * N;
      const int k = j & (Ls - 1);
      const float2 a = xr[j], wb = cmul(xr[j + half], tw[k * tstep]);
      const int o = ((j >> s) << (s + 1)) + k;
      yr[o] = make_float2(a.x + wb.x, a.y + wb.y);
      yr[o + Ls] = make_float2(a.x - wb.x, a.y - wb.y);
    }
    __syncthreads();
    float2* t2 = x;
    x = y;
    y = t2;
  }
  for (int i = tid; i < nrows * N; i += FFT_THREADS) {
    const float2 v = x[i];
    out[row0 * N + i] = make_float2(v.x * scale, v.y * scale);
  }
}

}  // namespace

// in / out: [rows][N] complex64 (may alias); N a power of two, 2 ≤ N ≤ 4096 (N == 1: copy).
PIAMD_EXPORT int piamd_fft_c2c(const void* in, void* out, long long rows, int N, int inverse,
                               float scale, hipStream_t st) {
  if (N < 1 || N > FFT_MAX_N || (N & (N - 1)) || rows < 0) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  int logN = 0;
  while ((1 << logN) < N) ++logN;
  if (N == 1) {
    hipMemcpyAsync(out, in, rows * sizeof(float2), hipMemcpyDeviceToDevice, st);
    return (int)hipGetLastError();
  }
  const int R = N >= 1024 ? 1 : 1024 / N;
  const long long grid = (rows + R - 1) / R;
  if (grid > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  const size_t lds = ((size_t)2 * R * N + N) * sizeof(float2);
  // N ≥ 2048: one workgroup per row holds 96 KiB of LDS (one per CU), so give it 1024 threads
  // (16 waves, one radix-4 butterfly each per stage at N = 4096) instead of 4 idle-heavy waves.
  if (N >= 2048)
    hipLaunchKernelGGL(fft_pow2_kernel<1024>, dim3((unsigned)grid), dim3(1024), lds, st,
                       (const float2*)in, (float2*)out, rows, N, logN, inverse, scale);
  else
    hipLaunchKernelGGL(fft_pow2_kernel<256>, dim3((unsigned)grid), dim3(256), lds, st,
                       (const float2*)in, (float2*)out, rows, N, logN, inverse, scale);
  return (int)hipGetLastError();
}
