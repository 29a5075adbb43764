// Batched complex-to-complex FFT of power-of-two length N ≤ 4096 along contiguous rows
// (complex64, interleaved re/im) — the transform kernel behind paddle.fft (fft / ifft / rfft /
// irfft / hfft / fftn ...; other lengths: Bluestein, longer power-of-two rows: four-step, both
// composed in ops/fft.py over this kernel).
//
// Parity: reference `paddle/phi/kernels/funcs/fft.cu` (cuFFT plans behind fft_c2c / fft_r2c /
// fft_c2r). Here a self-sorting Stockham radix-2 transform entirely in LDS:
//   * a 256-thread workgroup owns R = max(1, 1024 / N) rows (small transforms are batched so every
//     thread has butterflies), rows are loaded with coalesced 8-byte loads into one LDS buffer;
//   * log2(N) stages ping-pong between the two halves of a 2·R·N·8-byte LDS image (≤ 64 KiB),
//     stage s: y[(j / Ls)·2Ls + k] = a + w·b, y[… + Ls] = a − w·b with a = x[j], b = x[j + N/2],
//     k = j mod Ls, w = exp(∓iπk/Ls) — natural-order input and output, no bit reversal;
//   * twiddles from sincospif-style accurate sincos of (k / Ls), scale (1, 1/N or 1/√N) fused in
//     the store.
#include "common.h"

namespace {

constexpr int FFT_THREADS = 256;
constexpr int FFT_MAX_N = 4096;

__global__ __launch_bounds__(FFT_THREADS) void fft_pow2_kernel(const float2* __restrict__ in,
                                                              float2* __restrict__ out, long long rows,
                                                              int N, int logN, int inverse,
                                                              float scale) {
  extern __shared__ float2 buf[];  // [2][R * N]
  const int R = N >= 1024 ? 1 : 1024 / N;
  const int RN = R * N;
  const long long row0 = (long long)blockIdx.x * R;
  const int nrows = (int)min((long long)R, rows - row0);
  const int tid = threadIdx.x;
  float2* x = buf;
  float2* y = buf + RN;
  for (int i = tid; i < nrows * N; i += FFT_THREADS) x[i] = in[row0 * N + i];
  __syncthreads();
  const float sgn = inverse ? 1.f : -1.f;
  const int half = N >> 1;
  for (int s = 0; s < logN; ++s) {
    const int Ls = 1 << s;
    for (int t = tid; t < nrows * half; t += FFT_THREADS) {
      const int r = t >> (logN - 1), j = t & (half - 1);
      const float2* xr = x + r * N;
      float2* yr = y + r * N;
      const int k = j & (Ls - 1);
      float sn, cs;
      sincospif(sgn * (float)k / (float)Ls, &sn, &cs);
      const float2 a = xr[j], b = xr[j + half];
      const float2 wb = make_float2(b.x * cs - b.y * sn, b.x * sn + b.y * cs);
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
  const size_t lds = (size_t)2 * R * N * sizeof(float2);
  hipLaunchKernelGGL(fft_pow2_kernel, dim3((unsigned)grid), dim3(FFT_THREADS), lds, st,
                     (const float2*)in, (float2*)out, rows, N, logN, inverse, scale);
  return (int)hipGetLastError();
}
