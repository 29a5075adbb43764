// Batched Viterbi decoding (max-product dynamic programming over a linear-chain CRF) in ONE
// kernel launch: one workgroup per sequence walks all time steps with the running scores in LDS
// (double-buffered, one barrier per step), records the arg-max back-pointers, and backtraces on
// the device — no per-step launches and no host round trip.
//
// Parity: reference `paddle/phi/kernels/gpu/viterbi_decode_kernel.cu` / `python/paddle/text/
// viterbi_decode.py` (scores [B], paths [B, T] with positions past a sequence's length zeroed;
// with include_bos_eos_tag the last two tags are BOS / EOS: alpha_0 += trans[BOS, :], the final
// scores += trans[:, EOS]). Ties resolve to the lowest tag index.
#include "common.h"

namespace {

constexpr int VT_THREADS = 256;

__global__ __launch_bounds__(VT_THREADS) void viterbi_kernel(const float* __restrict__ pot,
                                                             const float* __restrict__ trans,
                                                             const long long* __restrict__ lengths,
                                                             int T, int N, int bos_eos,
                                                             float* __restrict__ scores,
                                                             long long* __restrict__ path,
                                                             int* __restrict__ hist) {
  extern __shared__ float sm[];  // alpha[2][N], then the reduction scratch
  float* alpha0 = sm;
  float* alpha1 = sm + N;
  float* rv = sm + 2 * N;                      // [VT_THREADS] values
  int* ri = reinterpret_cast<int*>(rv + VT_THREADS);  // [VT_THREADS] indices
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* p = pot + (long long)b * T * N;
  int* h = hist + (long long)b * T * N;
  const long long len = lengths[b];
  for (int j = tid; j < N; j += VT_THREADS)
    alpha0[j] = p[j] + (bos_eos ? trans[(long long)(N - 2) * N + j] : 0.f);
  __syncthreads();
  float* cur = alpha0;
  float* nxt = alpha1;
  for (int t = 1; t < T; ++t) {
    const bool live = t < len;
    for (int j = tid; j < N; j += VT_THREADS) {
      float best = -INFINITY;
      int arg = 0;
      for (int i = 0; i < N; ++i) {
        const float s = cur[i] + trans[(long long)i * N + j];
        if (s > best) {
          best = s;
          arg = i;
        }
      }
      nxt[j] = live ? best + p[(long long)t * N + j] : cur[j];
      h[(long long)(t - 1) * N + j] = live ? arg : j;
    }
    __syncthreads();
    float* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  // final scores (+ transition to EOS) and the arg-max tag
  float best = -INFINITY;
  int arg = 0x7fffffff;
  for (int j = tid; j < N; j += VT_THREADS) {
    const float s = cur[j] + (bos_eos ? trans[(long long)j * N + (N - 1)] : 0.f);
    if (s > best || (s == best && j < arg)) {
      best = s;
      arg = j;
    }
  }
  rv[tid] = best;
  ri[tid] = arg;
  __syncthreads();
  for (int w = VT_THREADS / 2; w > 0; w >>= 1) {
    if (tid < w) {
      const float o = rv[tid + w];
      const int oi = ri[tid + w];
      if (o > rv[tid] || (o == rv[tid] && oi < ri[tid])) {
        rv[tid] = o;
        ri[tid] = oi;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    scores[b] = rv[0];
    long long* out = path + (long long)b * T;
    int last = ri[0];
    out[T - 1] = last;
    for (int t = T - 2; t >= 0; --t) {
      last = h[(long long)t * N + last];
      out[t] = last;
    }
    for (int t = 0; t < T; ++t)
      if (t >= len) out[t] = 0;
  }
}

}  // namespace

// potentials f32 [B, T, N], transitions f32 [N, N], lengths int64 [B] → scores f32 [B],
// paths int64 [B, T] (positions ≥ length zeroed); hist: int32 workspace [B, T, N].
PIAMD_EXPORT int piamd_viterbi_decode(const float* pot, const float* trans, const long long* lengths,
                                      int B, int T, int N, int bos_eos, float* scores, long long* path,
                                      int* hist, hipStream_t stream) {
  if (B <= 0 || T <= 0) return 0;
  if (N <= 0 || (size_t)(2 * N + 2 * VT_THREADS) * 4 > 64 * 1024) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(2 * N + 2 * VT_THREADS) * 4;
  hipLaunchKernelGGL(viterbi_kernel, dim3(B), dim3(VT_THREADS), lds, stream, pot, trans, lengths, T, N,
                     bos_eos, scores, path, hist);
  return (int)hipGetLastError();
}
