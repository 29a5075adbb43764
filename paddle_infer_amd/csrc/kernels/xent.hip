// Softmax cross-entropy over (optionally vocab-sharded) logits, forward + backward.
//
// Parity: reference `paddle/phi/kernels/gpu/cross_entropy_kernel.cu`
// (softmax_with_cross_entropy, hard labels, ignore_index) and the tensor-parallel
// `paddle/fluid/operators/collective/c_softmax_with_cross_entropy_op.cu` (ParallelCrossEntropy).
//
// MI355X design: one 256-thread block per row, single HBM pass with an online (running max,
// running sum) softmax in registers over 16 B bf16 vectors; the backward writes the logit
// gradient (softmax − onehot)·dloss IN PLACE over the logits when asked, so the 0.8 GB
// [tokens × vocab] logits tensor never has a second copy. The vocab-parallel form exports the
// per-row partial statistics (local max, local Σexp, target logit) so the caller combines them
// with three tiny all-reduces over the model-parallel group.
#include "common.h"

namespace {

__device__ __forceinline__ void online_update(float& m, float& s, float x) {
  if (x > m) { s = s * __expf(m - x) + 1.f; m = x; }
  else s += __expf(x - m);
}
__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  float M = fmaxf(m, m2);
  if (M == -INFINITY) { m = M; s = 0.f; return; }
  s = s * __expf(m - M) + s2 * __expf(m2 - M);
  m = M;
}

template <int DT>  // 0 = f32, 1 = bf16, 2 = fp16
__global__ __launch_bounds__(256) void xent_stats_kernel(
    const void* __restrict__ logits, const long long* __restrict__ labels, int V,
    long long vocab_start, int ignore_index, float* __restrict__ out_max,
    float* __restrict__ out_sum, float* __restrict__ out_target) {
  constexpr bool BF16 = DT != 0, F16 = DT == 2;  // BF16: any 16-bit storage
  const int row = blockIdx.x;
  const size_t base = (size_t)row * V;
  float m = -INFINITY, s = 0.f;
  if (BF16 && (V % 8) == 0) {
    const u16x8* p = reinterpret_cast<const u16x8*>((const bf16_t*)logits + base);
    for (int i = threadIdx.x; i < V / 8; i += 256) {
      u16x8 r = p[i];
      float x[8], lm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) { x[j] = h2f<F16>(r[j]); lm = fmaxf(lm, x[j]); }
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ls += __expf(x[j] - lm);
      online_merge(m, s, lm, ls);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += 256) {
      float x = BF16 ? h2f<F16>(((const bf16_t*)logits)[base + i]) : ((const float*)logits)[base + i];
      online_update(m, s, x);
    }
  }
  // wave merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
  }
  __shared__ float sm[4], ss[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int i = 1; i < 4; ++i) online_merge(M, S, sm[i], ss[i]);
    out_max[row] = M;
    out_sum[row] = S;
    const long long lab = labels[row];
    float t = 0.f;
    if (lab != ignore_index && lab >= vocab_start && lab < vocab_start + V) {
      const size_t k = base + (size_t)(lab - vocab_start);
      t = BF16 ? h2f<F16>(((const bf16_t*)logits)[k]) : ((const float*)logits)[k];
    }
    out_target[row] = t;
  }
}

// grad[row, j] = (exp(x - lse) - [j == label]) * dloss[row]   (0 for ignored rows)
template <int DT>  // 0 = f32, 1 = bf16, 2 = fp16
__global__ __launch_bounds__(256) void xent_bwd_kernel(
    const void* __restrict__ logits, const long long* __restrict__ labels,
    const float* __restrict__ lse, const float* __restrict__ dloss, float dloss_scalar, int V,
    long long vocab_start, int ignore_index, void* __restrict__ grad) {
  constexpr bool BF16 = DT != 0, F16 = DT == 2;  // BF16: any 16-bit storage
  const int row = blockIdx.x;
  const size_t base = (size_t)row * V;
  const long long lab = labels[row];
  const float L = lse[row];
  const float d = lab == ignore_index ? 0.f : (dloss ? dloss[row] : dloss_scalar);
  const long long tl = lab - vocab_start;
  if (BF16 && (V % 8) == 0) {
    const u16x8* p = reinterpret_cast<const u16x8*>((const bf16_t*)logits + base);
    u16x8* q = reinterpret_cast<u16x8*>((bf16_t*)grad + base);
    for (int i = threadIdx.x; i < V / 8; i += 256) {
      u16x8 r = p[i], o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float g = __expf(h2f<F16>(r[j]) - L);
        if ((long long)(i * 8 + j) == tl) g -= 1.f;
        o[j] = f2h<F16>(g * d);
      }
      q[i] = o;
    }
  } else {
    for (int i = threadIdx.x; i < V; i += 256) {
      float x = BF16 ? h2f<F16>(((const bf16_t*)logits)[base + i]) : ((const float*)logits)[base + i];
      float g = __expf(x - L);
      if ((long long)i == tl) g -= 1.f;
      g *= d;
      if (BF16) ((bf16_t*)grad)[base + i] = f2h<F16>(g);
      else ((float*)grad)[base + i] = g;
    }
  }
}

}  // namespace

// dtype: 0 = f32, 1 = bf16, 2 = fp16.
// Per-row local statistics: max, Σexp(x - max), target logit (0 if label not in this shard).
PIAMD_EXPORT int piamd_xent_stats(int dtype, const void* logits, const long long* labels, int rows,
                                  int V, long long vocab_start, int ignore_index, float* out_max,
                                  float* out_sum, float* out_target, hipStream_t stream) {
  if (rows == 0) return 0;
#define XS(D)                                                                                     \
  hipLaunchKernelGGL((xent_stats_kernel<D>), dim3(rows), dim3(256), 0, stream, logits, labels, V, \
                     vocab_start, ignore_index, out_max, out_sum, out_target)
  if (dtype == 1) XS(1); else if (dtype == 2) XS(2); else if (dtype == 0) XS(0);
  else return (int)hipErrorInvalidValue;
#undef XS
  return (int)hipGetLastError();
}

// Backward; grad may alias logits (in-place). dloss: per-row device array or null (then the
// host scalar dloss_scalar applies to every row, e.g. 1/num_tokens for a mean loss).
PIAMD_EXPORT int piamd_xent_bwd(int dtype, const void* logits, const long long* labels,
                                const float* lse, const float* dloss, float dloss_scalar, int rows,
                                int V, long long vocab_start, int ignore_index, void* grad,
                                hipStream_t stream) {
  if (rows == 0) return 0;
#define XB(D)                                                                                     \
  hipLaunchKernelGGL((xent_bwd_kernel<D>), dim3(rows), dim3(256), 0, stream, logits, labels, lse, \
                     dloss, dloss_scalar, V, vocab_start, ignore_index, grad)
  if (dtype == 1) XB(1); else if (dtype == 2) XB(2); else if (dtype == 0) XB(0);
  else return (int)hipErrorInvalidValue;
#undef XB
  return (int)hipGetLastError();
}
