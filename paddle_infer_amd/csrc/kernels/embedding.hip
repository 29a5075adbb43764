// Token + position embedding lookup (forward) and its deterministic gradient (backward).
//
// Parity: reference `paddle/phi/kernels/gpu/embedding_kernel.cu` / `embedding_grad_kernel.cu`
// (lookup_table_v2), `c_embedding_op.cu` (vocab-parallel lookup: ids outside this rank's
// [start, start + V_local) produce zero rows) and the GPT embedding (word + learned position).
//
// Forward fuses the two gathers and the add: out[t] = W[id_t - start] + P[pos_t], 16-B vector
// loads / stores (H % 8 == 0), grid-stride; bf16 (the training path) or, through the *_dt entry
// points, f32 / fp16 tables (paddle.nn.functional.embedding; padding ids arrive as −1 = zero row).
//
// Backward is sort-based and atomic-free (deterministic, f32 accumulation — repeated tokens are
// summed in registers, not by bf16 atomics that would round at every add): the host side sorts
// the ids once on the device (`torch.sort`); block i handles sorted position i and exits unless it
// starts a run of equal ids, otherwise it sums the run's dy rows in f32 and adds the result into
// dW[id] (bf16 or f32 main-grad) with one read-modify-write — no two blocks touch the same row.
// Position gradients for the default positions (pos = t mod S) are a strided column sum over the
// batch, one block per (position, column chunk).
#include "common.h"

namespace {

// 8 consecutive elements of dtype DT (0 f32, 1 bf16, 2 fp16) ↔ f32 registers
template <int DT>
__device__ __forceinline__ void ld8(const void* base, long long idx, float (&v)[8]) {
  if constexpr (DT == 0) {
    const f32x4* q = reinterpret_cast<const f32x4*>((const float*)base + idx);
    const f32x4 a = q[0], b = q[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  } else {
    const u16x8 u = *reinterpret_cast<const u16x8*>((const unsigned short*)base + idx);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = DT == 1 ? bf2f(u[j]) : h2f<true>(u[j]);
  }
}

template <int DT>
__device__ __forceinline__ void st8(void* base, long long idx, const float (&v)[8]) {
  if constexpr (DT == 0) {
    f32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[4 + j]; }
    f32x4* q = reinterpret_cast<f32x4*>((float*)base + idx);
    q[0] = a;
    q[1] = b;
  } else {
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = DT == 1 ? f2bf(v[j]) : f2h<true>(v[j]);
    *reinterpret_cast<u16x8*>((unsigned short*)base + idx) = o;
  }
}

template <int DT>
__global__ void emb_fwd_kernel(const long long* __restrict__ ids, const void* __restrict__ w,
                               long long start, int vlocal, const void* __restrict__ p,
                               const long long* __restrict__ pos, int S,
                               void* __restrict__ out, long long T, int H) {
  const int hv = H / 8;
  const long long total = T * hv;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long t = i / hv;
    const int c = (int)(i % hv) * 8;
    const long long id = ids[t] - start;
    float v[8];
    if (id >= 0 && id < vlocal) {
      ld8<DT>(w, id * H + c, v);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
    if (p) {
      const long long ps = pos ? pos[t] : t % S;
      float b[8];
      ld8<DT>(p, ps * H + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += b[j];
    }
    st8<DT>(out, t * H + c, v);
  }
}

// one block (256 threads) per sorted position; columns in chunks of 256 x 8
template <bool F32OUT, int DT = 1>
__global__ __launch_bounds__(256) void emb_bwd_kernel(const long long* __restrict__ sorted,
                                                      const long long* __restrict__ order,
                                                      const void* __restrict__ dy,
                                                      void* __restrict__ dw, long long start,
                                                      int vlocal, long long T, int H,
                                                      int accumulate) {
  const long long i = blockIdx.x;
  const long long id = sorted[i];
  if (i > 0 && sorted[i - 1] == id) return;  // not the head of a run
  const long long row = id - start;
  if (row < 0 || row >= vlocal) return;  // another vocab shard's token
  long long end = i + 1;
  while (end < T && sorted[end] == id) ++end;
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (long long s = i; s < end; ++s) {
      float g[8];
      ld8<DT>(dy, order[s] * H + c, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += g[j];
    }
    if (F32OUT) {
      float* d = (float*)dw + row * H + c;
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = (accumulate ? d[j] : 0.f) + acc[j];
    } else {
      bf16_t* d = (bf16_t*)dw + row * H + c;
      u16x8 o;
      const u16x8 old = accumulate ? *reinterpret_cast<const u16x8*>(d) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j] + (accumulate ? bf2f(old[j]) : 0.f));
      *reinterpret_cast<u16x8*>(d) = o;
    }
  }
}

// dP[s][c] (+)= Σ_b dy[b*S + s][c]; grid (S, ceil(H / 2048)), 256 threads x 8 columns
template <bool F32OUT>
__global__ __launch_bounds__(256) void pos_bwd_kernel(const bf16_t* __restrict__ dy,
                                                      void* __restrict__ dp, int B, int S, int H,
                                                      int accumulate) {
  const int s = blockIdx.x, c = (blockIdx.y * 256 + threadIdx.x) * 8;
  if (c >= H) return;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int b = 0; b < B; ++b) {
    const u16x8 g = *reinterpret_cast<const u16x8*>(dy + ((long long)b * S + s) * H + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(g[j]);
  }
  if (F32OUT) {
    float* d = (float*)dp + (long long)s * H + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = (accumulate ? d[j] : 0.f) + acc[j];
  } else {
    bf16_t* d = (bf16_t*)dp + (long long)s * H + c;
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j] + (accumulate ? bf2f(d[j]) : 0.f));
    *reinterpret_cast<u16x8*>(d) = o;
  }
}

}  // namespace

// out [T][H] bf16 = W[ids - start] (zero outside [0, vlocal)) + P[pos] (P may be null; pos null →
// t mod S). H % 8 == 0, 16-B aligned rows.
PIAMD_EXPORT int piamd_embedding_fwd(const long long* ids, const void* w, long long start,
                                     int vlocal, const void* p, const long long* pos, int S,
                                     void* out, long long T, int H, hipStream_t st) {
  if (H % 8 || T < 0 || (p && !pos && S < 1)) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  hipLaunchKernelGGL(emb_fwd_kernel<1>, dim3(stride_grid(T * (H / 8), 256)), dim3(256), 0, st, ids, w,
                     start, vlocal, p, pos, S, out, T, H);
  return (int)hipGetLastError();
}

// Any element type (dtype 0 f32, 1 bf16, 2 fp16: weight, position table and output alike).
PIAMD_EXPORT int piamd_embedding_fwd_dt(int dtype, const long long* ids, const void* w, long long start,
                                        int vlocal, const void* p, const long long* pos, int S,
                                        void* out, long long T, int H, hipStream_t st) {
  if (H % 8 || T < 0 || (p && !pos && S < 1) || dtype < 0 || dtype > 2) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  const dim3 grid(stride_grid(T * (H / 8), 256));
  if (dtype == 0)
    hipLaunchKernelGGL(emb_fwd_kernel<0>, grid, dim3(256), 0, st, ids, w, start, vlocal, p, pos, S, out, T, H);
  else if (dtype == 2)
    hipLaunchKernelGGL(emb_fwd_kernel<2>, grid, dim3(256), 0, st, ids, w, start, vlocal, p, pos, S, out, T, H);
  else
    hipLaunchKernelGGL(emb_fwd_kernel<1>, grid, dim3(256), 0, st, ids, w, start, vlocal, p, pos, S, out, T, H);
  return (int)hipGetLastError();
}

// dW (f32) (+)= Σ dy rows per id for a dy of any element type (dtype as above).
PIAMD_EXPORT int piamd_embedding_bwd_dt(int dtype, const long long* sorted, const long long* order,
                                        const void* dy, float* dw, long long start, int vlocal, long long T,
                                        int H, int accumulate, hipStream_t st) {
  if (H % 8 || T < 0 || dtype < 0 || dtype > 2) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  if (dtype == 0)
    hipLaunchKernelGGL((emb_bwd_kernel<true, 0>), dim3(T), dim3(256), 0, st, sorted, order, dy, dw, start,
                       vlocal, T, H, accumulate);
  else if (dtype == 2)
    hipLaunchKernelGGL((emb_bwd_kernel<true, 2>), dim3(T), dim3(256), 0, st, sorted, order, dy, dw, start,
                       vlocal, T, H, accumulate);
  else
    hipLaunchKernelGGL((emb_bwd_kernel<true, 1>), dim3(T), dim3(256), 0, st, sorted, order, dy, dw, start,
                       vlocal, T, H, accumulate);
  return (int)hipGetLastError();
}

// dW[id - start] (+)= Σ dy rows of that id. sorted = ids sorted ascending, order = their
// original token rows (torch.sort). dw_f32: dW is f32 (else bf16).
PIAMD_EXPORT int piamd_embedding_bwd(const long long* sorted, const long long* order,
                                     const void* dy, void* dw, int dw_f32, long long start,
                                     int vlocal, long long T, int H, int accumulate,
                                     hipStream_t st) {
  if (H % 8 || T < 0) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  if (dw_f32)
    hipLaunchKernelGGL((emb_bwd_kernel<true, 1>), dim3(T), dim3(256), 0, st, sorted, order, dy, dw, start,
                       vlocal, T, H, accumulate);
  else
    hipLaunchKernelGGL((emb_bwd_kernel<false, 1>), dim3(T), dim3(256), 0, st, sorted, order, dy, dw, start,
                       vlocal, T, H, accumulate);
  return (int)hipGetLastError();
}

// dP[0:S] (+)= Σ over the batch of dy [B][S][H] (default positions).
PIAMD_EXPORT int piamd_pos_embedding_bwd(const void* dy, void* dp, int dp_f32, int B, int S,
                                         int H, int accumulate, hipStream_t st) {
  if (H % 8 || B < 1 || S < 1) return (int)hipErrorInvalidValue;
  dim3 grid(S, (H + 2047) / 2048);
  if (dp_f32)
    hipLaunchKernelGGL(pos_bwd_kernel<true>, grid, dim3(256), 0, st, (const bf16_t*)dy, dp, B, S,
                       H, accumulate);
  else
    hipLaunchKernelGGL(pos_bwd_kernel<false>, grid, dim3(256), 0, st, (const bf16_t*)dy, dp, B, S,
                       H, accumulate);
  return (int)hipGetLastError();
}
