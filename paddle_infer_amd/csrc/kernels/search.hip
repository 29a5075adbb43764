// Beam-search step: softmax + per-beam top-K + per-batch top-beam + beam-offset / cache-id update.
//
// Parity: reference `phi/kernels/fusion/gpu/beam_search_softmax.cu` (op `beam_search_softmax`,
// python `paddle/tensor/search.py:1111`): identical outputs (ids_this_time, out_cum_scores,
// cache_ids, beam_offsets, parent_idx, stop_flags_out, seq_lens_out, step_ids_out), the same
// ordering rule (score descending, ties → smaller token id, then earlier candidate), the
// length-penalty rescaling of the running score, finished beams (only end_id, score kept) and the
// early-stop variant (finished beams keep their slot, the rest are filled by the best live
// candidates).
//
// MI355X design — two launches per decode step, no host round trip (hipGraph-capturable):
//   stage 1: grid (rows = batch·beam, P vocab slices) × 256 threads. Every thread keeps a sorted
//            top-KP (KP = next power of two ≥ beam, ≤ 16) and an online (max, Σexp) pair over its
//            strided vocab elements (logits read once, f32 or bf16); the block merges them with KP
//            rounds of wave64-shuffle argmax over LDS-resident candidates.
//   stage 2: one wave per batch entry: merges the P slices of each beam row (softmax
//            normaliser + top-K in f32), applies the length penalty and the running score, picks
//            the best `beam` of the beam·K candidates, writes the per-beam outputs and rewrites
//            the beam-offset / cache-id histories of the batch entry with the 64 lanes.
#include "common.h"
#include <float.h>

namespace {

constexpr int S1_THREADS = 256;

struct Cand {
  float v;
  int id;
};

// "a ranks before b": larger value, ties → smaller id
__device__ __forceinline__ bool before(float av, int aid, float bv, int bid) {
  return av > bv || (av == bv && (unsigned)aid < (unsigned)bid);
}

// lane-parallel argmax over a wave: returns the winning (v, id, index) broadcast to all lanes
__device__ __forceinline__ void wave_best(float& v, int& id, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oid = __shfl_xor(id, o, 64), oidx = __shfl_xor(idx, o, 64);
    const bool take = before(ov, oid, v, id) || (ov == v && oid == id && oidx < idx);
    if (take) { v = ov; id = oid; idx = oidx; }
  }
}

template <int KP, typename T>
__global__ __launch_bounds__(S1_THREADS) void bss_stage1(
    const T* __restrict__ logits, const unsigned char* __restrict__ stop, const int* __restrict__ end_ids,
    float* __restrict__ part, int V, int K, int fuse_softmax) {
  const int row = blockIdx.x, P = gridDim.y, p = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int vs = (V + P - 1) / P, v0 = p * vs, v1 = min(V, v0 + vs);
  const bool fin = stop[row] != 0;
  const int eid = end_ids[0];
  const T* lg = logits + (long long)row * V;

  float tv[KP];
  int ti[KP];
#pragma unroll
  for (int i = 0; i < KP; ++i) { tv[i] = -FLT_MAX; ti[i] = -1; }
  float m = -FLT_MAX, s = 0.f;
  for (int e = v0 + tid; e < v1; e += S1_THREADS) {
    float x;
    if (fin) x = e == eid ? (fuse_softmax ? FLT_MAX : 0.f) : -FLT_MAX;
    else x = (float)lg[e];
    if (fuse_softmax) {  // online softmax statistics (exp relative to the running max)
      if (x > m) { s = s * __expf(m - x) + 1.f; m = x; }
      else s += __expf(x - m);
    }
    if (before(x, e, tv[KP - 1], ti[KP - 1]) || ti[KP - 1] == -1) {
      tv[KP - 1] = x; ti[KP - 1] = e;
#pragma unroll
      for (int k = KP - 2; k >= 0; --k) {
        if (ti[k] == -1 || before(tv[k + 1], ti[k + 1], tv[k], ti[k])) {
          const float a = tv[k]; tv[k] = tv[k + 1]; tv[k + 1] = a;
          const int b = ti[k]; ti[k] = ti[k + 1]; ti[k + 1] = b;
        }
      }
    }
  }
  // block softmax statistics
  __shared__ float red_m[S1_THREADS / 64], red_s[S1_THREADS / 64];
  if (fuse_softmax) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
      const float nm = fmaxf(m, om);
      s = (m == -FLT_MAX ? 0.f : s * __expf(m - nm)) + (om == -FLT_MAX ? 0.f : os * __expf(om - nm));
      m = nm;
    }
    if (lane == 0) { red_m[w] = m; red_s[w] = s; }
  }
  // candidates to LDS; K rounds of block argmax
  __shared__ Cand cand[S1_THREADS * KP];
  __shared__ Cand wbest[S1_THREADS / 64];
  __shared__ int wbidx[S1_THREADS / 64];
#pragma unroll
  for (int i = 0; i < KP; ++i) cand[tid * KP + i] = Cand{tv[i], ti[i]};
  __syncthreads();
  float* out = part + ((long long)row * P + p) * (2 * K + 2);
  int head = 0;  // this thread's candidates are sorted: the next unused one
  for (int r = 0; r < K; ++r) {
    float v = -FLT_MAX;
    int id = -1, idx = tid;
    if (head < KP) { v = cand[tid * KP + head].v; id = cand[tid * KP + head].id; }
    if (id == -1) v = -FLT_MAX, id = 0x7fffffff;
    wave_best(v, id, idx);
    if (lane == 0) { wbest[w] = Cand{v, id}; wbidx[w] = idx; }
    __syncthreads();
    float bv = wbest[0].v;
    int bid = wbest[0].id, bidx = wbidx[0];
#pragma unroll
    for (int i = 1; i < S1_THREADS / 64; ++i)
      if (before(wbest[i].v, wbest[i].id, bv, bid)) { bv = wbest[i].v; bid = wbest[i].id; bidx = wbidx[i]; }
    if (tid == bidx) ++head;
    if (tid == 0) {
      reinterpret_cast<int*>(out)[r] = bid == 0x7fffffff ? -1 : bid;
      out[K + r] = bv;
    }
    __syncthreads();
  }
  if (tid == 0) {
    float M = -FLT_MAX, Ssum = 0.f;
    if (fuse_softmax) {
#pragma unroll
      for (int i = 0; i < S1_THREADS / 64; ++i) M = fmaxf(M, red_m[i]);
#pragma unroll
      for (int i = 0; i < S1_THREADS / 64; ++i)
        Ssum += red_m[i] == -FLT_MAX ? 0.f : red_s[i] * __expf(red_m[i] - M);
    }
    out[2 * K] = M;
    out[2 * K + 1] = Ssum;
  }
}

// one wave per batch entry. cand scratch in LDS: beam rows x (P*K) slice candidates.
__global__ __launch_bounds__(64) void bss_stage2(
    const float* __restrict__ part, int P, int K, int beam, const float* __restrict__ cum,
    const int* __restrict__ seq_lens, const unsigned char* __restrict__ stop,
    const int* __restrict__ end_ids, const int* __restrict__ step_ids,
    const int* __restrict__ last_cache_ids, const int* __restrict__ last_beam_offsets,
    int* __restrict__ ids_out, float* __restrict__ cum_out, int* __restrict__ cache_ids,
    int* __restrict__ beam_offsets, int* __restrict__ parent_out, unsigned char* __restrict__ stop_out,
    int* __restrict__ seq_lens_out, int* __restrict__ step_ids_out, int fuse_softmax,
    int early_stop, float length_penalty, int max_len_off, int max_dec_len) {
  extern __shared__ char smem_raw[];
  float* row_v = reinterpret_cast<float*>(smem_raw);   // [beam][K] per-row top-K scores
  int* row_i = reinterpret_cast<int*>(row_v + beam * K);  // [beam][K] token ids
  int* sel_par = row_i + beam * K;                       // [beam] chosen parent
  const int bi = blockIdx.x, lane = threadIdx.x;
  const int NC = P * K;

  for (int j = 0; j < beam; ++j) {
    const int row = bi * beam + j;
    const float* pr = part + (long long)row * P * (2 * K + 2);
    float M = -FLT_MAX, Ssum = 0.f;
    if (fuse_softmax) {
      for (int q = lane; q < P; q += 64) M = fmaxf(M, pr[q * (2 * K + 2) + 2 * K]);
      M = wave_max(M);
      for (int q = lane; q < P; q += 64) {
        const float mq = pr[q * (2 * K + 2) + 2 * K], sq = pr[q * (2 * K + 2) + 2 * K + 1];
        Ssum += mq == -FLT_MAX ? 0.f : sq * __expf(mq - M);
      }
      Ssum = wave_sum(Ssum);
    }
    // running score with the length penalty restored (cum is stored penalised)
    float cl = cum[row], pen = 1.f;
    if (length_penalty != 0.f && !stop[row]) {
      const float prev = powf((float)step_ids[row], length_penalty);
      pen = powf((float)step_ids[row] + 1.f, length_penalty);
      cl = cl * prev / pen;
    }
    const float lse = fuse_softmax ? M + logf(Ssum) : 0.f;
    // K rounds of argmax over the P*K slice candidates (each slice list is sorted)
    for (int r = 0; r < K; ++r) {
      float v = -FLT_MAX;
      int id = 0x7fffffff, idx = 0x7fffffff;
      for (int c = lane; c < NC; c += 64) {
        const int q = c / K, t = c % K;
        const int cid = reinterpret_cast<const int*>(pr + q * (2 * K + 2))[t];
        if (cid < 0) continue;
        bool used = false;
        for (int u = 0; u < r; ++u) used |= row_i[j * K + u] == cid;
        if (used) continue;
        const float cv = pr[q * (2 * K + 2) + K + t];
        if (before(cv, cid, v, id)) { v = cv; id = cid; idx = c; }
      }
      wave_best(v, id, idx);
      if (lane == 0) {
        row_i[j * K + r] = id == 0x7fffffff ? -1 : id;
        row_v[j * K + r] = id == 0x7fffffff ? -FLT_MAX : (v - lse) / pen + cl;
      }
      __syncthreads();
    }
  }
  // batch selection over beam x K candidates
  const int first = step_ids[0] == 0;
  const int nc = first ? K : beam * K;
  int nstop = 0;
  if (early_stop)
    for (int j = 0; j < beam; ++j) nstop += stop[bi * beam + j] != 0;
  const int nsel = beam - nstop;
  for (int r = 0; r < nsel; ++r) {
    float v = -FLT_MAX;
    int id = 0x7fffffff, idx = 0x7fffffff;
    for (int c = lane; c < nc; c += 64) {
      const int par = c / K;
      if (early_stop && !first && stop[bi * beam + par]) continue;
      if (row_i[c] < 0) continue;
      if (before(row_v[c], row_i[c], v, id) || (row_v[c] == v && row_i[c] == id && c < idx)) {
        v = row_v[c]; id = row_i[c]; idx = c;
      }
    }
    wave_best(v, id, idx);
    if (lane == 0) {
      // slot: without early stop r; with early stop the r-th non-finished slot
      int slot = r;
      if (early_stop) {
        int seen = -1;
        for (int j = 0; j < beam; ++j)
          if (!stop[bi * beam + j] && ++seen == r) { slot = j; break; }
      }
      const int o = bi * beam + slot;
      const int par = idx == 0x7fffffff ? 0 : idx / K;
      ids_out[o] = id == 0x7fffffff ? -1 : id;
      cum_out[o] = v;
      parent_out[o] = par;
      sel_par[slot] = par;
      stop_out[o] = stop[bi * beam + par];
      seq_lens_out[o] = seq_lens[bi * beam + par];
      step_ids_out[o] = step_ids[bi * beam + par];
      if (idx != 0x7fffffff) row_i[idx] = -2;  // consumed
    }
    __syncthreads();
  }
  if (early_stop && lane == 0) {
    for (int j = 0; j < beam; ++j) {
      const int o = bi * beam + j;
      if (!stop[o]) continue;
      ids_out[o] = end_ids[0];
      cum_out[o] = cum[o];
      parent_out[o] = j;
      sel_par[j] = j;
      stop_out[o] = stop[o];
      seq_lens_out[o] = seq_lens[o];
      // step_ids_out keeps its (copied) value
    }
  }
  __syncthreads();
  // histories (outputs start as copies of the inputs, done by the host wrapper)
  const int max_len = max_len_off + max_dec_len;
  for (int j = 0; j < beam; ++j) {
    const int o = bi * beam + j, src_beam = sel_par[j], src = bi * beam + src_beam;
    const int sl = seq_lens[src];
    if (sl != 0) {
      const int tmax = min(sl + 1, max_len);
      for (int t = lane; t < tmax; t += 64)
        beam_offsets[(long long)o * max_len + t] =
            t == sl ? src_beam : last_beam_offsets[(long long)src * max_len + t];
      const int st = step_ids[src];
      const int cmax = min(st + 1, max_dec_len);
      for (int t = lane; t < cmax; t += 64)
        cache_ids[(long long)o * max_dec_len + t] =
            t == st ? ids_out[o] : last_cache_ids[(long long)src * max_dec_len + t];
    }
  }
}

}  // namespace

// logits [bs*beam, V] (f32 when logits_bf16 == 0, else bf16); cum/… [bs*beam]; stop bool bytes;
// last_cache_ids [bs*beam, max_dec_len]; last_beam_offsets [bs*beam, max_seq_len + max_dec_len].
// Outputs must be pre-initialised as copies (cache_ids, beam_offsets, stop_out, seq_lens_out,
// step_ids_out). part: f32 workspace of bs*beam*P*(2*beam+2). beam ≤ 16.
PIAMD_EXPORT int piamd_beam_search_softmax(
    const void* logits, int logits_bf16, const float* cum, const int* seq_lens,
    const unsigned char* stop, const int* end_ids, const int* step_ids, const int* last_cache_ids,
    const int* last_beam_offsets, int bs, int beam, int V, int max_seq_len, int max_dec_len,
    int fuse_softmax, int early_stop, float length_penalty, int P, float* part, int* ids_out,
    float* cum_out, int* cache_ids, int* beam_offsets, int* parent_out, unsigned char* stop_out,
    int* seq_lens_out, int* step_ids_out, hipStream_t st) {
  if (beam < 1 || beam > 16 || bs < 1 || V < 1 || P < 1 || P > 1024) return (int)hipErrorInvalidValue;
  const dim3 g1(bs * beam, P);
  const int KP = beam <= 1 ? 1 : beam <= 2 ? 2 : beam <= 4 ? 4 : beam <= 8 ? 8 : 16;
#define S1(KK)                                                                                    \
  if (logits_bf16)                                                                                \
    hipLaunchKernelGGL((bss_stage1<KK, __bf16>), g1, dim3(S1_THREADS), 0, st,                     \
                       (const __bf16*)logits, stop, end_ids, part, V, beam, fuse_softmax);        \
  else                                                                                            \
    hipLaunchKernelGGL((bss_stage1<KK, float>), g1, dim3(S1_THREADS), 0, st,                      \
                       (const float*)logits, stop, end_ids, part, V, beam, fuse_softmax)
  switch (KP) {
    case 1: S1(1); break;
    case 2: S1(2); break;
    case 4: S1(4); break;
    case 8: S1(8); break;
    default: S1(16); break;
  }
#undef S1
  const size_t sm = (size_t)beam * beam * 8 + beam * 4;
  hipLaunchKernelGGL(bss_stage2, dim3(bs), dim3(64), sm, st, part, P, beam, beam, cum, seq_lens,
                     stop, end_ids, step_ids, last_cache_ids, last_beam_offsets, ids_out, cum_out,
                     cache_ids, beam_offsets, parent_out, stop_out, seq_lens_out, step_ids_out,
                     fuse_softmax, early_stop, length_penalty, max_seq_len, max_dec_len);
  return (int)hipGetLastError();
}

// Greedy decoding: out[r] = argmax_v logits[r, v] (ties → the smaller id; NaNs are skipped unless
// the whole row is NaN — unlike torch.argmax, which returns a NaN's index; equal on finite rows), one 1024-thread workgroup per row: each
// lane keeps a running (max, id) over 16-B vector loads (8 bf16/fp16 or 4 f32), then one wave64
// shuffle argmax per wave and a 16-entry LDS merge. One launch, no workspace, capturable.
namespace {
template <typename T>
__device__ __forceinline__ float to_f(T v) { return (float)v; }
__device__ __forceinline__ void amax_merge(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}
template <typename T, int VEC>
__global__ __launch_bounds__(1024) void argmax_rows_kernel(const T* __restrict__ x, long long ld,
                                                           int V, long long* __restrict__ out) {
  const T* row = x + (long long)blockIdx.x * ld;
  float best = -INFINITY;
  int bid = 0x7fffffff;
  const int nvec = V / VEC;
  for (int c = threadIdx.x; c < nvec; c += 1024) {
    typedef T TV __attribute__((ext_vector_type(VEC)));
    const TV t = *reinterpret_cast<const TV*>(row + (long long)c * VEC);
#pragma unroll
    for (int j = 0; j < VEC; ++j) amax_merge(best, bid, to_f(t[j]), c * VEC + j);
  }
  for (int v = nvec * VEC + threadIdx.x; v < V; v += 1024) amax_merge(best, bid, to_f(row[v]), v);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bid, o, 64);
    amax_merge(best, bid, v2, i2);
  }
  __shared__ float sv[16];
  __shared__ int si[16];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sv[w] = best; si[w] = bid; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 16; ++k) amax_merge(best, bid, sv[k], si[k]);
    out[blockIdx.x] = bid == 0x7fffffff ? 0 : bid;
  }
}
}  // namespace

// logits rows [R][ld] (dtype 0 f32, 1 bf16, 2 fp16), R ≥ 1, V ≥ 1 → out int64 [R]. Vector loads
// need ld and the base 16-B aligned (the caller passes contiguous rows; else scalar path: VEC 1).
PIAMD_EXPORT int piamd_argmax_rows(const void* x, long long ld, int R, int V, int dtype, long long* out,
                                   hipStream_t st) {
  if (R < 1 || V < 1 || dtype < 0 || dtype > 2) return (int)hipErrorInvalidValue;
  const int esz = dtype == 0 ? 4 : 2;
  const bool vec = ((uintptr_t)x % 16 == 0) && ((ld * esz) % 16 == 0);
  if (dtype == 0) {
    if (vec) hipLaunchKernelGGL((argmax_rows_kernel<float, 4>), dim3(R), dim3(1024), 0, st, (const float*)x, ld, V, out);
    else hipLaunchKernelGGL((argmax_rows_kernel<float, 1>), dim3(R), dim3(1024), 0, st, (const float*)x, ld, V, out);
  } else if (dtype == 1) {
    if (vec) hipLaunchKernelGGL((argmax_rows_kernel<__bf16, 8>), dim3(R), dim3(1024), 0, st, (const __bf16*)x, ld, V, out);
    else hipLaunchKernelGGL((argmax_rows_kernel<__bf16, 1>), dim3(R), dim3(1024), 0, st, (const __bf16*)x, ld, V, out);
  } else {
    if (vec) hipLaunchKernelGGL((argmax_rows_kernel<_Float16, 8>), dim3(R), dim3(1024), 0, st, (const _Float16*)x, ld, V, out);
    else hipLaunchKernelGGL((argmax_rows_kernel<_Float16, 1>), dim3(R), dim3(1024), 0, st, (const _Float16*)x, ld, V, out);
  }
  return (int)hipGetLastError();
}
