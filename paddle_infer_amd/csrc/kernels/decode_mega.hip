// Persistent whole-stack decode step ("megakernel") for GPT decoding on gfx950 (1, 2 or 4 rows).
//
// Why: a decode step is a chain of 5 small launches per layer (QKV GEMV → attention → out GEMV →
// FFN1 GEMV → FFN2 GEMV). Each GEMV streams 8-33 MB of weights and sits at its ramp floor
// (profiles/gemv_decode_r3_nt.txt: 25 MB in ≈9 µs ≈ 2.8 TB/s) — HBM idles while a launch drains
// and the next ramps up. Weights do not depend on activations, so one persistent kernel can load
// the NEXT projection's weights while the current phase finishes and the grid syncs.
//
// Design (one launch per token for all layers):
//   * grid = 256 workgroups (one per CU) × 256 threads; every GEMV phase splits its N output
//     columns evenly: WG w owns rows [w·NPW, (w+1)·NPW) of the [N][K] (out, in) weight, a
//     CONTIGUOUS slice of ≤ 128 KiB held in LDS with every row padded by 16 B.
//   * waves 1..3 are loaders: right after a phase has consumed its LDS slice they issue the next
//     phase's slice with direct-to-LDS DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction),
//     while wave 0 publishes the phase's outputs and waits on the grid barrier — the weight stream
//     overlaps the barrier instead of following it. (A wave's loads retire in order, so the
//     barrier-polling wave must not own prefetches; hence the loader / control split.)
//   * the GEMV phases run on MFMA (gemv_mfma: activations staged in LDS, mfma_f32_16x16x32_bf16
//     straight on the padded weight rows; int8 / int4 weight-only codes widened in registers);
//     the VALU form (gemv_lds) remains for A/B instantiations.
//   * cross-workgroup data (residual, q / new k,v, attention partials, FFN hidden) is published
//     with agent-scope relaxed atomic stores into slots written once per launch (plain loads are
//     then coherent across the 8 per-XCD L2s); the barrier is a two-level arrival counter polled
//     by one lane with s_sleep back-off. The grid is launched COOPERATIVELY
//     (hipLaunchCooperativeKernel after an occupancy check), so all 256 workgroups are co-resident
//     by the runtime's guarantee; the spin stays bounded as a safety net (a timeout raises `err`
//     and runs the launch to completion, every wave exits).
//   * per layer: LN1 (recomputed per WG from the residual) + QKV GEMV + bias, new k/v written to
//     the cache → split-K attention over the cache (one workgroup per (row, head, split), base-2
//     softmax, optional whole-head RoPE) → partial combine + out GEMV + bias + residual → LN2 +
//     FFN1 GEMV + bias + GELU → FFN2 GEMV + bias + residual. Rounding points match the
//     launch-per-op path (bf16 LN output, bf16 cache / attention output / hidden / residual).
// Shapes: decode_mega_kernel<MegaCfg<E, D, Hq, Hk, F, ROT, W8, NB, MM>> — the instantiated
// variants are listed at mega_fn (GPT-3 1.3B and 350M widths, a GQA 4:1 variant, ± rotary
// embedding, bf16 / int8 / int4 weights, 1 / 2 / 4 rows). Anything else: the host launcher
// refuses and the Python side takes the per-op path.
// Reference parity: one decode step of FusedMultiTransformer with time_step
// (`paddle/fluid/operators/fused/fused_multi_transformer_op.cu`, masked_multihead_attention).
#include "common.h"

namespace {

constexpr int NT = 256;                // threads per workgroup (4 waves)
constexpr int NWG = 256;               // workgroups (one per CU)
constexpr int E = 2048, D = 128, HQ = 16, HK = 16, F = 8192;
constexpr int NQKV = (HQ + 2 * HK) * D;  // 6144
constexpr int WBYTES = 128 * 1024;     // LDS weight slice
// LDS placement per layer: QKV [0, 96K) → out [96K, 128K) (free during QKV) → FFN1 [0, 128K),
// whose first 96 KiB stream in during the attention phase (workgroups without attention work) or
// the out-projection prologue (the others) and the last 32 KiB once the out slice is consumed → FFN2 [0, 128K) → next QKV [0, 96K).
constexpr int OUT_OFF = 96 * 1024;
constexpr int FFN1_PRE = 96 * 1024;
// per loader wave: FFN1_PRE / 1 KiB / 3 waves DMA instructions (the out phase waits for every
// older one: `s_waitcnt vmcnt(32)` in phase_start)
static_assert(FFN1_PRE / 1024 / 3 == 32, "phase_start WAIT_OLDER count");
constexpr int PSTRIDE = D + 2;         // attention partial: acc[D], m, l
// per-layer partial block, padded to 256 B
__host__ __device__ constexpr long pstride(int nsplit) { return ((long)HQ * nsplit * PSTRIDE + 63) / 64 * 64; }

typedef unsigned long long u64;

struct MegaLayer {
  const bf16_t *ln1_g, *ln1_b, *wqkv, *bqkv, *wo, *bo, *ln2_g, *ln2_b, *w1, *b1, *w2, *b2;
  bf16_t *kc, *vc;
  // int8 weight-only mode (MegaArgs.w8): the four weights above are int8 [out][in] and these
  // are their per-output-channel f32 scales (null otherwise)
  const float *sqkv, *so, *s1, *s2;
};

struct MegaArgs {
  const MegaLayer* layers;
  int nl;
  int maxS;
  int nsplit;
  int act;  // 0 gelu (erf), 1 gelu (tanh)
  float eps;
  float scale_log2;
  const bf16_t* resid;  // [E] input residual (embedding output)
  bf16_t* rbuf;         // [2·nl][E] residual after each out / FFN2 phase; the last row is the output
  float* qn;            // [nl][HQ·D] q + bias
  float* kvn;           // [nl][2·HK·D] new k, v (+bias, bf16-rounded)
  float* part;          // [nl][pstride_l] attention partials [HQ][nsplit][PSTRIDE]
  bf16_t* h;            // [nl][F] FFN hidden
  unsigned* bar;        // barrier words (BAR_WORDS; zero before the first launch, re-zeroed by each)
  int* err;             // number of launches in which a grid barrier timed out
  const int* pos;       // [1] cache slot of the new token
  u64* trace;           // nullable: [NWG][5·nl][4] wall-clock (100 MHz): phase start, prologue done,
                        // GEMV done, barrier arrival
  int late_dma;         // bit 0: the FFN phases issue the next slice only after their GEMV; bit 1:
                        // attention workgroups queue their FFN1 head in the out prologue instead
                        // of at the end of the attention phase; bit 2: the FFN2 slice head is
                        // touched right behind the FFN1 head (decode_mega_kernel; A/B knobs)
  int loader;           // must be 0 (the retired dedicated-loader variant; field kept for the ABI)
  int rot;              // rotary dims: 0 or D (whole head)
  int neox;             // 1: rotate-half (NeoX), 0: interleaved pairs (GPT-J)
  float log2_base;      // log2 of the rotary base
  int w8;               // weight format: 0 bf16, 1 int8, 2 int4 weight-only (MegaLayer scales)
  int nb;               // batch rows per step (1, 2 or 4): resid / rbuf / qn / kvn / part / h hold
                        // nb rows per slot, pos nb entries, the caches are [rows][HK][maxS][D]
  int mm;               // 1 = MFMA GEMV phases, 0 = VALU (MegaCfg MM; the instantiated variant)
};

__device__ __forceinline__ u64 ld64(const void* p) { return *reinterpret_cast<const u64*>(p); }
__device__ __forceinline__ void st64(void* p, u64 v) {
  __hip_atomic_store((u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ u64 pack2f(float a, float b) {
  return (u64)__float_as_uint(a) | ((u64)__float_as_uint(b) << 32);
}
// 8 bf16 at p (16 B aligned) published by other workgroups → f32
__device__ __forceinline__ void ld_bf8(const bf16_t* p, float* v) {
  const u16x8 u = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = bf2f(u[i]);
}

// Wave 0 only: this wave's publishing stores have completed → arrive → wait for barrier `b`
// (1-based). Two levels so no word sees more than 32 requesters: workgroup w arrives on the
// counter of group w % 8 (32 members); the last member of a group arrives on the global counter
// (8 members); the last group raises all 8 group flags; members poll their group's flag.
// Every word sits on its own 256-B line.
// Lines 0-7: group counters, 8: global counter, 9-16: group flags, 17: this launch's "a barrier
// timed out" flag, 18: exited workgroups. The last workgroup to exit zeroes all of them;
// `err` counts timed-out launches and is never reset by the kernel (MegaDecoder.check()).
constexpr int BAR_LINE = 64, BAR_WORDS = 19 * BAR_LINE;
// Barrier words are read with a read-modify-write (compare-and-swap against a value the word
// never holds): RMW atomics execute memory-side and see every XCD's update, while a plain
// agent-scope load may be served by a stale line in the poller's own L2 for as long as that line
// stays resident (measured: ~160 µs release latency under hipGraph replay).
__device__ __forceinline__ unsigned poll(unsigned* p) {
  unsigned expect = 0xFFFFFFFFu;
  __hip_atomic_compare_exchange_strong(p, &expect, 0xFFFFFFFFu, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return expect;
}
__device__ __forceinline__ void grid_sync(const MegaArgs& a, unsigned b, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (a.trace && lane == 0) a.trace[((long)blockIdx.x * a.nl * 5 + b - 1) * 4 + 3] = wall_clock64();
  if (lane == 0) {
    const int g = blockIdx.x & 7;
    unsigned* xc = a.bar + g * BAR_LINE;
    unsigned* gc = a.bar + 8 * BAR_LINE;
    unsigned* fl = a.bar + (9 + g) * BAR_LINE;
    if (__hip_atomic_fetch_add(xc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == b * (NWG / 8) - 1 &&
        __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == b * 8 - 1) {
      for (int i = 0; i < 8; ++i)
        __hip_atomic_fetch_max(a.bar + (9 + i) * BAR_LINE, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned spins = 0;
    while (poll(fl) < b) {
      __builtin_amdgcn_s_sleep(1);
      if ((++spins & 1023) == 0) {  // bounded: one timeout makes the launch's later barriers fall through
        unsigned* failed = a.bar + 17 * BAR_LINE;
        if (poll(failed)) break;
        if (spins > (1u << 21)) {
          if (__hip_atomic_exchange(failed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
            __hip_atomic_fetch_add(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
}

__device__ __forceinline__ void tmark(const MegaArgs& a, unsigned ph, int k) {
  if (a.trace && threadIdx.x == 0) a.trace[((long)blockIdx.x * a.nl * 5 + ph) * 4 + k] = wall_clock64();
}

// Loader waves: DMA bytes [from, to) (multiples of 1 KiB) of the slice at `src` into the same
// offsets of the LDS slice.
__device__ __forceinline__ void prefetch(const bf16_t* src, int from, int to, char* wl, int wv, int lane) {
  if (wv == 0 || src == nullptr) return;
  const char* s = reinterpret_cast<const char*>(src) + lane * 16;
  for (int p = (from >> 10) + wv - 1; p < (to >> 10); p += 3)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(s + p * 1024),
                                     (__attribute__((address_space(3))) void*)(wl + p * 1024), 16, 0, 0);
}

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at their no-wait maxima; gfx9 encoding: vmcnt
// in bits [3:0] and [15:14])
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// Phase entry: loader waves wait for their DMA (all of it, all but the newest OLD
// wave-instructions = the FFN1 head, or none), then the whole workgroup meets (wave 0 arrives here
// after its grid barrier).
enum { WAIT_ALL, WAIT_OLDER, WAIT_NONE };
template <int OLD>
__device__ __forceinline__ void phase_start(const MegaArgs& a, int wv, unsigned ph, int wait = WAIT_ALL) {
  if (wv != 0 && wait == WAIT_ALL) wait_vm<0>();
  if (wv != 0 && wait == WAIT_OLDER) wait_vm<OLD>();
  __syncthreads();
  if (a.trace && threadIdx.x == 0) a.trace[((long)blockIdx.x * a.nl * 5 + ph) * 4] = wall_clock64();
}

// One exchange level of the column-halving butterfly: lanes with bit O set keep the upper HALF
// columns, the others the lower, each adding its partner's copy. Compile-time recursion keeps
// every register index static (a runtime loop here became dynamic-index select chains).
template <int HALF, int O>
__device__ __forceinline__ void butterfly(float* acc, int lane) {
  const bool up = (lane & O) != 0;
#pragma unroll
  for (int i = 0; i < HALF; ++i) {
    const float mine = up ? acc[i + HALF] : acc[i];
    const float oth = up ? acc[i] : acc[i + HALF];
    acc[i] = mine + __shfl_xor(oth, O, 64);
  }
  if constexpr (HALF > 1) butterfly<HALF / 2, O / 2>(acc, lane);
}

// y_b[c] = Σ_k x_b[k]·W[c][k] for the NPW columns of this workgroup's LDS slice `ws` ([NPW][K]
// bf16 or int8, row stride RS bytes) and NB activation rows b (batch rows share every weight read: one LDS read and convert
// feeds NB FMAs); thread t holds x_b[k] for k = (j·256 + t)·8 + i (threads past K hold nothing:
// K = 1024 leaves waves 2-3 out of the dot products). r[b] = column `tid`'s sum for tid < NPW.
// Reduction: a butterfly that halves the live columns per exchange (log2 P steps, P−1 shuffles
// instead of 6·P), then 4 waves through LDS (`red` holds 4·NB·32 floats).
// `mid()` runs once every wave has consumed the first half of the columns (slice bytes
// [0, SLICE/2) are free), `end()` once the whole slice is consumed: the loader waves issue the
// next slices' DMA there.
template <int NPW, int K, bool W8, int NB, int RS, class Mid, class End>
__device__ __forceinline__ void gemv_lds(const char* ws, const float (&x)[NB][(K + 2047) / 2048][8], float* red,
                                         int tid, Mid mid, End end, float (&r)[NB]) {
  constexpr int KCH = (K + 2047) / 2048;
  constexpr int P = NPW <= 8 ? 8 : 32;
  constexpr int LOGP = P == 8 ? 3 : 5;
  static_assert(NPW <= 32 && K % 1024 == 0, "gemv_lds shape");
  const int lane = tid & 63, wv = tid >> 6;
  float acc[NB][P];
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int c = 0; c < P; ++c) acc[b][c] = 0.f;
  auto cols = [&](auto c0, auto c1) {
#pragma unroll
    for (int c = decltype(c0)::value; c < decltype(c1)::value; ++c) {
#pragma unroll
      for (int j = 0; j < KCH; ++j) {
        if (K % 2048 != 0 && (j * 256 + tid) * 8 >= K) continue;  // wave-uniform
        float wf[8];
        if constexpr (W8) {  // int8 [NPW][K]: 8 weights per 8-B read, scaled after the sum
          const uint2 q = *reinterpret_cast<const uint2*>(ws + (long)c * RS + (j * 256 + tid) * 8);
#pragma unroll
          for (int i = 0; i < 8; ++i)
            wf[i] = (float)(int)(signed char)(((i < 4 ? q.x : q.y) >> (8 * (i & 3))) & 0xFF);
        } else {
          const u16x8 w = *reinterpret_cast<const u16x8*>(ws + (long)c * RS + (j * 256 + tid) * 16);
#pragma unroll
          for (int i = 0; i < 8; ++i) wf[i] = bf2f(w[i]);
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[b][c] += x[b][j][i] * wf[i];
      }
    }
  };
  cols(std::integral_constant<int, 0>{}, std::integral_constant<int, NPW / 2>{});
  __syncthreads();  // columns [0, NPW/2) = slice bytes [0, SLICE/2) consumed by every wave
  mid();
  cols(std::integral_constant<int, NPW / 2>{}, std::integral_constant<int, NPW>{});
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    butterfly<P / 2, 32>(acc[b], lane);
#pragma unroll
    for (int o = 32 >> LOGP; o > 0; o >>= 1) acc[b][0] += __shfl_xor(acc[b][0], o, 64);
    if ((lane & ((64 >> LOGP) - 1)) == 0) red[(wv * NB + b) * P + (lane >> (6 - LOGP))] = acc[b][0];
  }
  __syncthreads();
  end();
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    r[b] = 0.f;
    if (tid < NPW)
      r[b] = red[b * P + tid] + red[(NB + b) * P + tid] + red[(2 * NB + b) * P + tid] +
             red[(3 * NB + b) * P + tid];
  }
}

// N block-wide sums in one LDS round (blockDim 256; `red` holds 4·N floats).
template <int N>
__device__ __forceinline__ void block_sum_n(float (&v)[N], float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = wave_sum(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) red[w * N + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = red[i] + red[N + i] + red[2 * N + i] + red[3 * N + i];
  __syncthreads();
}

// x_b = bf16(LN(resid_b)) for NB rows r + b·EE, this thread's 8 elements k = 8·tid (threads with
// 8·tid ≥ EE hold 0). Every row's (Σv, Σv²) share one block reduction (`wred`: 8·NB floats).
template <int EE, int NB>
__device__ __forceinline__ void ln_prologue(const MegaArgs& a, const bf16_t* r, const bf16_t* g,
                                            const bf16_t* b, float (&x)[NB][1][8], float* wred, int tid) {
  const bool on = tid * 8 < EE;
  // gamma / beta first: their latency then hides under the residual load and the reductions
  // (a load is not hoisted across the __syncthreads of block_sum_n)
  u16x8 gg{}, bb{};
  float v[NB][8];
#pragma unroll
  for (int n = 0; n < NB; ++n)
#pragma unroll
    for (int i = 0; i < 8; ++i) v[n][i] = 0.f;
  if (on) {
    gg = *reinterpret_cast<const u16x8*>(g + tid * 8);
    bb = *reinterpret_cast<const u16x8*>(b + tid * 8);
#pragma unroll
    for (int n = 0; n < NB; ++n) ld_bf8(r + (long)n * EE + tid * 8, v[n]);
  }
  // one reduction of (Σv, Σv²) per row: var = E[v²] − mean² (f32 over ≤ 2048 bf16 values)
  float sq[2 * NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    sq[n] = sq[NB + n] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sq[n] += v[n][i];
      sq[NB + n] += v[n][i] * v[n][i];
    }
  }
  block_sum_n<2 * NB>(sq, wred);
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const float mean = sq[n] * (1.f / EE);
    const float rs = rsqrtf(fmaxf(sq[NB + n] * (1.f / EE) - mean * mean, 0.f) + a.eps);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      x[n][0][i] = on ? bf2f(f2bf((v[n][i] - mean) * rs * bf2f(gg[i]) + bf2f(bb[i]))) : 0.f;
  }
}

// Lanes 0..NC-1 of wave 0 each hold one bf16 `y`; publish them as NC/4 64-bit stores at dst.
// Every lane of the wave must call this (shuffles).
__device__ __forceinline__ void publish_bf16(bf16_t* dst, float y, int lane, int NC) {
  const unsigned u = (unsigned)f2bf(y);
  const unsigned pair = u | ((unsigned)__shfl_down((int)u, 1, 64) << 16);
  const unsigned pair2 = (unsigned)__shfl_down((int)pair, 2, 64);
  if (lane < NC && (lane & 3) == 0) st64(dst + lane, (u64)pair | ((u64)pair2 << 32));
}

// Loader waves: DMA bytes [from, to) (multiples of 1 KiB) of the [rows][RB-byte] slice at `src`
// into the padded LDS image (row r at r·(RB + 16)); a 1 KiB piece never straddles a row.
template <int RB>
__device__ __forceinline__ void prefetch_p(const bf16_t* src, int from, int to, char* wl, int wv, int lane) {
  if (wv == 0 || src == nullptr) return;
  const char* s = reinterpret_cast<const char*>(src) + lane * 16;
  for (int p = (from >> 10) + wv - 1; p < (to >> 10); p += 3) {
    const int off = p * 1024, dst = off / RB * (RB + 16) + off % RB;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(s + off),
                                     (__attribute__((address_space(3))) void*)(wl + dst), 16, 0, 0);
  }
}

// Loader waves: read bytes [from, to) of `src` through the cache hierarchy into ONE 1 KiB LDS
// scratch piece (the data is dropped): an early touch of a later phase's slice, so its real DMA
// is served from the memory-side cache instead of HBM (MegaArgs.late_dma bit 2, A/B).
__device__ __forceinline__ void touch(const bf16_t* src, int from, int to, char* scratch, int wv, int lane) {
  if (wv == 0 || src == nullptr) return;
  const char* s = reinterpret_cast<const char*>(src) + lane * 16;
  for (int p = (from >> 10) + wv - 1; p < (to >> 10); p += 3)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(s + p * 1024),
                                     (__attribute__((address_space(3))) void*)scratch, 16, 0, 0);
}

// MFMA form of gemv_lds for bf16 slices (same contract: x as gemv_lds, r[b] = column tid's sum
// for tid < NPW; `mid` and `end` both run once the whole slice is consumed). The activation rows
// are staged in LDS (`xs`: NB rows of KP = min(K, 8192 / NB) k, 16-B padded; one pass for every
// K ≤ KP, else K / KP passes); each wave takes a quarter of a pass's k and runs
// mfma_f32_16x16x32_bf16 over column tiles of 16: A = activations, B = the weight rows straight
// from the padded LDS image (one 16-B read per lane, conflict-free thanks to the row padding).
// Slices narrower than a tile (NPW = 8 / 4) put HS = 16 / NPW k-sets of the wave's range side by
// side instead of idle columns: A row b·HS + h holds row b's activations of k-set h, B column
// h·NPW + c column c's weights of k-set h, and only those diagonal blocks of C are kept. A rows /
// B columns past the real ones read a clamped (valid) row and land in C entries nobody keeps, so
// no read is predicated. Operands are read SB k-steps at a time, the next batch's reads issued
// before this batch's MFMAs (one wave per SIMD: nothing else hides the LDS latency). The partial
// sums (4 waves × HS k-sets) meet in `red`. No per-column butterfly and no bf16 → f32 converts:
// NB rows cost the same MFMAs as one. WQ = 1 / 2: int8 / int4 weight rows (8 / 4 B per lane and
// k-step), widened to bf16 in registers right before their MFMA (exact), scaled per column by
// the caller.
template <int NPW, int K, int NB, int RS, int WQ = 0, class Mid, class End>
__device__ __forceinline__ void gemv_mfma(const char* ws, const float (&x)[NB][(K + 2047) / 2048][8], float* red,
                                          bf16_t* xs, int tid, Mid mid, End end, float (&r)[NB]) {
  constexpr int KPM = 8192 / NB;
  constexpr int KP = K < KPM ? K : KPM;           // k per staging pass
  constexpr int JP = KP >= 2048 ? KP / 2048 : 1;  // thread x-chunks per pass
  constexpr int NPASS = K / KP;
  constexpr int XS = KP + 8;                      // xs row stride (elements)
  constexpr int HS = NPW >= 16 ? 1 : 16 / NPW;    // k-sets side by side in a tile
  constexpr int NCT = NPW >= 16 ? (NPW + 15) / 16 : 1;  // column tiles
  constexpr int P = NPW >= 16 ? NCT * 16 : NPW;   // red row length
  constexpr int DK = KP / 4 / HS;                 // k per k-set of a wave's quarter
  constexpr int SPW = DK / 32;                    // k-steps per wave per pass
  constexpr int SB0 = NCT == 1 ? 8 : 4;
  constexpr int SB = SPW < SB0 ? SPW : SB0;       // k-steps per operand batch
  constexpr int NBT = SPW / SB;
  static_assert(NPW <= 32 && K % 1024 == 0 && NB <= 4 && NB * HS <= 16 && K % KP == 0 && SPW % SB == 0,
                "gemv_mfma shape");
  constexpr int WBITS = WQ == 0 ? 16 : WQ == 1 ? 8 : 4;
  typedef typename std::conditional<WQ == 0, u16x8, typename std::conditional<WQ == 1, uint2, unsigned>::type>::type BRaw;
  auto widen = [](const BRaw& w) -> u16x8 {
    if constexpr (WQ == 1) {  // 8 int8 codes
      u16x8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        o[i] = (unsigned short)(__float_as_uint((float)(int)(signed char)(((i < 4 ? w.x : w.y) >> (8 * (i & 3))) & 0xFF)) >> 16);
      return o;
    } else if constexpr (WQ == 2) {  // 8 int4 codes, k ascending from the low nibble
      u16x8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        o[i] = (unsigned short)(__float_as_uint((float)((int)(w << (28 - 4 * i)) >> 28)) >> 16);
      return o;
    } else {
      return w;
    }
  };
  const int lane = tid & 63, wv = tid >> 6, lr = lane & 15, g = lane >> 4;
  // per-lane operand bases (every k-step is then a constant offset)
  const int arow = lr < NB * HS ? lr : NB * HS - 1;
  const bf16_t* ap = xs + (arow / HS) * XS + wv * (KP / 4) + (arow % HS) * DK + g * 8;
  const char* bp[NCT];
#pragma unroll
  for (int t = 0; t < NCT; ++t) {
    const int c = NPW >= 16 ? (t * 16 + lr < NPW ? t * 16 + lr : NPW - 1) : lr % NPW;
    const int h = NPW >= 16 ? 0 : lr / NPW;
    bp[t] = ws + (long)c * RS + (wv * (KP / 4) + h * DK + g * 8) * WBITS / 8;
  }
  f32x4 acc[NCT];
#pragma unroll
  for (int t = 0; t < NCT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < NPASS; ++q) {
    if (q) __syncthreads();  // the previous pass's A reads are done
#pragma unroll
    for (int jj = 0; jj < JP; ++jj) {
      const int kk = (jj * 256 + tid) * 8;
      if (kk < KP) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          u16x8 o;
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] = f2bf(x[b][q * JP + jj][i]);  // exact: x holds bf16 values
          *reinterpret_cast<u16x8*>(xs + b * XS + kk) = o;
        }
      }
    }
    __syncthreads();
    auto load = [&](int bt, u16x8 (&av)[SB], BRaw (&bw)[SB][NCT]) {
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int st = bt * SB + u;
        av[u] = *reinterpret_cast<const u16x8*>(ap + st * 32);
#pragma unroll
        for (int t = 0; t < NCT; ++t)
          bw[u][t] = *reinterpret_cast<const BRaw*>(bp[t] + (q * KP + st * 32) * WBITS / 8);
      }
    };
    u16x8 a0[SB];
    BRaw b0[SB][NCT];
    load(0, a0, b0);
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      u16x8 a1[SB];
      BRaw b1[SB][NCT];
      if (bt + 1 < NBT) load(bt + 1, a1, b1);
#pragma unroll
      for (int u = 0; u < SB; ++u)
#pragma unroll
        for (int t = 0; t < NCT; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a0[u]),
                                                           __builtin_bit_cast(bf16x8, widen(b0[u][t])), acc[t], 0, 0, 0);
      if (bt + 1 < NBT) {
#pragma unroll
        for (int u = 0; u < SB; ++u) {
          a0[u] = a1[u];
#pragma unroll
          for (int t = 0; t < NCT; ++t) b0[u][t] = b1[u][t];
        }
      }
    }
  }
  // C[row g·4 + i][col lr]; row = b·HS + h is kept where col belongs to k-set h
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = g * 4 + i, b = row / HS, h = row % HS;
    if (row < NB * HS) {
#pragma unroll
      for (int t = 0; t < NCT; ++t) {
        const int c = NPW >= 16 ? t * 16 + lr : lr % NPW;
        const bool keep = NPW >= 16 ? c < NPW : lr / NPW == h;
        if (keep) red[((wv * HS + h) * NB + b) * P + c] = acc[t][i];
      }
    }
  }
  __syncthreads();
  mid();
  end();
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    r[b] = 0.f;
    if (tid < NPW) {
#pragma unroll
      for (int wh = 0; wh < 4 * HS; ++wh) r[b] += red[(wh * NB + b) * P + tid];
    }
  }
}

// Model shape of the single-launch step. E / D / HQ / HK / F: hidden width, head dim, query and
// key/value heads (GQA when HK < HQ), FFN width; ROT: rotary embedding over the whole head dim
// (NeoX rotate-half or GPT-J interleaved per MegaArgs.neox, angles pos·base^(−2f/D)) applied to q
// and the new k. Every projection splits its output columns evenly over the 256 workgroups and
// each workgroup's weight slice must fit the 128 KiB LDS image.
// NB: batch rows per step (each GEMV phase applies its LDS slice to all NB rows; attention runs
// one workgroup per (row, head, split)). MM: the GEMV phases run on MFMA (gemv_mfma, the default;
// int8 weights widened in registers), else on the VALU (gemv_lds; A/B variants).
template <int E_, int D_, int HQ_, int HK_, int F_, int ROT_, int W8_ = 0, int NB_ = 1, int MM_ = 1>
struct MegaCfg {
  static constexpr int E = E_, D = D_, HQ = HQ_, HK = HK_, F = F_, ROT = ROT_, W8 = W8_, NB = NB_, MM = MM_;
  static_assert(NB == 1 || NB == 2 || NB == 4, "rows per step");
  // W8: weight format (0 bf16, 1 int8, 2 int4 weight-only with per-output-channel scales)
  static_assert(W8 >= 0 && W8 <= 2 && (W8 != 2 || MM), "int4 weights run on the MFMA phases");
  static constexpr int WBITS = W8 == 0 ? 16 : W8 == 1 ? 8 : 4;
  static constexpr int NQKV = (HQ + 2 * HK) * D;
  static constexpr int NPQ = NQKV / NWG, NPO = E / NWG, NP1 = F / NWG, NP2 = E / NWG;
  // slice bytes (global, [rows][in] contiguous): QKV [0, QB) → out [QB, QB + OB) (free during
  // QKV) → FFN1 [0, F1B), whose first F1PRE bytes stream in during the attention phase
  // (workgroups without attention work) or the out-projection prologue (the others) and the rest
  // once the out slice is consumed → FFN2 [0, F2B) → next QKV [0, QB)
  static constexpr int QB = NPQ * E * WBITS / 8, OB = NPO * E * WBITS / 8, F1B = NP1 * E * WBITS / 8,
                       F2B = NP2 * F * WBITS / 8;
  // LDS image: every weight row is padded by 16 B (row strides RSE / RSF), so the 16 rows of an
  // MFMA B fragment (one 16-B read per lane, same k) start on 16 different bank quads
  static constexpr int RBE = E * WBITS / 8, RBF = F * WBITS / 8, RSE = RBE + 16, RSF = RBF + 16;
  static constexpr int OUT_OFF = NPQ * RSE;
  static constexpr int F1PRE = QB < F1B ? QB : F1B;
  static constexpr int WL = (NPQ + NPO) * RSE > NP1 * RSE ? (NPQ + NPO) * RSE : NP1 * RSE;
  static constexpr int WLB = ((WL > NP2 * RSF ? WL : NP2 * RSF) + 1023) / 1024 * 1024;
  // early half-slice DMA (MegaArgs.late_dma = 0): whole rows of the next slice whose LDS extent
  // stays inside the half (by columns) the running GEMV has already consumed
  static constexpr int MID1 = F2B < (NP1 / 2) * RSE / RSF * RBF ? F2B : (NP1 / 2) * RSE / RSF * RBF;
  static constexpr int MID2 = QB < (NP2 / 2) * RSF / RSE * RBE ? QB : (NP2 / 2) * RSF / RSE * RBE;
  // the out phase of a non-attention workgroup waits for every DMA older than its FFN1 head: the
  // newest F1PRE/1 KiB/3 wave-instructions per loader wave (floor: the minimum over the waves)
  static constexpr int WAIT_OLD = F1PRE / 1024 / 3;
  // FFN2 touch (late_dma bit 2): the first TOUCHB bytes of the slice right behind the FFN1 head,
  // TWAIT wave-instructions per loader wave outstanding in all (vmcnt holds ≤ 63)
  static constexpr int TOUCHB = (63 - WAIT_OLD) * 3 * 1024 < F2B ? (63 - WAIT_OLD) * 3 * 1024 : F2B;
  static constexpr int TWAIT = WAIT_OLD + TOUCHB / 1024 / 3;
  static constexpr int LPR = D / 8;  // lanes per head row (16 B each)
  static_assert(NQKV % NWG == 0 && E % NWG == 0 && F % NWG == 0, "columns split evenly over the grid");
  static_assert(WLB <= 132 * 1024, "slices fit the LDS image");
  static_assert(RBE % 1024 == 0 && RBF % 1024 == 0, "1 KiB pieces never straddle a row");
  static_assert(HQ * D == E && HQ % HK == 0 && E % 1024 == 0 && E <= 2048 && F % 2048 == 0, "widths");
  static_assert(D == 64 || D == 128, "head dim");
  static_assert(NPQ <= 32 && NP1 <= 32 && (NPO & (NPO - 1)) == 0 && (NP1 & (NP1 - 1)) == 0 &&
                NPO >= 4 && NP1 >= 4, "per-workgroup column counts");
};

// One GEMV phase of decode_mega_kernel<C> over a slice with LDS row stride RS.
template <class C, int NPW, int K, int RS, class Mid, class End>
__device__ __forceinline__ void gemv_phase(const char* ws, const float (&x)[C::NB][(K + 2047) / 2048][8],
                                           float* red, bf16_t* xs, int tid, Mid mid, End end, float (&r)[C::NB]) {
  if constexpr (C::MM)
    gemv_mfma<NPW, K, C::NB, RS, C::W8>(ws, x, red, xs, tid, mid, end, r);
  else
    gemv_lds<NPW, K, C::W8 != 0, C::NB, RS>(ws, x, red, tid, mid, end, r);
}

__host__ __device__ constexpr long pstride_hd(int hq, int d, int nsplit) {
  return ((long)hq * nsplit * (d + 2) + 63) / 64 * 64;
}

template <class C>
__global__ __launch_bounds__(NT, 1) void decode_mega_kernel(MegaArgs a) {
  constexpr int E = C::E, D = C::D, HQ = C::HQ, HK = C::HK, F = C::F, LPR = C::LPR;
  constexpr int NPQ = C::NPQ, NPO = C::NPO, NP1 = C::NP1, NP2 = C::NP2;
  constexpr int PSTR = D + 2;
  constexpr int NB = C::NB;
  constexpr bool W8 = C::W8 != 0;
  // a workgroup's weight slice: `rows` [out] rows of `in` weights, C::WBITS bits each
  auto slice = [](const bf16_t* w, long row0, long in) {
    return reinterpret_cast<const bf16_t*>(reinterpret_cast<const char*>(w) + row0 * in * C::WBITS / 8);
  };
  constexpr int RSE = C::RSE, RSF = C::RSF, RBE = C::RBE, RBF = C::RBF;
  __shared__ __attribute__((aligned(1024))) char wl[C::WLB];
  __shared__ __attribute__((aligned(16))) bf16_t xs[C::MM ? NB * (8192 / NB + 8) : 8];  // gemv_mfma staging
  __shared__ float red[4 * NB * 32];
  __shared__ float wred[8 * NB];
  __shared__ float sc[256];
  __shared__ float pv[4][D];
  __shared__ __attribute__((aligned(1024))) char tch[1024];  // touch() scratch

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, w = blockIdx.x;
  const long pst = pstride_hd(HQ, D, a.nsplit);  // one row's partial block
  const bool tou = (a.late_dma & 4) != 0;
  unsigned nbar = 0;

  prefetch_p<RBE>(slice(a.layers[0].wqkv, (long)w * NPQ, E), 0, C::QB, wl, wv, lane);
  for (int l = 0; l < a.nl; ++l) {
    const MegaLayer& Ly = a.layers[l];
    // this layer's buffer slots (NB rows each): every published vector has its own address per
    // launch, so a reader's L2 can never hold a stale copy and plain (cached) loads are coherent
    const bf16_t* rin = l == 0 ? a.resid : a.rbuf + (long)(2 * l - 1) * NB * E;
    bf16_t* rmid = a.rbuf + (long)(2 * l) * NB * E;
    bf16_t* rout = a.rbuf + (long)(2 * l + 1) * NB * E;
    float* qn = a.qn + (long)l * NB * HQ * D;
    float* kvn = a.kvn + (long)l * NB * 2 * HK * D;
    float* part = a.part + (long)l * NB * pst;
    bf16_t* hb = a.h + (long)l * NB * F;
    // ---------------------------------------------------------------- QKV
    phase_start<C::WAIT_OLD>(a, wv, nbar);
    {
      // epilogue operands requested first: their latency hides under the prologue and GEMV
      const float bq = lane < NPQ ? bf2f(Ly.bqkv[w * NPQ + lane]) : 0.f;
      const float sq = W8 && lane < NPQ ? Ly.sqkv[w * NPQ + lane] : 1.f;
      float x[NB][1][8];
      ln_prologue<E, NB>(a, rin, Ly.ln1_g, Ly.ln1_b, x, wred, tid);
      tmark(a, nbar, 1);
      // out slice into the region QKV does not use, behind this GEMV
      float y[NB];
      gemv_phase<C, NPQ, E, RSE>(wl, x, red, xs, tid, [] {}, [&] {
        prefetch_p<RBE>(slice(Ly.wo, (long)w * NPO, E), 0, C::OB, wl + C::OUT_OFF, wv, lane);
      }, y);
      tmark(a, nbar, 2);
      if (wv == 0) {
        if (lane < NPQ) {
          const int col = w * NPQ + lane;
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const float v = bf2f(f2bf(sq * y[b])) + bq;
            if (col < HQ * D) {
              __hip_atomic_store(qn + b * HQ * D + col, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
              const int kv = col - HQ * D;          // [0, 2·HK·D)
              const int which = kv / (HK * D), r = kv % (HK * D), kh = r / D, d = r % D;
              const bf16_t vb = f2bf(v);
              if (which || !C::ROT) {  // rotated k is cached by the attention phase (needs all of D)
                bf16_t* cache = which ? Ly.vc : Ly.kc;
                cache[(((long)b * HK + kh) * a.maxS + a.pos[b]) * D + d] = vb;
              }
              // rotary k stays unrounded until rotated (the per-op path rounds after the rotation)
              __hip_atomic_store(kvn + b * 2 * HK * D + kv, (C::ROT && !which) ? v : bf2f(vb),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
          }
        }
        grid_sync(a, ++nbar, lane);
      } else {
        ++nbar;
      }
    }
    // ---------------------------------------------------------------- attention
    // (attention reads no weights: the out slice keeps streaming)
    phase_start<C::WAIT_OLD>(a, wv, nbar, WAIT_NONE);
    const bf16_t* w1s = slice(Ly.w1, (long)w * NP1, E);
    if (w < NB * HQ * a.nsplit) {
      // one workgroup per (row, head, split)
      const int bi = w / (HQ * a.nsplit), wr = w % (HQ * a.nsplit);
      const int h = wr / a.nsplit, s = wr % a.nsplit, kh = h / (HQ / HK);
      const int pos = a.pos[bi], L = pos + 1;
      const float* qn_b = qn + bi * HQ * D;
      const float* kvn_b = kvn + bi * 2 * HK * D;
      const int chunk = (L + a.nsplit - 1) / a.nsplit;
      const int j0 = s * chunk, n = min(L, j0 + chunk) - j0;
      constexpr int RIF = NT / LPR;                    // key rows in flight per workgroup
      const int sub = tid % LPR, kslot = tid / LPR;    // LPR lanes per key row
      const long kvbase = ((long)bi * HK + kh) * a.maxS * D;
      float rc[8], rsn[8];
      if (C::ROT) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = sub * 8 + j;
          const int f = a.neox ? (i % (D / 2)) : (i >> 1);
          sincosf((float)pos * exp2f(-(2.f * f / (float)D) * a.log2_base), &rsn[j], &rc[j]);
        }
      }
      // same rotation as decode_attn_kernel (infer.hip): partner element from lane sub ^ LPR/2
      // (rotate-half) or the neighbouring element (interleaved)
      auto rotate = [&](float* v) {
        float pr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (a.neox) {
            pr[j] = __shfl_xor(v[j], LPR / 2, 64) * (sub < LPR / 2 ? -1.f : 1.f);
          } else {
            pr[j] = (j & 1) ? v[j - 1] : -v[j + 1];
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] * rc[j] + pr[j] * rsn[j];
      };
      float q[8], kn[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        q[i] = ldf(qn_b + h * D + sub * 8 + i);
        kn[i] = ldf(kvn_b + kh * D + sub * 8 + i);
      }
      // the cached K and V rows of this thread's first two key slots do not depend on q or the
      // new k: requested before either is used (one round trip for short splits)
      u16x8 kraw[2], vraw[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int j = j0 + kslot + RIF * u;
        if (kslot + RIF * u < n && j != pos) {
          kraw[u] = *reinterpret_cast<const u16x8*>(Ly.kc + kvbase + (long)j * D + sub * 8);
          vraw[u] = *reinterpret_cast<const u16x8*>(Ly.vc + kvbase + (long)j * D + sub * 8);
        }
      }
      if (C::ROT) {
        rotate(q);
        rotate(kn);
#pragma unroll
        for (int i = 0; i < 8; ++i) kn[i] = bf2f(f2bf(kn[i]));
        if (h % (HQ / HK) == 0 && s == 0 && kslot == 0) {  // one writer per kv head
          u16x8 ko;
#pragma unroll
          for (int i = 0; i < 8; ++i) ko[i] = f2bf(kn[i]);
          *reinterpret_cast<u16x8*>(Ly.kc + kvbase + (long)pos * D + sub * 8) = ko;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) q[i] *= a.scale_log2;
      auto row = [&](const bf16_t* cache, int which, int j, float* r) {
        if (j == pos) {
          if (which == 0) {
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = kn[i];
          } else {
            const float* p = kvn_b + HK * D + kh * D + sub * 8;
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
              const u64 u = ld64(p + i);
              r[i] = __uint_as_float((unsigned)u);
              r[i + 1] = __uint_as_float((unsigned)(u >> 32));
            }
          }
        } else {
          const u16x8 u = *reinterpret_cast<const u16x8*>(cache + kvbase + (long)j * D + sub * 8);
#pragma unroll
          for (int i = 0; i < 8; ++i) r[i] = bf2f(u[i]);
        }
      };
      float kp[2][8], vp[2][8];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int j = j0 + kslot + RIF * u;
        if (kslot + RIF * u < n) {
          if (j == pos) {
            row(Ly.kc, 0, j, kp[u]);
            row(Ly.vc, 1, j, vp[u]);
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              kp[u][i] = bf2f(kraw[u][i]);
              vp[u][i] = bf2f(vraw[u][i]);
            }
          }
        }
      }
      auto score = [&](int i, const float* k) {
        float d = 0.f;
#pragma unroll
        for (int t = 0; t < 8; ++t) d += q[t] * k[t];
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
        if (sub == 0 && i < n) sc[i] = d;
      };
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (RIF * u < n) score(kslot + RIF * u, kp[u]);  // workgroup-uniform bound
      for (int i = kslot + 2 * RIF; i < n; i += RIF) {
        float k[8];
        row(Ly.kc, 0, j0 + i, k);
        score(i, k);
      }
      __syncthreads();
      const float sv = tid < n ? sc[tid] : -INFINITY;
      const float m = block_max<4>(sv, wred);
      const float p = tid < n ? exp2f(sv - m) : 0.f;
      const float lsum = block_sum<4>(p, wred);
      if (tid < n) sc[tid] = p;
      __syncthreads();
      float acc[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (kslot + RIF * u < n) {
          const float pi = sc[kslot + RIF * u];
#pragma unroll
          for (int t = 0; t < 8; ++t) acc[t] += pi * vp[u][t];
        }
      }
      for (int i = kslot + 2 * RIF; i < n; i += RIF) {
        float v[8];
        row(Ly.vc, 1, j0 + i, v);
        const float pi = sc[i];
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] += pi * v[t];
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
#pragma unroll
        for (int o = LPR; o < 64; o <<= 1) acc[t] += __shfl_xor(acc[t], o, 64);
      }
      if (lane < LPR) {
#pragma unroll
        for (int t = 0; t < 8; ++t) pv[wv][sub * 8 + t] = acc[t];
      }
      __syncthreads();
      if (wv == 0) {
        float* dst = part + bi * pst + (long)(h * a.nsplit + s) * PSTR;
        const int d0 = lane * 2;
        if (d0 < D) {
          const float v0 = pv[0][d0] + pv[1][d0] + pv[2][d0] + pv[3][d0];
          const float v1 = pv[0][d0 + 1] + pv[1][d0 + 1] + pv[2][d0 + 1] + pv[3][d0 + 1];
          st64(dst + d0, pack2f(n > 0 ? v0 : 0.f, n > 0 ? v1 : 0.f));
        }
        if (lane == 0) st64(dst + D, pack2f(n > 0 ? m : -INFINITY, n > 0 ? lsum : 0.f));
      }
      // K/V are consumed: the loader waves queue the FFN1 head now, behind wave 0's partial
      // stores and grid barrier, so it no longer stalls their out-projection GEMV work
      if (!(a.late_dma & 2)) prefetch_p<RBE>(w1s, 0, C::F1PRE, wl, wv, lane);
      if (tou) touch(slice(Ly.w2, (long)w * NP2, F), 0, C::TOUCHB, tch, wv, lane);
    } else {
      prefetch_p<RBE>(w1s, 0, C::F1PRE, wl, wv, lane);
      if (tou) touch(slice(Ly.w2, (long)w * NP2, F), 0, C::TOUCHB, tch, wv, lane);
    }
    if (wv == 0) grid_sync(a, ++nbar, lane); else ++nbar;
    // ---------------------------------------------------------------- out projection
    // every workgroup has its FFN1 head in flight (queued at the attention phase start, or at its
    // end by attention workgroups) and waits for the older out slice only; with late_dma bit 1 the
    // attention workgroups queue the head only here (every older load has to land first)
    const bool attn_late = w < NB * HQ * a.nsplit && (a.late_dma & 2);
    if (tou && !attn_late)  // the FFN2 touches are queued behind the FFN1 head
      phase_start<C::TWAIT>(a, wv, nbar, WAIT_OLDER);
    else
      phase_start<C::WAIT_OLD>(a, wv, nbar, attn_late ? WAIT_ALL : WAIT_OLDER);
    {
      const int ocol = w * NPO + (lane & (NPO - 1));
      const float bo = bf2f(Ly.bo[ocol]);
      float ro[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) ro[b] = bf2f(rin[b * E + ocol]);
      const float so = W8 ? Ly.so[ocol] : 1.f;
      float x[NB][1][8];
      {
        const int h = tid / LPR, d0 = (tid % LPR) * 8;  // thread t holds elements 8t … 8t+7
        const bool on = h < HQ;
        // online combine; SPR splits' partials of every row requested at once (no load waits on
        // another; HQ·nsplit·NB ≤ 256 keeps nsplit ≤ SPR for the instantiated head counts)
        constexpr int SPR = NB == 4 ? 4 : 8;
        float M[NB], lt[NB], o[NB][8];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          M[b] = -INFINITY;
          lt[b] = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) o[b][i] = 0.f;
        }
        for (int s0 = 0; s0 < a.nsplit; s0 += SPR) {
          u64 ml[NB][SPR], ov[NB][SPR][4];
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const float* base = part + b * pst + (long)min(h, HQ - 1) * a.nsplit * PSTR;
#pragma unroll
            for (int t = 0; t < SPR; ++t) {
              const float* ps = base + min(s0 + t, a.nsplit - 1) * PSTR;
              ml[b][t] = ld64(ps + D);
#pragma unroll
              for (int i = 0; i < 4; ++i) ov[b][t][i] = ld64(ps + d0 + 2 * i);
            }
          }
#pragma unroll
          for (int b = 0; b < NB; ++b) {
#pragma unroll
            for (int t = 0; t < SPR; ++t) {
              const float ms = __uint_as_float((unsigned)ml[b][t]);
              if (s0 + t >= a.nsplit || ms == -INFINITY) continue;
              const float nM = fmaxf(M[b], ms), c = exp2f(M[b] - nM), e = exp2f(ms - nM);
              lt[b] = lt[b] * c + e * __uint_as_float((unsigned)(ml[b][t] >> 32));
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                o[b][2 * i] = o[b][2 * i] * c + e * __uint_as_float((unsigned)ov[b][t][i]);
                o[b][2 * i + 1] = o[b][2 * i + 1] * c + e * __uint_as_float((unsigned)(ov[b][t][i] >> 32));
              }
              M[b] = nM;
            }
          }
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const float inv = 1.f / lt[b];
#pragma unroll
          for (int i = 0; i < 8; ++i) x[b][0][i] = on ? bf2f(f2bf(o[b][i] * inv)) : 0.f;
        }
      }
      if (attn_late) prefetch_p<RBE>(w1s, 0, C::F1PRE, wl, wv, lane);
      tmark(a, nbar, 1);
      float y[NB];
      gemv_phase<C, NPO, E, RSE>(wl + C::OUT_OFF, x, red, xs, tid, [] {}, [&] {
        prefetch_p<RBE>(w1s, C::F1PRE, C::F1B, wl, wv, lane);
      }, y);
      tmark(a, nbar, 2);
      if (wv == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) publish_bf16(rmid + b * E + w * NPO, so * y[b] + bo + ro[b], lane, NPO);
        grid_sync(a, ++nbar, lane);
      } else {
        ++nbar;
      }
    }
    // ---------------------------------------------------------------- FFN1
    phase_start<C::WAIT_OLD>(a, wv, nbar);
    {
      const float b1 = bf2f(Ly.b1[w * NP1 + (lane & (NP1 - 1))]);
      const float s1 = W8 ? Ly.s1[w * NP1 + (lane & (NP1 - 1))] : 1.f;
      float x[NB][1][8];
      ln_prologue<E, NB>(a, rmid, Ly.ln2_g, Ly.ln2_b, x, wred, tid);
      tmark(a, nbar, 1);
      const bf16_t* w2s = slice(Ly.w2, (long)w * NP2, F);
      const int mid = (a.late_dma & 1) ? 0 : C::MID1;
      float y[NB];
      gemv_phase<C, NP1, E, RSE>(wl, x, red, xs, tid, [&] { prefetch_p<RBF>(w2s, 0, mid, wl, wv, lane); },
                                 [&] { prefetch_p<RBF>(w2s, mid, C::F2B, wl, wv, lane); }, y);
      tmark(a, nbar, 2);
      if (wv == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          const float t = s1 * y[b] + b1;
          publish_bf16(hb + b * F + w * NP1, a.act ? gelu_tanh(t) : gelu_erf(t), lane, NP1);
        }
        grid_sync(a, ++nbar, lane);
      } else {
        ++nbar;
      }
    }
    // ---------------------------------------------------------------- FFN2
    phase_start<C::WAIT_OLD>(a, wv, nbar);
    {
      const int fcol = w * NP2 + (lane & (NP2 - 1));
      const float b2 = bf2f(Ly.b2[fcol]);
      float rm[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) rm[b] = bf2f(rmid[b * E + fcol]);
      const float s2 = W8 ? Ly.s2[fcol] : 1.f;
      constexpr int KCH2 = F / 2048;
      float x[NB][KCH2][8];
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int j = 0; j < KCH2; ++j) ld_bf8(hb + b * F + (j * 256 + tid) * 8, x[b][j]);
      tmark(a, nbar, 1);
      const bf16_t* nq = l + 1 < a.nl ? slice(a.layers[l + 1].wqkv, (long)w * NPQ, E) : nullptr;
      const int mid = (a.late_dma & 1) ? 0 : C::MID2;
      float y[NB];
      gemv_phase<C, NP2, F, RSF>(wl, x, red, xs, tid, [&] { prefetch_p<RBE>(nq, 0, mid, wl, wv, lane); },
                                 [&] { prefetch_p<RBE>(nq, mid, C::QB, wl, wv, lane); }, y);
      tmark(a, nbar, 2);
      if (wv == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) publish_bf16(rout + b * E + w * NP2, s2 * y[b] + b2 + rm[b], lane, NP2);
        if (l + 1 < a.nl) grid_sync(a, ++nbar, lane);
      } else {
        ++nbar;
      }
    }
  }
  if (wv != 0) wait_vm<0>();
  // the last workgroup out re-zeroes the barrier words for the next launch (stream-ordered), so
  // a launch needs no memset node in front of it
  if (tid == 0 &&
      __hip_atomic_fetch_add(a.bar + 18 * BAR_LINE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NWG - 1) {
    for (int i = 0; i < 19; ++i)
      __hip_atomic_exchange(a.bar + i * BAR_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------------------------------
// Greedy tail of a batch-1 decode step, one launch: final LayerNorm → LM-head GEMV → argmax →
// token bookkeeping → the next step's embedding. On the launch-per-op tail these are ~8 small
// kernels per token (LN, head GEMM, argmax, pad masking, token-column store, position increment,
// embedding gather + add), ≈110 µs of a 1.39 ms step (profiles/decode_step_anatomy_r4.txt).
//   * 256 workgroups × 16 waves; every workgroup recomputes the LN of the [E] residual (4 KB from
//     L2), then each wave streams column quads of the [V][E] head table (16 × 16-B loads per lane
//     in flight) and keeps its best (bf16-rounded logit, smallest id) as one 64-bit key.
//   * argmax: per-group 64-bit atomic max (8 groups of 32 workgroups, one 256-B line each), then
//     a two-level arrival counter; the last workgroup reads the 8 maxima, applies
//     `where(done, pad, tok)`, stores the token into out[0, t], raises `done` on EOS, advances
//     `pos`, writes word_emb[tok] + pos_emb[pos] for the next step and re-zeroes the words.
// Same rounding points as the per-op tail (bf16 LN output, bf16 logits, ties → smaller id).
// Parity: reference greedy search in `fused_multi_transformer` decoding loops
// (`paddlenlp` generation `greedy_search`: argmax → where(unfinished) → append; `top_k=1`).
struct HeadArgs {
  const bf16_t *y, *g, *b;  // [E] final residual, final-LN gamma / beta
  float eps;
  int V;                    // vocabulary rows of `w`
  const bf16_t* w;          // [V][E] LM head
  u64* best;                // 8 words, 256-B apart (zero before the first launch)
  unsigned* cnt;            // 9 words, 256-B apart (zero before the first launch)
  long long* out;           // &out[0, t]
  unsigned char* done;      // [1] bool
  long long eos;            // < 0: no EOS
  long long pad;
  int* pos;                 // [1] slot of the token just decoded; advanced by one
  long long* tok;           // [1] chosen token (pad-masked)
  const bf16_t* wemb;       // [V][E] word embedding
  const bf16_t* pemb;       // [P][E] learned position embedding
  int P;
  bf16_t* resid;            // [E] next step's embedding output (written when pos + 1 < P)
};
constexpr int HNT = 1024, HNWG = 256;

__device__ __forceinline__ u64 logit_key(float v, int col) {
  const unsigned u = __float_as_uint(v);
  const unsigned k = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // order-preserving
  return ((u64)k << 32) | (u64)(0xFFFFFFFFu - (unsigned)col);     // ties → smaller id
}

__global__ __launch_bounds__(HNT) void decode_head_kernel(HeadArgs a) {
  __shared__ float xs[E];
  __shared__ float wred[16];
  __shared__ u64 wbest[16];
  __shared__ long long sh_tok;
  __shared__ int sh_pos, sh_last;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, w = blockIdx.x;
  {
    const unsigned yy = reinterpret_cast<const unsigned*>(a.y)[tid];
    const unsigned gg = reinterpret_cast<const unsigned*>(a.g)[tid];
    const unsigned bb = reinterpret_cast<const unsigned*>(a.b)[tid];
    const float v0 = bf2f((bf16_t)(yy & 0xFFFF)), v1 = bf2f((bf16_t)(yy >> 16));
    const float mean = block_sum<16>(v0 + v1, wred) * (1.f / E);
    const float d0 = v0 - mean, d1 = v1 - mean;
    const float rs = rsqrtf(block_sum<16>(d0 * d0 + d1 * d1, wred) * (1.f / E) + a.eps);
    xs[2 * tid] = bf2f(f2bf(d0 * rs * bf2f((bf16_t)(gg & 0xFFFF)) + bf2f((bf16_t)(bb & 0xFFFF))));
    xs[2 * tid + 1] = bf2f(f2bf(d1 * rs * bf2f((bf16_t)(gg >> 16)) + bf2f((bf16_t)(bb >> 16))));
  }
  __syncthreads();
  float x[4][8];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[j][i] = xs[(j * 64 + lane) * 8 + i];
  u64 best = 0;
  const int nq = (a.V + 3) >> 2, stride = gridDim.x * 16;
  for (int q = w * 16 + wv; q < nq; q += stride) {
    u16x8 wt[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const long col = min(q * 4 + c, a.V - 1);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wt[c][j] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(a.w + col * E + (j * 64 + lane) * 8));
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) s += x[j][i] * bf2f(wt[c][j][i]);
      s = wave_sum(s);
      const int col = q * 4 + c;
      if (col < a.V) {
        const u64 k = logit_key(bf2f(f2bf(s)), col);
        best = k > best ? k : best;
      }
    }
  }
  if (lane == 0) wbest[wv] = best;
  __syncthreads();
  if (tid == 0) {
    u64 m = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) m = wbest[i] > m ? wbest[i] : m;
    const int g = w & 7;
    __hip_atomic_fetch_max(a.best + g * 32, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the max has landed before the arrival
    int last = 0;
    if (__hip_atomic_fetch_add(a.cnt + g * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == HNWG / 8 - 1 &&
        __hip_atomic_fetch_add(a.cnt + 8 * 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 7)
      last = 1;
    sh_last = last;
    if (last) {
      u64 mm = 0;
      for (int i = 0; i < 8; ++i) {
        const u64 v = __hip_atomic_exchange(a.best + i * 32, (u64)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mm = v > mm ? v : mm;
      }
      for (int i = 0; i < 9; ++i)
        __hip_atomic_exchange(a.cnt + i * 64, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      long long id = (long long)(0xFFFFFFFFu - (unsigned)mm);
      if (*a.done) id = a.pad;
      *a.out = id;
      *a.tok = id;
      if (a.eos >= 0 && id == a.eos) *a.done = 1;
      const int p = *a.pos + 1;
      *a.pos = p;
      sh_tok = id;
      sh_pos = p;
    }
  }
  __syncthreads();
  if (!sh_last) return;
  const long long id = sh_tok;
  const int p = sh_pos;
  if (tid < E / 8 && p < a.P && id >= 0 && id < a.V) {
    const u16x8 u = *reinterpret_cast<const u16x8*>(a.wemb + id * E + tid * 8);
    const u16x8 v = *reinterpret_cast<const u16x8*>(a.pemb + (long)p * E + tid * 8);
    u16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f2bf(bf2f(u[i]) + bf2f(v[i]));
    *reinterpret_cast<u16x8*>(a.resid + tid * 8) = o;
  }
}

}  // namespace

// Occupancy-checked cooperative launch capability of a kernel (cached per kernel).
static int coop_ok(const void* fn, int threads) {
  static const void* fns[16];
  static int ok[16];
  static int n = 0;
  for (int i = 0; i < n; ++i)
    if (fns[i] == fn) return ok[i];
  int dev = 0, attr = 0, per_cu = 0, cus = 0;
  const int r = hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&attr, hipDeviceAttributeCooperativeLaunch, dev) == hipSuccess && attr &&
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0) == hipSuccess &&
                per_cu * cus >= NWG;
  if (n < 16) {
    fns[n] = fn;
    ok[n++] = r;
  }
  return r;
}

// The instantiated model shapes (E, D, Hq, Hk, F) × rotary off / on; the GEMV phases run on MFMA
// (MegaCfg MM default) for bf16 and int8 weight-only.
typedef MegaCfg<2048, 128, 16, 16, 8192, 0> CfgGpt13;    // GPT-3 1.3B
typedef MegaCfg<2048, 128, 16, 16, 8192, 1> CfgGpt13R;
typedef MegaCfg<2048, 128, 16, 4, 8192, 0> CfgGqa4;      // 1.3B width, 4 KV heads (GQA 4:1)
typedef MegaCfg<2048, 128, 16, 4, 8192, 1> CfgGqa4R;
typedef MegaCfg<1024, 64, 16, 16, 4096, 0> CfgGpt350;    // GPT-3 350M
typedef MegaCfg<1024, 64, 16, 16, 4096, 1> CfgGpt350R;
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 1> CfgGpt13W8;  // int8 weight-only
typedef MegaCfg<2048, 128, 16, 4, 8192, 1, 1> CfgGqa4RW8;
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 1, 1, 0> CfgGpt13W8V;  // int8 on the VALU (A/B)
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 2> CfgGpt13W4;  // int4 weight-only
typedef MegaCfg<2048, 128, 16, 4, 8192, 1, 2> CfgGqa4RW4;
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 2, 2> CfgGpt13W4B2;
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 2, 4> CfgGpt13W4B4;
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 0, 1, 0> CfgGpt13V;  // 1.3B on the VALU (A/B)
// batched steps (2 / 4 rows: small serving batches, beams)
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 0, 2> CfgGpt13B2;
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 0, 4> CfgGpt13B4;
typedef MegaCfg<2048, 128, 16, 16, 8192, 1, 0, 2> CfgGpt13RB2;
typedef MegaCfg<2048, 128, 16, 16, 8192, 1, 0, 4> CfgGpt13RB4;
typedef MegaCfg<2048, 128, 16, 4, 8192, 0, 0, 2> CfgGqa4B2;
typedef MegaCfg<2048, 128, 16, 4, 8192, 0, 0, 4> CfgGqa4B4;
typedef MegaCfg<2048, 128, 16, 4, 8192, 1, 0, 2> CfgGqa4RB2;
typedef MegaCfg<2048, 128, 16, 4, 8192, 1, 0, 4> CfgGqa4RB4;
typedef MegaCfg<1024, 64, 16, 16, 4096, 0, 0, 2> CfgGpt350B2;
typedef MegaCfg<1024, 64, 16, 16, 4096, 0, 0, 4> CfgGpt350B4;
typedef MegaCfg<1024, 64, 16, 16, 4096, 1, 0, 2> CfgGpt350RB2;
typedef MegaCfg<1024, 64, 16, 16, 4096, 1, 0, 4> CfgGpt350RB4;
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 1, 2> CfgGpt13W8B2;  // int8 weight-only, batched
typedef MegaCfg<2048, 128, 16, 16, 8192, 0, 1, 4> CfgGpt13W8B4;
typedef MegaCfg<2048, 128, 16, 4, 8192, 1, 1, 2> CfgGqa4RW8B2;
typedef MegaCfg<2048, 128, 16, 4, 8192, 1, 1, 4> CfgGqa4RW8B4;

// mm: 1 = MFMA GEMV phases, 0 = VALU, -1 = whichever is instantiated (MFMA first)
static const void* mega_fn(int E_, int D_, int hq, int hk, int F_, int rot, int w8, int nb, int mm = -1) {
#define MEGA_CFG(C)                                                                           \
  if (E_ == C::E && D_ == C::D && hq == C::HQ && hk == C::HK && F_ == C::F &&                 \
      (rot != 0) == C::ROT && w8 == C::W8 && nb == C::NB && (mm < 0 || (mm != 0) == C::MM)) \
    return (const void*)decode_mega_kernel<C>;
  MEGA_CFG(CfgGpt13) MEGA_CFG(CfgGpt13R) MEGA_CFG(CfgGqa4) MEGA_CFG(CfgGqa4R)
  MEGA_CFG(CfgGpt350) MEGA_CFG(CfgGpt350R) MEGA_CFG(CfgGpt13W8) MEGA_CFG(CfgGqa4RW8) MEGA_CFG(CfgGpt13V) MEGA_CFG(CfgGpt13W8V)
  MEGA_CFG(CfgGpt13W4) MEGA_CFG(CfgGqa4RW4) MEGA_CFG(CfgGpt13W4B2) MEGA_CFG(CfgGpt13W4B4)
  MEGA_CFG(CfgGpt13B2) MEGA_CFG(CfgGpt13B4) MEGA_CFG(CfgGpt13RB2) MEGA_CFG(CfgGpt13RB4)
  MEGA_CFG(CfgGqa4B2) MEGA_CFG(CfgGqa4B4) MEGA_CFG(CfgGqa4RB2) MEGA_CFG(CfgGqa4RB4)
  MEGA_CFG(CfgGpt350B2) MEGA_CFG(CfgGpt350B4) MEGA_CFG(CfgGpt350RB2) MEGA_CFG(CfgGpt350RB4)
  MEGA_CFG(CfgGpt13W8B2) MEGA_CFG(CfgGpt13W8B4) MEGA_CFG(CfgGqa4RW8B2) MEGA_CFG(CfgGqa4RW8B4)
#undef MEGA_CFG
  return nullptr;
}

// 1 when the variant (GEMV kind mm as in mega_fn) is instantiated and this device can run it.
PIAMD_EXPORT int piamd_decode_mega_variant_supported(int E_, int D_, int hq, int hk, int F_, int rot, int w8,
                                                     int nb, int mm) {
  const void* fn = mega_fn(E_, D_, hq, hk, F_, rot, w8, nb, mm);
  return fn != nullptr && coop_ok(fn, NT);
}
// 1 when this device can run the single-launch step for the shape at `nb` rows: an instantiated
// shape, cooperative launches supported and all NWG workgroups co-resident.
PIAMD_EXPORT int piamd_decode_mega_batch_supported(int E_, int D_, int hq, int hk, int F_, int rot, int w8,
                                                   int nb) {
  const void* fn = mega_fn(E_, D_, hq, hk, F_, rot, w8, nb);
  return fn != nullptr && coop_ok(fn, NT);
}
PIAMD_EXPORT int piamd_decode_mega_shape_supported(int E_, int D_, int hq, int hk, int F_, int rot, int w8) {
  return piamd_decode_mega_batch_supported(E_, D_, hq, hk, F_, rot, w8, 1);
}
PIAMD_EXPORT int piamd_decode_mega_supported() { return piamd_decode_mega_shape_supported(E, D, HQ, HK, F, 0, 0); }

// Launch one decode step over `nl` layers of the shape (E_, D_, hq, hk, F_) with a.rot rotary
// dims (0 or D_). `layers` is a device array of MegaLayer; scratch buffers per MegaArgs (part:
// nl · pstride_hd(hq, D_, nsplit) floats); a.loader must be 0 (the round-4 dedicated-loader
// variant was retired once the MFMA GEMV phases made this kernel faster). Returns hipError_t.
PIAMD_EXPORT int piamd_decode_mega(const MegaArgs* args, int E_, int D_, int hq, int hk, int F_,
                                   hipStream_t st) {
  const MegaArgs& a = *args;
  const void* fn = mega_fn(E_, D_, hq, hk, F_, a.rot, a.w8, a.nb, a.mm);
  if (!fn || (a.rot != 0 && a.rot != D_) || a.nl < 1 || a.loader != 0 || a.nsplit < 1 ||
      a.nb * hq * a.nsplit > NWG ||
      (a.maxS + a.nsplit - 1) / a.nsplit > 256 || !a.layers || !a.resid || !a.rbuf || !a.qn ||
      !a.kvn || !a.part || !a.h || !a.bar || !a.err || !a.pos)
    return (int)hipErrorInvalidValue;
  // cooperative launch: the runtime guarantees all NWG workgroups are co-resident (the grid
  // barriers rely on it) or refuses the launch; checked once against the kernel's occupancy
  MegaArgs arg = a;
  void* kargs[] = {&arg};
  if (!coop_ok(fn, NT)) return (int)hipErrorCooperativeLaunchTooLarge;
  return (int)hipLaunchCooperativeKernel(fn, dim3(NWG), dim3(NT), kargs, 0, st);
}

// Greedy tail of one batch-1 decode step (see decode_head_kernel). Returns hipError_t.
PIAMD_EXPORT int piamd_decode_head_greedy(const HeadArgs* args, int E_, hipStream_t st) {
  const HeadArgs& a = *args;
  if (E_ != E || a.V < 1 || !a.y || !a.g || !a.b || !a.w || !a.best || !a.cnt || !a.out || !a.done ||
      !a.pos || !a.tok || !a.wemb || !a.pemb || !a.resid || a.P < 1)
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(decode_head_kernel, dim3(HNWG), dim3(HNT), 0, st, a);
  return (int)hipGetLastError();
}
