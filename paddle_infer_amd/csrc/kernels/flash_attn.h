// Flash attention forward / backward on CDNA4 MFMA (bf16 or fp16 in, f32 accumulate), with
// in-kernel attention dropout and an additive attention mask / bias.
//
// Parity: reference `python/paddle/nn/functional/flash_attention.py:142` (flash_attention with
// `dropout`, scaled_dot_product_attention, flash_attn_unpadded), `paddle/phi/kernels/gpu/
// flash_attn_kernel.cu`, and the fork's CUTLASS `phi/kernels/fusion/cutlass/
// memory_efficient_attention*.cu` / `variable_length_memory_efficient_attention.cu` (LSE output,
// causal mask, additive mask, GQA via kv-head grouping, packed variable-length batches).
//
// This header holds the kernels; flash_attn.hip (bf16) and flash_attn_f16.hip (fp16) instantiate
// them in two translation units so the two halves compile in parallel.
//
// MI355X design (cdna_hip_programming.md §3, T2, T10, T12, App. B "Fused attention prefill",
// "Attention backward"):
//   * Layout [B, S, H, D] with free b/s/h strides, so Q/K/V are consumed straight out of the fused
//     QKV projection output and dQ/dK/dV are written straight into the fused dQKV gradient.
//   * Head dims: D in {64, 96, 128} (forward and backward) and 256 (forward). LDS rows are DP = 64 /
//     128 / 256 elements (power of two, so the XOR swizzle stays closed); D = 96 uses 128-element
//     rows whose last 4 chunks are never read.
//   * Forward: workgroup = 4 waves = 128 query rows (32 per wave), K/V tiles of 64 keys DMA'd
//     straight into LDS (global_load_lds_dwordx4), double buffered. SWAPPED products with
//     v_mfma_f32_32x32x16_{bf16,f16}: Sᵀ = K·Qᵀ puts one query row per lane, so the online-softmax
//     row max/sum is 31 in-lane ops + one cross-half shuffle, and the Sᵀ accumulator is directly
//     the B operand of Oᵀ = Vᵀ·Pᵀ (no LDS round trip for P). Vᵀ fragments come from the row-major
//     V image with ds_read_b64_tr_b16 (hardware transpose).
//   * Backward = two atomic-free kernels. dK/dV: workgroup = 128 keys (key on the MFMA lane),
//     dKᵀ/dVᵀ kept in accumulators across the whole sweep over query tiles and the q-heads of a GQA
//     group. dQ: the forward's structure (query row on the lane), dSᵀ feeds dQᵀ = Kᵀ·dSᵀ from
//     registers. Recomputing S/dP in the dQ kernel removes the f32 dQ atomics and keeps the
//     result bitwise deterministic. (A stored-dS variant — dK/dV writes 16-bit dS, dQ only runs
//     Kᵀ·dSᵀ — measured net-neutral at the GPT shape and slower elsewhere; removed in round 5,
//     A/B record profiles/fa_persist_r4.txt.)
//   * Dropout: keep(q, key) is a stateless counter hash of (seed, offset, row, key) — the same
//     keyed two-round lowbias32 as the LayerNorm dropout (common.h), one 32-bit hash per PAIR of
//     adjacent keys (two 16-bit uniforms). The forward, dK/dV and dQ kernels regenerate the same
//     mask; nothing is stored. The row sum l uses the undropped P (softmax normaliser), O uses
//     P∘M, and 1/(1-p) is folded into the epilogue scale.
//   * Mask: additive [B|1, H|1, Sq, Sk] bias in the input dtype (element strides, 0 = broadcast),
//     added to the scaled logits before the softmax in all three kernels; rows padded to a
//     multiple of 4 keys by the caller so each lane reads 8 B per 4 keys.
//   * Every global load is unconditional (row indices clamped, out-of-range rows masked in the
//     softmax), so hipcc can count `vmcnt` and the K/V prefetch stays in flight under the MFMAs.
//   * Grids are XCD-grouped (fa_map): the tiles of one (batch, head) run together on one XCD and
//     share its L2; inside a group causal tiles go heaviest-first.
#pragma once
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

// C ABI argument block (ops/attention.py mirrors it as a ctypes.Structure).
#include "fa_args.h"

// hand-scheduled assembly dK/dV and dQ kernels (fa_asm_host.hip): 1 = launched, 0 = shape not taken
int fa_dkdv_asm(const FaArgs& a, hipStream_t st);
int fa_dq_asm(const FaArgs& a, hipStream_t st);
int fa_fwd_asm(const FaArgs& a, hipStream_t st);


namespace fa {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
enum { F_DROP = 1, F_MASK = 2 };

template <bool F16>
struct ET;
template <>
struct ET<false> {
  typedef bf16x8 V8;
  static __device__ __forceinline__ f32x16 mfma(V8 a, V8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float tof(unsigned short u) { return bf2f(u); }
  static __device__ __forceinline__ unsigned short fromf(float f) { return f2bf(f); }
  static __device__ __forceinline__ V8 frag(const f32x16& acc, int s) {
    V8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)acc[8 * s + j];
    return r;
  }
};
template <>
struct ET<true> {
  typedef f16x8 V8;
  static __device__ __forceinline__ f32x16 mfma(V8 a, V8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float tof(unsigned short u) {
    return (float)__builtin_bit_cast(_Float16, u);
  }
  static __device__ __forceinline__ unsigned short fromf(float f) {
    return __builtin_bit_cast(unsigned short, (_Float16)f);
  }
  static __device__ __forceinline__ V8 frag(const f32x16& acc, int s) {
    V8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (_Float16)acc[8 * s + j];
    return r;
  }
};
template <bool F16>
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
  return (unsigned)ET<F16>::fromf(lo) | ((unsigned)ET<F16>::fromf(hi) << 16);
}

template <bool F16>
__device__ __forceinline__ typename ET<F16>::V8 cat44(s16x4_t a, s16x4_t b) {
  s16x8 t = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(typename ET<F16>::V8, t);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Direct-to-LDS DMA (global_load_lds_dwordx4) of a [ROWS][ROWB] tile into the dual-use XOR image.
// The LDS destination of one wave-instruction is lane-linear (1 KiB), so the swizzle is applied
// to the per-lane SOURCE address (guide §5.4 rule 21): physical chunk pc of row r holds logical
// chunk pc ^ x(r). Rows past `rmax` are clamped (masked later); logical chunks past the head dim
// (D < DP) re-read chunk 0 (in bounds, never consumed).
template <int ROWS, int ROWB, int DCH, int NWV = 4>
__device__ __forceinline__ void glds_tile(const unsigned short* gbase, long long rstride, int row0,
                                          int rmax, char* tile, int w, int lane) {
  constexpr int CH = ROWB / 16;
  constexpr int PIECES = ROWS * CH / 64;
  constexpr int PPW = PIECES / NWV;
  static_assert(PPW * NWV == PIECES, "tile pieces must split evenly over the waves");
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int P = w * PPW + i;
    const int L = P * 64 + lane, r = L / CH, pc = L % CH;
    const int x = (((r & 3) << 2) | ((r >> 2) & 3)) & (CH - 1);
    const long long row = min(row0 + r, rmax);
    int lc = pc ^ x;
    if (DCH < CH) lc = lc < DCH ? lc : 0;
    const unsigned short* src = gbase + row * rstride + (lc << 3);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(tile + P * 1024),
                                     16, 0, 0);
  }
}

// XCD-aware work mapping (guide T1): workgroup ids are dealt round-robin to the 8 XCDs, so the
// launcher pads the grid to a multiple of 8 and the kernel reads its logical id as
// (bid % 8) · (G / 8) + bid / 8. The `per` tiles of one (batch, head) group are then consecutive
// logical ids = consecutive dispatches on ONE XCD: they run together and share that head's K/V
// (forward, dQ) or Q/dO (dK/dV) panels in the XCD's L2 instead of fetching them from HBM once
// per tile. Returns false for the padding ids. `sub` = tile index inside the group (0 first).
__device__ __forceinline__ bool fa_map(int per, int ngroups, int& grp, int& sub) {
  const int G = (int)gridDim.x, bid = (int)blockIdx.x;
  const int lid = (bid & 7) * (G >> 3) + (bid >> 3);
  if (lid >= per * ngroups) return false;
  grp = lid / per;
  sub = lid - grp * per;
  return true;
}
__host__ __forceinline__ dim3 fa_grid(long long n) { return dim3((unsigned)((n + 7) / 8 * 8)); }

// glds_tile with the per-lane part of every piece's source address precomputed (bytes from the
// tile's first row; valid while no row of the tile needs clamping): a full-tile issue is then a
// wave-uniform base + one VGPR per piece, with no per-issue address arithmetic.
template <int ROWS, int ROWB, int DCH>
struct DmaOffs {
  static constexpr int PPW = ROWS * (ROWB / 16) / 64 / 4;
  unsigned off[PPW];
};
template <int ROWS, int ROWB, int DCH>
__device__ __forceinline__ void dma_offs(long long rstride, int w, int lane, DmaOffs<ROWS, ROWB, DCH>& o) {
  constexpr int CH = ROWB / 16;
#pragma unroll
  for (int i = 0; i < DmaOffs<ROWS, ROWB, DCH>::PPW; ++i) {
    const int P = w * DmaOffs<ROWS, ROWB, DCH>::PPW + i;
    const int L = P * 64 + lane, r = L / CH, pc = L % CH;
    const int x = (((r & 3) << 2) | ((r >> 2) & 3)) & (CH - 1);
    int lc = pc ^ x;
    if (DCH < CH) lc = lc < DCH ? lc : 0;
    o.off[i] = (unsigned)(((long long)r * rstride + (lc << 3)) * 2);
  }
}
template <int ROWS, int ROWB, int DCH>
__device__ __forceinline__ void glds_tile_pre(const unsigned short* gtile, const DmaOffs<ROWS, ROWB, DCH>& o,
                                              char* tile, int w) {
#pragma unroll
  for (int i = 0; i < DmaOffs<ROWS, ROWB, DCH>::PPW; ++i) {
    const int P = w * DmaOffs<ROWS, ROWB, DCH>::PPW + i;
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void*)(reinterpret_cast<const char*>(gtile) + o.off[i]),
        (__attribute__((address_space(3))) void*)(tile + P * 1024), 16, 0, 0);
  }
}

// Dropout key: (seed, offset) folded into two 32-bit round keys, uniform over the grid.
struct DropKey {
  uint32_t lo, hi, thr;  // thr = p * 65536: keep iff 16-bit uniform >= thr
  float inv;             // 1 / (1 - p)
};
__device__ __forceinline__ DropKey drop_key(float p, uint64_t seed, uint64_t offset) {
  DropKey k;
  k.lo = rng_key(seed, offset);
  k.hi = lowbias32(k.lo ^ 0x632BE5ABu);
  k.thr = (uint32_t)(p * 65536.f);
  k.inv = 1.f / (1.f - p);
  return k;
}
// 32-bit hash of the key pair (key >> 1) of attention row `row` (row = lse index: every (batch,
// head, query) has its own). half = key & 1 selects the 16-bit uniform.
__device__ __forceinline__ uint32_t drop_hash(const DropKey& k, long long row, int sk_half,
                                              int key) {
  const uint64_t pair = (uint64_t)row * (uint64_t)sk_half + (uint64_t)(key >> 1);
  return lowbias32(lowbias32((uint32_t)pair + k.lo) ^ (k.hi ^ ((uint32_t)(pair >> 32) * 0x85EBCA6Bu)));
}
__device__ __forceinline__ bool drop_keep(const DropKey& k, uint32_t h, int key) {
  return ((key & 1) ? (h >> 16) : (h & 0xFFFFu)) >= k.thr;
}

// 4 consecutive mask values (keys key0..key0+3, key0 % 4 == 0) of one mask row, as f32 * log2e.
template <bool F16>
__device__ __forceinline__ f32x4 mask4(const unsigned short* mrow, int key0, int Sk) {
  const int kk = key0 < Sk ? key0 : 0;
  const u16x4 m = *reinterpret_cast<const u16x4*>(mrow + kk);
  f32x4 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = ET<F16>::tof(m[e]) * kLog2e;
  return r;
}

// Per-lane LDS offsets, computed once per kernel (they are loop-invariant; every read then is one
// of these VGPRs + a compile-time immediate, so the tile loops carry no address arithmetic):
//   row[kk]     row read of 16-B chunk (2kk + hh) of image row l32 (rows 32t + l32 share the
//               swizzle of l32: +32t·ROWB is an immediate)
//   tr[jj][dt]  transposed read (ds_read_b64_tr_b16 of a 4-row x 16-col block) at rows
//               r0 = 16ks + 4hh + 8jj, cols c0 = 32dt + 16(g&1): +16ks·ROWB is an immediate.
//               d-block dt only flips chunk bits 2-3 (byte bits 6-7) of the dt = 0 offset, so
//               tr[jj][dt] == tr[jj][0] ^ (dt << 6): kernels at two waves per SIMD keep only
//               tr[.][0] live and pay one v_xor per read (tr_x)
template <int ROWB, int KSTEPS, int DT>
struct LaneOffs {
  int row[KSTEPS];
  int tr[2][DT];
};
// row[kk] == row[0] ^ (kk << 5) likewise (kk flips chunk bits 1-3 = byte bits 5-7)
template <int ROWB, int KSTEPS, int DT>
__device__ __forceinline__ int row_x(const LaneOffs<ROWB, KSTEPS, DT>& L, int kk) {
  return L.row[0] ^ (kk << 5);
}
template <int ROWB, int KSTEPS, int DT>
__device__ __forceinline__ int tr_x(const LaneOffs<ROWB, KSTEPS, DT>& L, int jj, int dt) {
  return L.tr[jj][0] ^ (dt << 6);
}
template <int ROWB, int KSTEPS, int DT>
__device__ __forceinline__ void lane_offs(int lane, LaneOffs<ROWB, KSTEPS, DT>& L) {
  constexpr int CH = ROWB / 16;
  const int l32 = lane & 31, hh = lane >> 5, gi = lane & 15, g = lane >> 4;
  const int xl = (((l32 & 3) << 2) | ((l32 >> 2) & 3)) & (CH - 1);
#pragma unroll
  for (int kk = 0; kk < KSTEPS; ++kk) L.row[kk] = l32 * ROWB + (((2 * kk + hh) ^ xl) << 4);
#pragma unroll
  for (int jj = 0; jj < 2; ++jj)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int rl = 4 * hh + 8 * jj + (gi >> 2);
      const int col = 32 * dt + 16 * (g & 1) + 4 * (gi & 3);
      const int xr = (((rl & 3) << 2) | ((rl >> 2) & 3)) & (CH - 1);
      L.tr[jj][dt] = rl * ROWB + ((((col >> 3)) ^ xr) << 4) + ((col & 7) << 1);
    }
}
template <bool F16>
__device__ __forceinline__ typename ET<F16>::V8 lds_at(const char* smem, int off) {
  return *reinterpret_cast<const typename ET<F16>::V8*>(smem + off);
}
__device__ __forceinline__ s16x4_t lds_tr_at(const char* smem, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + off));
}

// ------------------------------------------------------------------------------------------
// Forward
// ------------------------------------------------------------------------------------------
// NW waves per workgroup, 32 query rows each (BM = 32·NW); NW = 8 shares every K/V tile fill
// between twice the rows (half the LDS fill traffic per FLOP) at one workgroup per CU.
// D = 256 (wide heads): 512-byte LDS rows (K+V double buffer 128 KiB) and one workgroup per CU —
// the 16 Q fragments + 8 O accumulators need the whole 512-register file of one wave per SIMD.
template <int D, bool F16, bool CAUSAL, int FEAT, int NW = 4>
__global__ __launch_bounds__(64 * NW, D > 128 ? 1 : 8 / NW) void fwd_kernel(FaArgs a) {
  typedef ET<F16> E;
  typedef typename E::V8 V8;
  constexpr int DP = D > 128 ? 256 : D > 64 ? 128 : 64;
  constexpr int BM = 32 * NW, BN = 64;
  constexpr int KSTEPS = D / 16;
  constexpr int DT = D / 32;
  constexpr int ROWB = DP * 2;
  constexpr int TILE_B = BN * ROWB;  // bytes per K or V tile
  // one LDS object per buffer: the waitcnt pass can then prove the reads of buffer t
  // independent of the DMA still landing in buffer t+1 (a single array made hipcc put a
  // vmcnt(0) before the PV reads of every tile, exposing the next tile's HBM fetch)
  __shared__ __attribute__((aligned(16))) char kv0[2 * TILE_B];
  __shared__ __attribute__((aligned(16))) char kv1[2 * TILE_B];

  const unsigned short* q = (const unsigned short*)a.q;
  const unsigned short* k = (const unsigned short*)a.k;
  const unsigned short* v = (const unsigned short*)a.v;
  unsigned short* o = (unsigned short*)a.o;
  const int B = a.B, SqMax = a.Sq, Hq = a.Hq, Hk = a.Hk;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5, gi = lane & 15, g = lane >> 4;
  const int nmb = (SqMax + BM - 1) / BM;
  int grp, sub;
  if (!fa_map(nmb, Hq * B, grp, sub)) return;
  const int mb = CAUSAL ? nmb - 1 - sub : sub;  // causal: heaviest query block first
  const int hq = grp % Hq, b = grp / Hq;
  const int hk = hq / (Hq / Hk);
  const int m0 = mb * BM;
  int Sq = SqMax, Sk = a.Sk;
  long long lbase = ((long long)b * Hq + hq) * SqMax;
  if (a.cu_q) {  // variable-length: b = sequence, rows [cu[b], cu[b+1]) of the packed tensors
    const int q0s = a.cu_q[b], k0s = a.cu_k[b];
    Sq = a.cu_q[b + 1] - q0s;
    Sk = a.cu_k[b + 1] - k0s;
    if (m0 >= Sq) return;  // block-uniform: this sequence is shorter than the longest
    q += (long long)q0s * a.sqs;
    o += (long long)q0s * a.sos;
    k += (long long)k0s * a.sks;
    v += (long long)k0s * a.svs;
    lbase = (long long)hq * a.ltot + q0s;
  }
  const int qrow0 = m0 + w * 32;
  const int coff = Sk - Sq;  // bottom-right aligned causal offset
  const float c = a.scale * kLog2e;
  const int qpos = qrow0 + l32;

  const unsigned short* kbase = k + b * a.skb + hk * a.skh;
  const unsigned short* vbase = v + b * a.svb + hk * a.svh;
  const unsigned short* mrow = nullptr;
  if (FEAT & F_MASK)
    mrow = (const unsigned short*)a.mask + b * a.smb + hq * a.smh + (long long)min(qpos, Sq - 1) * a.smq;
  DropKey dk;
  if (FEAT & F_DROP) dk = drop_key(a.p_drop, a.seed, a.offset);
  const int sk_half = (a.Sk + 1) >> 1;

  V8 qf[KSTEPS];
  {
    const int qr = min(qpos, Sq - 1);
    const unsigned short* qp = q + b * a.sqb + (long long)qr * a.sqs + hq * a.sqh + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) qf[kk] = *reinterpret_cast<const V8*>(qp + 16 * kk);
  }

  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, m0 + BM + coff);
  const int ntiles = n_end <= 0 ? 0 : (n_end + BN - 1) / BN;

  f32x16 oacc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) oacc[i][j] = 0.f;
  float m_i = -INFINITY, l_i = 0.f;

  auto issue = [&](int t, auto bufc) {
    char* ks = decltype(bufc)::value ? kv1 : kv0;
    glds_tile<BN, ROWB, D / 8, NW>(kbase, a.sks, t * BN, Sk - 1, ks, w, lane);
    glds_tile<BN, ROWB, D / 8, NW>(vbase, a.svs, t * BN, Sk - 1, ks + TILE_B, w, lane);
  };
  if (ntiles > 0) issue(0, std::integral_constant<int, 0>{});
  __syncthreads();

  LaneOffs<ROWB, KSTEPS, DT> L;
  lane_offs(lane, L);
  const bool wave_rows_valid = qrow0 < Sq;
  // key (relative to n0 + 4hh) valid for this lane's row iff < lim - n0
  const int m_lim = min(CAUSAL ? qpos + coff + 1 : 0x40000000, Sk) - 4 * hh;
  auto tile = [&](int t, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    constexpr int KS = 0, VS = TILE_B;
    const char* smem = BUF ? kv1 : kv0;
    if (t + 1 < ntiles) issue(t + 1, std::integral_constant<int, BUF ^ 1>{});
    const int n0 = t * BN;
    const bool active = wave_rows_valid && (!CAUSAL || n0 <= qrow0 + 31 + coff);
    if (active) {
      f32x16 sacc[2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int j = 0; j < 16; ++j) sacc[tt][j] = 0.f;
#pragma unroll
      for (int kk = 0; kk < KSTEPS; ++kk)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
          sacc[tt] = E::mfma(lds_at<F16>(smem, L.row[kk] + KS + tt * 32 * ROWB), qf[kk], sacc[tt]);
      const bool need_mask = (n0 + BN > Sk) || (CAUSAL && n0 + BN - 1 > qrow0 + coff);
      // scaled logits x = c·s (+ mask); on unmasked tiles without an additive mask the scale is
      // folded into the exponent below (p = exp2(c·s − m): one fma per element, and the row max
      // taken on the raw scores, c > 0)
      const bool fold = !(FEAT & F_MASK) && !need_mask;
      float mx = -INFINITY;
      auto scale_mask = [&](auto maskc) {
        constexpr bool MASKED = decltype(maskc)::value;
        const int lim = m_lim - n0;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            f32x4 mb4 = {0.f, 0.f, 0.f, 0.f};
            if (FEAT & F_MASK) mb4 = mask4<F16>(mrow, n0 + tt * 32 + 8 * g4 + 4 * hh, Sk);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 4 * g4 + e;
              float x = sacc[tt][r] * c + mb4[e];
              if (MASKED) x = (tt * 32 + 8 * g4 + e) < lim ? x : -INFINITY;
              sacc[tt][r] = x;
              mx = fmaxf(mx, x);
            }
          }
      };
      if (fold) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[tt][r]);
        mx *= c;
      } else if (need_mask) {
        scale_mask(std::true_type{});
      } else {
        scale_mask(std::false_type{});
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      // lazy rescale: the running max m_i moves only when a row's tile max exceeds it by more than
      // 8 (log2 units); p = exp2(x − m_i) ≤ 256 is exact in f32 / bf16 range and l_i, O use the same
      // m_i, so the result is unchanged while most tiles skip the O rescale
      const float m_new = mx > m_i + 8.f ? mx : m_i;
      const float msub = m_new == -INFINITY ? 0.f : m_new;
      float rs = 0.f;
      if (fold) {
        const float nm = -msub;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float p = fast_exp2(fmaf(sacc[tt][r], c, nm));
            sacc[tt][r] = p;
            rs += p;
          }
      } else {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float p = fast_exp2(sacc[tt][r] - msub);
            sacc[tt][r] = p;
            rs += p;
          }
      }
      rs += __shfl_xor(rs, 32, 64);
      if (FEAT & F_DROP) {  // O accumulates P∘M; the normaliser l keeps the undropped sum
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const int key = n0 + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const uint32_t h = drop_hash(dk, lbase + qpos, sk_half, key);
            if (!drop_keep(dk, h, key)) sacc[tt][r] = 0.f;
            if (!drop_keep(dk, h, key + 1)) sacc[tt][r + 1] = 0.f;
          }
      }
      // rescale only when some row's running max moved (T13-style skip of an O-wide pass)
      if (__any(m_new > m_i)) {
        const float alpha = fast_exp2(m_i - msub);
        l_i *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int j = 0; j < 16; ++j) oacc[dt][j] *= alpha;
      }
      l_i += rs;
      m_i = m_new;
      V8 pf[4];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int s = 0; s < 2; ++s) pf[2 * tt + s] = E::frag(sacc[tt], s);
      // Oᵀ += Vᵀ · Pᵀ
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) {
          const int ro = VS + 16 * ks4 * ROWB;
          oacc[dt] = E::mfma(cat44<F16>(lds_tr_at(smem, L.tr[0][dt] + ro), lds_tr_at(smem, L.tr[1][dt] + ro)),
                             pf[ks4], oacc[dt]);
        }
    }
    __syncthreads();
  };
  for (int t = 0; t < ntiles; t += 2) {
    tile(t, std::integral_constant<int, 0>{});
    if (t + 1 < ntiles) tile(t + 1, std::integral_constant<int, 1>{});
  }

  // epilogue: lane = query row, registers = d
  if (qpos < Sq) {
    float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    if (FEAT & F_DROP) inv *= dk.inv;
    unsigned short* op = o + b * a.sob + (long long)qpos * a.sos + hq * a.soh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * hh;
        uint2 pk;
        pk.x = pack2<F16>(oacc[dt][4 * g4 + 0] * inv, oacc[dt][4 * g4 + 1] * inv);
        pk.y = pack2<F16>(oacc[dt][4 * g4 + 2] * inv, oacc[dt][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(op + d0) = pk;
      }
    if (hh == 0 && a.lse)
      a.lse[lbase + qpos] = l_i > 0.f ? (m_i + log2f(l_i)) * kLn2 : INFINITY;
  }
}

// ------------------------------------------------------------------------------------------
// Persistent forward (padded layout, D <= 128, 4 waves): the grid is the resident workgroups
// (2 per CU) and each walks a static list of (batch, head, query-block) items. The items of one
// (batch, head) stay on one XCD (its K/V panel shared in that L2, as fa_map arranges for the
// one-item kernel) and every XCD's list runs the heaviest causal blocks first. The K/V tiles form
// ONE continuous sequence alternating between the two LDS buffers across item boundaries: the
// next item's first tile is DMA'd during the current item's last tile, and its Q fragments load
// right after the last S product — the prologue (Q fetch + first tile landing) of an item hides
// under the previous one instead of idling the CU, which short causal sequences (S = 1024: 2-16
// tiles per item) pay on every workgroup of the one-item kernel.
// ------------------------------------------------------------------------------------------
template <int D, bool F16, bool CAUSAL, int FEAT>
__global__ __launch_bounds__(256, 2) void fwd_persist_kernel(FaArgs a) {
  typedef ET<F16> E;
  typedef typename E::V8 V8;
  constexpr int DP = D > 64 ? 128 : 64;
  constexpr int BM = 128, BN = 64;
  constexpr int KSTEPS = D / 16;
  constexpr int DT = D / 32;
  constexpr int ROWB = DP * 2;
  constexpr int TILE_B = BN * ROWB;
  __shared__ __attribute__((aligned(16))) char kv0[2 * TILE_B];
  __shared__ __attribute__((aligned(16))) char kv1[2 * TILE_B];

  const unsigned short* q = (const unsigned short*)a.q;
  const unsigned short* k = (const unsigned short*)a.k;
  const unsigned short* v = (const unsigned short*)a.v;
  unsigned short* o = (unsigned short*)a.o;
  const int Sq = a.Sq, Sk = a.Sk, Hq = a.Hq, Hk = a.Hk;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int nmb = (Sq + BM - 1) / BM;
  const int ngroups = Hq * a.B;
  // static schedule: this workgroup runs on XCD blockIdx % 8 (round-robin dispatch) as local
  // worker blockIdx / 8 of gridDim / 8; XCD x owns the (batch, head) groups x, x + 8, ...
  const int xcd = (int)blockIdx.x & 7, nl = (int)gridDim.x >> 3, li = (int)blockIdx.x >> 3;
  const int gx = ngroups > xcd ? (ngroups - xcd + 7) / 8 : 0;
  const int nitems = gx * nmb;  // item j = sub · gx + group slot (sub 0 = heaviest block first)
  const int coff = Sk - Sq;
  const float c = a.scale * kLog2e;
  DropKey dk;
  if (FEAT & F_DROP) dk = drop_key(a.p_drop, a.seed, a.offset);
  const int sk_half = (a.Sk + 1) >> 1;

  struct Item {
    int b, hq, m0, ntiles;
    const unsigned short *kb, *vb;
  };
  // Worker li's kk-th item. Diagonal schedule (nl a multiple of nmb, at least nl groups per XCD):
  // step kk covers nl / nmb groups, the nmb workers of one group take its nmb query blocks
  // TOGETHER (its K/V panel is read into L2 once for all of them) and each worker rotates through
  // the block weights, so every worker gets the same causal work per nmb steps. Fewer groups (a
  // worker runs fewer than nmb items, the rotation would not balance): items sub-major, heaviest
  // first. Measured (B, S, H, D causal bf16): 96,1024,16,128 fwd 0.851 -> 0.816 ms diagonal (sub-major
  // 0.987: each head's K/V re-read per block), 8,2048,16,128 0.222 -> 0.199 and 4,4096,16,128
  // 0.366 -> 0.361 sub-major (diagonal 0.285 / 0.555), profiles/fa_persist_r4.txt.
  const bool diag = nl >= nmb && nl % nmb == 0 && gx >= nl;
  auto setup = [&](int kk, Item& it) -> bool {
    int slot, sub;
    if (diag) {
      slot = kk * (nl / nmb) + li / nmb;
      sub = (li % nmb + kk) % nmb;
    } else {
      const int jj = li + kk * nl;
      if (jj >= nitems) return false;
      sub = jj / gx;
      slot = jj - sub * gx;
    }
    if (slot >= gx) return false;
    const int grp = xcd + 8 * slot;
    const int mb = CAUSAL ? nmb - 1 - sub : sub;
    it.hq = grp % Hq;
    it.b = grp / Hq;
    it.m0 = mb * BM;
    const int hk = it.hq / (Hq / Hk);
    it.kb = k + it.b * a.skb + hk * a.skh;
    it.vb = v + it.b * a.svb + hk * a.svh;
    int n_end = Sk;
    if (CAUSAL) n_end = min(Sk, it.m0 + BM + coff);
    // at least one (masked) tile: rows are clamped, so the DMA stays in bounds
    it.ntiles = n_end <= 0 ? 1 : (n_end + BN - 1) / BN;
    return true;
  };
  auto issue = [&](const Item& it, int t, auto bufc) {
    char* ks = decltype(bufc)::value ? kv1 : kv0;
    glds_tile<BN, ROWB, D / 8, 4>(it.kb, a.sks, t * BN, Sk - 1, ks, w, lane);
    glds_tile<BN, ROWB, D / 8, 4>(it.vb, a.svs, t * BN, Sk - 1, ks + TILE_B, w, lane);
  };
  V8 qf[KSTEPS];
  auto load_q = [&](const Item& it) {
    const int qr = min(it.m0 + w * 32 + l32, Sq - 1);
    const unsigned short* qp = q + it.b * a.sqb + (long long)qr * a.sqs + it.hq * a.sqh + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) qf[kk] = *reinterpret_cast<const V8*>(qp + 16 * kk);
  };

  int kk = 0;
  Item cur, nxt;
  if (nitems == 0 || !setup(0, cur)) return;
  bool has_next = setup(1, nxt);
  issue(cur, 0, std::integral_constant<int, 0>{});
  load_q(cur);
  __syncthreads();

  LaneOffs<ROWB, KSTEPS, DT> L;
  lane_offs(lane, L);
  f32x16 oacc[DT];
  float m_i, l_i;
  auto reset = [&]() {
#pragma unroll
    for (int i = 0; i < DT; ++i)
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) oacc[i][jj] = 0.f;
    m_i = -INFINITY;
    l_i = 0.f;
  };
  reset();
  int t = 0;
  bool done = false;

  auto tile = [&](auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    constexpr int KS = 0, VS = TILE_B;
    const char* smem = BUF ? kv1 : kv0;
    const bool last = t + 1 == cur.ntiles;
    if (!last) issue(cur, t + 1, std::integral_constant<int, BUF ^ 1>{});
    else if (has_next) issue(nxt, 0, std::integral_constant<int, BUF ^ 1>{});
    const int qrow0 = cur.m0 + w * 32, qpos = qrow0 + l32;
    const int n0 = t * BN;
    const bool active = qrow0 < Sq && (!CAUSAL || n0 <= qrow0 + 31 + coff) && n0 < Sk;
    if (active) {
      f32x16 sacc[2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) sacc[tt][jj] = 0.f;
#pragma unroll
      for (int kk = 0; kk < KSTEPS; ++kk)
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
          sacc[tt] = E::mfma(lds_at<F16>(smem, L.row[kk] + KS + tt * 32 * ROWB), qf[kk], sacc[tt]);
      if (last && has_next) load_q(nxt);  // qf is dead for this item: the next item's Q lands under the softmax / PV
      const int m_lim = min(CAUSAL ? qpos + coff + 1 : 0x40000000, Sk) - 4 * hh;
      const bool need_mask = (n0 + BN > Sk) || (CAUSAL && n0 + BN - 1 > qrow0 + coff);
      const unsigned short* mrow = nullptr;
      if (FEAT & F_MASK)
        mrow = (const unsigned short*)a.mask + cur.b * a.smb + cur.hq * a.smh + (long long)min(qpos, Sq - 1) * a.smq;
      // scaled logits x = c·s (+ mask); on unmasked tiles without an additive mask the scale is
      // folded into the exponent below (p = exp2(c·s − m): one fma per element, and the row max
      // taken on the raw scores, c > 0)
      const bool fold = !(FEAT & F_MASK) && !need_mask;
      float mx = -INFINITY;
      auto scale_mask = [&](auto maskc) {
        constexpr bool MASKED = decltype(maskc)::value;
        const int lim = m_lim - n0;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            f32x4 mb4 = {0.f, 0.f, 0.f, 0.f};
            if (FEAT & F_MASK) mb4 = mask4<F16>(mrow, n0 + tt * 32 + 8 * g4 + 4 * hh, Sk);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 4 * g4 + e;
              float x = sacc[tt][r] * c + mb4[e];
              if (MASKED) x = (tt * 32 + 8 * g4 + e) < lim ? x : -INFINITY;
              sacc[tt][r] = x;
              mx = fmaxf(mx, x);
            }
          }
      };
      if (fold) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, sacc[tt][r]);
        mx *= c;
      } else if (need_mask) {
        scale_mask(std::true_type{});
      } else {
        scale_mask(std::false_type{});
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      // lazy rescale: the running max m_i moves only when a row's tile max exceeds it by more than
      // 8 (log2 units); p = exp2(x − m_i) ≤ 256 is exact in f32 / bf16 range and l_i, O use the same
      // m_i, so the result is unchanged while most tiles skip the O rescale
      const float m_new = mx > m_i + 8.f ? mx : m_i;
      const float msub = m_new == -INFINITY ? 0.f : m_new;
      float rs = 0.f;
      if (fold) {
        const float nm = -msub;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float p = fast_exp2(fmaf(sacc[tt][r], c, nm));
            sacc[tt][r] = p;
            rs += p;
          }
      } else {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float p = fast_exp2(sacc[tt][r] - msub);
            sacc[tt][r] = p;
            rs += p;
          }
      }
      rs += __shfl_xor(rs, 32, 64);
      if (FEAT & F_DROP) {
        const long long lbase = ((long long)cur.b * Hq + cur.hq) * Sq;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const int key = n0 + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const uint32_t hsh = drop_hash(dk, lbase + qpos, sk_half, key);
            if (!drop_keep(dk, hsh, key)) sacc[tt][r] = 0.f;
            if (!drop_keep(dk, hsh, key + 1)) sacc[tt][r + 1] = 0.f;
          }
      }
      if (__any(m_new > m_i)) {
        const float alpha = fast_exp2(m_i - msub);
        l_i *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int jj = 0; jj < 16; ++jj) oacc[dt][jj] *= alpha;
      }
      l_i += rs;
      m_i = m_new;
      V8 pf[4];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) pf[2 * tt + s2] = E::frag(sacc[tt], s2);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) {
          const int ro = VS + 16 * ks4 * ROWB;
          oacc[dt] = E::mfma(cat44<F16>(lds_tr_at(smem, L.tr[0][dt] + ro), lds_tr_at(smem, L.tr[1][dt] + ro)),
                             pf[ks4], oacc[dt]);
        }
    } else if (last && has_next) {
      load_q(nxt);
    }
    __syncthreads();
    if (!last) {
      ++t;
      return;
    }
    // item done: epilogue (lane = query row, registers = d), then switch to the next item
    if (qpos < Sq) {
      float inv = l_i > 0.f ? 1.f / l_i : 0.f;
      if (FEAT & F_DROP) inv *= dk.inv;
      unsigned short* op = o + cur.b * a.sob + (long long)qpos * a.sos + cur.hq * a.soh;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * dt + 8 * g4 + 4 * hh;
          uint2 pk;
          pk.x = pack2<F16>(oacc[dt][4 * g4 + 0] * inv, oacc[dt][4 * g4 + 1] * inv);
          pk.y = pack2<F16>(oacc[dt][4 * g4 + 2] * inv, oacc[dt][4 * g4 + 3] * inv);
          *reinterpret_cast<uint2*>(op + d0) = pk;
        }
      if (hh == 0 && a.lse)
        a.lse[((long long)cur.b * Hq + cur.hq) * Sq + qpos] = l_i > 0.f ? (m_i + log2f(l_i)) * kLn2 : INFINITY;
    }
    if (!has_next) {
      done = true;
      return;
    }
    ++kk;
    cur = nxt;
    has_next = setup(kk + 1, nxt);
    t = 0;
    reset();
  };
  while (true) {
    tile(std::integral_constant<int, 0>{});
    if (done) break;
    tile(std::integral_constant<int, 1>{});
    if (done) break;
  }
}

// ------------------------------------------------------------------------------------------
// Backward pre-pass, per attention row (f32, [rows] then [rows] again):
//   nrow[r]        = −Σ_d dO·O            (−δ: the dP accumulators start from it)
//   nrow[rows + r] = −lse / scale          (the S accumulators start from it)
// "Row constants as the initial accumulator" (guide App. B, attention backward): S' = Q·Kᵀ −
// lse/scale and dP' = dO·Vᵀ − δ leave the MFMA chains ready, so p = exp2(c·S') and dS = p·dP'
// need no per-element subtraction. 16 B per lane, DP/8 lanes per row.
// ------------------------------------------------------------------------------------------
template <int D, bool F16>
__global__ __launch_bounds__(256) void bwd_pre_kernel(const unsigned short* __restrict__ o,
                                                      const unsigned short* __restrict__ dout,
                                                      const float* __restrict__ lse,
                                                      float* __restrict__ nrow, float inv_scale,
                                                      int Sq, int Hq, long long sob, long long sos,
                                                      long long soh, int total) {
  constexpr int TPR = D > 64 ? 16 : 8;  // threads per row (power of two)
  const int row = (blockIdx.x * 256 + threadIdx.x) / TPR, sub = threadIdx.x % TPR;
  const bool ok = row < total;
  const int rr = ok ? row : 0;
  const int qr = rr % Sq, hq = (rr / Sq) % Hq, b = rr / (Sq * Hq);
  const int sc = sub < D / 8 ? sub : 0;
  const long long off = b * sob + (long long)qr * sos + hq * soh + sc * 8;
  u16x8 x = *reinterpret_cast<const u16x8*>(o + off);
  u16x8 d = *reinterpret_cast<const u16x8*>(dout + off);
  float s = 0.f;
  if (sub < D / 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += ET<F16>::tof(x[j]) * ET<F16>::tof(d[j]);
#pragma unroll
  for (int m = TPR / 2; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
  if (ok && sub == 0) {
    const long long r = ((long long)b * Hq + hq) * Sq + qr;
    nrow[r] = -s;
    nrow[total + r] = -lse[r] * inv_scale;
  }
}

// ------------------------------------------------------------------------------------------
// Backward dK/dV: workgroup = 128 keys of one (batch, kv-head); sweeps the q-heads of the GQA
// group and all query tiles of 64 rows. Key on the MFMA lane.
// ------------------------------------------------------------------------------------------
template <int D, bool F16, bool CAUSAL, int FEAT>
__global__ __launch_bounds__(256, 1) void bwd_dkdv_kernel(FaArgs a) {
  typedef ET<F16> E;
  typedef typename E::V8 V8;
  constexpr int DP = D > 64 ? 128 : 64;
  constexpr int BK = 128, BQ = 64;
  constexpr int KSTEPS = D / 16;
  constexpr int DT = D / 32;
  constexpr int ROWB = DP * 2;
  constexpr int QTILE_B = BQ * ROWB;    // Q or dO tile [64][DP]
  constexpr int KIMG_B = BK * ROWB;     // resident K and V images of the block's 128 keys
  constexpr int OFF_K = 0;
  constexpr int OFF_V = OFF_K + KIMG_B;
  constexpr int OFF_STAT = 2 * QTILE_B;  // per buffer: (−lse/scale, −δ) x 64 f32 after Q, dO
  constexpr int QBUF_B = OFF_STAT + 2 * BQ * 4;
  // resident K/V images and the two Q/dO buffers as separate LDS objects: the waitcnt pass can
  // then prove reads of one buffer independent of the DMA landing in the other (one array made
  // hipcc wait vmcnt(0) before the first transposed read of every tile)
  __shared__ __attribute__((aligned(16))) char smem[2 * KIMG_B];
  __shared__ __attribute__((aligned(16))) char qb0[QBUF_B];
  __shared__ __attribute__((aligned(16))) char qb1[QBUF_B];

  const unsigned short* q = (const unsigned short*)a.q;
  const unsigned short* k = (const unsigned short*)a.k;
  const unsigned short* v = (const unsigned short*)a.v;
  const unsigned short* dout = (const unsigned short*)a.dout;
  unsigned short* dk = (unsigned short*)a.dk;
  unsigned short* dv = (unsigned short*)a.dv;
  const float* nd = a.delta;                 // −δ
  const long long rows = a.cu_q ? (long long)a.Hq * a.ltot : (long long)a.B * a.Hq * a.Sq;
  const float* nl = a.delta + rows;  // −lse/scale
  const int B = a.B, SqMax = a.Sq, Hq = a.Hq, Hk = a.Hk;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int HB = Hk * B;
  // causal: low key blocks see the most queries -> first
  int kb = (int)blockIdx.x / HB, hk = (int)blockIdx.x % Hk, b = ((int)blockIdx.x % HB) / Hk;
  if (a.map & 2) {
    int grp;
    if (!fa_map((a.Sk + BK - 1) / BK, HB, grp, kb)) return;
    hk = grp % Hk;
    b = grp / Hk;
  }
  const int n0 = kb * BK;
  int Sq = SqMax, Sk = a.Sk;
  long long lrow = (long long)b * Hq * SqMax, lhead = SqMax;  // stats index = lrow + hq*lhead + q
  if (a.cu_q) {
    const int q0s = a.cu_q[b], k0s = a.cu_k[b];
    Sq = a.cu_q[b + 1] - q0s;
    Sk = a.cu_k[b + 1] - k0s;
    if (n0 >= Sk) return;
    q += (long long)q0s * a.sqs;
    dout += (long long)q0s * a.sos;
    k += (long long)k0s * a.sks;
    v += (long long)k0s * a.svs;
    dk += (long long)k0s * a.sks;
    dv += (long long)k0s * a.svs;
    lrow = q0s;
    lhead = a.ltot;
  }
  const int kw0 = n0 + 32 * w;  // this wave's first key
  const int key = kw0 + l32;
  const int coff = Sk - Sq;
  const int group = Hq / Hk;
  const float c = a.scale * kLog2e;
  DropKey drk;
  if (FEAT & F_DROP) drk = drop_key(a.p_drop, a.seed, a.offset);
  const int sk_half = (a.Sk + 1) >> 1;
  const int keyc = min(key, Sk - 1);

  // K / V of the block's keys stay resident in LDS (B operands of S and dP are row reads)
  glds_tile<BK, ROWB, D / 8>(k + b * a.skb + hk * a.skh, a.sks, n0, Sk - 1, smem + OFF_K, w, lane);
  glds_tile<BK, ROWB, D / 8>(v + b * a.svb + hk * a.svh, a.svs, n0, Sk - 1, smem + OFF_V, w, lane);

  LaneOffs<ROWB, KSTEPS, DT> L;
  lane_offs(lane, L);
  int kvo[KSTEPS];  // this wave's K rows (V = +KIMG_B)
#pragma unroll
  for (int kk = 0; kk < KSTEPS; ++kk) kvo[kk] = OFF_K + 32 * w * ROWB + L.row[kk];

  f32x16 dkacc[DT], dvacc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) { dkacc[i][j] = 0.f; dvacc[i][j] = 0.f; }

  const int q_start = CAUSAL ? max(0, n0 - coff) : 0;
  const int qt0 = q_start / BQ;
  const int nqt = (Sq + BQ - 1) / BQ;
  const int tiles_per_head = nqt - qt0;
  const int total = (n0 < Sk && tiles_per_head > 0) ? tiles_per_head * group : 0;
  // causal / bounds mask in lane-relative form: row qr = q0 + 4hh + cq (cq compile-time) is
  // valid for this lane's key iff lo <= q0 + cq < hi  (lo, hi per lane; q0 added per tile)
  const int m_hi = key < Sk ? Sq - 4 * hh : -0x40000000;
  const int m_lo = CAUSAL ? key - coff - 4 * hh : -0x40000000;

  DmaOffs<BQ, ROWB, D / 8> dmq, dmo;
  dma_offs(a.sqs, w, lane, dmq);
  dma_offs(a.sos, w, lane, dmo);
  auto issue = [&](int it, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    char* qb = buf ? qb1 : qb0;
    const int hq = hk * group + it / tiles_per_head;
    const int q0 = (qt0 + it % tiles_per_head) * BQ;
    char* qs = qb;
    const unsigned short* qh = q + b * a.sqb + hq * a.sqh;
    const unsigned short* oh = dout + b * a.sob + hq * a.soh;
    if (q0 + BQ <= Sq) {  // full tile: precomputed lane offsets
      glds_tile_pre<BQ, ROWB, D / 8>(qh + (long long)q0 * a.sqs, dmq, qs, w);
      glds_tile_pre<BQ, ROWB, D / 8>(oh + (long long)q0 * a.sos, dmo, qs + QTILE_B, w);
    } else {
      glds_tile<BQ, ROWB, D / 8>(qh, a.sqs, q0, Sq - 1, qs, w, lane);
      glds_tile<BQ, ROWB, D / 8>(oh, a.sos, q0, Sq - 1, qs + QTILE_B, w, lane);
    }
    if (w < 2) {  // wave 0: −lse/scale row, wave 1: −δ row (64 f32 = one 4-B/lane DMA)
      const float* s = (w == 0 ? nl : nd) + lrow + hq * lhead + min(q0 + lane, Sq - 1);
      char* st = qb + OFF_STAT + w * BQ * 4;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)s,
                                       (__attribute__((address_space(3))) void*)st, 4, 0, 0);
    }
  };
  if (total > 0) issue(0, std::integral_constant<int, 0>{});
  __syncthreads();

  // one query tile; every LDS address below is a precomputed lane offset + an immediate. The
  // buffer parity is a template constant (two tile bodies) so each body reads one LDS object
  // while the DMA lands in the other.
  auto tile = [&](int it, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    const char* qb = BUF ? qb1 : qb0;
    constexpr int QS = 0, DOS = QTILE_B;
    const float* lst = reinterpret_cast<const float*>(qb + OFF_STAT);
    const float* dst = lst + BQ;
    const int hq = hk * group + it / tiles_per_head;
    const int q0 = (qt0 + it % tiles_per_head) * BQ;
    if (it + 1 < total) issue(it + 1, std::integral_constant<int, BUF ^ 1>{});
    f32x16 sacc[2], pacc[2];
    // S' = Q·Kᵀ − lse/scale, dP' = dO·Vᵀ − δ: row constants as the initial accumulators
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int qi0 = qt * 32 + 8 * g4 + 4 * hh;
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(lst + qi0);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(dst + qi0);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sacc[qt][4 * g4 + e] = l4[e];
          pacc[qt][4 * g4 + e] = (FEAT & F_DROP) ? 0.f : d4[e];
        }
      }
    V8 fr[2][6];
    auto ld = [&](int kk, V8* f) {
      f[0] = lds_at<F16>(smem, kvo[kk]);
      f[1] = lds_at<F16>(smem, kvo[kk] + KIMG_B);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f[2 + qt] = lds_at<F16>(qb, L.row[kk] + QS + qt * 32 * ROWB);
        f[4 + qt] = lds_at<F16>(qb, L.row[kk] + DOS + qt * 32 * ROWB);
      }
    };
    ld(0, fr[0]);
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) {
      if (kk + 1 < KSTEPS) ld(kk + 1, fr[(kk + 1) & 1]);
      const V8* f = fr[kk & 1];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        sacc[qt] = E::mfma(f[2 + qt], f[0], sacc[qt]);
        pacc[qt] = E::mfma(f[4 + qt], f[1], pacc[qt]);
      }
    }
    const bool need_mask = (kw0 + 31 >= Sk) || (q0 + BQ > Sq) || (CAUSAL && kw0 + 31 > q0 + coff);
    const unsigned short* mbase = nullptr;
    if (FEAT & F_MASK) mbase = (const unsigned short*)a.mask + b * a.smb + hq * a.smh + keyc;
    auto finish = [&](auto maskc) {
      constexpr bool MASKED = decltype(maskc)::value;
      const int lo = m_lo - q0, hi = m_hi - q0;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          f32x4 d4;
          if (FEAT & F_DROP) d4 = *reinterpret_cast<const f32x4*>(dst + qt * 32 + 8 * g4 + 4 * hh);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * g4 + e;
            const int cq = qt * 32 + 8 * g4 + e;  // query row - q0 - 4hh
            float x = sacc[qt][r] * c;
            if (FEAT & F_MASK)
              x += E::tof(mbase[(long long)min(q0 + 4 * hh + cq, Sq - 1) * a.smq]) * kLog2e;
            float p = fast_exp2(x);
            if (MASKED) p = (cq >= lo && cq < hi) ? p : 0.f;
            float ds = pacc[qt][r];
            float pd = p;
            if (FEAT & F_DROP) {
              const int qr = q0 + 4 * hh + cq;
              const bool kp = drop_keep(drk, drop_hash(drk, lrow + hq * lhead + qr, sk_half, key), key);
              pd = kp ? p : 0.f;
              ds = (kp ? ds * drk.inv : 0.f) + d4[e];
            }
            sacc[qt][r] = pd;
            pacc[qt][r] = p * ds;
          }
        }
    };
    if (need_mask) finish(std::true_type{});
    else finish(std::false_type{});
    // dVᵀ += dOᵀ·(P∘M) ; dKᵀ += Qᵀ·dS   (A operands via transposed reads of the dO / Q images)
    V8 pb[4], db[4];
#pragma unroll
    for (int qt = 0; qt < 2; ++qt)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        pb[2 * qt + s] = E::frag(sacc[qt], s);
        db[2 * qt + s] = E::frag(pacc[qt], s);
      }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int ro = 16 * ks * ROWB;
        const V8 fo = cat44<F16>(lds_tr_at(qb, L.tr[0][dt] + DOS + ro), lds_tr_at(qb, L.tr[1][dt] + DOS + ro));
        const V8 fq = cat44<F16>(lds_tr_at(qb, L.tr[0][dt] + QS + ro), lds_tr_at(qb, L.tr[1][dt] + QS + ro));
        dvacc[dt] = E::mfma(fo, pb[ks], dvacc[dt]);
        dkacc[dt] = E::mfma(fq, db[ks], dkacc[dt]);
      }
    __syncthreads();
  };
  for (int it = 0; it < total; it += 2) {
    tile(it, std::integral_constant<int, 0>{});
    if (it + 1 < total) tile(it + 1, std::integral_constant<int, 1>{});
  }

  if (key < Sk) {
    const float vs = (FEAT & F_DROP) ? drk.inv : 1.f;
    unsigned short* dkp = dk + b * a.skb + (long long)key * a.sks + hk * a.skh;
    unsigned short* dvp = dv + b * a.svb + (long long)key * a.svs + hk * a.svh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * hh;
        uint2 pk;
        pk.x = pack2<F16>(dkacc[dt][4 * g4 + 0] * a.scale, dkacc[dt][4 * g4 + 1] * a.scale);
        pk.y = pack2<F16>(dkacc[dt][4 * g4 + 2] * a.scale, dkacc[dt][4 * g4 + 3] * a.scale);
        *reinterpret_cast<uint2*>(dkp + d0) = pk;
        pk.x = pack2<F16>(dvacc[dt][4 * g4 + 0] * vs, dvacc[dt][4 * g4 + 1] * vs);
        pk.y = pack2<F16>(dvacc[dt][4 * g4 + 2] * vs, dvacc[dt][4 * g4 + 3] * vs);
        *reinterpret_cast<uint2*>(dvp + d0) = pk;
      }
  }
}

// ------------------------------------------------------------------------------------------
// Backward dQ: the forward's structure (query row on the lane).
// ------------------------------------------------------------------------------------------
template <int D, bool F16, bool CAUSAL, int FEAT>
__global__ __launch_bounds__(256, 2) void bwd_dq_kernel(FaArgs a) {
  typedef ET<F16> E;
  typedef typename E::V8 V8;
  constexpr int DP = D > 64 ? 128 : 64;
  constexpr int BM = 128, BN = 64;
  constexpr int KSTEPS = D / 16;
  constexpr int DT = D / 32;
  constexpr int ROWB = DP * 2;
  constexpr int TILE_B = BN * ROWB;
  // one LDS object per buffer (see fwd_kernel)
  __shared__ __attribute__((aligned(16))) char kv0[2 * TILE_B];
  __shared__ __attribute__((aligned(16))) char kv1[2 * TILE_B];

  const unsigned short* q = (const unsigned short*)a.q;
  const unsigned short* k = (const unsigned short*)a.k;
  const unsigned short* v = (const unsigned short*)a.v;
  const unsigned short* dout = (const unsigned short*)a.dout;
  unsigned short* dq = (unsigned short*)a.dq;
  const int B = a.B, SqMax = a.Sq, Hq = a.Hq, Hk = a.Hk;
  const long long rows = a.cu_q ? (long long)Hq * a.ltot : (long long)B * Hq * SqMax;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int nmb = (SqMax + BM - 1) / BM;
  const int HB = Hq * B;
  int mb = CAUSAL ? (nmb - 1 - (int)blockIdx.x / HB) : (int)blockIdx.x / HB;
  int hq = (int)blockIdx.x % Hq, b = ((int)blockIdx.x % HB) / Hq;
  if (a.map & 1) {  // grouped per (batch, head) on one XCD, heaviest query block first
    int grp, sub;
    if (!fa_map(nmb, HB, grp, sub)) return;
    mb = CAUSAL ? nmb - 1 - sub : sub;
    hq = grp % Hq;
    b = grp / Hq;
  }
  const int hk = hq / (Hq / Hk);
  const int m0 = mb * BM;
  int Sq = SqMax, Sk = a.Sk;
  long long lbase = ((long long)b * Hq + hq) * SqMax;
  if (a.cu_q) {
    const int q0s = a.cu_q[b], k0s = a.cu_k[b];
    Sq = a.cu_q[b + 1] - q0s;
    Sk = a.cu_k[b + 1] - k0s;
    if (m0 >= Sq) return;
    q += (long long)q0s * a.sqs;
    dq += (long long)q0s * a.sqs;
    dout += (long long)q0s * a.sos;
    k += (long long)k0s * a.sks;
    v += (long long)k0s * a.svs;
    lbase = (long long)hq * a.ltot + q0s;
  }
  const int qrow0 = m0 + w * 32;
  const int qpos = qrow0 + l32;
  const int coff = Sk - Sq;
  const float c = a.scale * kLog2e;

  const unsigned short* kbase = k + b * a.skb + hk * a.skh;
  const unsigned short* vbase = v + b * a.svb + hk * a.svh;
  const unsigned short* mrow = nullptr;
  if (FEAT & F_MASK)
    mrow = (const unsigned short*)a.mask + b * a.smb + hq * a.smh + (long long)min(qpos, Sq - 1) * a.smq;
  DropKey drk;
  if (FEAT & F_DROP) drk = drop_key(a.p_drop, a.seed, a.offset);
  const int sk_half = (a.Sk + 1) >> 1;

  V8 qf[KSTEPS], df[KSTEPS];
  float nlse, ndlt;  // −lse/scale, −δ of this lane's row
  {
    const long long qr = min(qpos, Sq - 1);
    const unsigned short* qp = q + b * a.sqb + qr * a.sqs + hq * a.sqh + 8 * hh;
    const unsigned short* dp = dout + b * a.sob + qr * a.sos + hq * a.soh + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) {
      qf[kk] = *reinterpret_cast<const V8*>(qp + 16 * kk);
      df[kk] = *reinterpret_cast<const V8*>(dp + 16 * kk);
    }
    const long long si = lbase + qr;
    ndlt = a.delta[si];
    nlse = a.delta[rows + si];
  }

  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, m0 + BM + coff);
  const int ntiles = n_end <= 0 ? 0 : (n_end + BN - 1) / BN;

  LaneOffs<ROWB, KSTEPS, DT> L;
  lane_offs(lane, L);

  f32x16 qacc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) qacc[i][j] = 0.f;

  auto issue = [&](int t, auto bufc) {
    char* ks = decltype(bufc)::value ? kv1 : kv0;
    glds_tile<BN, ROWB, D / 8>(kbase, a.sks, t * BN, Sk - 1, ks, w, lane);
    glds_tile<BN, ROWB, D / 8>(vbase, a.svs, t * BN, Sk - 1, ks + TILE_B, w, lane);
  };
  if (ntiles > 0) issue(0, std::integral_constant<int, 0>{});
  __syncthreads();

  const bool wave_rows_valid = qrow0 < Sq;
  // key (relative to the tile start n0, minus 4hh) valid for this lane's row iff < lim - n0
  const int m_lim = (CAUSAL ? qpos + coff + 1 : 0x40000000) - 4 * hh;
  auto tile = [&](int t, auto bufc) {
    constexpr int BUF = decltype(bufc)::value;
    constexpr int KS = 0, VS = TILE_B;
    const char* smem = BUF ? kv1 : kv0;
    if (t + 1 < ntiles) issue(t + 1, std::integral_constant<int, BUF ^ 1>{});
    const int n0 = t * BN;
    const bool active = wave_rows_valid && (!CAUSAL || n0 <= qrow0 + 31 + coff);
    if (active) {
      // opaque per-tile copies of the 3 base offsets: at two waves per SIMD hipcc would otherwise
      // hoist all 24 derived addresses out of the tile loop and spill
      LaneOffs<ROWB, KSTEPS, DT> Lt;
      Lt.row[0] = L.row[0];
      Lt.tr[0][0] = L.tr[0][0];
      Lt.tr[1][0] = L.tr[1][0];
      asm volatile("" : "+v"(Lt.row[0]), "+v"(Lt.tr[0][0]), "+v"(Lt.tr[1][0]));
      const bool need_mask = (n0 + BN > Sk) || (CAUSAL && n0 + BN - 1 > qrow0 + coff);
      const int lim = min(m_lim, Sk - 4 * hh) - n0;
      // the tile's 64 keys as two 32-key halves (S / dP accumulators of one half live at a time:
      // two waves per SIMD leave 256 registers)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        f32x16 sacc, pacc;
#pragma unroll
        for (int j = 0; j < 16; ++j) { sacc[j] = nlse; pacc[j] = (FEAT & F_DROP) ? 0.f : ndlt; }
#pragma unroll
        for (int kk = 0; kk < KSTEPS; ++kk) {
          sacc = E::mfma(lds_at<F16>(smem, row_x(Lt, kk) + KS + tt * 32 * ROWB), qf[kk], sacc);
          pacc = E::mfma(lds_at<F16>(smem, row_x(Lt, kk) + VS + tt * 32 * ROWB), df[kk], pacc);
        }
        auto finish = [&](auto maskc) {
          constexpr bool MASKED = decltype(maskc)::value;
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int key0 = n0 + tt * 32 + 8 * g4 + 4 * hh;
            f32x4 mb4 = {0.f, 0.f, 0.f, 0.f};
            if (FEAT & F_MASK) mb4 = mask4<F16>(mrow, key0, Sk);
            uint32_t h = 0, h2 = 0;
            if (FEAT & F_DROP) {
              h = drop_hash(drk, lbase + qpos, sk_half, key0);
              h2 = drop_hash(drk, lbase + qpos, sk_half, key0 + 2);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 4 * g4 + e;
              const int ck = tt * 32 + 8 * g4 + e;  // key - n0 - 4hh
              float p = fast_exp2(sacc[r] * c + mb4[e]);
              if (MASKED) p = ck < lim ? p : 0.f;
              float ds = pacc[r];
              if (FEAT & F_DROP) ds = (drop_keep(drk, e < 2 ? h : h2, key0 + e) ? ds * drk.inv : 0.f) + ndlt;
              pacc[r] = p * ds;
            }
          }
        };
        if (need_mask) finish(std::true_type{});
        else finish(std::false_type{});
        const V8 ds0 = E::frag(pacc, 0), ds1 = E::frag(pacc, 1);
        // dQᵀ += Kᵀ · dSᵀ over this half's 32 keys
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            const int ro = KS + 16 * (2 * tt + h2) * ROWB;
            qacc[dt] = E::mfma(cat44<F16>(lds_tr_at(smem, tr_x(Lt, 0, dt) + ro), lds_tr_at(smem, tr_x(Lt, 1, dt) + ro)),
                               h2 ? ds1 : ds0, qacc[dt]);
          }
      }
    }
    __syncthreads();
  };
  for (int t = 0; t < ntiles; t += 2) {
    tile(t, std::integral_constant<int, 0>{});
    if (t + 1 < ntiles) tile(t + 1, std::integral_constant<int, 1>{});
  }

  if (qpos < Sq) {
    unsigned short* qp = dq + b * a.sqb + (long long)qpos * a.sqs + hq * a.sqh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * hh;
        uint2 pk;
        pk.x = pack2<F16>(qacc[dt][4 * g4 + 0] * a.scale, qacc[dt][4 * g4 + 1] * a.scale);
        pk.y = pack2<F16>(qacc[dt][4 * g4 + 2] * a.scale, qacc[dt][4 * g4 + 3] * a.scale);
        *reinterpret_cast<uint2*>(qp + d0) = pk;
      }
  }
}


// ------------------------------------------------------------------------------------------
// Launchers (one per element type; the exported entry points in flash_attn.hip dispatch).
// ------------------------------------------------------------------------------------------
// forward waves per workgroup: PIAMD_FA_FWD_WAVES (4 or 8), read once
inline int fwd_waves() {
  static const int nw = [] {
    const char* e = getenv("PIAMD_FA_FWD_WAVES");
    return (e && atoi(e) == 8) ? 8 : 4;
  }();
  return nw;
}

template <bool F16, int D, bool C, int NW>
int launch_fwd_nw(const FaArgs& a, hipStream_t st) {
  const dim3 grid = fa_grid((long long)((a.Sq + 32 * NW - 1) / (32 * NW)) * a.Hq * a.B);
  const dim3 blk(64 * NW);
  const int feat = (a.p_drop > 0.f ? F_DROP : 0) | (a.mask ? F_MASK : 0);
  switch (feat) {
    case 0: hipLaunchKernelGGL((fwd_kernel<D, F16, C, 0, NW>), grid, blk, 0, st, a); break;
    case 1: hipLaunchKernelGGL((fwd_kernel<D, F16, C, 1, NW>), grid, blk, 0, st, a); break;
    case 2: hipLaunchKernelGGL((fwd_kernel<D, F16, C, 2, NW>), grid, blk, 0, st, a); break;
    default: hipLaunchKernelGGL((fwd_kernel<D, F16, C, 3, NW>), grid, blk, 0, st, a); break;
  }
  return (int)hipGetLastError();
}

// persistent forward: PIAMD_FA_PERSIST (1 = on, default; 0 = the one-item-per-workgroup grid)
inline bool fwd_persist() {
  static const bool on = [] {
    const char* e = getenv("PIAMD_FA_PERSIST");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <bool F16, int D, bool C>
int launch_fwd_persist(const FaArgs& a, hipStream_t st) {
  const long long items = (long long)((a.Sq + 127) / 128) * a.Hq * a.B;
  // 2 resident workgroups per CU on 256 CUs; a multiple of 8 (one worker list per XCD)
  const unsigned grid = (unsigned)std::min<long long>(512, (items + 7) / 8 * 8);
  const int feat = (a.p_drop > 0.f ? F_DROP : 0) | (a.mask ? F_MASK : 0);
  switch (feat) {
    case 0: hipLaunchKernelGGL((fwd_persist_kernel<D, F16, C, 0>), dim3(grid), dim3(256), 0, st, a); break;
    case 1: hipLaunchKernelGGL((fwd_persist_kernel<D, F16, C, 1>), dim3(grid), dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((fwd_persist_kernel<D, F16, C, 2>), dim3(grid), dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((fwd_persist_kernel<D, F16, C, 3>), dim3(grid), dim3(256), 0, st, a); break;
  }
  return (int)hipGetLastError();
}

template <bool F16, int D, bool C>
int launch_fwd_feat(const FaArgs& a, dim3 /*grid*/, hipStream_t st) {
  if constexpr (D > 128) return launch_fwd_nw<F16, D, C, 4>(a, st);
  else {
    if (!a.cu_q && fwd_persist() && fwd_waves() == 4) return launch_fwd_persist<F16, D, C>(a, st);
    return fwd_waves() == 8 ? launch_fwd_nw<F16, D, C, 8>(a, st) : launch_fwd_nw<F16, D, C, 4>(a, st);
  }
}

template <bool F16>
int launch_fwd(const FaArgs& a, hipStream_t st) {
  const dim3 grid(1);
#define FWD_D(DD) return a.causal ? launch_fwd_feat<F16, DD, true>(a, grid, st) \
                                  : launch_fwd_feat<F16, DD, false>(a, grid, st)
  switch (a.D) {
    case 64: FWD_D(64);
    case 96: FWD_D(96);
    case 128: FWD_D(128);
    case 256: FWD_D(256);
    default: return (int)hipErrorInvalidValue;
  }
#undef FWD_D
}

template <bool F16, int D, bool C>
int launch_bwd_feat(const FaArgs& a, dim3 gkv, dim3 gq, hipStream_t st) {
  const int feat = (a.p_drop > 0.f ? F_DROP : 0) | (a.mask ? F_MASK : 0);
#define BWD_F(FF)                                                                              \
  if (!(FF == 0 && D == 128 && !F16 && fa_dkdv_asm(a, st) == 1))                               \
    hipLaunchKernelGGL((bwd_dkdv_kernel<D, F16, C, FF>), gkv, dim3(256), 0, st, a);            \
  if (!(FF == 0 && D == 128 && !F16 && fa_dq_asm(a, st) == 1))                                 \
    hipLaunchKernelGGL((bwd_dq_kernel<D, F16, C, FF>), gq, dim3(256), 0, st, a);               \
  break;
  switch (feat) {
    case 0: BWD_F(0)
    case 1: BWD_F(1)
    case 2: BWD_F(2)
    default: BWD_F(3)
  }
#undef BWD_F
  return (int)hipGetLastError();
}

// backward grid order (FaArgs::map). Measured at B96 S1024 H16 D128 causal: grouping the dQ
// grid saves 7 % (954 -> 886 us) when the grid is large; at small grids (B8 S2048, 2k workgroups)
// it loses 12 % to the tail, and grouping the dK/dV grid loses at both (profiles/fa_bwd_experiments_r3.txt).
// PIAMD_FA_BWD_MAP=<bits> overrides.
inline int fa_bwd_map(const FaArgs& a) {
  static const int env = [] {
    const char* e = getenv("PIAMD_FA_BWD_MAP");
    return e ? atoi(e) : -1;
  }();
  if (env >= 0) return env;
  const long long nq = (long long)((a.Sq + 127) / 128) * a.Hq * a.B;
  return nq >= 8192 ? 1 : 0;
}

template <bool F16>
int launch_bwd(const FaArgs& a, hipStream_t st) {
  // delta rows: padded [B, Hq, Sq]; packed [Hq, ltot] == the padded layout with B = 1, Sq = ltot
  const int pB = a.cu_q ? 1 : a.B, pS = a.cu_q ? a.ltot : a.Sq;
  const int total = pB * a.Hq * pS;
  const int tpr = a.D > 64 ? 16 : 8;
  const int pre_blocks = (int)(((long long)total * tpr + 255) / 256);
  const long long nkv = (long long)((a.Sk + 127) / 128) * a.Hk * a.B, nq = (long long)((a.Sq + 127) / 128) * a.Hq * a.B;
  const dim3 gkv = (a.map & 2) ? fa_grid(nkv) : dim3((unsigned)nkv), gq = (a.map & 1) ? fa_grid(nq) : dim3((unsigned)nq);
#define BWD_D(DD)                                                                                  \
  hipLaunchKernelGGL((bwd_pre_kernel<DD, F16>), dim3(pre_blocks), dim3(256), 0, st,              \
                     (const unsigned short*)a.o, (const unsigned short*)a.dout, a.lse, a.delta,  \
                     1.f / a.scale, pS, a.Hq, a.sob, a.sos, a.soh, total);                        \
  return a.causal ? launch_bwd_feat<F16, DD, true>(a, gkv, gq, st)                               \
                  : launch_bwd_feat<F16, DD, false>(a, gkv, gq, st)
  switch (a.D) {
    case 64: BWD_D(64);
    case 96: BWD_D(96);
    case 128: BWD_D(128);
    default: return (int)hipErrorInvalidValue;
  }
#undef BWD_D
}

}  // namespace fa
