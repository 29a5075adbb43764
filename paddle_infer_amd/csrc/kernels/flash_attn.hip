// Flash attention forward / backward on CDNA4 MFMA (bf16 in, f32 accumulate).
//
// Parity: reference `python/paddle/nn/functional/flash_attention.py` (flash_attention,
// scaled_dot_product_attention, flash_attn_unpadded), `paddle/phi/kernels/gpu/flash_attn_kernel.cu`,
// and the fork's CUTLASS `phi/kernels/fusion/cutlass/memory_efficient_attention*.cu`
// (memory_efficient_attention fwd/bwd, LSE output, causal mask, GQA via kv-head grouping).
//
// MI355X design (cdna_hip_programming.md §3, T2, T10, T12, App. B "Fused attention prefill",
// "Attention backward"):
//   * Layout [B, S, H, D] with free b/s/h strides, so Q/K/V are consumed straight out of the fused
//     QKV projection output and dQ/dK/dV are written straight into the fused dQKV gradient — no
//     transposes around the kernel.
//   * Forward: workgroup = 4 waves = 128 query rows (32 per wave), K/V tiles of 64 keys,
//     register-staged double buffer in LDS (next tile's global loads issued before the current
//     tile's MFMAs, written to LDS after them: T14). SWAPPED products with
//     v_mfma_f32_32x32x16_bf16: Sᵀ = K·Qᵀ puts one query row per lane, so the online-softmax row
//     max/sum is 31 in-lane ops + one cross-half shuffle, and the Sᵀ accumulator is directly the B
//     operand of Oᵀ = Vᵀ·Pᵀ (no LDS round trip for P). Vᵀ fragments come from the row-major V
//     image with ds_read_b64_tr_b16 (hardware transpose). LDS images use the dual-use XOR
//     layout (row reads and transposed reads both conflict-free at D = 128).
//   * Backward = two atomic-free kernels. dK/dV: workgroup = 4 waves = 128 keys (32 per wave, key
//     on the MFMA lane), dKᵀ/dVᵀ kept in accumulators across the whole sweep over query tiles and
//     over the q-heads of a GQA group, so dK/dV need no cross-workgroup sum. dQ: the forward's
//     structure (query row on the lane): Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ, and the dSᵀ accumulator feeds
//     dQᵀ = Kᵀ·dSᵀ straight from registers (Kᵀ via transposed LDS reads). Recomputing S/dP in the dQ
//     kernel costs 2 extra MFMA products but removes the f32 dQ atomics, whose chip-wide rate
//     (≈1.3 TB/s) would floor the backward, and keeps the result bitwise deterministic.
//   * Every global load is unconditional (row indices clamped, out-of-range rows masked in the
//     softmax), so hipcc can count `vmcnt` and the K/V prefetch stays in flight under the MFMAs.
//   * Causal grids are flattened and launched heaviest-first (LPT order across all heads).
#include "common.h"

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// Dual-use LDS image (guide T10 layout (b)): byte offset of 16-B chunk `ch` of row `row` in an
// image with ROWB-byte rows.
template <int ROWB>
__device__ __forceinline__ int lds_off(int row, int ch) {
  constexpr int CH = ROWB / 16;
  const int x = (((row & 3) << 2) | ((row >> 2) & 3)) & (CH - 1);
  return row * ROWB + ((ch ^ x) << 4);
}

__device__ __forceinline__ bf16x8 lds_row8(const char* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}

// Transposed read: 16-lane group reads a 4-row x 16-col block starting at (r0, c0 elems); lane i
// of the group receives column c0+i of rows r0..r0+3.
template <int ROWB>
__device__ __forceinline__ s16x4_t lds_tr4(const char* base, int r0, int c0, int gi) {
  const int q = gi >> 2, p = gi & 3;
  const int col = c0 + 4 * p;
  const int off = lds_off<ROWB>(r0 + q, col >> 3) + ((col & 7) << 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off));
}

__device__ __forceinline__ bf16x8 cat44(s16x4_t a, s16x4_t b) {
  s16x8 t = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, t);
}

__device__ __forceinline__ bf16x8 zero_bf16x8() {
  s16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  return __builtin_bit_cast(bf16x8, z);
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 pack_frag(const f32x16& acc, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)acc[8 * s + j];
  return r;
}


__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Direct-to-LDS DMA (global_load_lds_dwordx4) of a [ROWS][ROWB] bf16 tile into the dual-use
// XOR image. The LDS destination of one wave-instruction is lane-linear (1 KiB), so the swizzle is
// applied to the per-lane SOURCE address (guide §5.4 rule 21): physical chunk pc of row r holds
// logical chunk pc ^ x(r). Rows past `rmax` are clamped (masked later). Each of the 4 waves issues
// ROWS*ROWB/4096 pieces.
template <int ROWS, int ROWB>
__device__ __forceinline__ void glds_tile(const bf16_t* gbase, long long rstride, int row0, int rmax,
                                          char* tile, int w, int lane) {
  constexpr int CH = ROWB / 16;
  constexpr int PIECES = ROWS * CH / 64;
  constexpr int PPW = PIECES / 4;
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int P = w * PPW + i;
    const int L = P * 64 + lane, r = L / CH, pc = L % CH;
    const int x = (((r & 3) << 2) | ((r >> 2) & 3)) & (CH - 1);
    const long long row = min(row0 + r, rmax);
    const bf16_t* src = gbase + row * rstride + ((pc ^ x) << 3);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(tile + P * 1024),
                                     16, 0, 0);
  }
}

// ------------------------------------------------------------------------------------------
// Forward
// ------------------------------------------------------------------------------------------
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    bf16_t* __restrict__ o, float* __restrict__ lse, int B, int SqMax, int SkMax, int Hq, int Hk,
    long long sqb, long long sqs, long long sqh, long long skb, long long sks, long long skh,
    long long svb, long long svs, long long svh, long long sob, long long sos, long long soh,
    float scale, const int* __restrict__ cu_q, const int* __restrict__ cu_k, int ltot) {
  constexpr int BM = 128, BN = 64;
  constexpr int KSTEPS = D / 16;
  constexpr int DT = D / 32;
  constexpr int CH = D / 8;          // 16-B chunks per row
  constexpr int ROWB = D * 2;
  constexpr int TILE_B = BN * ROWB;  // bytes per K or V tile
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_B];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5, gi = lane & 15, g = lane >> 4;
  const int nmb = (SqMax + BM - 1) / BM;
  const int HB = Hq * B;
  const int mb = CAUSAL ? (nmb - 1 - (int)blockIdx.x / HB) : (int)blockIdx.x / HB;
  const int hq = (int)blockIdx.x % Hq, b = ((int)blockIdx.x % HB) / Hq;
  const int hk = hq / (Hq / Hk);
  const int m0 = mb * BM;
  int Sq = SqMax, Sk = SkMax;
  long long lbase = ((long long)b * Hq + hq) * SqMax;
  if (cu_q) {  // variable-length: b = sequence, rows [cu[b], cu[b+1]) of the packed tensors
    const int q0s = cu_q[b], k0s = cu_k[b];
    Sq = cu_q[b + 1] - q0s;
    Sk = cu_k[b + 1] - k0s;
    if (m0 >= Sq) return;  // block-uniform: this sequence is shorter than the longest
    q += (long long)q0s * sqs;
    o += (long long)q0s * sos;
    k += (long long)k0s * sks;
    v += (long long)k0s * svs;
    lbase = (long long)hq * ltot + q0s;
  }
  const int qrow0 = m0 + w * 32;
  const int coff = Sk - Sq;  // bottom-right aligned causal offset
  const float c = scale * kLog2e;

  const bf16_t* kbase = k + b * skb + hk * skh;
  const bf16_t* vbase = v + b * svb + hk * svh;

  bf16x8 qf[KSTEPS];
  {
    const int qr = min(qrow0 + l32, Sq - 1);
    const bf16_t* qp = q + b * sqb + (long long)qr * sqs + hq * sqh + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(qp + 16 * kk);
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

  auto issue = [&](int t, int buf) {
    char* ks = smem + buf * 2 * TILE_B;
    glds_tile<BN, ROWB>(kbase, sks, t * BN, Sk - 1, ks, w, lane);
    glds_tile<BN, ROWB>(vbase, svs, t * BN, Sk - 1, ks + TILE_B, w, lane);
  };
  if (ntiles > 0) issue(0, 0);
  __syncthreads();

  const bool wave_rows_valid = qrow0 < Sq;
  const int qpos = qrow0 + l32;
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) issue(t + 1, buf ^ 1);
    const int n0 = t * BN;
    const bool active = wave_rows_valid && (!CAUSAL || n0 <= qrow0 + 31 + coff);
    if (active) {
      const char* ks = smem + buf * 2 * TILE_B;
      const char* vs = ks + TILE_B;
      f32x16 sacc[2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int j = 0; j < 16; ++j) sacc[tt][j] = 0.f;
#pragma unroll
      for (int kk = 0; kk < KSTEPS; ++kk) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          bf16x8 a = lds_row8(ks, lds_off<ROWB>(tt * 32 + l32, 2 * kk + hh));
          sacc[tt] = mfma32(a, qf[kk], sacc[tt]);
        }
      }
      const bool need_mask = (n0 + BN > Sk) || (CAUSAL && n0 + BN - 1 > qrow0 + coff);
      float mx = -INFINITY;
      if (need_mask) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = n0 + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const bool ok = (key < Sk) & (!CAUSAL | (key <= qpos + coff));
            const float x = ok ? sacc[tt][r] * c : -INFINITY;
            sacc[tt][r] = x;
            mx = fmaxf(mx, x);
          }
      } else {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float x = sacc[tt][r] * c;
            sacc[tt][r] = x;
            mx = fmaxf(mx, x);
          }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_i, mx);
      const float msub = m_new == -INFINITY ? 0.f : m_new;
      float rs = 0.f;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(sacc[tt][r] - msub);
          sacc[tt][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 32, 64);
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
      bf16x8 pf[4];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int s = 0; s < 2; ++s) pf[2 * tt + s] = pack_frag(sacc[tt], s);
      // Oᵀ += Vᵀ · Pᵀ
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int c0 = 32 * dt + 16 * (g & 1);
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) {
          const int r0 = 16 * ks4 + 4 * hh;
          s16x4_t lo = lds_tr4<ROWB>(vs, r0, c0, gi);
          s16x4_t hi = lds_tr4<ROWB>(vs, r0 + 8, c0, gi);
          oacc[dt] = mfma32(cat44(lo, hi), pf[ks4], oacc[dt]);
        }
      }
    }
    __syncthreads();
  }

  // epilogue: lane = query row, registers = d
  if (qpos < Sq) {
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    bf16_t* op = o + b * sob + (long long)qpos * sos + hq * soh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * hh;
        uint2 pk;
        pk.x = pack_bf16x2(oacc[dt][4 * g4 + 0] * inv, oacc[dt][4 * g4 + 1] * inv);
        pk.y = pack_bf16x2(oacc[dt][4 * g4 + 2] * inv, oacc[dt][4 * g4 + 3] * inv);
        *reinterpret_cast<uint2*>(op + d0) = pk;
      }
    if (hh == 0 && lse)
      lse[lbase + qpos] = l_i > 0.f ? (m_i + log2f(l_i)) * kLn2 : INFINITY;
  }
}

// ------------------------------------------------------------------------------------------
// Backward pre-pass: delta[b, h, q] = Σ_d dO·O (f32). 16 B per lane, D/8 lanes per row.
// ------------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void fa_bwd_pre_kernel(
    const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout, float* __restrict__ delta,
    int Sq, int Hq, long long sob, long long sos, long long soh, int total) {
  constexpr int TPR = D / 8;  // threads per row
  const int row = (blockIdx.x * 256 + threadIdx.x) / TPR, sub = threadIdx.x % TPR;
  const bool ok = row < total;
  const int rr = ok ? row : 0;
  const int qr = rr % Sq, hq = (rr / Sq) % Hq, b = rr / (Sq * Hq);
  const long long off = b * sob + (long long)qr * sos + hq * soh + sub * 8;
  u16x8 a = *reinterpret_cast<const u16x8*>(o + off);
  u16x8 d = *reinterpret_cast<const u16x8*>(dout + off);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += bf2f(a[j]) * bf2f(d[j]);
#pragma unroll
  for (int x = TPR / 2; x > 0; x >>= 1) s += __shfl_xor(s, x, 64);
  if (ok && sub == 0) delta[((long long)b * Hq + hq) * Sq + qr] = s;
}

// ------------------------------------------------------------------------------------------
// Backward dK/dV: workgroup = 128 keys of one (batch, kv-head); sweeps the q-heads of the GQA
// group and all query tiles of 64 rows. Key on the MFMA lane.
// ------------------------------------------------------------------------------------------
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dk, bf16_t* __restrict__ dv, int B,
    int SqMax, int SkMax, int Hq, int Hk, long long sqb, long long sqs, long long sqh, long long skb,
    long long sks, long long skh, long long svb, long long svs, long long svh, long long sdob,
    long long sdos, long long sdoh, float scale, const int* __restrict__ cu_q,
    const int* __restrict__ cu_k, int ltot) {
  constexpr int BK = 128, BQ = 64;
  constexpr int KSTEPS = D / 16;
  constexpr int DT = D / 32;
  constexpr int CH = D / 8;
  constexpr int ROWB = D * 2;
  constexpr int QTILE_B = BQ * ROWB;    // Q or dO tile [64][D]
  constexpr int KIMG_B = BK * ROWB;     // resident K and V images of the block's 128 keys
  constexpr int OFF_K = 2 * 2 * QTILE_B;
  constexpr int OFF_V = OFF_K + KIMG_B;
  constexpr int OFF_STAT = OFF_V + KIMG_B;  // 2 buffers x (lse, delta) x 64 f32
  constexpr int SMEM = OFF_STAT + 2 * 2 * BQ * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5, gi = lane & 15, g = lane >> 4;
  const int HB = Hk * B;
  const int kb = (int)blockIdx.x / HB;  // causal: low key blocks see the most queries -> first
  const int hk = (int)blockIdx.x % Hk, b = ((int)blockIdx.x % HB) / Hk;
  const int n0 = kb * BK;
  int Sq = SqMax, Sk = SkMax;
  long long lrow = (long long)b * Hq * SqMax, lhead = SqMax;  // stats index = lrow + hq*lhead + q
  if (cu_q) {
    const int q0s = cu_q[b], k0s = cu_k[b];
    Sq = cu_q[b + 1] - q0s;
    Sk = cu_k[b + 1] - k0s;
    if (n0 >= Sk) return;
    q += (long long)q0s * sqs;
    dout += (long long)q0s * sdos;
    k += (long long)k0s * sks;
    v += (long long)k0s * svs;
    dk += (long long)k0s * sks;
    dv += (long long)k0s * svs;
    lrow = q0s;
    lhead = ltot;
  }
  const int kw0 = n0 + 32 * w;  // this wave's first key
  const int key = kw0 + l32;
  const int coff = Sk - Sq;
  const int group = Hq / Hk;
  const float c = scale * kLog2e;

  // K / V of the block's keys stay resident in LDS (B operands of S and dP are row reads)
  glds_tile<BK, ROWB>(k + b * skb + hk * skh, sks, n0, Sk - 1, smem + OFF_K, w, lane);
  glds_tile<BK, ROWB>(v + b * svb + hk * svh, svs, n0, Sk - 1, smem + OFF_V, w, lane);
  const char* kimg = smem + OFF_K;
  const char* vimg = smem + OFF_V;

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

  auto issue = [&](int it, int buf) {
    const int hq = hk * group + it / tiles_per_head;
    const int q0 = (qt0 + it % tiles_per_head) * BQ;
    char* qs = smem + buf * 2 * QTILE_B;
    glds_tile<BQ, ROWB>(q + b * sqb + hq * sqh, sqs, q0, Sq - 1, qs, w, lane);
    glds_tile<BQ, ROWB>(dout + b * sdob + hq * sdoh, sdos, q0, Sq - 1, qs + QTILE_B, w, lane);
    if (w < 2) {  // wave 0: lse row, wave 1: delta row (64 f32 = one 4-B/lane DMA)
      const float* s = (w == 0 ? lse : delta) + lrow + hq * lhead + min(q0 + lane, Sq - 1);
      char* st = smem + OFF_STAT + (buf * 2 + w) * BQ * 4;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)s,
                                       (__attribute__((address_space(3))) void*)st, 4, 0, 0);
    }
  };
  if (total > 0) issue(0, 0);
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int buf = it & 1;
    const int q0 = (qt0 + it % tiles_per_head) * BQ;
    if (it + 1 < total) issue(it + 1, buf ^ 1);
    const char* qs = smem + buf * 2 * QTILE_B;
    const char* dos = qs + QTILE_B;
    const float* lst = reinterpret_cast<const float*>(smem + OFF_STAT) + buf * 2 * BQ;
    const float* dst = lst + BQ;
    // Re-derive every lane-dependent LDS address inside the iteration (an opaque copy of the lane
    // id): otherwise hipcc hoists ~60 loop-invariant swizzled addresses into VGPRs and evicts the
    // accumulators to AGPRs with per-iteration copies.
    int lx = lane;
    asm volatile("" : "+v"(lx));
    const int l32 = lx & 31, hh = lx >> 5, gi = lx & 15, g = lx >> 4;
    // no per-wave skip: a wave whose keys are all above this tile's diagonal computes a fully
    // masked tile (only the first q tile of a block); a branch here would make hipcc shuttle the
    // 128 loop-carried dK/dV accumulators between AGPRs and VGPRs every iteration.
    {
      f32x16 sacc[2], pacc[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int j = 0; j < 16; ++j) { sacc[qt][j] = 0.f; pacc[qt][j] = 0.f; }
      // S = Q·Kᵀ, dP = dO·Vᵀ with the next k-step's 6 fragments loaded one step ahead
      bf16x8 fr[2][6];
      auto ld = [&](int kk, bf16x8* f) {
        const int koff = lds_off<ROWB>(32 * w + l32, 2 * kk + hh);
        f[0] = lds_row8(kimg, koff);
        f[1] = lds_row8(vimg, koff);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const int qoff = lds_off<ROWB>(qt * 32 + l32, 2 * kk + hh);
          f[2 + qt] = lds_row8(qs, qoff);
          f[4 + qt] = lds_row8(dos, qoff);
        }
      };
      ld(0, fr[0]);
#pragma unroll
      for (int kk = 0; kk < KSTEPS; ++kk) {
        if (kk + 1 < KSTEPS) ld(kk + 1, fr[(kk + 1) & 1]);
        const bf16x8* f = fr[kk & 1];
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          sacc[qt] = mfma32(f[2 + qt], f[0], sacc[qt]);
          pacc[qt] = mfma32(f[4 + qt], f[1], pacc[qt]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_sched_barrier(0);
      const bool need_mask = (kw0 + 31 >= Sk) || (q0 + BQ > Sq) ||
                             (CAUSAL && kw0 + 31 > q0 + coff);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int qi0 = qt * 32 + 8 * g4 + 4 * hh;
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(lst + qi0);
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(dst + qi0);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * g4 + e;
            float p = fast_exp2(sacc[qt][r] * c - l4[e] * kLog2e);
            if (need_mask) {
              const int qr = q0 + qi0 + e;
              const bool ok = (key < Sk) & (qr < Sq) & (!CAUSAL | (key <= qr + coff));
              p = ok ? p : 0.f;
            }
            sacc[qt][r] = p;
            pacc[qt][r] = p * (pacc[qt][r] - d4[e]);
          }
        }
      // dVᵀ += dOᵀ·P ; dKᵀ += Qᵀ·dS   (A operands via transposed reads of the dO / Q images)
      bf16x8 pb[4], db[4];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          pb[2 * qt + s] = pack_frag(sacc[qt], s);
          db[2 * qt + s] = pack_frag(pacc[qt], s);
        }
      __builtin_amdgcn_sched_barrier(0);
      // dVᵀ += dOᵀ·P ; dKᵀ += Qᵀ·dS, transposed-read fragments one (dt, half) step ahead
      bf16x8 tf[2][4];
      auto ldt = [&](int st, bf16x8* f) {  // st = 2*dt + half: ks in {2*half, 2*half+1}
        const int c0 = 32 * (st >> 1) + 16 * (g & 1);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int r0 = 16 * (2 * (st & 1) + j) + 4 * hh;
          f[2 * j] = cat44(lds_tr4<ROWB>(dos, r0, c0, gi), lds_tr4<ROWB>(dos, r0 + 8, c0, gi));
          f[2 * j + 1] = cat44(lds_tr4<ROWB>(qs, r0, c0, gi), lds_tr4<ROWB>(qs, r0 + 8, c0, gi));
        }
      };
      ldt(0, tf[0]);
#pragma unroll
      for (int st = 0; st < 2 * DT; ++st) {
        if (st + 1 < 2 * DT) ldt(st + 1, tf[(st + 1) & 1]);
        const bf16x8* f = tf[st & 1];
        const int dt = st >> 1;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int ks = 2 * (st & 1) + j;
          dvacc[dt] = mfma32(f[2 * j], pb[ks], dvacc[dt]);
          dkacc[dt] = mfma32(f[2 * j + 1], db[ks], dkacc[dt]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();
  }

  if (key < Sk) {
    bf16_t* dkp = dk + b * skb + (long long)key * sks + hk * skh;
    bf16_t* dvp = dv + b * svb + (long long)key * svs + hk * svh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * hh;
        uint2 pk;
        pk.x = pack_bf16x2(dkacc[dt][4 * g4 + 0] * scale, dkacc[dt][4 * g4 + 1] * scale);
        pk.y = pack_bf16x2(dkacc[dt][4 * g4 + 2] * scale, dkacc[dt][4 * g4 + 3] * scale);
        *reinterpret_cast<uint2*>(dkp + d0) = pk;
        pk.x = pack_bf16x2(dvacc[dt][4 * g4 + 0], dvacc[dt][4 * g4 + 1]);
        pk.y = pack_bf16x2(dvacc[dt][4 * g4 + 2], dvacc[dt][4 * g4 + 3]);
        *reinterpret_cast<uint2*>(dvp + d0) = pk;
      }
  }
}

// ------------------------------------------------------------------------------------------
// Backward dQ: the forward's structure (query row on the lane).
// ------------------------------------------------------------------------------------------
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void fa_bwd_dq_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dq, int B, int SqMax, int SkMax, int Hq,
    int Hk, long long sqb, long long sqs, long long sqh, long long skb, long long sks,
    long long skh, long long svb, long long svs, long long svh, long long sdob, long long sdos,
    long long sdoh, float scale, const int* __restrict__ cu_q, const int* __restrict__ cu_k,
    int ltot) {
  constexpr int BM = 128, BN = 64;
  constexpr int KSTEPS = D / 16;
  constexpr int DT = D / 32;
  constexpr int CH = D / 8;
  constexpr int ROWB = D * 2;
  constexpr int TILE_B = BN * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_B];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5, gi = lane & 15, g = lane >> 4;
  const int nmb = (SqMax + BM - 1) / BM;
  const int HB = Hq * B;
  const int mb = CAUSAL ? (nmb - 1 - (int)blockIdx.x / HB) : (int)blockIdx.x / HB;
  const int hq = (int)blockIdx.x % Hq, b = ((int)blockIdx.x % HB) / Hq;
  const int hk = hq / (Hq / Hk);
  const int m0 = mb * BM;
  int Sq = SqMax, Sk = SkMax;
  long long lbase = ((long long)b * Hq + hq) * SqMax;
  if (cu_q) {
    const int q0s = cu_q[b], k0s = cu_k[b];
    Sq = cu_q[b + 1] - q0s;
    Sk = cu_k[b + 1] - k0s;
    if (m0 >= Sq) return;
    q += (long long)q0s * sqs;
    dq += (long long)q0s * sqs;
    dout += (long long)q0s * sdos;
    k += (long long)k0s * sks;
    v += (long long)k0s * svs;
    lbase = (long long)hq * ltot + q0s;
  }
  const int qrow0 = m0 + w * 32;
  const int qpos = qrow0 + l32;
  const int coff = Sk - Sq;
  const float c = scale * kLog2e;

  const bf16_t* kbase = k + b * skb + hk * skh;
  const bf16_t* vbase = v + b * svb + hk * svh;

  bf16x8 qf[KSTEPS], df[KSTEPS];
  float lse2, dlt;
  {
    const long long qr = min(qpos, Sq - 1);
    const bf16_t* qp = q + b * sqb + qr * sqs + hq * sqh + 8 * hh;
    const bf16_t* dp = dout + b * sdob + qr * sdos + hq * sdoh + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) {
      qf[kk] = *reinterpret_cast<const bf16x8*>(qp + 16 * kk);
      df[kk] = *reinterpret_cast<const bf16x8*>(dp + 16 * kk);
    }
    const long long si = lbase + qr;
    lse2 = lse[si] * kLog2e;
    dlt = delta[si];
  }

  int n_end = Sk;
  if (CAUSAL) n_end = min(Sk, m0 + BM + coff);
  const int ntiles = n_end <= 0 ? 0 : (n_end + BN - 1) / BN;

  f32x16 qacc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) qacc[i][j] = 0.f;

  auto issue = [&](int t, int buf) {
    char* ks = smem + buf * 2 * TILE_B;
    glds_tile<BN, ROWB>(kbase, sks, t * BN, Sk - 1, ks, w, lane);
    glds_tile<BN, ROWB>(vbase, svs, t * BN, Sk - 1, ks + TILE_B, w, lane);
  };
  if (ntiles > 0) issue(0, 0);
  __syncthreads();

  const bool wave_rows_valid = qrow0 < Sq;
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) issue(t + 1, buf ^ 1);
    const int n0 = t * BN;
    const bool active = wave_rows_valid && (!CAUSAL || n0 <= qrow0 + 31 + coff);
    if (active) {
      const char* ks = smem + buf * 2 * TILE_B;
      const char* vs = ks + TILE_B;
      f32x16 sacc[2], pacc[2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int j = 0; j < 16; ++j) { sacc[tt][j] = 0.f; pacc[tt][j] = 0.f; }
#pragma unroll
      for (int kk = 0; kk < KSTEPS; ++kk) {
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int off = lds_off<ROWB>(tt * 32 + l32, 2 * kk + hh);
          sacc[tt] = mfma32(lds_row8(ks, off), qf[kk], sacc[tt]);
          pacc[tt] = mfma32(lds_row8(vs, off), df[kk], pacc[tt]);
        }
      }
      const bool need_mask = (n0 + BN > Sk) || (CAUSAL && n0 + BN - 1 > qrow0 + coff);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = fast_exp2(sacc[tt][r] * c - lse2);
          if (need_mask) {
            const int key = n0 + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const bool ok = (key < Sk) & (!CAUSAL | (key <= qpos + coff));
            p = ok ? p : 0.f;
          }
          pacc[tt][r] = p * (pacc[tt][r] - dlt);
        }
      bf16x8 dsf[4];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int s = 0; s < 2; ++s) dsf[2 * tt + s] = pack_frag(pacc[tt], s);
      // dQᵀ += Kᵀ · dSᵀ
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int c0 = 32 * dt + 16 * (g & 1);
#pragma unroll
        for (int ks4 = 0; ks4 < 4; ++ks4) {
          const int r0 = 16 * ks4 + 4 * hh;
          s16x4_t lo = lds_tr4<ROWB>(ks, r0, c0, gi);
          s16x4_t hi = lds_tr4<ROWB>(ks, r0 + 8, c0, gi);
          qacc[dt] = mfma32(cat44(lo, hi), dsf[ks4], qacc[dt]);
        }
      }
    }
    __syncthreads();
  }

  if (qpos < Sq) {
    bf16_t* qp = dq + b * sqb + (long long)qpos * sqs + hq * sqh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * hh;
        uint2 pk;
        pk.x = pack_bf16x2(qacc[dt][4 * g4 + 0] * scale, qacc[dt][4 * g4 + 1] * scale);
        pk.y = pack_bf16x2(qacc[dt][4 * g4 + 2] * scale, qacc[dt][4 * g4 + 3] * scale);
        *reinterpret_cast<uint2*>(qp + d0) = pk;
      }
  }
}

}  // namespace

PIAMD_EXPORT int piamd_flash_attn_varlen_fwd(const void*, const void*, const void*, void*, float*,
                                             int, int, int, int, int, int, long long, long long,
                                             long long, long long, long long, long long, long long,
                                             long long, long long, long long, long long, long long,
                                             float, int, const int*, const int*, int, hipStream_t);
PIAMD_EXPORT int piamd_flash_attn_varlen_bwd(const void*, const void*, const void*, const void*,
                                             const void*, const float*, float*, void*, void*, void*,
                                             int, int, int, int, int, int, long long, long long,
                                             long long, long long, long long, long long, long long,
                                             long long, long long, long long, long long, long long,
                                             float, int, const int*, const int*, int, hipStream_t);

// q,k,v,o: bf16 [B, S, H, D] with element strides (b, s, h); d contiguous. lse: f32 [B, Hq, Sq]
// (nullable). D in {64, 128}; Hq % Hk == 0.
PIAMD_EXPORT int piamd_flash_attn_fwd(const void* q, const void* k, const void* v, void* o,
                                      float* lse, int B, int Sq, int Sk, int Hq, int Hk, int D,
                                      long long sqb, long long sqs, long long sqh, long long skb,
                                      long long sks, long long skh, long long svb, long long svs,
                                      long long svh, long long sob, long long sos, long long soh,
                                      float scale, int causal, hipStream_t stream) {
  return piamd_flash_attn_varlen_fwd(q, k, v, o, lse, B, Sq, Sk, Hq, Hk, D, sqb, sqs, sqh, skb, sks,
                                     skh, svb, svs, svh, sob, sos, soh, scale, causal, nullptr,
                                     nullptr, 0, stream);
}

// Variable-length (packed) form: cu_q / cu_k int32 [B+1] row offsets on the device, q/k/v/o packed
// [total, H, D] (batch strides ignored), Sq / Sk = the longest sequence, lse f32 [Hq, total_q]
// (ltot = total_q). With cu_q == null this is the padded [B, S, H, D] kernel above.
PIAMD_EXPORT int piamd_flash_attn_varlen_fwd(const void* q, const void* k, const void* v, void* o,
                                             float* lse, int B, int Sq, int Sk, int Hq, int Hk,
                                             int D, long long sqb, long long sqs, long long sqh,
                                             long long skb, long long sks, long long skh,
                                             long long svb, long long svs, long long svh,
                                             long long sob, long long sos, long long soh,
                                             float scale, int causal, const int* cu_q,
                                             const int* cu_k, int ltot, hipStream_t stream) {
  if (Hk <= 0 || Hq % Hk || (cu_q && !cu_k)) return (int)hipErrorInvalidValue;
  if (cu_q) sqb = skb = svb = sob = 0;
  if (B == 0 || Sq == 0) return 0;
  if (Sk == 0) return (int)hipErrorInvalidValue;
  dim3 grid(((Sq + 127) / 128) * Hq * B), block(256);
#define FAF(DD, CC)                                                                               \
  hipLaunchKernelGGL((fa_fwd_kernel<DD, CC>), grid, block, 0, stream, (const bf16_t*)q,          \
                     (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse, B, Sq, Sk, Hq, Hk, sqb, \
                     sqs, sqh, skb, sks, skh, svb, svs, svh, sob, sos, soh, scale, cu_q, cu_k, ltot)
  if (D == 128) { if (causal) FAF(128, true); else FAF(128, false); }
  else if (D == 64) { if (causal) FAF(64, true); else FAF(64, false); }
  else return (int)hipErrorInvalidValue;
#undef FAF
  return (int)hipGetLastError();
}

// Backward. Strides: q/dq share (sqb, sqs, sqh); k/dk share (skb, sks, skh); v/dv share
// (svb, svs, svh); o and dout share (sdb, sds, sdh). delta: f32 [B, Hq, Sq] workspace.
// dq_acc / reserved: unused (kept for ABI stability).
PIAMD_EXPORT int piamd_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o,
                                      const void* dout, const float* lse, float* delta,
                                      float* dq_acc, void* dq, void* dk, void* dv,
                                      void* reserved, int B, int Sq, int Sk, int Hq, int Hk, int D,
                                      long long sqb, long long sqs, long long sqh, long long skb,
                                      long long sks, long long skh, long long svb, long long svs,
                                      long long svh, long long sdb, long long sds, long long sdh,
                                      float scale, int causal, hipStream_t stream) {
  (void)reserved; (void)dq_acc;
  return piamd_flash_attn_varlen_bwd(q, k, v, o, dout, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, D,
                                     sqb, sqs, sqh, skb, sks, skh, svb, svs, svh, sdb, sds, sdh,
                                     scale, causal, nullptr, nullptr, 0, stream);
}

// Variable-length backward (see piamd_flash_attn_varlen_fwd); lse / delta f32 [Hq, total_q].
PIAMD_EXPORT int piamd_flash_attn_varlen_bwd(const void* q, const void* k, const void* v,
                                             const void* o, const void* dout, const float* lse,
                                             float* delta, void* dq, void* dk, void* dv, int B,
                                             int Sq, int Sk, int Hq, int Hk, int D, long long sqb,
                                             long long sqs, long long sqh, long long skb,
                                             long long sks, long long skh, long long svb,
                                             long long svs, long long svh, long long sdb,
                                             long long sds, long long sdh, float scale,
                                             int causal, const int* cu_q, const int* cu_k,
                                             int ltot, hipStream_t stream) {
  if (Hk <= 0 || Hq % Hk || (cu_q && !cu_k)) return (int)hipErrorInvalidValue;
  if (cu_q) sqb = skb = svb = sdb = 0;
  if (B == 0 || Sq == 0 || Sk == 0) return 0;
  // delta rows: padded [B, Hq, Sq]; packed [Hq, ltot] == the padded layout with B = 1, Sq = ltot
  const int pB = cu_q ? 1 : B, pS = cu_q ? ltot : Sq;
  const int total = pB * Hq * pS;
  const int tpr = D / 8;
  const int pre_blocks = (int)(((long long)total * tpr + 255) / 256);
#define PRE(DD)                                                                                   \
  hipLaunchKernelGGL((fa_bwd_pre_kernel<DD>), dim3(pre_blocks), dim3(256), 0, stream,            \
                     (const bf16_t*)o, (const bf16_t*)dout, delta, pS, Hq, sdb, sds, sdh, total)
  if (D == 128) PRE(128); else if (D == 64) PRE(64); else return (int)hipErrorInvalidValue;
#undef PRE
  dim3 gkv(((Sk + 127) / 128) * Hk * B), gq(((Sq + 127) / 128) * Hq * B), block(256);
#define FAB(DD, CC)                                                                               \
  hipLaunchKernelGGL((fa_bwd_dkdv_kernel<DD, CC>), gkv, block, 0, stream, (const bf16_t*)q,      \
                     (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, lse, delta,         \
                     (bf16_t*)dk, (bf16_t*)dv, B, Sq, Sk, Hq, Hk, sqb, sqs, sqh, skb, sks, skh,   \
                     svb, svs, svh, sdb, sds, sdh, scale, cu_q, cu_k, ltot);                      \
  hipLaunchKernelGGL((fa_bwd_dq_kernel<DD, CC>), gq, block, 0, stream, (const bf16_t*)q,         \
                     (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, lse, delta,         \
                     (bf16_t*)dq, B, Sq, Sk, Hq, Hk, sqb, sqs, sqh, skb, sks, skh, svb, svs, svh, \
                     sdb, sds, sdh, scale, cu_q, cu_k, ltot)
  if (D == 128) { if (causal) { FAB(128, true); } else { FAB(128, false); } }
  else { if (causal) { FAB(64, true); } else { FAB(64, false); } }
#undef FAB
  return (int)hipGetLastError();
}
