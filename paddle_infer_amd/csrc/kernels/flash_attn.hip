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
//   * Backward: workgroup = 4 waves = 128 keys (32 per wave, key on the MFMA lane), dKᵀ/dVᵀ kept in
//     accumulators across the whole sweep over query tiles (and over the q-heads of a GQA group),
//     so dK/dV need no cross-workgroup sum; dQ is summed over key blocks with f32 atomics whose
//     wave-instructions are two 128-B row segments (full atomic rate, MI355X_MICROARCH §atomics).
//   * Causal blocks are launched heaviest-first.
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

// ------------------------------------------------------------------------------------------
// Forward
// ------------------------------------------------------------------------------------------
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    bf16_t* __restrict__ o, float* __restrict__ lse, int Sq, int Sk, int Hq, int Hk,
    long long sqb, long long sqs, long long sqh, long long skb, long long sks, long long skh,
    long long svb, long long svs, long long svh, long long sob, long long sos, long long soh,
    float scale) {
  constexpr int BM = 128, BN = 64;
  constexpr int KSTEPS = D / 16;
  constexpr int DT = D / 32;
  constexpr int CH = D / 8;          // 16-B chunks per row
  constexpr int ROWB = D * 2;
  constexpr int TILE_B = BN * ROWB;  // bytes per K or V tile
  constexpr int LPT = BN * CH / 256; // 16-B loads per thread per tile
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_B];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5, gi = lane & 15, g = lane >> 4;
  const int nmb = (Sq + BM - 1) / BM;
  const int mb = CAUSAL ? (nmb - 1 - (int)blockIdx.x) : (int)blockIdx.x;
  const int hq = blockIdx.y, b = blockIdx.z;
  const int hk = hq / (Hq / Hk);
  const int m0 = mb * BM;
  const int qrow0 = m0 + w * 32;
  const int coff = Sk - Sq;  // bottom-right aligned causal offset
  const float c = scale * kLog2e;

  const bf16_t* kbase = k + b * skb + hk * skh;
  const bf16_t* vbase = v + b * svb + hk * svh;

  bf16x8 qf[KSTEPS];
  {
    const int qr = qrow0 + l32;
    const bf16_t* qp = q + b * sqb + (long long)qr * sqs + hq * sqh + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk)
      qf[kk] = qr < Sq ? *reinterpret_cast<const bf16x8*>(qp + 16 * kk) : zero_bf16x8();
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

  u16x8 kreg[LPT], vreg[LPT];
  auto gload = [&](int t) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, r = id / CH, cc = id % CH;
      const int key = t * BN + r;
      if (key < Sk) {
        kreg[i] = *reinterpret_cast<const u16x8*>(kbase + (long long)key * sks + cc * 8);
        vreg[i] = *reinterpret_cast<const u16x8*>(vbase + (long long)key * svs + cc * 8);
      } else {
        kreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        vreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  };
  auto lstore = [&](int buf) {
    char* ks = smem + buf * 2 * TILE_B;
    char* vs = ks + TILE_B;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, r = id / CH, cc = id % CH;
      *reinterpret_cast<u16x8*>(ks + lds_off<ROWB>(r, cc)) = kreg[i];
      *reinterpret_cast<u16x8*>(vs + lds_off<ROWB>(r, cc)) = vreg[i];
    }
  };

  if (ntiles > 0) { gload(0); lstore(0); }
  __syncthreads();

  const bool wave_rows_valid = qrow0 < Sq;
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) gload(t + 1);
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
      // scale, mask, row max (query row = lane)
      const int qpos = qrow0 + l32;
      const bool need_mask = (n0 + BN > Sk) || (CAUSAL && n0 + BN - 1 > qrow0 + coff);
      float mx = -INFINITY;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float x = sacc[tt][r] * c;
          if (need_mask) {
            const int key = n0 + tt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (key >= Sk || (CAUSAL && key > qpos + coff)) x = -INFINITY;
          }
          sacc[tt][r] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_i, mx);
      const float msub = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = exp2f(m_i - msub);
      float rs = 0.f;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = exp2f(sacc[tt][r] - msub);
          sacc[tt][r] = p;
          rs += p;
        }
      rs += __shfl_xor(rs, 32, 64);
      l_i = l_i * alpha + rs;
      m_i = m_new;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int j = 0; j < 16; ++j) oacc[dt][j] *= alpha;
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
    if (t + 1 < ntiles) lstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane = query row, registers = d
  const int qr = qrow0 + l32;
  if (qr < Sq) {
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    bf16_t* op = o + b * sob + (long long)qr * sos + hq * soh;
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
      lse[((long long)b * Hq + hq) * Sq + qr] = l_i > 0.f ? (m_i + log2f(l_i)) * kLn2 : INFINITY;
  }
}

// ------------------------------------------------------------------------------------------
// Backward pre-pass: delta[b, h, q] = Σ_d dO·O (f32), one wave per (row, head).
// ------------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void fa_bwd_pre_kernel(
    const bf16_t* __restrict__ o, const bf16_t* __restrict__ dout, float* __restrict__ delta,
    int Sq, int Hq, long long sob, long long sos, long long soh, long long sdb, long long sds,
    long long sdh, int total) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wid >= total) return;
  const int qr = wid % Sq, hq = (wid / Sq) % Hq, b = wid / (Sq * Hq);
  const bf16_t* op = o + b * sob + (long long)qr * sos + hq * soh;
  const bf16_t* dp = dout + b * sdb + (long long)qr * sds + hq * sdh;
  float s = 0.f;
  for (int d = lane * 2; d < D; d += 128) {
    s += bf2f(op[d]) * bf2f(dp[d]) + bf2f(op[d + 1]) * bf2f(dp[d + 1]);
  }
  s = wave_sum(s);
  if (lane == 0) delta[((long long)b * Hq + hq) * Sq + qr] = s;
}

// ------------------------------------------------------------------------------------------
// Backward main: workgroup = 128 keys of one (batch, kv-head); sweeps the q-heads of the GQA
// group and all query tiles of 64 rows.
// ------------------------------------------------------------------------------------------
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void fa_bwd_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k, const bf16_t* __restrict__ v,
    const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dq_acc, bf16_t* __restrict__ dk,
    bf16_t* __restrict__ dv, int Sq, int Sk, int Hq, int Hk, long long sqb, long long sqs,
    long long sqh, long long skb, long long sks, long long skh, long long svb, long long svs,
    long long svh, long long sdob, long long sdos, long long sdoh, long long sdkb,
    long long sdks, long long sdkh, long long sdvb, long long sdvs, long long sdvh,
    float scale) {
  constexpr int BK = 128, BQ = 64;
  constexpr int KSTEPS = D / 16;
  constexpr int DT = D / 32;
  constexpr int CH = D / 8;
  constexpr int ROWB = D * 2;
  constexpr int KIMG_B = BK * ROWB;     // K image [128 keys][D]
  constexpr int QTILE_B = BQ * ROWB;    // Q or dO tile [64][D]
  constexpr int DS_ROWB = BQ * 2;       // dSᵀ image [128 keys][64 q] bf16
  constexpr int DS_B = BK * DS_ROWB;
  constexpr int LPT = BQ * CH / 256;    // 16-B loads per thread per Q (or dO) tile
  constexpr int OFF_K = 0;
  constexpr int OFF_Q = OFF_K + KIMG_B;               // 2 buffers x (Q, dO)
  constexpr int OFF_DS = OFF_Q + 2 * 2 * QTILE_B;
  constexpr int OFF_STAT = OFF_DS + DS_B;             // 2 buffers x (lse, delta) x 64 f32
  constexpr int SMEM = OFF_STAT + 2 * 2 * BQ * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5, gi = lane & 15, g = lane >> 4;
  const int nkb = (Sk + BK - 1) / BK;
  const int kb = CAUSAL ? (int)blockIdx.x : (int)blockIdx.x;  // (light blocks are the late ones)
  const int hk = blockIdx.y, b = blockIdx.z;
  const int n0 = kb * BK;
  const int kw0 = n0 + 32 * w;  // this wave's first key
  const int coff = Sk - Sq;
  const int group = Hq / Hk;
  const float c = scale * kLog2e;
  (void)nkb;

  // ---- stage K image (all 128 keys) into LDS; K and V fragments of this wave's keys to regs.
  {
    const bf16_t* kbp = k + b * skb + hk * skh;
#pragma unroll
    for (int i = 0; i < BK * CH / 256; ++i) {
      const int id = tid + 256 * i, r = id / CH, cc = id % CH;
      const int key = n0 + r;
      u16x8 val = key < Sk ? *reinterpret_cast<const u16x8*>(kbp + (long long)key * sks + cc * 8)
                           : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      *reinterpret_cast<u16x8*>(smem + OFF_K + lds_off<ROWB>(r, cc)) = val;
    }
  }
  bf16x8 kf[KSTEPS], vf[KSTEPS];
  {
    const int key = kw0 + l32;
    const bf16_t* kp = k + b * skb + (long long)key * sks + hk * skh + 8 * hh;
    const bf16_t* vp = v + b * svb + (long long)key * svs + hk * svh + 8 * hh;
#pragma unroll
    for (int kk = 0; kk < KSTEPS; ++kk) {
      kf[kk] = key < Sk ? *reinterpret_cast<const bf16x8*>(kp + 16 * kk) : zero_bf16x8();
      vf[kk] = key < Sk ? *reinterpret_cast<const bf16x8*>(vp + 16 * kk) : zero_bf16x8();
    }
  }

  f32x16 dkacc[DT], dvacc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) { dkacc[i][j] = 0.f; dvacc[i][j] = 0.f; }

  // first query tile that can see any key of this block
  const int q_start = CAUSAL ? max(0, n0 - coff) : 0;
  const int qt0 = q_start / BQ;
  const int nqt = (Sq + BQ - 1) / BQ;
  const int tiles_per_head = nqt - qt0;
  const int total = tiles_per_head > 0 ? tiles_per_head * group : 0;

  u16x8 qreg[LPT], doreg[LPT];
  float lreg = 0.f, dreg = 0.f;
  auto gload = [&](int it) {
    const int hq = hk * group + it / tiles_per_head;
    const int q0 = (qt0 + it % tiles_per_head) * BQ;
    const bf16_t* qbp = q + b * sqb + hq * sqh;
    const bf16_t* dbp = dout + b * sdob + hq * sdoh;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, r = id / CH, cc = id % CH;
      const int qr = q0 + r;
      if (qr < Sq) {
        qreg[i] = *reinterpret_cast<const u16x8*>(qbp + (long long)qr * sqs + cc * 8);
        doreg[i] = *reinterpret_cast<const u16x8*>(dbp + (long long)qr * sdos + cc * 8);
      } else {
        qreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        doreg[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
    if (tid < BQ) {
      const int qr = q0 + tid;
      const long long si = ((long long)b * Hq + hq) * Sq + qr;
      lreg = qr < Sq ? lse[si] * kLog2e : INFINITY;
      dreg = qr < Sq ? delta[si] : 0.f;
    }
  };
  auto lstore = [&](int buf) {
    char* qs = smem + OFF_Q + buf * 2 * QTILE_B;
    char* ds = qs + QTILE_B;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, r = id / CH, cc = id % CH;
      *reinterpret_cast<u16x8*>(qs + lds_off<ROWB>(r, cc)) = qreg[i];
      *reinterpret_cast<u16x8*>(ds + lds_off<ROWB>(r, cc)) = doreg[i];
    }
    float* st = reinterpret_cast<float*>(smem + OFF_STAT) + buf * 2 * BQ;
    if (tid < BQ) { st[tid] = lreg; st[BQ + tid] = dreg; }
  };

  if (total > 0) { gload(0); lstore(0); }
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int buf = it & 1;
    const int hq = hk * group + it / tiles_per_head;
    const int q0 = (qt0 + it % tiles_per_head) * BQ;
    if (it + 1 < total) gload(it + 1);
    const char* qs = smem + OFF_Q + buf * 2 * QTILE_B;
    const char* dos = qs + QTILE_B;
    const float* lst = reinterpret_cast<const float*>(smem + OFF_STAT) + buf * 2 * BQ;
    const float* dst = lst + BQ;
    char* dsimg = smem + OFF_DS;
    // wave fully masked for this q tile? (all its keys beyond every query row)
    const bool active = !CAUSAL || (kw0 <= q0 + BQ - 1 + coff);
    if (active) {
      // S = Q·Kᵀ and dP = dO·Vᵀ, key on lane, query in registers; 2 q-subtiles of 32
      f32x16 sacc[2], pacc[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int j = 0; j < 16; ++j) { sacc[qt][j] = 0.f; pacc[qt][j] = 0.f; }
#pragma unroll
      for (int kk = 0; kk < KSTEPS; ++kk) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          bf16x8 a = lds_row8(qs, lds_off<ROWB>(qt * 32 + l32, 2 * kk + hh));
          sacc[qt] = mfma32(a, kf[kk], sacc[qt]);
          bf16x8 a2 = lds_row8(dos, lds_off<ROWB>(qt * 32 + l32, 2 * kk + hh));
          pacc[qt] = mfma32(a2, vf[kk], pacc[qt]);
        }
      }
      // P = exp2(S·c − lse·log2e), dS = P·(dP − delta)
      const int key = kw0 + l32;
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qi = qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          const int qr = q0 + qi;
          float p = exp2f(sacc[qt][r] * c - lst[qi]);
          if (key >= Sk || (CAUSAL && key > qr + coff)) p = 0.f;
          sacc[qt][r] = p;
          pacc[qt][r] = p * (pacc[qt][r] - dst[qi]);
        }
      // dVᵀ += dOᵀ·P ; dKᵀ += Qᵀ·dS   (A operands via transposed reads of the dO / Q images)
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pb = pack_frag(sacc[qt], s);
          const bf16x8 db = pack_frag(pacc[qt], s);
          const int r0 = 32 * qt + 16 * s + 4 * hh;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const int c0 = 32 * dt + 16 * (g & 1);
            bf16x8 ado = cat44(lds_tr4<ROWB>(dos, r0, c0, gi), lds_tr4<ROWB>(dos, r0 + 8, c0, gi));
            dvacc[dt] = mfma32(ado, pb, dvacc[dt]);
            bf16x8 aq = cat44(lds_tr4<ROWB>(qs, r0, c0, gi), lds_tr4<ROWB>(qs, r0 + 8, c0, gi));
            dkacc[dt] = mfma32(aq, db, dkacc[dt]);
          }
        }
      // dSᵀ image [key][q]: lane's key row, 4 consecutive q per register group
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int qc = 32 * qt + 8 * g4 + 4 * hh;  // first of 4 q columns
          uint2 pk;
          pk.x = pack_bf16x2(pacc[qt][4 * g4 + 0], pacc[qt][4 * g4 + 1]);
          pk.y = pack_bf16x2(pacc[qt][4 * g4 + 2], pacc[qt][4 * g4 + 3]);
          *reinterpret_cast<uint2*>(dsimg + lds_off<DS_ROWB>(32 * w + l32, qc >> 3) + ((qc & 7) << 1)) = pk;
        }
    } else {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int qc = 32 * qt + 8 * g4 + 4 * hh;
          *reinterpret_cast<uint2*>(dsimg + lds_off<DS_ROWB>(32 * w + l32, qc >> 3) + ((qc & 7) << 1)) = uint2{0u, 0u};
        }
    }
    __syncthreads();
    // dQ[q][d] (this wave: d columns 32w..32w+31) = Σ_key dS[q][key]·K[key][d]
    {
      bool any = true;
      if (CAUSAL) any = n0 <= q0 + BQ - 1 + coff;
      if (any && 32 * w < D) {
        f32x16 qacc[2];
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int j = 0; j < 16; ++j) qacc[qt][j] = 0.f;
        const char* kimg = smem + OFF_K;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
          const int r0 = 16 * ks + 4 * hh;
          const int cb = 32 * w + 16 * (g & 1);
          bf16x8 bk = cat44(lds_tr4<ROWB>(kimg, r0, cb, gi), lds_tr4<ROWB>(kimg, r0 + 8, cb, gi));
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) {
            const int qb = 32 * qt + 16 * (g & 1);
            bf16x8 ads = cat44(lds_tr4<DS_ROWB>(dsimg, r0, qb, gi), lds_tr4<DS_ROWB>(dsimg, r0 + 8, qb, gi));
            qacc[qt] = mfma32(ads, bk, qacc[qt]);
          }
        }
        // atomics: lane = d column, registers = q rows
        const int d = 32 * w + l32;
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int qr = q0 + 32 * qt + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (qr < Sq)
              atomicAdd(dq_acc + (((long long)b * Sq + qr) * Hq + hq) * D + d, qacc[qt][r] * scale);
          }
      }
    }
    if (it + 1 < total) lstore(buf ^ 1);
    __syncthreads();
  }

  // write dK (scaled) and dV: lane = key, registers = d
  const int key = kw0 + l32;
  if (key < Sk) {
    bf16_t* dkp = dk + b * sdkb + (long long)key * sdks + hk * sdkh;
    bf16_t* dvp = dv + b * sdvb + (long long)key * sdvs + hk * sdvh;
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

// dq (bf16, strided) = dq_acc (f32, [B, Sq, Hq, D] contiguous)
template <int D>
__global__ __launch_bounds__(256) void fa_dq_convert_kernel(const float* __restrict__ acc,
                                                           bf16_t* __restrict__ dq, int Sq,
                                                           int Hq, long long sb, long long ss,
                                                           long long sh, long long total8) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total8) return;
  const long long e = i * 8;
  const int d = e % D;
  const long long row = e / D;  // (b*Sq + s)*Hq + h
  const int h = row % Hq;
  const long long bs = row / Hq;
  const int s = bs % Sq;
  const int b = bs / Sq;
  f32x4 a = *reinterpret_cast<const f32x4*>(acc + e), c2 = *reinterpret_cast<const f32x4*>(acc + e + 4);
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) { o[j] = f2bf(a[j]); o[4 + j] = f2bf(c2[j]); }
  *reinterpret_cast<u16x8*>(dq + b * sb + (long long)s * ss + h * sh + d) = o;
}

}  // namespace

// q,k,v,o: bf16 [B, S, H, D] with element strides (b, s, h); d contiguous. lse: f32 [B, Hq, Sq]
// (nullable). D in {64, 128}; Hq % Hk == 0.
PIAMD_EXPORT int piamd_flash_attn_fwd(const void* q, const void* k, const void* v, void* o,
                                      float* lse, int B, int Sq, int Sk, int Hq, int Hk, int D,
                                      long long sqb, long long sqs, long long sqh, long long skb,
                                      long long sks, long long skh, long long svb, long long svs,
                                      long long svh, long long sob, long long sos, long long soh,
                                      float scale, int causal, hipStream_t stream) {
  if (Hk <= 0 || Hq % Hk) return (int)hipErrorInvalidValue;
  if (B == 0 || Sq == 0) return 0;
  dim3 grid((Sq + 127) / 128, Hq, B), block(256);
#define FAF(DD, CC)                                                                               \
  hipLaunchKernelGGL((fa_fwd_kernel<DD, CC>), grid, block, 0, stream, (const bf16_t*)q,          \
                     (const bf16_t*)k, (const bf16_t*)v, (bf16_t*)o, lse, Sq, Sk, Hq, Hk, sqb,  \
                     sqs, sqh, skb, sks, skh, svb, svs, svh, sob, sos, soh, scale)
  if (D == 128) { if (causal) FAF(128, true); else FAF(128, false); }
  else if (D == 64) { if (causal) FAF(64, true); else FAF(64, false); }
  else return (int)hipErrorInvalidValue;
#undef FAF
  return (int)hipGetLastError();
}

// Backward. dq_acc: f32 workspace [B, Sq, Hq, D] (zeroed here). delta: f32 [B, Hq, Sq] workspace.
PIAMD_EXPORT int piamd_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o,
                                      const void* dout, const float* lse, float* delta,
                                      float* dq_acc, void* dq, void* dk, void* dv,
                                      void* reserved, int B, int Sq, int Sk, int Hq, int Hk, int D,
                                      long long sqb, long long sqs, long long sqh, long long skb,
                                      long long sks, long long skh, long long svb, long long svs,
                                      long long svh, long long sdb, long long sds, long long sdh,
                                      float scale, int causal, hipStream_t stream) {
  // Strides: q/dq share (sqb, sqs, sqh); k/dk share (skb, sks, skh); v/dv share (svb, svs, svh);
  // o and dout share (sdb, sds, sdh).
  (void)reserved;
  if (Hk <= 0 || Hq % Hk) return (int)hipErrorInvalidValue;
  if (B == 0 || Sq == 0 || Sk == 0) return 0;
  hipMemsetAsync(dq_acc, 0, sizeof(float) * (size_t)B * Sq * Hq * D, stream);
  const int total = B * Hq * Sq;
#define PRE(DD)                                                                                   \
  hipLaunchKernelGGL((fa_bwd_pre_kernel<DD>), dim3((total + 3) / 4), dim3(256), 0, stream,       \
                     (const bf16_t*)o, (const bf16_t*)dout, delta, Sq, Hq, sdb, sds, sdh, sdb,  \
                     sds, sdh, total)
  if (D == 128) PRE(128); else if (D == 64) PRE(64); else return (int)hipErrorInvalidValue;
#undef PRE
  dim3 grid((Sk + 127) / 128, Hk, B), block(256);
#define FAB(DD, CC)                                                                               \
  hipLaunchKernelGGL((fa_bwd_kernel<DD, CC>), grid, block, 0, stream, (const bf16_t*)q,          \
                     (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, lse, delta, dq_acc, \
                     (bf16_t*)dk, (bf16_t*)dv, Sq, Sk, Hq, Hk, sqb, sqs, sqh, skb, sks, skh, svb, \
                     svs, svh, sdb, sds, sdh, skb, sks, skh, svb, svs, svh, scale)
  if (D == 128) { if (causal) FAB(128, true); else FAB(128, false); }
  else { if (causal) FAB(64, true); else FAB(64, false); }
#undef FAB
  const long long total8 = (long long)B * Sq * Hq * D / 8;
  const int cg = (int)((total8 + 255) / 256);
  if (D == 128)
    hipLaunchKernelGGL((fa_dq_convert_kernel<128>), dim3(cg), dim3(256), 0, stream, dq_acc,
                       (bf16_t*)dq, Sq, Hq, sqb, sqs, sqh, total8);
  else
    hipLaunchKernelGGL((fa_dq_convert_kernel<64>), dim3(cg), dim3(256), 0, stream, dq_acc,
                       (bf16_t*)dq, Sq, Hq, sqb, sqs, sqh, total8);
  return (int)hipGetLastError();
}
