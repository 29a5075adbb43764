// Skinny MFMA GEMM: C[M][N] = act(alpha · A[M][K] · B[N][K]ᵀ + bias) (+ resid) for few-row
// products — inference linears, prefill of short prompts, small batched matmuls — where the
// 256×256-tile assembly GEMM (csrc/asm/gemm_gen.py) would leave most of the 256 CUs idle.
//
// Parity: reference `paddle/phi/kernels/funcs/blas/blas_impl.cu.h` (cublas GEMM behind matmul /
// fc / linear at small M) and `fused/fused_gemm_epilogue_op.cu` (bias / activation epilogue).
//
// Structure (gfx950, bf16 or fp16 operands, f32 accumulation):
//   * A and B both K-contiguous (weights in their cached [N][K] copy), so every operand fragment
//     is a direct 32-B-per-lane global load — no LDS staging: few rows means little reuse to win,
//     and the weight bytes (the dominant stream) are read exactly once per workgroup.
//   * workgroup = 4 waves over ONE output tile of TM = 16·MB rows × TN = 16·NB·WN columns: WN
//     waves side by side along N (they read the same A fragments — L1 hits) and 4/WN waves
//     splitting the tile's K range (k64 steps w_k, w_k + 4/WN, …) that meet in LDS, so a short
//     K range still keeps every wave busy and a long one keeps four load streams in flight.
//     Grid (N/TN, M/TM, KS): KS > 1 splits K over workgroups. Fixup mode (cnt != null): every
//     slice adds its partial into a zeroed f32 tile with memory-side atomics and the last slice
//     to arrive (per-tile counter) runs the epilogue and re-zeroes the tile — one launch. Slice
//     mode (cnt == null): f32 slices ws[KS][M][N] summed in a fixed order by small_gemm_finish.
//   * v_mfma_f32_16x16x32_{bf16,f16} with the operands swapped (D = B·Aᵀ blocks), so a lane owns
//     4 consecutive output columns of one row: 8-B (16-bit) / 16-B (f32) stores. Lane group g of
//     a k64 step loads k = 16g … 16g+15 of its row; MFMA sub-step s uses elements 8s … 8s+7 of it
//     (a permutation of the k sum, identical for A and B).
//   * rows ≥ M / columns ≥ N read a clamped (valid) row and are never stored.
//   * LayerNorm fold (LN, bf16 / fp16, KS = 1): C = act(LN(A)·Bᵀ + bias) with the host-side fold
//     B' = B∘γ, c1[n] = Σ_k B'[n][k], b2[n] = bias[n] + Σ_k β[k]·B[n][k], so that
//     LN(a)·B = rstd·(a·B'ᵀ − mean·c1) + b2. The kernel runs on the RAW rows: every lane adds up
//     Σa and Σa² of the A fragments it already loads, the four lane groups and the K-splitting
//     waves combine them, and the epilogue applies rstd·(acc − mean·c1[n]) + b2[n]. No separate
//     LayerNorm launch (serving-batch decode: reference fused_multi_transformer pre-LN; post-LN
//     BERT inference at few rows, where the producer of the raw rows skips its LayerNorm and the
//     statistics computed here also feed the residual epilogue of a later GEMM via ln_stats).
// Contract: K % 64 == 0, N % 4 == 0, lda / ldb % 8 == 0, 16-B aligned operands.
#include "common.h"

namespace {

typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));

template <bool F16>
__device__ __forceinline__ f32x4 mma16(const u16x8& b, const u16x8& a, const f32x4& c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, b),
                                                  __builtin_bit_cast(f16x8_t, a), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, b),
                                                   __builtin_bit_cast(bf16x8, a), c, 0, 0, 0);
}

__device__ __forceinline__ float sg_act(float v, int act) {
  switch (act) {
    case 1: return gelu_tanh(v);
    case 2: return gelu_erf(v);
    case 3: return fmaxf(v, 0.f);
    case 4: return v / (1.f + __expf(-v));
    case 5: return tanhf(v);  // skinny-kernel only (e.g. the BERT pooler fc)
    default: return v;
  }
}

struct SgArgs {
  const bf16_t* a;
  long long lda;
  const bf16_t* b;
  long long ldb;
  void* c;
  long long ldc;
  float* ws;  // KS > 1: f32 slices [KS][M][N]
  const bf16_t* bias;
  const bf16_t* resid;
  long long ldr;
  float alpha;
  int M, N, K, c_f32, act;
  const float* ln_c1;  // LN fold: [N] column sums of B' (null: no LayerNorm)
  const float* ln_b2;  // LN fold: [N] bias + B·β
  float ln_eps;
  float* ln_stats;         // LN fold: [M] (mean, rstd) of the raw A rows written out (nullable)
  const float* rln_stats;  // deferred LayerNorm of the residual: [M] (mean, rstd) of its raw rows
  const bf16_t* rln_g;     // ... and its 16-bit γ / β [N] (resid added as LN(resid) when set)
  const bf16_t* rln_b;
};

// Epilogue value of (m, n..n+3) → C.
template <bool F16, bool LN = false>
__device__ __forceinline__ void sg_store(const SgArgs& p, int m, int n, f32x4 v, float mu = 0.f,
                                         float rs = 1.f) {
  float2 rst = make_float2(0.f, 1.f);
  if (p.rln_stats) rst = reinterpret_cast<const float2*>(p.rln_stats)[m];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float x;
    if constexpr (LN) x = rs * (v[j] - mu * p.ln_c1[n + j]) + p.ln_b2[n + j];
    else x = v[j] * p.alpha + (p.bias ? h2f<F16>(p.bias[n + j]) : 0.f);
    x = sg_act(x, p.act);
    if (p.resid) {
      float r = h2f<F16>(p.resid[(long long)m * p.ldr + n + j]);
      if (p.rln_stats)  // residual kept raw by its producer: LN applied here (post-LN chains)
        r = (r - rst.x) * rst.y * h2f<F16>(p.rln_g[n + j]) + h2f<F16>(p.rln_b[n + j]);
      x += r;
    }
    v[j] = x;
  }
  if (p.c_f32) {
    *reinterpret_cast<f32x4*>((float*)p.c + (long long)m * p.ldc + n) = v;
  } else {
    u16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f2h<F16>(v[j]);
    *reinterpret_cast<u16x4*>((bf16_t*)p.c + (long long)m * p.ldc + n) = o;
  }
}

template <bool F16, int MB, int NB, int WN, int D, bool LN = false, int DB = D>
__global__ __launch_bounds__(256) void small_gemm_kernel(SgArgs p, int* __restrict__ cnt) {
  static_assert(DB >= D && DB % D == 0, "B ring depth must be a multiple of the A ring depth");
  constexpr int WK = 4 / WN;
  __shared__ f32x4 red[WK > 1 ? 4 : 1][MB * NB][64];
  __shared__ float2 lst[LN && WK > 1 ? 4 : 1][MB][16];  // LN: per-wave row (Σa, Σa²)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r16 = lane & 15;
  const int wn = w % WN, wk = w / WN;
  const int n0 = blockIdx.x * (16 * NB * WN) + wn * (16 * NB), m0 = blockIdx.y * (16 * MB);
  const int kz = blockIdx.z, KS = gridDim.z;
  const int nkb = p.K >> 6;
  const int kb_beg = (int)((long long)nkb * kz / KS), kb_end = (int)((long long)nkb * (kz + 1) / KS);

  const bf16_t* arow[MB];
  const bf16_t* brow[NB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
    arow[mb] = p.a + (long long)min(m0 + 16 * mb + r16, p.M - 1) * p.lda + 16 * g;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
    brow[nb] = p.b + (long long)min(n0 + 16 * nb + r16, p.N - 1) * p.ldb + 16 * g;

  f32x4 acc[MB][NB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // LN: Σa of row r16 of block mb (every column of the ones·Aᵀ block) and the A·Aᵀ block whose
  // diagonal holds Σa² (row r16's at lane r16 + 16·(r16 >> 2), element r16 & 3)
  f32x4 accS[LN ? MB : 1], accQ[LN ? MB : 1];
#pragma unroll
  for (int mb = 0; mb < (LN ? MB : 1); ++mb) accS[mb] = accQ[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = F16 ? 0x3C00 : 0x3F80;  // 1.0 in the operand type

  // Register rings of operand fragments: step i computes on A slot i % D and B slot i % DB, then
  // refills them with steps i + D / i + DB — D k64 steps of A loads (L2-resident activations) and
  // DB of B loads (the weight stream from HBM) in flight per wave. DB > D: the weight stream of a
  // wave's whole K range is issued up front (one HBM round trip) while A follows in L2 trips.
  u16x8 ar[D][MB][2], br[DB][NB][2];
  auto loadA = [&](int kb, u16x8 (&ad)[MB][2]) {
    const long long k = (long long)kb << 6;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const u16x8* s = reinterpret_cast<const u16x8*>(arow[mb] + k);
      ad[mb][0] = s[0];
      ad[mb][1] = s[1];
    }
  };
  auto loadB = [&](int kb, u16x8 (&bd)[NB][2]) {
    const long long k = (long long)kb << 6;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const u16x8* s = reinterpret_cast<const u16x8*>(brow[nb] + k);
      bd[nb][0] = s[0];
      bd[nb][1] = s[1];
    }
  };
  const int kb0 = kb_beg + wk;
  if constexpr (DB == D) {
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (kb0 + d * WK < kb_end) {
        loadB(kb0 + d * WK, br[d]);
        loadA(kb0 + d * WK, ar[d]);
      }
  } else {  // A of the first step first: its wait then covers no later-issued B load
    if (kb0 < kb_end) loadA(kb0, ar[0]);
#pragma unroll
    for (int d = 0; d < DB; ++d)
      if (kb0 + d * WK < kb_end) loadB(kb0 + d * WK, br[d]);
#pragma unroll
    for (int d = 1; d < D; ++d)
      if (kb0 + d * WK < kb_end) loadA(kb0 + d * WK, ar[d]);
  }
  for (int kb = kb0; kb < kb_end; kb += DB * WK) {
#pragma unroll
    for (int d = 0; d < DB; ++d) {
      const int k = kb + d * WK;
      if (k >= kb_end) break;
      const int da = d % D;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int nb = 0; nb < NB; ++nb)
            acc[mb][nb] = mma16<F16>(br[d][nb][s], ar[da][mb][s], acc[mb][nb]);
      if constexpr (LN) {  // row statistics on the matrix cores: ones·Aᵀ and A·Aᵀ blocks
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) {
            accS[mb] = mma16<F16>(ones, ar[da][mb][s], accS[mb]);
            accQ[mb] = mma16<F16>(ar[da][mb][s], ar[da][mb][s], accQ[mb]);
          }
      }
      if constexpr (DB == D) {
        if (k + D * WK < kb_end) {
          loadB(k + D * WK, br[d]);
          loadA(k + D * WK, ar[da]);
        }
      } else {
        if (k + D * WK < kb_end) loadA(k + D * WK, ar[da]);
        if (k + DB * WK < kb_end) loadB(k + DB * WK, br[d]);
      }
    }
  }
  float s1[MB], s2[MB];  // LN: Σa / Σa² of row r16 of block mb over this wave's K range
  if constexpr (LN) {
    const int j = r16 & 3;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      const f32x4 q = accQ[mb];
      const float dq = j == 0 ? q[0] : j == 1 ? q[1] : j == 2 ? q[2] : q[3];
      s1[mb] = accS[mb][0];
      s2[mb] = __shfl(dq, r16 + 16 * (r16 >> 2));
      if (WK > 1 && g == 0) lst[WK > 1 ? w : 0][mb][r16] = make_float2(s1[mb], s2[mb]);
    }
  }
  if constexpr (WK > 1) {
    // the K-splitting waves of one column group meet in LDS; wave (wn, wk) finishes the blocks
    // i ≡ wk (mod WK) of its column group
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) red[w][mb * NB + nb][lane] = acc[mb][nb];
    __syncthreads();
  }
  float mu[MB], rs[MB];
  if constexpr (LN) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      float a = s1[mb], b = s2[mb];
      if constexpr (WK > 1) {
        a = b = 0.f;
#pragma unroll
        for (int j = 0; j < WK; ++j) {
          const float2 t = lst[wn + j * WN][mb][r16];
          a += t.x;
          b += t.y;
        }
      }
      mu[mb] = a / p.K;
      rs[mb] = rsqrtf(fmaxf(b / p.K - mu[mb] * mu[mb], 0.f) + p.ln_eps);
    }
    // row statistics out (for a later consumer of the same raw rows, e.g. the residual epilogue
    // of the next GEMM): column block 0, wave 0, one lane per row
    if (p.ln_stats && blockIdx.x == 0 && w == 0 && g == 0) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int m = m0 + 16 * mb + r16;
        if (m < p.M) reinterpret_cast<float2*>(p.ln_stats)[m] = make_float2(mu[mb], rs[mb]);
      }
    }
  }
  // D = B·Aᵀ block: lane holds rows m = r16 of the A block, columns n = 4g + j of the B block
  float sink = 0.f;
  bool any = false;
#pragma unroll
  for (int i = 0; i < MB * NB; ++i) {
    if (WK > 1 && i % WK != wk) continue;
    const int mb = i / NB, nb = i % NB;
    const int m = m0 + 16 * mb + r16, n = n0 + 16 * nb + 4 * g;
    f32x4 v = acc[mb][nb];
    if constexpr (WK > 1) {
      v = red[wn][i][lane];
#pragma unroll
      for (int j = 1; j < WK; ++j) v += red[wn + j * WN][i][lane];
    }
    if (m >= p.M || n >= p.N) continue;
    if (KS == 1) {
      if constexpr (LN) sg_store<F16, true>(p, m, n, v, mu[mb], rs[mb]);
      else sg_store<F16>(p, m, n, v);
    } else if (cnt == nullptr) {
      *reinterpret_cast<f32x4*>(p.ws + ((long long)kz * p.M + m) * p.N + n) = v;
    } else {
      float* t = p.ws + (long long)m * p.N + n;
#pragma unroll
      for (int j = 0; j < 4; ++j) sink += xcd_add(t + j, v[j]);
      any = true;
    }
  }
  if (KS == 1 || cnt == nullptr) return;
  // fixup: the workgroup's adds are complete (returning atomics + drain) before its arrival
  xcd_drain(sink);
  (void)any;
  __syncthreads();
  __shared__ int last_s;
  const int tile = blockIdx.y * gridDim.x + blockIdx.x;
  if (threadIdx.x == 0) last_s = atomicAdd(&cnt[tile], 1) == KS - 1;
  __syncthreads();
  if (!last_s) return;
  // last arrival: every slice's adds landed (memory-side, coherent across XCDs); take + epilogue
  const int cols = 16 * NB * WN;
  const int c0 = blockIdx.x * cols;
  for (int e = threadIdx.x; e < 16 * MB * cols / 4; e += 256) {
    const int r = e / (cols / 4), cq = e % (cols / 4);
    const int m = m0 + r, n = c0 + 4 * cq;
    if (m >= p.M || n >= p.N) continue;
    float* t = p.ws + (long long)m * p.N + n;
    f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = xcd_take(t + j);
    sg_store<F16>(p, m, n, v);
  }
  if (threadIdx.x == 0) atomicExch(&cnt[tile], 0);
}

// C = epilogue(Σ_z ws[z]) in a fixed order; 4 columns per thread (N % 4 == 0).
template <bool F16>
__global__ __launch_bounds__(256) void small_gemm_finish(SgArgs p, int KS) {
  const long long MN = (long long)p.M * p.N, q = MN / 4;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < q; i += (long long)gridDim.x * 256) {
    const long long e = i * 4;
    const int m = (int)(e / p.N), n = (int)(e - (long long)m * p.N);
    f32x4 v = *reinterpret_cast<const f32x4*>(p.ws + e);
    for (int z = 1; z < KS; ++z) v += *reinterpret_cast<const f32x4*>(p.ws + z * MN + e);
    sg_store<F16>(p, m, n, v);
  }
}

template <bool F16, int MB, int NB, int WN>
void sg_launch(const SgArgs& p, int ks, int depth, int* cnt, hipStream_t st) {
  dim3 grid((p.N + 16 * NB * WN - 1) / (16 * NB * WN), (p.M + 16 * MB - 1) / (16 * MB), ks);
  if (p.ln_c1) {  // LayerNorm fold (ks == 1 checked by the caller)
    if constexpr (WN == 1) {
      if ((depth >> 4) == 4) {  // weight stream 4 k64 steps deep (the M = 128 BERT configs)
        hipLaunchKernelGGL((small_gemm_kernel<F16, MB, NB, 1, 1, true, 4>), grid, dim3(256), 0, st, p, cnt);
        return;
      }
      if ((depth >> 4) == 2) {  // 2 deep (serving-batch decode, M = 32)
        hipLaunchKernelGGL((small_gemm_kernel<F16, MB, NB, 1, 1, true, 2>), grid, dim3(256), 0, st, p, cnt);
        return;
      }
    }
    if ((depth & 15) >= 2)
      hipLaunchKernelGGL((small_gemm_kernel<F16, MB, NB, WN, 2, true>), grid, dim3(256), 0, st, p, cnt);
    else
      hipLaunchKernelGGL((small_gemm_kernel<F16, MB, NB, WN, 1, true>), grid, dim3(256), 0, st, p, cnt);
    return;
  }
  // depth = A depth | (B depth << 4); B depths 2 / 4 / 8 with A depth 1, one wave column (WN = 1)
  const int db = depth >> 4;
  if constexpr (WN == 1) {
    if (db == 2 || db == 4 || db == 8) {
      if ((depth & 15) != 1) return;
      if (db == 2)
        hipLaunchKernelGGL((small_gemm_kernel<F16, MB, NB, 1, 1, false, 2>), grid, dim3(256), 0, st, p, cnt);
      else if (db == 4)
        hipLaunchKernelGGL((small_gemm_kernel<F16, MB, NB, 1, 1, false, 4>), grid, dim3(256), 0, st, p, cnt);
      else
        hipLaunchKernelGGL((small_gemm_kernel<F16, MB, NB, 1, 1, false, 8>), grid, dim3(256), 0, st, p, cnt);
      return;
    }
  }
  if ((depth & 15) >= 2)
    hipLaunchKernelGGL((small_gemm_kernel<F16, MB, NB, WN, 2>), grid, dim3(256), 0, st, p, cnt);
  else
    hipLaunchKernelGGL((small_gemm_kernel<F16, MB, NB, WN, 1>), grid, dim3(256), 0, st, p, cnt);
}

template <bool F16, int WN>
int sg_dispatch_wn(const SgArgs& p, int mb, int nb, int ks, int depth, int* cnt, hipStream_t st) {
#define SG_CASE(M_, N_) \
  if (mb == M_ && nb == N_) { sg_launch<F16, M_, N_, WN>(p, ks, depth, cnt, st); return 0; }
  SG_CASE(1, 1) SG_CASE(1, 2) SG_CASE(1, 4)
  SG_CASE(2, 1) SG_CASE(2, 2) SG_CASE(2, 4)
  SG_CASE(4, 1) SG_CASE(4, 2) SG_CASE(4, 4)
  SG_CASE(8, 1) SG_CASE(8, 2)
#undef SG_CASE
  return (int)hipErrorInvalidValue;
}

template <bool F16>
int sg_dispatch(const SgArgs& p, int mb, int nb, int wn, int ks, int depth, int* cnt, hipStream_t st) {
  if (wn == 1) return sg_dispatch_wn<F16, 1>(p, mb, nb, ks, depth, cnt, st);
  if (wn == 2) return sg_dispatch_wn<F16, 2>(p, mb, nb, ks, depth, cnt, st);
  if (wn == 4) return sg_dispatch_wn<F16, 4>(p, mb, nb, ks, depth, cnt, st);
  return (int)hipErrorInvalidValue;
}

}  // namespace

// f16: fp16 operands / 16-bit output (else bf16). mb ∈ {1,2,4,8} (TM = 16·mb rows), nb ∈ {1,2,4}
// (mb·nb ≤ 16), wn ∈ {1,2,4} waves along N (TN = 16·nb·wn columns; the other 4/wn waves split K),
// depth ∈ {1,2} k64 steps of loads in flight per wave (| DB << 4, DB ∈ {2,4,8}: with depth 1 and
// wn 1, DB steps of B — the weight stream — in flight, A one step), ks ≥ 1 K slices. ks > 1: cnt != null → fixup mode (ws = M·N f32 and cnt = tiles ints, both
// zeroed, left zeroed); cnt == null → slice mode (ws = ks·M·N f32 + a finish launch).
// bias / resid: 16-bit, nullable. act: 0 none, 1 gelu_tanh, 2 gelu_erf, 3 relu, 4 silu, 5 tanh.
// ln_c1 / ln_b2 (f32 [N], both or neither): LayerNorm fold — C = act(LN(A)·Bᵀ + bias) with B the
// folded weight B∘γ, c1 its row sums and b2 = bias + B·β (the bias argument is then ignored);
// ks == 1, alpha == 1; ln_stats (f32 [M][2], nullable): the (mean, rstd) of each raw A row out.
// rln_stats (f32 [M][2]) + rln_g / rln_b (16-bit [N]), with resid: the residual is a raw row whose
// LayerNorm its producer deferred — LN(resid) = (r − mean)·rstd·γ + β is added instead of r.
PIAMD_EXPORT int piamd_small_gemm_ln(int f16, const void* a, long long lda, const void* b,
                                     long long ldb, void* c, long long ldc, int c_f32, int M, int N,
                                     int K, int mb, int nb, int wn, int depth, int ks, float alpha,
                                     const void* bias, int act, const void* resid, long long ldr,
                                     float* ws, int* cnt, const float* ln_c1, const float* ln_b2,
                                     float ln_eps, float* ln_stats, const float* rln_stats,
                                     const void* rln_g, const void* rln_b, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || N % 4 || lda % 8 || ldb % 8 || ldc % 4 || ks < 1 ||
      ks > K / 64 || (ks > 1 && !ws) || ((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) % 16)
    return (int)hipErrorInvalidValue;
  if ((ln_c1 != nullptr) != (ln_b2 != nullptr) || (ln_c1 && (ks != 1 || alpha != 1.f)) ||
      (ln_stats && !ln_c1))
    return (int)hipErrorInvalidValue;
  if (rln_stats && (!resid || !rln_g || !rln_b)) return (int)hipErrorInvalidValue;
  {  // depth: A depth 1 | 2, optionally | (B depth 2 / 4 / 8) << 4 with A depth 1, wn 1 (LN fold: 2 / 4)
    const int da = depth & 15, db = depth >> 4;
    if (da < 1 || da > 2 || (db && (da != 1 || wn != 1 || (ln_c1 && db != 2 && db != 4) || (db != 2 && db != 4 && db != 8))))
      return (int)hipErrorInvalidValue;
  }
  SgArgs p{(const bf16_t*)a, lda, (const bf16_t*)b, ldb, c, ldc, ws, (const bf16_t*)bias,
           (const bf16_t*)resid, ldr, alpha, M, N, K, c_f32, act, ln_c1, ln_b2, ln_eps, ln_stats,
           rln_stats, (const bf16_t*)rln_g, (const bf16_t*)rln_b};
  int* kc = ks > 1 ? cnt : nullptr;
  const int rc = f16 ? sg_dispatch<true>(p, mb, nb, wn, ks, depth, kc, st)
                     : sg_dispatch<false>(p, mb, nb, wn, ks, depth, kc, st);
  if (rc) return rc;
  if (ks > 1 && !cnt) {
    const int grid = stride_grid((long long)M * N / 4, 256);
    if (f16) hipLaunchKernelGGL(small_gemm_finish<true>, dim3(grid), dim3(256), 0, st, p, ks);
    else hipLaunchKernelGGL(small_gemm_finish<false>, dim3(grid), dim3(256), 0, st, p, ks);
  }
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_small_gemm(int f16, const void* a, long long lda, const void* b, long long ldb,
                                  void* c, long long ldc, int c_f32, int M, int N, int K, int mb,
                                  int nb, int wn, int depth, int ks, float alpha, const void* bias,
                                  int act, const void* resid, long long ldr, float* ws, int* cnt,
                                  hipStream_t st) {
  return piamd_small_gemm_ln(f16, a, lda, b, ldb, c, ldc, c_f32, M, N, K, mb, nb, wn, depth, ks,
                             alpha, bias, act, resid, ldr, ws, cnt, nullptr, nullptr, 0.f, nullptr,
                             nullptr, nullptr, nullptr, st);
}
