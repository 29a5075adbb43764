// bf16 MFMA GEMM with fused epilogues, C[M,N] = A[M,K] · B[K,N] (f32 accumulate).
//
// Parity: reference `paddle/phi/kernels/funcs/blas` matmul + `fused_gemm_epilogue_op.cu`
// (cublasLt epilogues: bias, bias+GELU with aux, dGELU) used by FusedFeedForward / fused_linear.
// The dense GEMMs of the framework run on the assembly GEMM (csrc/asm/gemm_gen.py) and the skinny
// kernel (gemm_small.hip); this file's main loop and epilogue serve the grouped MoE expert GEMMs
// and the implicit-GEMM convolutions below.
//
// Structure (cdna_hip_programming.md §5: 256² tile, glds, BK = 64):
//   * workgroup = 8 waves (2 M × 4 N), tile 256 × 256, each wave 128 × 64 = 4 × 2 blocks of
//     v_mfma_f32_32x32x16_bf16; SWAPPED operands (Cᵀ = Bᵀ·Aᵀ) so each lane owns one output row
//     and 4 consecutive columns per register quad → 8-byte epilogue stores;
//   * both operands staged global → LDS with global_load_lds_dwordx4 (no VGPR round trip) into two
//     LDS stages (128 KiB), the next K-tile's DMA in flight under the current tile's MFMAs;
//   * operand layouts: K-contiguous (row-major A, or B given as [N][K]) images are read with
//     ds_read_b128; M/N-contiguous images (row-major B = weights [K][N], or A given as [K][M] for
//     weight gradients) with the hardware transpose read ds_read_b64_tr_b16 — so forward,
//     data-gradient and weight-gradient GEMMs all run without a transpose kernel;
//   * XOR-swizzled LDS images (swizzle applied to the per-lane global SOURCE address, the LDS
//     side of a DMA being lane-linear) keep both read kinds bank-conflict free;
//   * bijective XCD-aware tile order: consecutive tiles of one XCD share an A row-panel in L2.
#include "common.h"

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;

constexpr int BM = 256, BN = 256, BK = 64, NWAVE = 8, NTHR = NWAVE * 64;
constexpr int TILE_BYTES = 256 * BK * 2;            // one operand image per stage (32 KiB)
constexpr int STAGE_BYTES = 2 * TILE_BYTES;
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));

// One 32×32×16 MFMA step on 16-bit operand fragments carried as raw bits: bf16 or IEEE fp16.
template <bool F16>
__device__ __forceinline__ f32x16 mma32(bf16x8 a, bf16x8 b, f32x16 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a),
                                                  __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// XOR image with ROWB-byte rows (16-B chunks permuted by the low row bits).
template <int ROWB>
__device__ __forceinline__ int img_off(int row, int ch) {
  constexpr int CH = ROWB / 16;
  const int x = ((((row & 3) << 2) | ((row >> 2) & 3)) ^ ((row >> 4) & 0)) & (CH - 1);
  return row * ROWB + ((ch ^ x) << 4);
}

__device__ __forceinline__ bf16x8 rd_row(const char* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}

template <int ROWB>
__device__ __forceinline__ s16x4_t rd_tr4(const char* base, int r0, int c0, int gi) {
  const int q = gi >> 2, p = gi & 3;
  const int col = c0 + 4 * p;
  const int off = img_off<ROWB>(r0 + q, col >> 3) + ((col & 7) << 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off));
}

__device__ __forceinline__ bf16x8 cat44(s16x4_t a, s16x4_t b) {
  s16x8 t = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, t);
}

// DMA a [ROWS][ROWB] bf16 tile (row r at gbase + min(r0 + r, rmax) * ld, 16-B chunk c at +8c)
// into the XOR image at `img`; NWAVE waves share the pieces (1 KiB per wave-instruction).
template <int ROWS, int ROWB>
__device__ __forceinline__ void dma_tile(const bf16_t* gbase, long long ld, int r0, int rmax,
                                         char* img, int w, int lane) {
  constexpr int CH = ROWB / 16;
  constexpr int PIECES = ROWS * ROWB / 1024;
  constexpr int PPW = PIECES / NWAVE;
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int P = w * PPW + i;
    const int L = P * 64 + lane, r = L / CH, pc = L % CH;
    const int x = (((r & 3) << 2) | ((r >> 2) & 3)) & (CH - 1);
    const long long row = min(r0 + r, rmax);
    const bf16_t* src = gbase + row * ld + ((pc ^ x) << 3);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(img + P * 1024),
                                     16, 0, 0);
  }
}

__device__ __forceinline__ float act_fwd(float v, int act) {
  switch (act) {
    case 1: return gelu_tanh(v);
    case 2: return gelu_erf(v);
    case 3: return fmaxf(v, 0.f);
    case 4: return v / (1.f + __expf(-v));
    default: return v;
  }
}
__device__ __forceinline__ float act_grad(float h, int act) {
  switch (act) {
    case 1: return gelu_tanh_grad(h);
    case 2: return gelu_erf_grad(h);
    case 3: return h > 0.f ? 1.f : 0.f;
    case 4: { const float s = 1.f / (1.f + __expf(-h)); return s * (1.f + h * (1.f - s)); }
    default: return 1.f;
  }
}

// Epilogue kinds
enum { EPI_STORE = 0, EPI_BIAS_ACT = 1, EPI_DACT = 2 };

// Main loop: acc = A[m0:m0+256, kbase:kbase+64·nk] · B[kbase:…, n0:n0+256].
// A_KC: A[m][k] at a + m*lda + k (rows clamped to amax) — else A[m][k] at a + k*lda + m.
// B_KC: B[k][n] at b + n*ldb + k (rows clamped to bmax) — else B[k][n] at b + k*ldb + n.
template <bool A_KC, bool B_KC>
__device__ __forceinline__ void gemm_mainloop(const bf16_t* __restrict__ a, long long lda, int amax,
                                              const bf16_t* __restrict__ b, long long ldb, int bmax,
                                              int m0, int n0, long long kbase, int nk, char* smem,
                                              f32x16 (&acc)[4][2]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;  // 2 (M) x 4 (N) waves
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  if (nk <= 0) return;

  auto stage_load = [&](int kt, int s) {
    char* ai = smem + s * STAGE_BYTES;
    char* bi = ai + TILE_BYTES;
    const long long k0 = kbase + (long long)kt * BK;
    if (A_KC) dma_tile<256, 128>(a + k0, lda, m0, amax, ai, w, lane);         // [256 m][64 k]
    else      dma_tile<64, 512>(a + k0 * lda + m0, lda, 0, 63, ai, w, lane);  // [64 k][256 m]
    if (B_KC) dma_tile<256, 128>(b + k0, ldb, n0, bmax, bi, w, lane);         // [256 n][64 k]
    else      dma_tile<64, 512>(b + k0 * ldb + n0, ldb, 0, 63, bi, w, lane);  // [64 k][256 n]
  };

  stage_load(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int gi = lane & 15, hi = lane >> 5, half16 = (lane >> 4) & 1, l31 = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt & 1;
    if (kt + 1 < nk) stage_load(kt + 1, s ^ 1);
    const char* ai = smem + s * STAGE_BYTES;
    const char* bi = ai + TILE_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 af[4], bf[2];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        const int mrow = wr * 128 + mb * 32;
        if (A_KC) af[mb] = rd_row(ai, img_off<128>(mrow + l31, 2 * ks + hi));
        else af[mb] = cat44(rd_tr4<512>(ai, 16 * ks + 8 * hi, mrow + 16 * half16, gi),
                            rd_tr4<512>(ai, 16 * ks + 8 * hi + 4, mrow + 16 * half16, gi));
      }
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int ncol = wc * 64 + nb * 32;
        if (B_KC) bf[nb] = rd_row(bi, img_off<128>(ncol + l31, 2 * ks + hi));
        else bf[nb] = cat44(rd_tr4<512>(bi, 16 * ks + 8 * hi, ncol + 16 * half16, gi),
                            rd_tr4<512>(bi, 16 * ks + 8 * hi + 4, ncol + 16 * half16, gi));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[nb], af[mb], acc[mb][nb], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// Epilogue: waves laid out WM (M) × 8/WM (N), each MB × NB blocks of 32 × 32 (default: the 256²
// tile, 2 × 4 waves of 4 × 2). Lane owns row m0 + wr·32MB + mb·32 + l31 (stored while < mend);
// columns n = n0 + wc·32NB + nb·32 + 8g + 4·hi + (0..3) (stored while < N).
// Output-row remap of a phase convolution (the strided data gradient): row m = (img, oh, ow) of
// the OHp × OWp phase grid lands on pixel (img, oh·st_h + ph, ow·st_w + pw) of an H × W output.
struct RowMap {
  int ohw_p, ow_p, hw_d, w_d, st_h, st_w, ph, pw;
  __device__ __forceinline__ long long row(int m) const {
    const int img = m / ohw_p, rem = m - img * ohw_p, oh = rem / ow_p, ow = rem - oh * ow_p;
    return (long long)img * hw_d + (long long)(oh * st_h + ph) * w_d + ow * st_w + pw;
  }
};

template <int WM = 2, int MB = 4, int NB = 2, bool F16 = false>
__device__ __forceinline__ void gemm_epilogue(const f32x16 (&acc)[MB][NB], void* __restrict__ c,
                                              long long ldc, int c_f32, int accumulate, int m0,
                                              int mend, int n0, int N, int epi, int act,
                                              const bf16_t* __restrict__ bias,
                                              bf16_t* __restrict__ aux, long long ldaux,
                                              const RowMap* rmap = nullptr) {
  constexpr int WC = NWAVE / WM;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w / WC, wc = w % WC;
  const int hi = lane >> 5, l31 = lane & 31;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int m = m0 + wr * (32 * MB) + mb * 32 + l31;
    if (m >= mend) continue;
    const long long mr = rmap ? rmap->row(m) : (long long)m;  // destination row
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wc * (32 * NB) + nb * 32 + 8 * g + 4 * hi;
        if (n >= N) continue;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = acc[mb][nb][4 * g + j];
        if (epi == EPI_BIAS_ACT) {
          u16x4 pre;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] += bias ? h2f<F16>(bias[n + j]) : 0.f;
            pre[j] = f2h<F16>(v[j]);
            v[j] = act_fwd(h2f<F16>(pre[j]), act);
          }
          if (aux) *reinterpret_cast<u16x4*>(aux + (long long)m * ldaux + n) = pre;
        } else if (epi == EPI_DACT) {
          const u16x4 h = *reinterpret_cast<const u16x4*>(aux + (long long)m * ldaux + n);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] *= act_grad(h2f<F16>(h[j]), act);
        }
        if (c_f32) {
          f32x4* p = reinterpret_cast<f32x4*>((float*)c + mr * ldc + n);
          f32x4 o = accumulate ? *p : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] += v[j];
          *p = o;
        } else {
          u16x4 o;
          bf16_t* p = (bf16_t*)c + mr * ldc + n;
          if (accumulate) {
            const u16x4 old = *reinterpret_cast<const u16x4*>(p);
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = f2h<F16>(v[j] + h2f<F16>(old[j]));
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = f2h<F16>(v[j]);
          }
          *reinterpret_cast<u16x4*>(p) = o;
        }
      }
    }
  }
}

// bijective XCD-aware tile order (guide T1): consecutive tiles of one XCD share an A row-panel
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig % 8, q = nwg / 8, rr = nwg % 8;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
}

// ---- grouped (MoE expert) GEMMs over expert-sorted rows --------------------------------------
// Parity: reference `fluid/operators/fused/moe_expert_gemm.h` / `fused_moe_op.cu` (CUTLASS grouped
// GEMM over per-expert row ranges). Rows of expert e occupy [offs[e], offs[e+1]) of the sorted
// activation matrix; the offsets live on the device, so routing never synchronises with the host
// and the launch is hipGraph-capturable. The grid is sized for the worst case
// (ceil(rows_cap/256) + E row tiles × N tiles); every workgroup finds its expert by scanning the
// per-expert tile counts (wave-uniform scalar loads), surplus workgroups exit at once.
__device__ __forceinline__ bool moe_find_tile(const int* __restrict__ offs, int E, int t, int& e,
                                              int& r0, int& r1) {
  int acc = 0;
  for (int i = 0; i < E; ++i) {
    const int b0 = offs[i], b1 = offs[i + 1];
    const int nt = (b1 - b0 + BM - 1) / BM;
    if (t < acc + nt) {
      e = i;
      r0 = b0 + (t - acc) * BM;
      r1 = b1;
      return true;
    }
    acc += nt;
  }
  return false;
}

// Y[rows] = X[rows] · W_e (+ bias_e, act): B_KC=false → W_e stored [K][N] (w + e*sw);
// B_KC=true → W_e stored [N][K] (also the data-gradient dX = dY · W_eᵀ of a [K_in][N] weight).
template <bool B_KC>
__global__ __launch_bounds__(NTHR, 1) void moe_gemm_kernel(
    const bf16_t* __restrict__ x, long long ldx, const bf16_t* __restrict__ w, long long ldw,
    long long sw, const int* __restrict__ offs, int E, void* __restrict__ y, long long ldy,
    int y_f32, int N, int K, int tm_max, int epi, int act, const bf16_t* __restrict__ bias,
    bf16_t* __restrict__ aux, long long ldaux) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES];
  const int tn = (N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, tm_max * tn);
  int e, r0, r1;
  if (!moe_find_tile(offs, E, wg / tn, e, r0, r1)) return;
  const int n0 = (wg % tn) * BN;
  f32x16 acc[4][2];
  gemm_mainloop<true, B_KC>(x, ldx, r1 - 1, w + e * sw, ldw, N - 1, r0, n0, 0, K / BK, smem, acc);
  gemm_epilogue(acc, y, ldy, y_f32, 0, r0, r1, n0, N, epi, act,
                bias ? bias + (long long)e * N : nullptr, aux, ldaux);
}

// Weight gradient per expert: dW_e[M=K_in][N] (+)= X_eᵀ · dY_e, reduced over the expert's rows.
// Segments must be padded to multiples of 64 rows with ZERO rows (moe_permute(align=64)).
__global__ __launch_bounds__(NTHR, 1) void moe_wgrad_kernel(
    const bf16_t* __restrict__ x, long long ldx, const bf16_t* __restrict__ dy, long long lddy,
    const int* __restrict__ offs, int E, void* __restrict__ dw, long long sdw, int dw_f32,
    int accumulate, int M, int N) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES];
  const int tn = N / BN, per = (M / BM) * tn;
  const int wg = xcd_remap(blockIdx.x, per * E);
  const int e = wg / per, t = wg % per, m0 = (t / tn) * BM, n0 = (t % tn) * BN;
  const int r0 = offs[e], r1 = offs[e + 1];
  if (r1 == r0 && accumulate) return;  // empty expert: nothing to add
  f32x16 acc[4][2];
  gemm_mainloop<false, false>(x, ldx, 0, dy, lddy, 0, m0, n0, r0, (r1 - r0) / BK, smem, acc);
  void* out = dw_f32 ? (void*)((float*)dw + e * sdw) : (void*)((bf16_t*)dw + e * sdw);
  gemm_epilogue(acc, out, N, dw_f32, accumulate, m0, M, n0, N, EPI_STORE, 0, nullptr, nullptr, 0);
}

// ---- implicit-GEMM convolution (NHWC, bf16) ---------------------------------------------------
// Parity: reference `phi/kernels/gpudnn/conv_kernel.cu` / `conv_grad_kernel.cu` (cuDNN) — here an
// MFMA implicit GEMM: Y[m = (n, oh, ow)][k_out] = Σ_{(r, s, c)} X[n, oh·st − pad + r·dil,
// ow·st − pad + s·dil, c] · W[k_out][(r, s, c)], the A tile gathered straight from the NHWC
// activation by the global→LDS DMA (one 128-byte channel run of one input pixel per 8 lanes; out-of-
// image taps read a zero row), W in OHWI = [K_out][R·S·C] (K-contiguous B operand). Same 256² tile,
// XOR-swizzled LDS images and MFMA loop as gemm_kernel; bias + activation fused in the epilogue.
// Requires C % 64 == 0 (a 64-channel k-step never straddles two taps) and K_out % 4 == 0.
// Per-tile BatchNorm statistics of the stored (16-bit-rounded) conv outputs, for the BN that
// follows (it then skips its own statistics pass over the output): (count, mean, M2) of every
// column over the tile's valid rows → stats[(k·Kout + n)·P + tile_m] (k = 0 count, 1 mean, 2 M2;
// channel-major, so the finalize reads each channel's P partials contiguously).
// Each wave transposes its outputs through a private LDS image (rows of 64 columns, 136-B
// stride: the 8-B row writes of a lane column are conflict-free), ≤ 64 rows at a time; lane pair
// (c2, c2 + 32) then sums columns 2·c2 and 2·c2 + 1 down alternate rows (4-B reads), shifted by
// the columns' first values (no cancellation against a large mean). The WM waves of a column merge in LDS (Chan's formula).
template <int WM, int MB, int NB, bool F16>
__device__ __forceinline__ void conv_tile_stats(const f32x16 (&acc)[MB][NB], char* smem, float* __restrict__ stats,
                                                int m0, int M, int n0, int Kout, int tile_m, int P) {
  constexpr int WC = NWAVE / WM, TN = WC * NB * 32;
  constexpr int COLS = NB * 32;            // a wave's columns (one per lane)
  constexpr int RSB = COLS * 2 + 8;        // image row stride (bytes)
  constexpr int MBP = MB < 2 ? MB : 2;     // 32-row blocks per transposition pass
  constexpr int WIMG = 32 * MBP * RSB;     // a wave's image
  static_assert(COLS == 64, "one column per lane");
  static_assert(NWAVE * WIMG <= 2 * (256 * 64 * 2 + 64 * 64 * 2), "images fit the smallest tile's LDS");
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w / WC, wc = w % WC;
  const int hi = lane >> 5, l31 = lane & 31;
  const int rbase = m0 + wr * 32 * MB;
  const int nw = max(0, min(32 * MB, M - rbase));  // valid rows of this wave
  char* img = smem + w * WIMG;
  __syncthreads();  // the main loop's LDS images are dead
  const int half = lane >> 5, c2 = lane & 31;
  float sh0 = 0.f, sh1 = 0.f, s0 = 0.f, q0 = 0.f, s1 = 0.f, q1 = 0.f;
#pragma unroll
  for (int p = 0; p < MB / MBP; ++p) {
#pragma unroll
    for (int i = 0; i < MBP; ++i) {
      const int mb = p * MBP + i;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          u16x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = f2h<F16>(acc[mb][nb][4 * g + j]);
          *reinterpret_cast<u16x4*>(img + (i * 32 + l31) * RSB + (nb * 32 + 8 * g + 4 * hi) * 2) = o;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // lane (half, c2): columns 2·c2, 2·c2 + 1 over the pass's rows half, half + 2, … (one 4-B read
    // per row for two columns)
    const int rows = min(32 * MBP, nw - p * 32 * MBP);  // valid rows of this pass
    if (p == 0 && nw > 0) {
      const unsigned u = *reinterpret_cast<const unsigned*>(img + c2 * 4);
      sh0 = h2f<F16>((unsigned short)(u & 0xFFFF));
      sh1 = h2f<F16>((unsigned short)(u >> 16));
    }
#pragma unroll 8
    for (int r = half; r < 32 * MBP; r += 2) {
      if (r < rows) {
        const unsigned u = *reinterpret_cast<const unsigned*>(img + r * RSB + c2 * 4);
        const float d0 = h2f<F16>((unsigned short)(u & 0xFFFF)) - sh0;
        const float d1 = h2f<F16>((unsigned short)(u >> 16)) - sh1;
        s0 += d0;
        q0 += d0 * d0;
        s1 += d1;
        q1 += d1 * d1;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // the two row halves share the shift: their sums add
  s0 += __shfl_xor(s0, 32, 64);
  q0 += __shfl_xor(q0, 32, 64);
  s1 += __shfl_xor(s1, 32, 64);
  q1 += __shfl_xor(q1, 32, 64);
  __syncthreads();  // every image read; the merge table reuses the front of smem
  float* red = reinterpret_cast<float*>(smem);  // [WM][TN][3]
  {
    // lanes 0-31 hold column 2·c2, lanes 32-63 (same sums) store column 2·c2 + 1
    const int cl = wc * COLS + 2 * c2 + half;
    const float n = (float)nw, sh = half ? sh1 : sh0, s = half ? s1 : s0, q = half ? q1 : q0;
    float* r = red + (wr * TN + cl) * 3;
    r[0] = n;
    r[1] = nw ? sh + s / n : 0.f;
    r[2] = nw ? fmaxf(q - s * s / n, 0.f) : 0.f;
  }
  __syncthreads();
  for (int cl = tid; cl < TN; cl += NTHR) {
    const int n = n0 + cl;
    if (n >= Kout) continue;
    float cn = 0.f, cm = 0.f, cm2 = 0.f;
#pragma unroll
    for (int r = 0; r < WM; ++r) {
      const float* e = red + (r * TN + cl) * 3;
      const float nb = e[0];
      if (nb == 0.f) continue;
      const float nn = cn + nb, d = e[1] - cm;
      cm += d * nb / nn;
      cm2 += e[2] + d * d * cn * nb / nn;
      cn = nn;
    }
    stats[((long long)0 * Kout + n) * P + tile_m] = cn;
    stats[((long long)1 * Kout + n) * P + tile_m] = cm;
    stats[((long long)2 * Kout + n) * P + tile_m] = cm2;
  }
}

struct ConvGeom {
  int N, H, W, C, OH, OW, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w;
};

// Tile 256 (M) × TN (N), TN = 8/WM · 32·NB: WM=2,MB=4,NB=2 → 256² (K_out ≥ 256); WM=4,MB=2,NB=2 →
// 256 × 128; WM=8,MB=1,NB=2 → 256 × 64 (narrow layers keep every MFMA column useful).
// ksplit > 1: workgroup (tile, part) reduces k-steps [part·nk/ksplit, (part+1)·nk/ksplit) into an
// f32 partial plane ws[part][M][K_out]; conv_splitk_finish sums the planes (fixed order:
// deterministic) and applies bias + activation — fills the chip on the small late-stage layers.
// SC (small-channel stem mode, C == 8: image channels zero-padded to 8): a 64-deep k-step holds
// EIGHT taps × 8 channels — 16-B chunk j of k-step kt is tap 8·kt + j — so a 3-channel 7×7 stem runs
// 7 k-steps instead of 49 padded-to-64-channel ones; W is [K_out][ceil(R·S/8)·64] (taps ≥ R·S zero).
template <int WM, int MB, int NB, bool SC = false, bool F16 = false>
__global__ __launch_bounds__(NTHR, 1) void conv_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ wt, const bf16_t* __restrict__ zero,
    bf16_t* __restrict__ y, float* __restrict__ ws, int ksplit, ConvGeom g, int Kout, int act,
    const bf16_t* __restrict__ bias, int yf32, float* __restrict__ stats, RowMap rm, int yacc) {
  constexpr int WC = NWAVE / WM, TN = WC * NB * 32;
  constexpr int B_BYTES = TN * BK * 2, SBYTES = TILE_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[2 * SBYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w / WC, wc = w % WC;
  const int M = g.N * g.OH * g.OW;
  const int tm = (M + BM - 1) / BM, tn = (Kout + TN - 1) / TN;
  const int wg = xcd_remap(blockIdx.x, tm * tn * ksplit);
  const int part = wg % ksplit, tile = wg / ksplit;
  const int m0 = (tile / tn) * BM, n0 = (tile % tn) * TN;
  const int cpt = SC ? 1 : g.C / BK;  // 64-channel k-steps per tap
  const int nk_all = SC ? (g.R * g.S + 7) / 8 : g.R * g.S * cpt;
  const long long RSC = SC ? (long long)nk_all * BK : (long long)g.R * g.S * g.C;
  const int kt0 = (int)((long long)nk_all * part / ksplit);
  const int kt1 = (int)((long long)nk_all * (part + 1) / ksplit);

  // this lane's 4 DMA pieces of the A tile: fixed output pixel per piece, k-step invariant
  constexpr int PPW = 4;
  long long pbase[PPW];
  int ih0[PPW], iw0[PPW], choff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int P = w * PPW + i, L = P * 64 + lane, r = L / 8, pc = L % 8;
    const int xsw = (((r & 3) << 2) | ((r >> 2) & 3)) & 7;
    choff[i] = (pc ^ xsw) << 3;
    const int m = m0 + r;
    if (m < M) {
      const int n = m / (g.OH * g.OW), rem = m % (g.OH * g.OW);
      const int oh = rem / g.OW, ow = rem % g.OW;
      pbase[i] = (long long)n * g.H * g.W;
      ih0[i] = oh * g.st_h - g.pad_h;
      iw0[i] = ow * g.st_w - g.pad_w;
    } else {
      pbase[i] = -1;
      ih0[i] = iw0[i] = 0;
    }
  }
  auto stage_load = [&](int kt, int s) {
    char* ai = smem + s * SBYTES;
    char* bi = ai + TILE_BYTES;
    const int rs = kt / cpt, c0 = (kt % cpt) * BK;
    const int rr = rs / g.S, ss = rs % g.S;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const bf16_t* src;
      if (SC) {
        const int tap = kt * 8 + (choff[i] >> 3), tr = tap / g.S, ts = tap - tr * g.S;
        const int ih = ih0[i] + tr * g.dil_h, iw = iw0[i] + ts * g.dil_w;
        const bool ok = pbase[i] >= 0 && tap < g.R * g.S && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        src = ok ? x + (pbase[i] + (long long)ih * g.W + iw) * 8 : zero;
      } else {
        const int ih = ih0[i] + rr * g.dil_h, iw = iw0[i] + ss * g.dil_w;
        const bool ok = pbase[i] >= 0 && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        src = ok ? x + (pbase[i] + (long long)ih * g.W + iw) * g.C + c0 + choff[i] : zero + choff[i];
      }
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(ai + (w * PPW + i) * 1024),
                                       16, 0, 0);
    }
    dma_tile<TN, 128>(wt + (long long)kt * BK, RSC, n0, Kout - 1, bi, w, lane);
  };

  f32x16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  if (kt1 > kt0) {
    stage_load(kt0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int hi = lane >> 5, l31 = lane & 31;
  for (int kt = kt0; kt < kt1; ++kt) {
    const int s = (kt - kt0) & 1;
    if (kt + 1 < kt1) stage_load(kt + 1, s ^ 1);
    const char* ai = smem + s * SBYTES;
    const char* bi = ai + TILE_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 af[MB], bf[NB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        af[mb] = rd_row(ai, img_off<128>(wr * (32 * MB) + mb * 32 + l31, 2 * ks + hi));
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        bf[nb] = rd_row(bi, img_off<128>(wc * (32 * NB) + nb * 32 + l31, 2 * ks + hi));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[mb][nb] = mma32<F16>(bf[nb], af[mb], acc[mb][nb]);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (ksplit > 1)
    gemm_epilogue<WM, MB, NB>(acc, ws + (long long)part * M * Kout, Kout, 1, 0, m0, M, n0, Kout,
                              EPI_STORE, 0, nullptr, nullptr, 0);
  else if (yf32)  // f32 output (the split-bf16 fp32 convolution): plain store, no epilogue ops
    gemm_epilogue<WM, MB, NB>(acc, (float*)y, Kout, 1, 0, m0, M, n0, Kout, EPI_STORE, 0, nullptr,
                              nullptr, 0, rm.ohw_p ? &rm : nullptr);
  else
    gemm_epilogue<WM, MB, NB, F16>(acc, y, Kout, 0, yacc, m0, M, n0, Kout,
                              (bias || act) ? EPI_BIAS_ACT : EPI_STORE, act, bias, nullptr, 0,
                              rm.ohw_p ? &rm : nullptr);
  if (stats)  // (host: ksplit == 1, 16-bit output without bias / activation)
    conv_tile_stats<WM, MB, NB, F16>(acc, smem, stats, m0, M, n0, Kout, tile / tn, tm);
}

// y[m][n] = act(Σ_p ws[p][m][n] + bias[n]) — 4 outputs per thread (K_out % 4 == 0).
template <bool F16>
__global__ __launch_bounds__(256) void conv_splitk_finish(const float* __restrict__ ws, int ksplit,
                                                          long long MN, int Kout, int act,
                                                          const bf16_t* __restrict__ bias,
                                                          bf16_t* __restrict__ y) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= MN) return;
  f32x4 v = *reinterpret_cast<const f32x4*>(ws + i);
  for (int p = 1; p < ksplit; ++p) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(ws + p * MN + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += t[j];
  }
  const int n = (int)(i % Kout);
  u16x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float h = v[j];
    if (bias || act) h = h2f<F16>(f2h<F16>(h + (bias ? h2f<F16>(bias[n + j]) : 0.f)));
    o[j] = f2h<F16>(act_fwd(h, act));
  }
  *reinterpret_cast<u16x4*>(y + i) = o;
}

// ---- implicit-GEMM convolution weight gradient (NHWC, bf16) -----------------------------------
// Parity: reference `phi/kernels/gpudnn/conv_grad_kernel.cu:666` (cuDNN backward-filter). Here
// D[q = (r, s, c)][k] = Σ_m X[pixel(m, r, s)][c] · dY[m][k] over every output pixel m = (n, oh, ow)
// — a GEMM whose reduction runs over the N·OH·OW output pixels, with D in HWIO order [R][S][C][K].
// Both operands are reduction-major (!KC) LDS images [64 pixels][cols], read with the hardware
// transpose ds_read_b64_tr_b16:
//   * A (M' = the R·S·C filter taps × channels, 256 per tile): gathered by the LDS DMA, each 16-B
//     chunk (8 channels of ONE tap — C % 8 == 0) from the input pixel the tap sees, so a tile packs
//     several taps when C < 256 (a 64-channel 3×3 layer fills 576 rows = 2¼ tiles instead of 9
//     quarter-empty ones); out-of-image taps and pixels past the end read the zero row;
//   * B (N' = K_out, tile TN ∈ {64, 128, 256}): dY rows, plain DMA (K_out % TN == 0);
//   * the reduction (hundreds of thousands of pixels) is split over `ksplit` workgroups per output
//     tile writing f32 partial planes ws[part][RSC][K_out]; conv_splitk_finish-style fixed-order
//     sum (deterministic) into the f32 D.
// pixel(m): m → (n, oh, ow) by an f32 reciprocal with one integer correction (M < 2^24).
struct ConvWgradGeom {
  int N, H, W, C, OH, OW, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w;
  int M, RSC, Kout;
  float inv_ow, inv_ohw;
};

template <int WM, int MB, int NB, bool F16 = false>
__global__ __launch_bounds__(NTHR, 1) void conv_wgrad_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, const bf16_t* __restrict__ zero,
    float* __restrict__ out, int ksplit, ConvWgradGeom g) {
  constexpr int WC = NWAVE / WM, TN = WC * NB * 32;
  constexpr int A_BYTES = 64 * 512, B_BYTES = 64 * TN * 2, SBYTES = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[2 * SBYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w / WC, wc = w % WC;
  const int tm = (g.RSC + BM - 1) / BM, tn = g.Kout / TN;
  const int wg = xcd_remap(blockIdx.x, tm * tn * ksplit);
  const int part = wg % ksplit, tile = wg / ksplit;
  const int m0 = (tile / tn) * BM, n0 = (tile % tn) * TN;
  const int nk_all = (g.M + 63) / 64;
  const int kt0 = (int)((long long)nk_all * part / ksplit);
  const int kt1 = (int)((long long)nk_all * (part + 1) / ksplit);

  // A gather: this lane's 4 pieces (2 pixels × 512 B each); per piece a fixed pixel row r of the
  // 64-pixel step and a fixed 8-channel chunk (tap offset dh/dw, channel c) — k-step invariant
  constexpr int PPW = 4;
  int prow[PPW], pc_off[PPW], pdh[PPW], pdw[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int P = w * PPW + i, L = P * 64 + lane, r = L >> 5, pc = L & 31;
    const int xsw = ((r & 3) << 2) | ((r >> 2) & 3);
    const int q = m0 + ((pc ^ xsw) << 3);
    prow[i] = r;
    if (q < g.RSC) {
      const int tap = q / g.C, c = q - tap * g.C;
      const int rr = tap / g.S, ss = tap - rr * g.S;
      pc_off[i] = c;
      pdh[i] = rr * g.dil_h - g.pad_h;
      pdw[i] = ss * g.dil_w - g.pad_w;
    } else {
      pc_off[i] = -1;
      pdh[i] = pdw[i] = 0;
    }
  }
  const int ohw = g.OH * g.OW;
  auto stage_load = [&](int kt, int s) {
    char* ai = smem + s * SBYTES;
    char* bi = ai + A_BYTES;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int m = kt * 64 + prow[i];
      int n = (int)((float)m * g.inv_ohw);
      int rem = m - n * ohw;
      if (rem < 0) { --n; rem += ohw; } else if (rem >= ohw) { ++n; rem -= ohw; }
      int oh = (int)((float)rem * g.inv_ow);
      int ow = rem - oh * g.OW;
      if (ow < 0) { --oh; ow += g.OW; } else if (ow >= g.OW) { ++oh; ow -= g.OW; }
      const int ih = oh * g.st_h + pdh[i], iw = ow * g.st_w + pdw[i];
      const bool ok = m < g.M && pc_off[i] >= 0 && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
      const bf16_t* src = ok ? x + (((long long)n * g.H + ih) * g.W + iw) * g.C + pc_off[i] : zero;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(ai + (w * PPW + i) * 1024),
                                       16, 0, 0);
    }
    // dY rows past the end are clamped (finite data against the zero A rows)
    dma_tile<64, TN * 2>(dy + n0, g.Kout, kt * 64, g.M - 1, bi, w, lane);
  };

  f32x16 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  if (kt1 > kt0) {
    stage_load(kt0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int gi = lane & 15, hi = lane >> 5, half16 = (lane >> 4) & 1;
  for (int kt = kt0; kt < kt1; ++kt) {
    const int s = (kt - kt0) & 1;
    if (kt + 1 < kt1) stage_load(kt + 1, s ^ 1);
    const char* ai = smem + s * SBYTES;
    const char* bi = ai + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 af[MB], bf[NB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int mrow = wr * (32 * MB) + mb * 32;
        af[mb] = cat44(rd_tr4<512>(ai, 16 * ks + 8 * hi, mrow + 16 * half16, gi),
                       rd_tr4<512>(ai, 16 * ks + 8 * hi + 4, mrow + 16 * half16, gi));
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int ncol = wc * (32 * NB) + nb * 32;
        bf[nb] = cat44(rd_tr4<TN * 2>(bi, 16 * ks + 8 * hi, ncol + 16 * half16, gi),
                       rd_tr4<TN * 2>(bi, 16 * ks + 8 * hi + 4, ncol + 16 * half16, gi));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[mb][nb] = mma32<F16>(bf[nb], af[mb], acc[mb][nb]);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  gemm_epilogue<WM, MB, NB>(acc, out + (long long)part * g.RSC * g.Kout, g.Kout, 1, 0, m0, g.RSC,
                            n0, g.Kout, EPI_STORE, 0, nullptr, nullptr, 0);
}

// D (+)= Σ_p ws[p] in a fixed order (f32, 4 per thread). SL slices of the ksplit planes per output
// vector (slice s sums planes s, s + SL, …; then slices 0..SL-1 in order through LDS): with many
// split parts over a small filter (ks up to 256 planes of a 1×1 layer) a one-thread-per-output
// loop was a long serial chain on a handful of workgroups.
template <int SL>
__global__ __launch_bounds__(256) void wgrad_splitk_finish(const float* __restrict__ ws, int ksplit,
                                                           long long MN, float* __restrict__ d,
                                                           int accumulate, int Kout, int C) {
  constexpr int VPB = 256 / SL;  // output vectors per block
  const int t = threadIdx.x, vl = t % VPB, sl = t / VPB;
  const long long i = ((long long)blockIdx.x * VPB + vl) * 4;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (i < MN)
    for (int p = sl; p < ksplit; p += SL) v += *reinterpret_cast<const f32x4*>(ws + p * MN + i);
  if constexpr (SL > 1) {
    __shared__ f32x4 red[256];
    red[t] = v;
    __syncthreads();
    if (sl) return;
    for (int k = 1; k < SL; ++k) v += red[k * VPB + vl];
  }
  if (i >= MN) return;
  if (accumulate & 6) {  // OHWI d[k][rsc] (channels_last filter) or KCRS d[k][c][rs] (contiguous)
    const long long RSC = MN / Kout, rsc = i / Kout;
    const int k = (int)(i - rsc * Kout);
    long long off = rsc;
    if (accumulate & 4) {  // rsc = rs·C + c  →  c·RS + rs
      const long long rs = rsc / C, c = rsc - rs * C;
      off = c * (RSC / C) + rs;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float* o = d + (long long)(k + j) * RSC + off;
      *o = (accumulate & 1) ? *o + v[j] : v[j];
    }
    return;
  }
  f32x4* o = reinterpret_cast<f32x4*>(d + i);
  if (accumulate) v += *o;
  *o = v;
}

// ---- int8 × int8 → int32 GEMM with dequantising epilogue -------------------------------------
// Parity: reference `fused_multi_transformer_int8_op.cu` / `attn_gemm_int8.h` (cublasLt int8
// igemm between quantised activations and int8 weights, dequantised with per-channel out scales)
// and `llm_int8_linear`. Y[M][N] = act((Xq[M][K] · Wq[N][K]ᵀ) · xs[m] · ws[n] + bias[n]).
// Same 256×256 tile / glds double buffer / XOR images as the bf16 kernel: a 128-byte LDS row holds
// 128 int8 (instead of 64 bf16), so the DMA and the 16-byte fragment reads are unchanged and each
// 16-B fragment feeds one v_mfma_i32_32x32x32_i8 (k = 16·half + j) — twice the bf16 MFMA rate.
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x16_t __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(NTHR, 1) void gemm_i8_kernel(
    const signed char* __restrict__ x, long long ldx, const signed char* __restrict__ wq,
    long long ldw, const float* __restrict__ xs, float xs_const, const float* __restrict__ ws,
    const bf16_t* __restrict__ bias, bf16_t* __restrict__ y, long long ldy, int M, int N, int K,
    int act) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int tm = (M + BM - 1) / BM, tn = (N + BN - 1) / BN;
  const int wg = xcd_remap(blockIdx.x, tm * tn);
  const int m0 = (wg / tn) * BM, n0 = (wg % tn) * BN;
  // byte matrices viewed as 2-byte elements for the shared DMA helper
  const bf16_t* xa = reinterpret_cast<const bf16_t*>(x);
  const bf16_t* wa = reinterpret_cast<const bf16_t*>(wq);
  const long long lx = ldx / 2, lw = ldw / 2;
  i32x16_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
  auto stage_load = [&](int kt, int s) {
    char* ai = smem + s * STAGE_BYTES;
    const long long k0 = (long long)kt * 64;  // 128 int8 = 64 two-byte units
    dma_tile<256, 128>(xa + k0, lx, m0, M - 1, ai, w, lane);
    dma_tile<256, 128>(wa + k0, lw, n0, N - 1, ai + TILE_BYTES, w, lane);
  };
  const int nk = K / 128;
  stage_load(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int hi = lane >> 5, l31 = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt & 1;
    if (kt + 1 < nk) stage_load(kt + 1, s ^ 1);
    const char* ai = smem + s * STAGE_BYTES;
    const char* bi = ai + TILE_BYTES;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      i32x4_t af[4], bf[2];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
        af[mb] = *reinterpret_cast<const i32x4_t*>(ai + img_off<128>(wr * 128 + mb * 32 + l31, 2 * ks + hi));
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        bf[nb] = *reinterpret_cast<const i32x4_t*>(bi + img_off<128>(wc * 64 + nb * 32 + l31, 2 * ks + hi));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_i32_32x32x32_i8(bf[nb], af[mb], acc[mb][nb], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int mb = 0; mb < 4; ++mb) {
    const int m = m0 + wr * 128 + mb * 32 + l31;
    if (m >= M) continue;
    const float sm = xs ? xs[m] : xs_const;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wc * 64 + nb * 32 + 8 * g + 4 * hi;
        if (n >= N) continue;
        u16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = (float)acc[mb][nb][4 * g + j] * sm * ws[n + j];
          if (bias) v += bf2f(bias[n + j]);
          o[j] = f2bf(act_fwd(v, act));
        }
        *reinterpret_cast<u16x4*>(y + (long long)m * ldy + n) = o;
      }
    }
  }
}

// Row quantisation: q[m][k] = clamp(round(x[m][k] / s_m), -127, 127) with s_m = max|x[m]| / 127
// (dynamic, per token; written to scale[m]) or the static per-tensor scale `s_static` (> 0).
// One wave per row, 16-B loads.
__global__ __launch_bounds__(256) void quant_rows_kernel(const bf16_t* __restrict__ x, long long ldx,
                                                         signed char* __restrict__ q, long long ldq,
                                                         float* __restrict__ scale, float s_static,
                                                         int M, int K) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const bf16_t* xr = x + (long long)m * ldx;
  float s = s_static;
  if (s <= 0.f) {
    float mx = 0.f;
    for (int k = lane * 8; k < K; k += 512) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(xr + k);
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(bf2f(v[j])));
    }
    mx = wave_max(mx);
    s = mx > 0.f ? mx / 127.f : 1.f;
    if (lane == 0) scale[m] = s;
  }
  const float inv = 1.f / s;
  for (int k = lane * 8; k < K; k += 512) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(xr + k);
    unsigned lo = 0, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int qi = (int)fminf(127.f, fmaxf(-127.f, rintf(bf2f(v[j]) * inv)));
      const unsigned b = (unsigned)(qi & 255);
      if (j < 4) lo |= b << (8 * j); else hi |= b << (8 * (j - 4));
    }
    *reinterpret_cast<uint2*>(q + (long long)m * ldq + k) = make_uint2(lo, hi);
  }
}

}  // namespace

// x [M][K] int8 row-major (ldx bytes), wq [N][K] int8 (ldw bytes); xs [M] per-row activation
// scales (or null → xs_const), ws [N] per-channel weight scales; y [M][N] bf16. K % 128 == 0,
// 16-byte aligned rows, N % 4 == 0.
PIAMD_EXPORT int piamd_gemm_i8(const void* x, long long ldx, const void* wq, long long ldw,
                               const float* xs, float xs_const, const float* ws, const void* bias,
                               void* y, long long ldy, int M, int N, int K, int act,
                               hipStream_t st) {
  if (K % 128 || N % 4 || M <= 0 || N <= 0 || ldx % 16 || ldw % 16) return (int)hipErrorInvalidValue;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL(gemm_i8_kernel, dim3(tiles), dim3(NTHR), 0, st, (const signed char*)x, ldx,
                     (const signed char*)wq, ldw, xs, xs_const, ws, (const bf16_t*)bias,
                     (bf16_t*)y, ldy, M, N, K, act);
  return (int)hipGetLastError();
}

// f32 y[m][n] = Σ_p ws[p][m][n] in plane order (f32-output split-K finish).
__global__ __launch_bounds__(256) void conv_splitk_finish_f32(const float* __restrict__ ws, int ksplit,
                                                              long long MN, float* __restrict__ y) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= MN) return;
  f32x4 v = *reinterpret_cast<const f32x4*>(ws + i);
  for (int p = 1; p < ksplit; ++p) v += *reinterpret_cast<const f32x4*>(ws + p * MN + i);
  *reinterpret_cast<f32x4*>(y + i) = v;
}

// NHWC implicit-GEMM convolution forward: x [N][H][W][C], wt [Kout][R][S][C] (OHWI), y
// [N][OH][OW][Kout], 16-bit (bf16, or IEEE fp16 when f16 != 0: same tiles on the f16 MFMA);
// zero: ≥ 128 zero bytes (out-of-image taps); bias [Kout] (nullable, element type of x);
// act: epi 0 store / 1 bias+act (aux = pre-activation) / 2 dact. C % 64 == 0 (or C == 8: stem mode), Kout % 4 == 0.
// flags bit 0: fp16 (else bf16); bit 1: y is f32 (plain sum, bias and act must be off) — the
// split-bf16 fp32 convolution of ops/conv.py runs its three products through this.
template <bool F16>
static void conv_fwd_launch(int tile_n, bool sc, unsigned grid, hipStream_t st, const bf16_t* xb,
                            const bf16_t* wb, const bf16_t* zb, bf16_t* y, float* wsf, int ksplit,
                            const ConvGeom& g, int Kout, int act, const bf16_t* bb, int yf32, float* stats,
                            const RowMap& rm, int yacc) {
#define CONV_FWD(WM, MB, NB, SCV) \
  hipLaunchKernelGGL((conv_fwd_kernel<WM, MB, NB, SCV, F16>), dim3(grid), dim3(NTHR), 0, st, xb, wb, zb, y, wsf, ksplit, g, Kout, act, bb, yf32, stats, rm, yacc)
  if (tile_n == 64) {
    if (sc) CONV_FWD(8, 1, 2, true); else CONV_FWD(8, 1, 2, false);
  } else if (tile_n == 128) {
    if (sc) CONV_FWD(4, 2, 2, true); else CONV_FWD(4, 2, 2, false);
  } else {
    if (sc) CONV_FWD(2, 4, 2, true); else CONV_FWD(2, 4, 2, false);
  }
#undef CONV_FWD
}

// stats (nullable): f32 [3][Kout][ceil(M / 256)] per-tile BatchNorm statistics of y
// (conv_tile_stats) — ksplit == 1, 16-bit y, no bias / activation.
// dst_h > 0: y is an N × dst_h × dst_w × Kout tensor and this convolution's OH × OW outputs are
// its phase (ph, pw) of stride (rs_h, rs_w): pixel (oh, ow) lands on (oh·rs_h + ph, ow·rs_w + pw)
// (the strided data gradient's phases, written in place) — ksplit == 1.
PIAMD_EXPORT int piamd_conv2d_fwd3(const void* x, const void* wt, const void* zero, void* y, int N,
                                   int H, int W, int C, int OH, int OW, int R, int S, int st_h,
                                   int st_w, int pad_h, int pad_w, int dil_h, int dil_w, int Kout,
                                   int act, const void* bias, int tile_n, int ksplit, void* ws,
                                   int flags, float* stats, int dst_h, int dst_w, int rs_h, int rs_w,
                                   int ph, int pw, hipStream_t st) {
  const bool sc = C == 8;
  // flags bit 2: y += the convolution (16-bit y, ksplit == 1, no bias / activation / stats)
  const int f16 = flags & 1, yf32 = (flags >> 1) & 1, yacc = (flags >> 2) & 1;
  if (yf32 && (bias || act)) return (int)hipErrorInvalidValue;
  if (stats && (ksplit != 1 || yf32 || bias || act)) return (int)hipErrorInvalidValue;
  if (yacc && (ksplit != 1 || yf32 || bias || act || stats)) return (int)hipErrorInvalidValue;
  RowMap rm{0, 0, 0, 0, 0, 0, 0, 0};
  if (dst_h > 0) {
    if (ksplit != 1 || rs_h < 1 || rs_w < 1 || ph < 0 || pw < 0 || (OH - 1) * rs_h + ph >= dst_h ||
        (OW - 1) * rs_w + pw >= dst_w)
      return (int)hipErrorInvalidValue;
    rm = RowMap{OH * OW, OW, dst_h * dst_w, dst_w, rs_h, rs_w, ph, pw};
  }
  if ((C % BK && !sc) || Kout % 4 || N < 1 || OH < 1 || OW < 1 || R < 1 || S < 1 || !zero || ksplit < 1 ||
      (ksplit > 1 && !ws) || ksplit > (sc ? (R * S + 7) / 8 : R * S * (C / BK)) ||
      (tile_n != 64 && tile_n != 128 && tile_n != 256))
    return (int)hipErrorInvalidValue;
  ConvGeom g{N, H, W, C, OH, OW, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w};
  const long long M = (long long)N * OH * OW;
  if (M * ksplit > 0x7fffffffLL || M * Kout > (1LL << 40)) return (int)hipErrorInvalidValue;
  const int tm = (int)((M + BM - 1) / BM);
  const unsigned grid = (unsigned)(tm * ((Kout + tile_n - 1) / tile_n) * ksplit);
  const auto xb = (const bf16_t*)x;
  const auto wb = (const bf16_t*)wt;
  const auto zb = (const bf16_t*)zero;
  const auto bb = (const bf16_t*)bias;
  float* wsf = (float*)ws;
  if (f16) conv_fwd_launch<true>(tile_n, sc, grid, st, xb, wb, zb, (bf16_t*)y, wsf, ksplit, g, Kout, act, bb, yf32, stats, rm, yacc);
  else conv_fwd_launch<false>(tile_n, sc, grid, st, xb, wb, zb, (bf16_t*)y, wsf, ksplit, g, Kout, act, bb, yf32, stats, rm, yacc);
  if (ksplit > 1) {
    const long long MN = M * Kout;
    const dim3 fg((unsigned)((MN / 4 + 255) / 256));
    if (yf32)
      hipLaunchKernelGGL(conv_splitk_finish_f32, fg, dim3(256), 0, st, wsf, ksplit, MN, (float*)y);
    else if (f16) hipLaunchKernelGGL(conv_splitk_finish<true>, fg, dim3(256), 0, st, wsf, ksplit, MN, Kout, act, bb, (bf16_t*)y);
    else hipLaunchKernelGGL(conv_splitk_finish<false>, fg, dim3(256), 0, st, wsf, ksplit, MN, Kout, act, bb, (bf16_t*)y);
  }
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_conv2d_fwd(const void* x, const void* wt, const void* zero, void* y, int N,
                                  int H, int W, int C, int OH, int OW, int R, int S, int st_h,
                                  int st_w, int pad_h, int pad_w, int dil_h, int dil_w, int Kout,
                                  int act, const void* bias, int tile_n, int ksplit, void* ws,
                                  int flags, hipStream_t st) {
  return piamd_conv2d_fwd3(x, wt, zero, y, N, H, W, C, OH, OW, R, S, st_h, st_w, pad_h, pad_w, dil_h,
                           dil_w, Kout, act, bias, tile_n, ksplit, ws, flags, nullptr, 0, 0, 0, 0, 0, 0, st);
}

PIAMD_EXPORT int piamd_conv2d_fwd2(const void* x, const void* wt, const void* zero, void* y, int N,
                                   int H, int W, int C, int OH, int OW, int R, int S, int st_h,
                                   int st_w, int pad_h, int pad_w, int dil_h, int dil_w, int Kout,
                                   int act, const void* bias, int tile_n, int ksplit, void* ws,
                                   int flags, float* stats, hipStream_t st) {
  return piamd_conv2d_fwd3(x, wt, zero, y, N, H, W, C, OH, OW, R, S, st_h, st_w, pad_h, pad_w, dil_h,
                           dil_w, Kout, act, bias, tile_n, ksplit, ws, flags, stats, 0, 0, 0, 0, 0, 0, st);
}

// NHWC implicit-GEMM convolution weight gradient: x [N][H][W][C], dy [N][OH][OW][Kout] 16-bit
// (bf16, or fp16 when f16 != 0) → d [R][S][C][Kout] f32 (HWIO; accumulate bit 0 adds into d;
// bit 1: d is OHWI [Kout][R][S][C] instead — the channels_last layout of a [K][C][R][S] filter —
// bit 2: d is KCRS [Kout][C][R][S] — a contiguous filter — so the gradient lands in the
// parameter's own layout; bits 1-2 need ksplit > 1). zero: ≥ 16 zero bytes.
// C % 8 == 0, Kout % tile_n == 0 (tile_n ∈ {64, 128, 256}), N·OH·OW < 2^24; ksplit > 1 needs ws
// with ksplit·R·S·C·Kout floats (ksplit == 1 writes d directly, requires accumulate == 0).
PIAMD_EXPORT int piamd_conv2d_wgrad(const void* x, const void* dy, const void* zero, float* d, int N,
                                    int H, int W, int C, int OH, int OW, int R, int S, int st_h,
                                    int st_w, int pad_h, int pad_w, int dil_h, int dil_w, int Kout,
                                    int tile_n, int ksplit, float* ws, int accumulate, int f16,
                                    hipStream_t st) {
  const long long M = (long long)N * OH * OW;
  const long long RSC = (long long)R * S * C;
  if (C % 8 || Kout % tile_n || N < 1 || OH < 1 || OW < 1 || R < 1 || S < 1 || !zero ||
      ksplit < 1 || (ksplit > 1 && !ws) || (ksplit == 1 && accumulate) || M >= (1LL << 24) ||
      RSC * Kout >= (1LL << 31) || ksplit > (M + 63) / 64 ||
      (tile_n != 64 && tile_n != 128 && tile_n != 256))
    return (int)hipErrorInvalidValue;
  ConvWgradGeom g{N, H, W, C, OH, OW, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w,
                  (int)M, (int)RSC, Kout, 1.f / (float)OW, 1.f / (float)(OH * OW)};
  const int tm = (int)((RSC + BM - 1) / BM);
  const long long wgs = (long long)tm * (Kout / tile_n) * ksplit;
  if (wgs > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  float* out = ksplit > 1 ? ws : d;
  const auto xb = (const bf16_t*)x;
  const auto db = (const bf16_t*)dy;
  const auto zb = (const bf16_t*)zero;
#define CONV_WG(WM, MB, NB)                                                                       \
  do {                                                                                            \
    if (f16) hipLaunchKernelGGL((conv_wgrad_kernel<WM, MB, NB, true>), dim3((unsigned)wgs),       \
                                dim3(NTHR), 0, st, xb, db, zb, out, ksplit, g);                   \
    else hipLaunchKernelGGL((conv_wgrad_kernel<WM, MB, NB, false>), dim3((unsigned)wgs),          \
                            dim3(NTHR), 0, st, xb, db, zb, out, ksplit, g);                       \
  } while (0)
  if (tile_n == 64) CONV_WG(8, 1, 2);
  else if (tile_n == 128) CONV_WG(4, 2, 2);
  else CONV_WG(2, 4, 2);
#undef CONV_WG
  if (ksplit > 1) {
    const long long MN = RSC * Kout;
    const long long nv = MN / 4;
    if (ksplit >= 64 && nv < 65536)
      hipLaunchKernelGGL(wgrad_splitk_finish<16>, dim3((unsigned)((nv + 15) / 16)), dim3(256), 0, st,
                         (const float*)ws, ksplit, MN, d, accumulate, Kout, C);
    else if (ksplit >= 8 && nv < 262144)
      hipLaunchKernelGGL(wgrad_splitk_finish<4>, dim3((unsigned)((nv + 63) / 64)), dim3(256), 0, st,
                         (const float*)ws, ksplit, MN, d, accumulate, Kout, C);
    else
      hipLaunchKernelGGL(wgrad_splitk_finish<1>, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st,
                         (const float*)ws, ksplit, MN, d, accumulate, Kout, C);
  }
  return (int)hipGetLastError();
}

// bf16 [M][K] → int8 [M][K]; s_static > 0: per-tensor scale, else dynamic per-row (scale[M] out).
PIAMD_EXPORT int piamd_quant_rows(const void* x, long long ldx, void* q, long long ldq,
                                  float* scale, float s_static, int M, int K, hipStream_t st) {
  if (K % 8 || M <= 0 || (s_static <= 0.f && !scale)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(quant_rows_kernel, dim3((M + 3) / 4), dim3(256), 0, st, (const bf16_t*)x,
                     ldx, (signed char*)q, ldq, scale, s_static, M, K);
  return (int)hipGetLastError();
}

// Grouped expert GEMM. x [rows][K] expert-sorted (offs[E+1] int32 on device, rows ≤ rows_cap);
// w: trans_w=0 → [E][K][N] (N % 256 == 0), trans_w=1 → [E][N][K]; per-expert stride sw elements.
// y [rows][N] bf16 (or f32 when y_f32); epi/act/aux as the conv kernels (0 store, 1 bias+act, 2 dact), bias [E][N] (may be null).
PIAMD_EXPORT int piamd_moe_gemm(const void* x, long long ldx, const void* w, long long ldw,
                                long long sw, int trans_w, const int* offs, int E, int rows_cap,
                                void* y, long long ldy, int y_f32, int N, int K, int epi, int act,
                                const void* bias, void* aux, long long ldaux, hipStream_t st) {
  if (K % BK || N % 4 || (!trans_w && N % BN) || E < 1 || rows_cap < 0 ||
      (epi == EPI_DACT && !aux))
    return (int)hipErrorInvalidValue;
  const int tm_max = (rows_cap + BM - 1) / BM + E, tn = (N + BN - 1) / BN;
  dim3 grid(tm_max * tn), block(NTHR);
  if (trans_w)
    hipLaunchKernelGGL(moe_gemm_kernel<true>, grid, block, 0, st, (const bf16_t*)x, ldx,
                       (const bf16_t*)w, ldw, sw, offs, E, y, ldy, y_f32, N, K, tm_max, epi, act,
                       (const bf16_t*)bias, (bf16_t*)aux, ldaux);
  else
    hipLaunchKernelGGL(moe_gemm_kernel<false>, grid, block, 0, st, (const bf16_t*)x, ldx,
                       (const bf16_t*)w, ldw, sw, offs, E, y, ldy, y_f32, N, K, tm_max, epi, act,
                       (const bf16_t*)bias, (bf16_t*)aux, ldaux);
  return (int)hipGetLastError();
}

// dW_e [M][N] (+)= X_eᵀ · dY_e for every expert; x [rows][M], dy [rows][N], expert segments
// 64-row aligned and zero padded; M, N multiples of 256; dw per-expert stride sdw elements.
PIAMD_EXPORT int piamd_moe_wgrad(const void* x, long long ldx, const void* dy, long long lddy,
                                 const int* offs, int E, void* dw, long long sdw, int dw_f32,
                                 int accumulate, int M, int N, hipStream_t st) {
  if (M % BM || N % BN || E < 1) return (int)hipErrorInvalidValue;
  dim3 grid(E * (M / BM) * (N / BN)), block(NTHR);
  hipLaunchKernelGGL(moe_wgrad_kernel, grid, block, 0, st, (const bf16_t*)x, ldx,
                     (const bf16_t*)dy, lddy, offs, E, dw, sdw, dw_f32, accumulate, M, N);
  return (int)hipGetLastError();
}
