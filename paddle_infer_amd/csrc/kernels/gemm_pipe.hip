// Persistent, ring-pipelined bf16 MFMA GEMM for the training hot path:
// C[M,N] = A[M,K] · B[K,N] with f32 accumulation and fused epilogues (bias / bias + activation
// with the saved pre-activation / activation-gradient / accumulate into an existing bf16 or f32 C)
// plus deterministic split-K for small-MN, long-K shapes (weight gradients).
//
// Parity: reference `paddle/phi/kernels/funcs/blas/blas_impl.cu.h` (cublas GEMM behind matmul /
// linear and their gradients) and `paddle/fluid/operators/fused/fused_gemm_epilogue_op.cu:30`
// (cublasLt bias / bias+GELU(aux) / dGELU epilogues used by fused_linear / FusedFeedForward).
//
// MI355X design:
//   * workgroup = 8 waves (2 M × 4 N; two per SIMD), 256 × 256 output tile, every wave owns a
//     128 × 64 sub-tile: 8 × 4 blocks of v_mfma_f32_16x16x32_bf16 (the 16x16 shape holds a higher
//     clock under load than 32x32, MI355X_MICROARCH.md "DVFS give-back" 7). Operands are SWAPPED
//     (Cᵀ = Bᵀ·Aᵀ) so each lane owns one output row and 4 consecutive columns;
//   * K is consumed in 32-deep SLOTS (A 256×32 + B 256×32 = 32 KiB); the LDS (all 160 KiB, ONE
//     __shared__ array) is a ring of 5 slots. Per slot each wave reads 8 + 4 fragments and issues
//     32 MFMAs, with one raw `s_barrier` per slot. With one wave per SIMD the LDS-DMA issue cost
//     (≈60 cycles per 1 KiB piece among MFMAs, MI355X_MICROARCH.md cycle constants) and the reads
//     sat in series with the MFMAs; with two, waves 4-7 run half of each slot's MFMAs before
//     their DMA issue, so each SIMD's matrix pipe is fed while the partner issues loads;
//   * slots are filled by global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip) THREE slots ahead:
//     the DMA for slot g+4 goes out right after slot g's barrier into the ring position slot g-1
//     just vacated, and the counted `s_waitcnt vmcnt(8)` before each barrier retires only slot g+1
//     (never vmcnt(0) in the loop; `__syncthreads()` would drain the DMA queue);
//   * fragments of slot g+1 are read while slot g's MFMAs run: B into a second register set (loop
//     unrolled by 2: static indexing), A into the SAME set, each m-block's register refilled right
//     after its 4 MFMAs consumed it (keeps the wave at ≤ 256 registers: two waves per SIMD);
//   * PERSISTENT: the grid is at most one workgroup per CU and the slot stream runs across the
//     workgroup's tiles — the next tile's first DMAs are already in flight while the finished
//     tile's epilogue is stored, so tile prologue latency and epilogue store tail overlap;
//   * XOR-swizzled LDS images with the swizzle on the per-lane DMA SOURCE address (the LDS side of
//     an LDS-DMA is lane-linear): K-contiguous operands → [256 rows][64 B] images, chunk ^=
//     (row>>1)&3, read with conflict-free ds_read_b128; M/N-contiguous operands → [32 k][512 B]
//     images, chunk ^= ((k&3)<<2)|((k>>2)&3), read with the hardware transpose ds_read_b64_tr_b16
//     (conflict-free). Forward (A, Bᵀ K-contiguous), data-gradient and weight-gradient (A, B both
//     M/N-contiguous) GEMMs therefore all run without transpose kernels;
//   * work order: 32 consecutive tiles per XCD per round (workgroup w on XCD w % 8 takes units
//     (8i + w%8)·32 + w/8), tiles in group-M order (8 M-tiles × all N), so the tiles an XCD holds
//     at once share A and B panels in its L2 (guide T1).
#include "common.h"

#include <type_traits>

namespace {

typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;

constexpr int TBM = 256, TBN = 256, KSL = 32, NTHR = 512;
// LDS holds 64-deep IMAGES (two 32-deep slots: every operand row a whole 128-byte line), 2 of them
constexpr int OPB = 256 * 2 * KSL * 2;  // one operand image: 32 KiB
constexpr int IMGB = 2 * OPB;           // 64 KiB
constexpr int LDSB = 2 * IMGB;          // 128 KiB
constexpr int GROUP_M = 8;

__device__ __forceinline__ int sw8(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int sw16(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

__device__ __forceinline__ void bar() { asm volatile("s_barrier" ::: "memory"); }
// s_waitcnt immediate (gfx9 encoding): lgkmcnt(0), vmcnt / expcnt left at their maxima
constexpr int LGKM0 = 0xF | (3 << 14) | (7 << 4);

// DMA of this wave's 4 pieces of one operand image (64 deep). The 32 pieces (1 KiB each) of an
// image are shared by the 8 waves: wave w takes w, w+8, w+16, w+24. Every piece covers whole
// 128-byte lines: KC — operand [rows][K] (leading dim ld), piece = 8 rows × 128 B, rows clamped to
// rlim; !KC — operand [K][cols], piece = 2 k-rows × 512 B, 8-col chunks clamped to rlim. `base`:
// uniform address of the image's first element (KC: tile row 0, k0; !KC: k-row k0, tile col 0).
// The per-lane offsets are recomputed per issue (a few VALU) rather than held in registers.
template <bool KC>
__device__ __forceinline__ void dma_op(const char* base, int ld, int rlim, char* img, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int L = (i * 8 + w) * 64 + lane;
    unsigned off;
    if (KC) {
      const int r = L >> 3, pc = L & 7;
      off = (unsigned)(min(r, rlim) * ld + ((pc ^ sw8(r)) << 3)) * 2u;
    } else {
      const int r = L >> 5, pc = L & 31;
      off = (unsigned)(r * ld + min((pc ^ sw16(r)) << 3, rlim)) * 2u;
    }
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(base + off),
                                     (__attribute__((address_space(3))) void*)(img + (i * 8 + w) * 1024),
                                     16, 0, 0);
  }
}

// 16 × 32 fragment of the 16x16x32 MFMA from half `ks` (32-deep slot) of an image: lane l holds
// row/col `base + (l&15)`, k = 32·ks + 8·(l>>4) + j. KC image [256 rows][128 B], 16-B chunk c of
// row r stored at c ^ ((r>>1)&7) (conflict-free ds_read_b128 for this operand); !KC image
// [64 k][512 B], chunk ^ (((k&3)<<2) | ((k>>2)&3)) on the low 4 bits (conflict-free
// ds_read_b64_tr_b16).
template <bool KC>
__device__ __forceinline__ bf16x8 ld_frag(const char* img, int base, int ks, int lane) {
  if (KC) {
    const int row = base + (lane & 15), c = 4 * ks + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + ((c ^ sw8(row)) << 4));
  }
  const int gi = lane & 15;
  const int k = 32 * ks + 8 * (lane >> 4) + (gi >> 2);
  const int col = base + 4 * (gi & 3);
  const int o0 = k * 512 + (((col >> 3) ^ sw16(k)) << 4) + ((col & 7) << 1);
  const int o1 = (k + 4) * 512 + (((col >> 3) ^ sw16(k + 4)) << 4) + ((col & 7) << 1);
  const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o0));
  const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + o1));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <bool B_KC>
__device__ __forceinline__ void read_b(bf16x8 (&b)[4], const char* img, int ks, int wc, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) b[i] = ld_frag<B_KC>(img + OPB, wc * 64 + i * 16, ks, lane);
}

// row mb of the slot: 4 MFMAs on the current A fragment, then (if `next`) that fragment's register
// is refilled with m-block mb of the next slot (single A register set, refilled row by row; the
// reads sit between the MFMAs)
template <bool A_KC, int MB>
__device__ __forceinline__ void mma_row(f32x4 (&acc)[8][4], bf16x8 (&a)[8], const bf16x8 (&b)[4],
                                        const char* next, int nks, int wr, int lane) {
#ifndef PIAMD_ABL_NO_MFMA
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
    acc[MB][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nb], a[MB], acc[MB][nb], 0, 0, 0);
#else  // ablation build: operands kept live, no matrix work
  asm volatile("" ::"v"(a[MB]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]));
#endif
#ifndef PIAMD_ABL_NO_READS
  if (next) a[MB] = ld_frag<A_KC>(next, wr * 128 + MB * 16, nks, lane);
#endif
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

enum { EPI_STORE = 0, EPI_BIAS_ACT = 1, EPI_DACT = 2 };

struct Problem {
  const bf16_t* a;
  const bf16_t* b;
  long long lda, ldb;
  void* c;
  long long ldc;
  int c_f32, accumulate, M, N, K, epi, act;
  const bf16_t* bias;
  bf16_t* aux;
  long long ldaux;
  int ksplit;
  float* ws;               // split-K partials [ksplit][M][N]
  int tm, tn, units, nks;  // tile grid, work units (tiles × ksplit), slots per unit
};

// unit → (part, m0, n0), group-M tile order
__device__ __forceinline__ void unit_coords(const Problem& p, int u, int& part, int& m0, int& n0) {
  const int ntiles = p.tm * p.tn;
  part = u / ntiles;
  const int tile = u - part * ntiles;
  const int per_group = GROUP_M * p.tn;
  const int grp = tile / per_group, first_m = grp * GROUP_M;
  const int gm = min(p.tm - first_m, GROUP_M);
  const int in_g = tile - grp * per_group;
  m0 = (first_m + in_g % gm) * TBM;
  n0 = (in_g / gm) * TBN;
}

// this workgroup's i-th unit (or -1): 32 consecutive units per XCD per round
__device__ __forceinline__ int my_unit(const Problem& p, int i) {
  const int w = blockIdx.x, G = gridDim.x;
  if (p.units <= G) return i == 0 ? w : -1;  // grid == units (host): one unit each
  const int u = (i * 8 + (w & 7)) * (G >> 3) + (w >> 3);
  return u < p.units ? u : -1;
}

// DMA issue cursor: which slot of which unit goes out next
struct Issuer {
  int i, s, u;  // unit ordinal, image within unit, unit id (-1: stream exhausted)
  const char* abase;
  const char* bbase;
  long long astep, bstep;  // bytes per image along K
  int lda, ldb, alim, blim;
};

template <bool A_KC, bool B_KC>
__device__ __forceinline__ void issuer_load_unit(const Problem& p, Issuer& is, int w, int lane) {
  is.u = my_unit(p, is.i);
  if (is.u < 0) return;
  int part, m0, n0;
  unit_coords(p, is.u, part, m0, n0);
  const long long k0 = (long long)part * p.nks * KSL;
  is.abase = reinterpret_cast<const char*>(A_KC ? p.a + (long long)m0 * p.lda + k0 : p.a + k0 * p.lda + m0);
  is.bbase = reinterpret_cast<const char*>(B_KC ? p.b + (long long)n0 * p.ldb + k0 : p.b + k0 * p.ldb + n0);
  is.astep = A_KC ? 2 * KSL * 2 : (long long)2 * KSL * p.lda * 2;
  is.bstep = B_KC ? 2 * KSL * 2 : (long long)2 * KSL * p.ldb * 2;
  is.lda = (int)p.lda;
  is.ldb = (int)p.ldb;
  is.alim = (A_KC ? p.M - 1 : p.M - 8) - m0;
  is.blim = (B_KC ? p.N - 1 : p.N - 8) - n0;
}

// issue the next image of the stream into LDS image position `pos` (no-op once exhausted)
template <bool A_KC, bool B_KC>
__device__ __forceinline__ void issue_next(const Problem& p, Issuer& is, char* smem, int pos, int w,
                                           int lane) {
  if (is.u < 0) return;
  char* img = smem + pos * IMGB;
#ifndef PIAMD_ABL_NO_DMA
  dma_op<A_KC>(is.abase + is.s * is.astep, is.lda, is.alim, img, w, lane);
  dma_op<B_KC>(is.bbase + is.s * is.bstep, is.ldb, is.blim, img + OPB, w, lane);
#endif
  if (++is.s == p.nks / 2) {
    is.s = 0;
    ++is.i;
    issuer_load_unit<A_KC, B_KC>(p, is, w, lane);
  }
}

// wait until at most `pend` images (8 DMA instructions each) of this wave are outstanding
__device__ __forceinline__ void wait_images(int pend) {
  if (pend >= 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- epilogues ---------------------------------------------------------------------------------
// A lane owns rows m = mb·16 + (l&15) and columns n = nb·16 + 4(l>>4) + j (j < 4) of its wave's
// 128 × 64 sub-tile (coordinates relative to the quadrant origin; mlim / nlim = rows / columns of
// the quadrant inside C). Edge tiles use predicated stores and clamped (unconditional) loads: a
// branch around a load makes hipcc wait vmcnt(0) per element. Each kernel instantiation carries
// exactly one epilogue kind (register pressure: the 256 accumulators are live when it starts).
enum { EK_BF16 = 0, EK_BF16_ACC = 1, EK_F32 = 2, EK_F32_ACC = 3, EK_FUSED = 4 };

template <int EK>
__device__ __forceinline__ void epi_plain(const f32x4 (&acc)[8][4], char* c, long long ldc, int mlim,
                                          int nlim, int lane) {
  constexpr bool F32 = EK == EK_F32 || EK == EK_F32_ACC;
  constexpr bool ACC = EK == EK_BF16_ACC || EK == EK_F32_ACC;
  constexpr int ES = F32 ? 4 : 2;
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    const int m = mb * 16 + (lane & 15);
    const bool mok = m < mlim;
    char* row = c + (long long)min(m, mlim - 1) * ldc * ES;
    f32x4 old[4];
    if (ACC) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int n = min(nb * 16 + 4 * (lane >> 4), nlim - 4);
        if (F32) {
          old[nb] = *reinterpret_cast<const f32x4*>(row + n * 4);
        } else {
          const u16x4 o = *reinterpret_cast<const u16x4*>(row + n * 2);
          old[nb] = f32x4{bf2f(o[0]), bf2f(o[1]), bf2f(o[2]), bf2f(o[3])};
        }
      }
    }
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int n = nb * 16 + 4 * (lane >> 4);
      f32x4 v = acc[mb][nb];
      if (ACC) v += old[nb];
      if (mok && n < nlim) {
        if (F32) *reinterpret_cast<f32x4*>(row + n * 4) = v;
        else *reinterpret_cast<u16x4*>(row + n * 2) = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
      }
    }
  }
}

// EPI_BIAS_ACT: pre = bf16(acc + bias) → aux (if any), C = act(pre); EPI_DACT: C = acc ⊙ act'(aux).
// bf16 C, no accumulation.
template <int EPI, int ACT>
__device__ __forceinline__ void epi_fused(const f32x4 (&acc)[8][4], bf16_t* c, long long ldc,
                                          bf16_t* aux, long long ldaux, const bf16_t* bias, int mlim,
                                          int nlim, int lane) {
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    const int m = mb * 16 + (lane & 15);
    const bool mok = m < mlim;
    const long long mr = min(m, mlim - 1);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int n = nb * 16 + 4 * (lane >> 4);
      const int nc = min(n, nlim - 4);
      const bool ok = mok && n < nlim;
      u16x4 o;
      if (EPI == EPI_BIAS_ACT) {
        const u16x4 b = bias ? *reinterpret_cast<const u16x4*>(bias + nc) : u16x4{0, 0, 0, 0};
        u16x4 pre;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pre[j] = f2bf(acc[mb][nb][j] + bf2f(b[j]));
          o[j] = f2bf(act_fwd(bf2f(pre[j]), ACT));
        }
        if (aux && ok) *reinterpret_cast<u16x4*>(aux + mr * ldaux + n) = pre;
      } else {
        const u16x4 h = *reinterpret_cast<const u16x4*>(aux + mr * ldaux + nc);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(acc[mb][nb][j] * act_grad(bf2f(h[j]), ACT));
      }
      if (ok) *reinterpret_cast<u16x4*>(c + mr * ldc + n) = o;
    }
  }
}

template <int EK>
__device__ __forceinline__ void epilogue(const Problem& p, const f32x4 (&acc)[8][4], int part, int m0,
                                         int n0, int wr, int wc, int lane) {
  const int qm = m0 + wr * 128, qn = n0 + wc * 64;  // wave sub-tile origin
  const int mlim = p.M - qm, nlim = p.N - qn;
  if (mlim <= 0 || nlim <= 0) return;
  if (EK != EK_FUSED) {
    if (p.ksplit > 1) {
      char* c = reinterpret_cast<char*>(p.ws + (long long)part * p.M * p.N + (long long)qm * p.N + qn);
      epi_plain<EK_F32>(acc, c, p.N, mlim, nlim, lane);
    } else {
      constexpr int es = (EK == EK_F32 || EK == EK_F32_ACC) ? 4 : 2;
      char* c = reinterpret_cast<char*>(p.c) + ((long long)qm * p.ldc + qn) * es;
      epi_plain<EK>(acc, c, p.ldc, mlim, nlim, lane);
    }
  } else {
    bf16_t* c = reinterpret_cast<bf16_t*>(p.c) + (long long)qm * p.ldc + qn;
    bf16_t* aux = p.aux ? p.aux + (long long)qm * p.ldaux + qn : nullptr;
    const bf16_t* bias = p.bias ? p.bias + qn : nullptr;
    switch (p.epi * 8 + p.act) {
      case EPI_BIAS_ACT * 8 + 1: epi_fused<EPI_BIAS_ACT, 1>(acc, c, p.ldc, aux, p.ldaux, bias, mlim, nlim, lane); break;
      case EPI_BIAS_ACT * 8 + 2: epi_fused<EPI_BIAS_ACT, 2>(acc, c, p.ldc, aux, p.ldaux, bias, mlim, nlim, lane); break;
      case EPI_BIAS_ACT * 8 + 3: epi_fused<EPI_BIAS_ACT, 3>(acc, c, p.ldc, aux, p.ldaux, bias, mlim, nlim, lane); break;
      case EPI_BIAS_ACT * 8 + 4: epi_fused<EPI_BIAS_ACT, 4>(acc, c, p.ldc, aux, p.ldaux, bias, mlim, nlim, lane); break;
      case EPI_DACT * 8 + 1: epi_fused<EPI_DACT, 1>(acc, c, p.ldc, aux, p.ldaux, bias, mlim, nlim, lane); break;
      case EPI_DACT * 8 + 2: epi_fused<EPI_DACT, 2>(acc, c, p.ldc, aux, p.ldaux, bias, mlim, nlim, lane); break;
      case EPI_DACT * 8 + 3: epi_fused<EPI_DACT, 3>(acc, c, p.ldc, aux, p.ldaux, bias, mlim, nlim, lane); break;
      case EPI_DACT * 8 + 4: epi_fused<EPI_DACT, 4>(acc, c, p.ldc, aux, p.ldaux, bias, mlim, nlim, lane); break;
      default: epi_fused<EPI_BIAS_ACT, 0>(acc, c, p.ldc, aux, p.ldaux, bias, mlim, nlim, lane); break;
    }
  }
}

template <bool A_KC, bool B_KC, int EK>
__global__ __launch_bounds__(NTHR, 1) void gemm_pipe_kernel(Problem p) {
  __shared__ __attribute__((aligned(1024))) char smem[LDSB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;
  // waves w and w+4 share a SIMD; the second of each pair (late = 1) issues the first half of a
  // slot's MFMAs BEFORE its LDS-DMA issue, so on every SIMD one wave feeds the matrix pipe while
  // its partner pays the DMA issue cost
  const int late = __builtin_amdgcn_readfirstlane(wr);
  int nunits = 0;
  while (my_unit(p, nunits) >= 0) ++nunits;
  if (nunits == 0) return;
  const int total = nunits * p.nks;  // slots in this workgroup's stream

  Issuer is;
  is.i = 0;
  is.s = 0;
  issuer_load_unit<A_KC, B_KC>(p, is, w, lane);
  // prologue: images 0 and 1 into LDS positions 0 and 1; wait for image 0
  issue_next<A_KC, B_KC>(p, is, smem, 0, w, lane);
  issue_next<A_KC, B_KC>(p, is, smem, 1, w, lane);
  wait_images(total > 2 ? 1 : 0);
  __builtin_amdgcn_s_waitcnt(LGKM0);
  bar();
  bf16x8 a[8], b0[4], b1[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = ld_frag<A_KC>(smem, wr * 128 + i * 16, 0, lane);
  read_b<B_KC>(b0, smem, 0, wc, lane);
  int g = 0;  // stream index of the slot being computed (image g >> 1, half g & 1)
  // step g: compute slot g (A in `a`, B in `bc`); read slot g+1's B into `bn` and its A into `a`.
  // ODD steps start a new image for the reads: wait for it (own DMAs, then everyone's via the
  // barrier) — the barrier also certifies that every wave finished reading image (g-1)/2, whose
  // LDS position then takes image (g+3)/2 (two steps of DMA latency budget)
  auto step = [&](f32x4 (&acc)[8][4], const bf16x8 (&bc)[4], bf16x8 (&bn)[4], auto odd) {
    constexpr bool ODD = decltype(odd)::value;
    if (ODD) {
      wait_images(0);
      // this wave's LDS reads of the previous image are complete: a real S_WAITCNT the
      // compiler's waitcnt pass sees (so it adds no lgkmcnt(0) behind the new reads)
      __builtin_amdgcn_s_waitcnt(LGKM0);
      bar();
    }
    const char* next = g + 1 < total ? smem + (((g + 1) >> 1) & 1) * IMGB : nullptr;
    constexpr int nks = ODD ? 0 : 1;  // half of the next slot inside its image
#ifndef PIAMD_ABL_NO_READS
    if (next) read_b<B_KC>(bn, next, nks, wc, lane);
#endif
    if (ODD && !late) issue_next<A_KC, B_KC>(p, is, smem, ((g - 1) >> 1) & 1, w, lane);
    __builtin_amdgcn_s_setprio(1);
    mma_row<A_KC, 0>(acc, a, bc, next, nks, wr, lane);
    mma_row<A_KC, 1>(acc, a, bc, next, nks, wr, lane);
    mma_row<A_KC, 2>(acc, a, bc, next, nks, wr, lane);
    mma_row<A_KC, 3>(acc, a, bc, next, nks, wr, lane);
    __builtin_amdgcn_s_setprio(0);
    if (ODD && late) issue_next<A_KC, B_KC>(p, is, smem, ((g - 1) >> 1) & 1, w, lane);
    __builtin_amdgcn_s_setprio(1);
    mma_row<A_KC, 4>(acc, a, bc, next, nks, wr, lane);
    mma_row<A_KC, 5>(acc, a, bc, next, nks, wr, lane);
    mma_row<A_KC, 6>(acc, a, bc, next, nks, wr, lane);
    mma_row<A_KC, 7>(acc, a, bc, next, nks, wr, lane);
    __builtin_amdgcn_s_setprio(0);
    ++g;
  };
  for (int ui = 0; ui < nunits; ++ui) {
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // units have an even slot count (whole images): the B register sets alternate in a fixed order
    for (int s = 0; s < p.nks; s += 2) {
      step(acc, b0, b1, std::false_type{});
      step(acc, b1, b0, std::true_type{});
    }
    // the next unit's first image is already in flight (DMA) and its first slot read meanwhile
    int part, m0, n0;
    unit_coords(p, my_unit(p, ui), part, m0, n0);
    epilogue<EK>(p, acc, part, m0, n0, wr, wc, lane);
  }
}

// C (+)= Σ_p ws[p] (fixed order: deterministic); 4 columns per thread
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int ksplit,
                                                            int M, int N, void* __restrict__ c,
                                                            long long ldc, int c_f32, int accumulate) {
  const long long MN = (long long)M * N;
  const int nq = N / 4;
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < MN / 4;
       q += (long long)gridDim.x * 256) {
    const long long m = q / nq;
    const int n = (int)(q - m * nq) * 4;
    f32x4 v = *reinterpret_cast<const f32x4*>(ws + m * N + n);
    for (int p = 1; p < ksplit; ++p) v += *reinterpret_cast<const f32x4*>(ws + p * MN + m * N + n);
    if (c_f32) {
      f32x4* pc = reinterpret_cast<f32x4*>((float*)c + m * ldc + n);
      if (accumulate) v += *pc;
      *pc = v;
    } else {
      u16x4* pc = reinterpret_cast<u16x4*>((bf16_t*)c + m * ldc + n);
      u16x4 o;
      if (accumulate) {
        const u16x4 old = *pc;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j] + bf2f(old[j]));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j]);
      }
      *pc = o;
    }
  }
}

constexpr int MAX_WG = 256;  // one workgroup per CU (160 KiB LDS each)

}  // namespace

// C[M][N] (+)= op(A) · op(B).
// trans_a: A stored [K][M] (lda ≥ M, M % 8 == 0), else [M][K] (lda ≥ K).
// trans_b: B stored [N][K] (ldb ≥ K), else [K][N] (ldb ≥ N, N % 8 == 0).
// K % (64·ksplit) == 0, N % 4 == 0, leading dims % 8 == 0 and < 2^22, 16-byte aligned operands.
// epi: 0 store, 1 bias + act (aux = pre-activation bf16 [M][N], may be null), 2 C = (A·B) ⊙
// act'(aux) — fused epilogues need A stored [M][K]. ksplit > 1 (epi 0 only): each tile's K range is
// split over ksplit work units writing f32 partials to ws [ksplit][M][N], summed in a fixed order
// by a second launch.
PIAMD_EXPORT int piamd_gemm_pipe(const void* a, long long lda, int trans_a, const void* b,
                                 long long ldb, int trans_b, void* c, long long ldc, int c_f32,
                                 int accumulate, int M, int N, int K, int epi, int act,
                                 const void* bias, void* aux, long long ldaux, int ksplit, void* ws,
                                 hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || ksplit < 1 || K % (2 * KSL * ksplit) || N % 4 ||
      (trans_a && M % 8) || (!trans_b && N % 8) || (epi == EPI_DACT && !aux) ||
      (ksplit > 1 && (epi != EPI_STORE || !ws)) || (trans_a && epi != EPI_STORE) ||
      (epi != EPI_STORE && (c_f32 || accumulate || (epi == EPI_DACT && (act < 1 || act > 4)))) || lda % 8 ||
      ldb % 8 || lda >= (1 << 22) || ldb >= (1 << 22) || ldc % 4)
    return (int)hipErrorInvalidValue;
  Problem p;
  p.a = (const bf16_t*)a; p.b = (const bf16_t*)b; p.lda = lda; p.ldb = ldb;
  p.c = c; p.ldc = ldc; p.c_f32 = c_f32; p.accumulate = accumulate;
  p.M = M; p.N = N; p.K = K; p.epi = epi; p.act = act;
  p.bias = (const bf16_t*)bias; p.aux = (bf16_t*)aux; p.ldaux = ldaux;
  p.ksplit = ksplit; p.ws = (float*)ws;
  p.tm = (M + TBM - 1) / TBM; p.tn = (N + TBN - 1) / TBN;
  const long long units = (long long)p.tm * p.tn * ksplit;
  if (units > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  p.units = (int)units;
  p.nks = K / KSL / ksplit;
  const int grid = p.units <= MAX_WG ? p.units : MAX_WG;
  // epilogue kind of the instantiation (split-K partials are f32 stores)
  const int ek = epi != EPI_STORE ? EK_FUSED
                 : ksplit > 1     ? EK_F32
                                  : c_f32 * 2 + accumulate;
#define PIPE_LAUNCH(AK, BKC, E) \
  hipLaunchKernelGGL((gemm_pipe_kernel<AK, BKC, E>), dim3(grid), dim3(NTHR), 0, st, p)
#define PIPE_EK(AK, BKC)                                  \
  switch (ek) {                                           \
    case EK_BF16: PIPE_LAUNCH(AK, BKC, EK_BF16); break;         \
    case EK_BF16_ACC: PIPE_LAUNCH(AK, BKC, EK_BF16_ACC); break; \
    case EK_F32: PIPE_LAUNCH(AK, BKC, EK_F32); break;           \
    default: PIPE_LAUNCH(AK, BKC, EK_F32_ACC); break;           \
  }
  if (!trans_a && trans_b) {
    if (ek == EK_FUSED) PIPE_LAUNCH(true, true, EK_FUSED);
    else PIPE_EK(true, true)
#ifndef PIAMD_GEMM_ONE
  } else if (!trans_a && !trans_b) {
    if (ek == EK_FUSED) PIPE_LAUNCH(true, false, EK_FUSED);
    else PIPE_EK(true, false)
  } else if (trans_a && !trans_b) {
    PIPE_EK(false, false)
  } else {
    PIPE_EK(false, true)
#endif
  }
#undef PIPE_EK
#undef PIPE_LAUNCH
  hipError_t err = hipGetLastError();
  if (err != hipSuccess || ksplit == 1) return (int)err;
  const long long q = (long long)M * N / 4;
  const int g = (int)std::min<long long>(2048, (q + 255) / 256);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(g), dim3(256), 0, st, (const float*)ws, ksplit, M,
                     N, c, ldc, c_f32, accumulate);
  return (int)hipGetLastError();
}
