// LayerNorm / RMSNorm forward + backward with an optional fused bias + dropout + residual-add
// prologue, for f32 / bf16 / fp16 rows of up to 16384 elements.
//
// Parity: reference `paddle/phi/kernels/gpu/layer_norm_kernel.cu` (f32/fp16/bf16 registrations at
// :218-240), `paddle/fluid/operators/fused/fused_layernorm_residual_dropout_bias.h` and
// `fused_bias_dropout_residual_layer_norm_op.cu` (out = LN(residual + dropout(x + bias))). RMSNorm
// (`rms = 1`: no mean subtraction, y = x * rsqrt(mean(x^2) + eps) * gamma) has no reference op; it
// shares every kernel here through one uniform runtime branch (LLaMA-style residual + RMSNorm).
//
// MI355X design:
//  * N <= 4096: one wave64 per row, the whole row in registers (16 B/lane loads: each vector
//    instruction moves 1 KiB contiguous), exact two-pass mean/variance from registers (no Welford,
//    no second HBM read); 4 rows per 256-thread block so an 8192 x 2048 activation gets 2048 blocks.
//  * N > 4096 (LLaMA-13B 5120, 65B 8192, up to 16384) and the few-row decode case: one workgroup per
//    row (256 or 512 threads), row still register-resident, block reductions through LDS.
//  * Backward: wave per row up to N = 1024, two waves per row with a prefetched second row for
//    1024 < N <= 2048, workgroup per row above.
//  * Backward fuses dgamma/dbeta (and the dbias of the prologue): every thread accumulates its
//    columns across a grid-stride set of rows in registers, each workgroup stores one row of a
//    [G][N] partial slab, and a 16-row-strip reduction folds it (G/16 atomics per column). Dropout masks are regenerated from
//    the stateless counter hash (common.h), never stored.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace {

enum { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2 };

template <int DT>
struct IO16 {
  typedef unsigned short T;
  typedef u16x8 Raw;  // 8 elements held in 4 VGPRs until used
  static __device__ __forceinline__ float cv(unsigned short v) {
    if (DT == DT_BF16) return bf2f(v);
    return (float)__builtin_bit_cast(_Float16, v);
  }
  static __device__ __forceinline__ unsigned short cvt(float f) {
    if (DT == DT_BF16) return f2bf(f);
    return __builtin_bit_cast(unsigned short, (_Float16)f);
  }
  static __device__ __forceinline__ Raw ldraw(const T* p) { return *reinterpret_cast<const Raw*>(p); }
  static __device__ __forceinline__ float el(const Raw& r, int j) { return cv(r[j]); }
  static __device__ __forceinline__ void load8(const T* p, float* v) {
    u16x8 r = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = cv(r[j]);
  }
  static __device__ __forceinline__ void store8(T* p, const float* v) {
    u16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = cvt(v[j]);
    __builtin_nontemporal_store(r, reinterpret_cast<u16x8*>(p));  // streamed rows: no L2 reuse
  }
  static __device__ __forceinline__ float load1(const T* p) { return cv(*p); }
  static __device__ __forceinline__ void store1(T* p, float v) { *p = cvt(v); }
};

template <int DT>
struct IO : IO16<DT> {};
template <>
struct IO<DT_F32> {
  typedef float T;
  struct Raw { f32x4 a, b; };
  static __device__ __forceinline__ Raw ldraw(const T* p) {
    return Raw{*reinterpret_cast<const f32x4*>(p), *reinterpret_cast<const f32x4*>(p + 4)};
  }
  static __device__ __forceinline__ float el(const Raw& r, int j) { return j < 4 ? r.a[j] : r.b[j - 4]; }
  static __device__ __forceinline__ void load8(const T* p, float* v) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  }
  static __device__ __forceinline__ void store8(T* p, const float* v) {
    f32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[4 + j]; }
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
  static __device__ __forceinline__ float load1(const T* p) { return *p; }
  static __device__ __forceinline__ void store1(T* p, float v) { *p = v; }
};

// Prologue of one 8-element vector: v = residual + dropout(x + bias). Stores h if asked.
template <int DT>
__device__ __forceinline__ void prologue8(float* v, const typename IO<DT>::T* bias,
                                          const typename IO<DT>::T* residual,
                                          typename IO<DT>::T* residual_out, size_t base, int col,
                                          float p_drop, float keep_scale, uint64_t seed,
                                          uint64_t offset) {
  typedef IO<DT> io;
  if (bias) {
    float b[8];
    io::load8(bias + col, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += b[j];
  }
  if (p_drop > 0.f) {
    float u[8];
    hash_uniform8(seed, offset, base + col, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = u[j] >= p_drop ? v[j] * keep_scale : 0.f;
  }
  if (residual) {
    float r[8];
    io::load8(residual + base + col, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += r[j];
  }
  if (residual_out) io::store8(residual_out + base + col, v);
}

// Two sums over a workgroup of NW waves with one LDS round (red holds 2 * NW floats).
template <int NW>
__device__ __forceinline__ void block_sum2(float& a, float& b, float* red) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { red[w] = a; red[NW + w] = b; }
  __syncthreads();
  a = 0.f; b = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) { a += red[i]; b += red[NW + i]; }
  __syncthreads();
}

// ---------------------------------------------------------------------------------- forward
// Wave per row. NV = 8-element vectors per lane (ceil(N / 512)), N <= 4096.
template <int NV, int DT>
__global__ __launch_bounds__(256) void ln_fwd_kernel(
    const typename IO<DT>::T* __restrict__ x, const typename IO<DT>::T* __restrict__ bias,
    const typename IO<DT>::T* __restrict__ residual, const typename IO<DT>::T* __restrict__ gamma,
    const typename IO<DT>::T* __restrict__ beta, typename IO<DT>::T* __restrict__ y,
    typename IO<DT>::T* __restrict__ residual_out, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int rows, int N, float eps, float p_drop, uint64_t seed,
    uint64_t offset, int rms) {
  typedef IO<DT> io;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = N >> 3;
  const size_t base = (size_t)row * N;
  float v[NV][8];
  float s = 0.f;
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * 64 + lane;
    if (vi < nvec) {
      io::load8(x + base + vi * 8, v[i]);
      prologue8<DT>(v[i], bias, residual, residual_out, base, vi * 8, p_drop, keep_scale, seed,
                    offset);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  const float mean = rms ? 0.f : wave_sum(s) / (float)N;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (i * 64 + lane < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { float d = v[i][j] - mean; ss += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)N + eps);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * 64 + lane;
    if (vi < nvec) {
      float g[8], b[8], o[8];
      if (gamma) io::load8(gamma + vi * 8, g); else for (int j = 0; j < 8; ++j) g[j] = 1.f;
      if (beta) io::load8(beta + vi * 8, b); else for (int j = 0; j < 8; ++j) b[j] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * g[j] + b[j];
      io::store8(y + base + vi * 8, o);
    }
  }
}

// Workgroup (NW waves) per row: the few-row decode case (NW = 4: every operand of the row is
// fetched in ONE round of 16 B loads issued up front, so the latency chain is load -> 2 block
// reductions -> store) and rows longer than 4096 (NW = 8, gamma/beta loaded late to bound VGPRs).
template <int NW, int NV, int DT>
__global__ __launch_bounds__(NW * 64) void ln_fwd_row_kernel(
    const typename IO<DT>::T* __restrict__ x, const typename IO<DT>::T* __restrict__ bias,
    const typename IO<DT>::T* __restrict__ residual, const typename IO<DT>::T* __restrict__ gamma,
    const typename IO<DT>::T* __restrict__ beta, typename IO<DT>::T* __restrict__ y,
    typename IO<DT>::T* __restrict__ residual_out, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int N, float eps, float p_drop, uint64_t seed, uint64_t offset,
    int rms) {
  typedef IO<DT> io;
  constexpr int T = NW * 64;
  constexpr bool EARLY = NW == 4;  // hold gamma/beta from the first load round
  __shared__ float red[2 * NW];
  const int row = blockIdx.x, t = threadIdx.x;
  const int nvec = N >> 3;
  const size_t base = (size_t)row * N;
  float v[NV][8], g[EARLY ? NV : 1][8], bb[EARLY ? NV : 1][8];
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * T + t;
    if (vi < nvec) {
      io::load8(x + base + vi * 8, v[i]);
      if (EARLY) {
        if (gamma) io::load8(gamma + vi * 8, g[i]); else for (int j = 0; j < 8; ++j) g[i][j] = 1.f;
        if (beta) io::load8(beta + vi * 8, bb[i]); else for (int j = 0; j < 8; ++j) bb[i][j] = 0.f;
      }
      prologue8<DT>(v[i], bias, residual, residual_out, base, vi * 8, p_drop, keep_scale, seed,
                    offset);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  float dummy = 0.f;
  if (!rms) block_sum2<NW>(s, dummy, red);
  const float mean = rms ? 0.f : s / (float)N;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (i * T + t < nvec)
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; ss += d * d; }
  block_sum2<NW>(ss, dummy, red);
  const float rstd = rsqrtf(ss / (float)N + eps);
  if (t == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * T + t;
    if (vi < nvec) {
      float o[8], gl[8], bl[8];
      const float* gp = g[EARLY ? i : 0];
      const float* bp = bb[EARLY ? i : 0];
      if (!EARLY) {
        if (gamma) io::load8(gamma + vi * 8, gl); else for (int j = 0; j < 8; ++j) gl[j] = 1.f;
        if (beta) io::load8(beta + vi * 8, bl); else for (int j = 0; j < 8; ++j) bl[j] = 0.f;
        gp = gl;
        bp = bl;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * gp[j] + bp[j];
      io::store8(y + base + vi * 8, o);
    }
  }
}

// ---------------------------------------------------------------------------------- backward
// x_hat is recomputed from the saved pre-norm input `h` (= residual_out of forward, or x when there
// is no prologue) and mean/rstd. Outputs:
//   dh = LN_bwd(dy) (+ d_res_in if given)      -> dres (grad of the residual input)
//   dx = dropout_bwd(dh)                        -> dx (grad of x / of x+bias), if dx
//   dgamma / dbeta / dbias(= column sums of dx)  -> f32 atomics into acc_*[N] (zeroed by launcher)
// RMSNorm: mean == 0 and the mean-gradient term m1 is dropped.

// Per-thread body over one row: TPR threads per row, the thread's vectors are vi = i * TPR + tid.
// Returns nothing; accumulates into dg/db/dbi.
template <int NV, int DT, int TPR, int NW>
__device__ __forceinline__ void ln_bwd_row(
    const typename IO<DT>::T* __restrict__ dy, const typename IO<DT>::T* __restrict__ h,
    const typename IO<DT>::T* __restrict__ gamma, float mean, float rstd,
    const typename IO<DT>::T* __restrict__ dres_in, typename IO<DT>::T* __restrict__ dres,
    typename IO<DT>::T* __restrict__ dx, size_t base, int tid, int nvec, int N, float p_drop,
    float keep_scale, uint64_t seed, uint64_t offset, int rms, float (&dg)[NV][8],
    float (&db)[NV][8], float (&dbi)[NV][8], float* red) {
  typedef IO<DT> io;
  // h, dy and the residual gradient of the row are loaded up front as raw vectors (all three
  // streams in flight together: one memory round trip per row) and x-hat / gamma*dy are recomputed
  // in the second pass instead of being held in f32 registers.
  typename io::Raw hr[NV], dr[NV], rr[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = min(i * TPR + tid, nvec - 1);
    hr[i] = io::ldraw(h + base + vi * 8);
    dr[i] = io::ldraw(dy + base + vi * 8);
    if (dres_in) rr[i] = io::ldraw(dres_in + base + vi * 8);
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * TPR + tid;
    if (vi < nvec) {
      float g[8];
      if (gamma) io::load8(gamma + vi * 8, g); else for (int j = 0; j < 8; ++j) g[j] = 1.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = io::el(dr[i], j);
        const float xh = (io::el(hr[i], j) - mean) * rstd;
        const float gd = d * g[j];
        dg[i][j] += d * xh;
        db[i][j] += d;
        s1 += gd;
        s2 += gd * xh;
      }
    }
  }
  if constexpr (NW == 0) {  // wave per row
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
  } else {
    block_sum2<NW>(s1, s2, red);
  }
  const float m1 = rms ? 0.f : s1 / (float)N, m2 = s2 / (float)N;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * TPR + tid;
    if (vi < nvec) {
      float g[8], o[8];
      if (gamma) io::load8(gamma + vi * 8, g); else for (int j = 0; j < 8; ++j) g[j] = 1.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (io::el(hr[i], j) - mean) * rstd;
        o[j] = rstd * (io::el(dr[i], j) * g[j] - m1 - xh * m2);
        if (dres_in) o[j] += io::el(rr[i], j);
      }
      if (dres) io::store8(dres + base + vi * 8, o);
      if (dx) {
        if (p_drop > 0.f) {
          float u[8];
          hash_uniform8(seed, offset, base + vi * 8, u);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = u[j] >= p_drop ? o[j] * keep_scale : 0.f;
        }
        io::store8(dx + base + vi * 8, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) dbi[i][j] += o[j];
      }
    }
  }
}

template <int NV, int DT>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const typename IO<DT>::T* __restrict__ dy, const typename IO<DT>::T* __restrict__ h,
    const typename IO<DT>::T* __restrict__ gamma, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const typename IO<DT>::T* __restrict__ dres_in,
    typename IO<DT>::T* __restrict__ dres, typename IO<DT>::T* __restrict__ dx,
    float* __restrict__ acc_dg, float* __restrict__ acc_db, float* __restrict__ acc_dbias,
    int rows, int N, float p_drop, uint64_t seed, uint64_t offset, int rms) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nvec = N >> 3;
  float dg[NV][8], db[NV][8], dbi[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { dg[i][j] = 0.f; db[i][j] = 0.f; dbi[i][j] = 0.f; }
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  typedef IO<DT> io;
  for (int row = blockIdx.x * 4 + w; row < rows; row += gridDim.x * 4) {
    const size_t base = (size_t)row * N;
    const float mean = mean_in[row], rstd = rstd_in[row];
    typename io::Raw hr[NV], dr[NV], rr[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = min(i * 64 + lane, nvec - 1);
      hr[i] = io::ldraw(h + base + vi * 8);
      dr[i] = io::ldraw(dy + base + vi * 8);
      if (dres_in) rr[i] = io::ldraw(dres_in + base + vi * 8);
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = i * 64 + lane;
      if (vi < nvec) {
        float g[8];
        if (gamma) io::load8(gamma + vi * 8, g); else for (int j = 0; j < 8; ++j) g[j] = 1.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = io::el(dr[i], j);
          const float xh = (io::el(hr[i], j) - mean) * rstd;
          const float gd = d * g[j];
          dg[i][j] += d * xh;
          db[i][j] += d;
          s1 += gd;
          s2 += gd * xh;
        }
      }
    }
    const float m1 = rms ? 0.f : wave_sum(s1) / (float)N, m2 = wave_sum(s2) / (float)N;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = i * 64 + lane;
      if (vi < nvec) {
        float g[8], o[8];
        if (gamma) io::load8(gamma + vi * 8, g); else for (int j = 0; j < 8; ++j) g[j] = 1.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (io::el(hr[i], j) - mean) * rstd;
          o[j] = rstd * (io::el(dr[i], j) * g[j] - m1 - xh * m2);
          if (dres_in) o[j] += io::el(rr[i], j);
        }
        if (dres) io::store8(dres + base + vi * 8, o);
        if (dx) {
          if (p_drop > 0.f) {
            float u[8];
            hash_uniform8(seed, offset, base + vi * 8, u);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = u[j] >= p_drop ? o[j] * keep_scale : 0.f;
          }
          io::store8(dx + base + vi * 8, o);
#pragma unroll
          for (int j = 0; j < 8; ++j) dbi[i][j] += o[j];
        }
      }
    }
  }
  // Block-reduce the 4 waves' column partials through LDS, then one plain coalesced store per
  // column into this block's row of the [G][N] slab (slab_reduce_kernel folds the G rows).
  __shared__ float red[4][512];
  float* outs[3] = {acc_dg, acc_db, acc_dbias};
  const size_t srow = (size_t)blockIdx.x * N;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (!outs[q]) continue;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[w][lane * 8 + j] = q == 0 ? dg[i][j] : (q == 1 ? db[i][j] : dbi[i][j]);
      __syncthreads();
      for (int c = threadIdx.x; c < 512; c += 256) {
        const int col = i * 512 + c;
        if (col < N) outs[q][srow + col] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
      }
      __syncthreads();
    }
  }
}

// 1024 < N <= 2048 (GPT-1.3B's 2048): TWO waves per row, each owning half the columns (2 vectors
// per lane), and the NEXT row's h / dy / mean / rstd prefetched into a second register stage, so
// every wave keeps two row fetches in flight (h, dy and the residual gradient of the next row
// prefetched) at <= 168 VGPRs (3 waves per SIMD); the wave-per-row
// kernel at this width holds 220 VGPRs for one row (2 waves per SIMD). The halves' row sums meet
// through LDS (parity-double-buffered: one barrier per row); the trip count is uniform over the
// workgroup so both row pairs reach every barrier.
template <int DT>
__device__ __forceinline__ void ln_bwd_pair_body(
    const typename IO<DT>::T* __restrict__ dy, const typename IO<DT>::T* __restrict__ h,
    const typename IO<DT>::T* __restrict__ gamma, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const typename IO<DT>::T* __restrict__ dres_in,
    typename IO<DT>::T* __restrict__ dres, typename IO<DT>::T* __restrict__ dx,
    float* __restrict__ acc_dg, float* __restrict__ acc_db, float* __restrict__ acc_dbias,
    int rows, int N, float p_drop, uint64_t seed, uint64_t offset, int rms) {
  typedef IO<DT> io;
  constexpr int NV = 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, half = w & 1, rp = w >> 1;
  const int nvec = N >> 3;
  __shared__ float red[2][2][2][2];  // [parity][row pair][half][s1, s2]
  float dg[NV][8], db[NV][8], dbi[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { dg[i][j] = 0.f; db[i][j] = 0.f; dbi[i][j] = 0.f; }
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  const bool one_store = dx == dres && p_drop == 0.f;  // dres and dx alias: the same values
  const int stride = gridDim.x * 2;
  const int row0 = blockIdx.x * 2 + rp;
  const int iters = rows > (int)blockIdx.x * 2 ? (rows - (int)blockIdx.x * 2 + stride - 1) / stride : 0;
  typename io::Raw hr2[2][NV], dr2[2][NV], rr2[2][NV];
  float mean2[2], rstd2[2];
  auto vcol = [&](int i) { return half * (NV * 64) + i * 64 + lane; };
  auto load = [&](int row, auto pc) {
    constexpr int P = decltype(pc)::value;
    const int r = min(row, rows - 1);
    const size_t base = (size_t)r * N;
    mean2[P] = mean_in[r];
    rstd2[P] = rstd_in[r];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = min(vcol(i), nvec - 1);
      hr2[P][i] = io::ldraw(h + base + vi * 8);
      dr2[P][i] = io::ldraw(dy + base + vi * 8);
      if (dres_in) rr2[P][i] = io::ldraw(dres_in + base + vi * 8);  // prefetched with h / dy
    }
  };
  auto body = [&](int k, auto pc) {
    constexpr int P = decltype(pc)::value;
    const int row = row0 + k * stride;
    const bool valid = row < rows;
    const size_t base = (size_t)min(row, rows - 1) * N;
    const float mean = mean2[P], rstd = rstd2[P];
    const auto& hr = hr2[P];
    const auto& dr = dr2[P];
    const auto& rr = rr2[P];
    typename io::Raw gr[NV];  // gamma: L1-resident, re-read per row (registers are the limit)
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (gamma) gr[i] = io::ldraw(gamma + min(vcol(i), nvec - 1) * 8);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (valid && vcol(i) < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = io::el(dr[i], j);
          const float xh = (io::el(hr[i], j) - mean) * rstd;
          const float gd = d * (gamma ? io::el(gr[i], j) : 1.f);
          dg[i][j] += d * xh;
          db[i][j] += d;
          s1 += gd;
          s2 += gd * xh;
        }
      }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      red[P][rp][half][0] = s1;
      red[P][rp][half][1] = s2;
    }
    __syncthreads();
    const float t1 = red[P][rp][0][0] + red[P][rp][1][0], t2 = red[P][rp][0][1] + red[P][rp][1][1];
    const float m1 = rms ? 0.f : t1 / (float)N, m2 = t2 / (float)N;
    if (!valid) return;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = vcol(i);
      if (vi < nvec) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (io::el(hr[i], j) - mean) * rstd;
          o[j] = rstd * (io::el(dr[i], j) * (gamma ? io::el(gr[i], j) : 1.f) - m1 - xh * m2);
          if (dres_in) o[j] += io::el(rr[i], j);
        }
        if (dres && !one_store) io::store8(dres + base + vi * 8, o);
        if (dx) {
          if (p_drop > 0.f) {
            float u[8];
            hash_uniform8(seed, offset, base + vi * 8, u);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = u[j] >= p_drop ? o[j] * keep_scale : 0.f;
          }
          io::store8(dx + base + vi * 8, o);
#pragma unroll
          for (int j = 0; j < 8; ++j) dbi[i][j] += o[j];
        }
      }
    }
  };
  if (iters > 0) load(row0, std::integral_constant<int, 0>{});
  for (int k = 0; k < iters; k += 2) {
    if (k + 1 < iters) load(row0 + (k + 1) * stride, std::integral_constant<int, 1>{});
    body(k, std::integral_constant<int, 0>{});
    if (k + 1 >= iters) break;
    if (k + 2 < iters) load(row0 + (k + 2) * stride, std::integral_constant<int, 0>{});
    body(k + 1, std::integral_constant<int, 1>{});
  }
  // the two row pairs' column partials of each half meet in LDS; one slab row per workgroup
  __shared__ float cmb[2][64][NV * 8];
  float* outs[3] = {acc_dg, acc_db, acc_dbias};
  const size_t srow = (size_t)blockIdx.x * N;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (!outs[q]) continue;
    if (rp == 1)
#pragma unroll
      for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) cmb[half][lane][i * 8 + j] = q == 0 ? dg[i][j] : (q == 1 ? db[i][j] : dbi[i][j]);
    __syncthreads();
    if (rp == 0) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int vi = vcol(i);
        if (vi >= nvec) continue;
        f32x4 a, b;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = (q == 0 ? dg[i][j] : (q == 1 ? db[i][j] : dbi[i][j])) + cmb[half][lane][i * 8 + j];
          b[j] = (q == 0 ? dg[i][4 + j] : (q == 1 ? db[i][4 + j] : dbi[i][4 + j])) + cmb[half][lane][i * 8 + 4 + j];
        }
        *reinterpret_cast<f32x4*>(outs[q] + srow + vi * 8) = a;
        *reinterpret_cast<f32x4*>(outs[q] + srow + vi * 8 + 4) = b;
      }
    }
    __syncthreads();
  }
}


// 16-bit: 3 waves per SIMD (<= 168 VGPRs with the residual-gradient prefetch); f32 rows hold
// twice the register bytes and keep the compiler's own allocation
#define LN_BWD_PAIR_PARAMS                                                                         \
  const typename IO<DT>::T *__restrict__ dy, const typename IO<DT>::T *__restrict__ h,             \
      const typename IO<DT>::T *__restrict__ gamma, const float *__restrict__ mean_in,             \
      const float *__restrict__ rstd_in, const typename IO<DT>::T *__restrict__ dres_in,           \
      typename IO<DT>::T *__restrict__ dres, typename IO<DT>::T *__restrict__ dx,                  \
      float *__restrict__ acc_dg, float *__restrict__ acc_db, float *__restrict__ acc_dbias, int rows, \
      int N, float p_drop, uint64_t seed, uint64_t offset, int rms
#define LN_BWD_PAIR_ARGS dy, h, gamma, mean_in, rstd_in, dres_in, dres, dx, acc_dg, acc_db, acc_dbias, \
                         rows, N, p_drop, seed, offset, rms
template <int DT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void ln_bwd_pair_kernel(
    LN_BWD_PAIR_PARAMS) {
  ln_bwd_pair_body<DT>(LN_BWD_PAIR_ARGS);
}
template <int DT>
__global__ __launch_bounds__(256) void ln_bwd_pair_kernel_f32(LN_BWD_PAIR_PARAMS) {
  ln_bwd_pair_body<DT>(LN_BWD_PAIR_ARGS);
}
#undef LN_BWD_PAIR_PARAMS
#undef LN_BWD_PAIR_ARGS
// Rows longer than 2048 (the wave-per-row variant would drop to 1 wave/SIMD): a 512-thread
// workgroup per row (NV = ceil(N / 4096) <= 4 vectors per thread), grid-stride over rows; every thread owns distinct columns, so the column partials go
// straight to the atomics without an LDS reduction.
template <int NV, int DT>
__global__ __launch_bounds__(512) void ln_bwd_wide_kernel(
    const typename IO<DT>::T* __restrict__ dy, const typename IO<DT>::T* __restrict__ h,
    const typename IO<DT>::T* __restrict__ gamma, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const typename IO<DT>::T* __restrict__ dres_in,
    typename IO<DT>::T* __restrict__ dres, typename IO<DT>::T* __restrict__ dx,
    float* __restrict__ acc_dg, float* __restrict__ acc_db, float* __restrict__ acc_dbias,
    int rows, int N, float p_drop, uint64_t seed, uint64_t offset, int rms) {
  __shared__ float red[16];
  const int nvec = N >> 3;
  float dg[NV][8], db[NV][8], dbi[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { dg[i][j] = 0.f; db[i][j] = 0.f; dbi[i][j] = 0.f; }
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  for (int row = blockIdx.x; row < rows; row += gridDim.x)
    ln_bwd_row<NV, DT, 512, 8>(dy, h, gamma, mean_in[row], rstd_in[row], dres_in, dres, dx,
                               (size_t)row * N, threadIdx.x, nvec, N, p_drop, keep_scale, seed,
                               offset, rms, dg, db, dbi, red);
  float* outs[3] = {acc_dg, acc_db, acc_dbias};
  const size_t srow = (size_t)blockIdx.x * N;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (!outs[q]) continue;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = i * 512 + threadIdx.x;
      if (vi < nvec) {
        f32x4 a, b;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = q == 0 ? dg[i][j] : (q == 1 ? db[i][j] : dbi[i][j]);
          b[j] = q == 0 ? dg[i][4 + j] : (q == 1 ? db[i][4 + j] : dbi[i][4 + j]);
        }
        *reinterpret_cast<f32x4*>(outs[q] + srow + vi * 8) = a;
        *reinterpret_cast<f32x4*>(outs[q] + srow + vi * 8 + 4) = b;
      }
    }
  }
}

// [G][N] slab of per-workgroup column partials -> acc[N] (zeroed): block (bx, gy, q) sums rows
// gy*16 .. +16 of 1024 columns with 16 B loads, then one f32 atomic per column. G x N x 4 B of
// plain traffic + (G / 16) x N atomics, instead of G x N contended atomics from the backward
// kernel itself (those dominated the N = 8192 / 16384 backward).
__global__ __launch_bounds__(256) void slab_reduce_kernel(float* __restrict__ s0, float* __restrict__ s1,
                                                          float* __restrict__ s2, float* __restrict__ a0,
                                                          float* __restrict__ a1, float* __restrict__ a2,
                                                          int G, int N) {
  const int q = blockIdx.z;
  const float* slab = q == 0 ? s0 : (q == 1 ? s1 : s2);
  float* acc = q == 0 ? a0 : (q == 1 ? a1 : a2);
  if (!slab) return;
  const int c4 = blockIdx.x * 1024 + threadIdx.x * 4;
  if (c4 >= N) return;
  const int g0 = blockIdx.y * 16, g1 = min(g0 + 16, G);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int g = g0; g < g1; ++g) s += *reinterpret_cast<const f32x4*>(slab + (size_t)g * N + c4);
#pragma unroll
  for (int j = 0; j < 4; ++j) atomicAdd(acc + c4 + j, s[j]);
}

// acc[N] (f32, summed over blocks) -> out[N] in the parameter dtype (or += into it).
template <int DT>
__global__ __launch_bounds__(256) void col_sum_kernel(const float* __restrict__ part, int G, int N,
                                                     typename IO<DT>::T* __restrict__ out,
                                                     int accumulate) {
  // 256 threads = 64 columns x 4 row-groups
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (col < N)
    for (int g = rg; g < G; g += 4) s += part[(size_t)g * N + col];
  __shared__ float red[4][64];
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && col < N) {
    float t = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    if (accumulate) t += IO<DT>::load1(out + col);
    IO<DT>::store1(out + col, t);
  }
}

template <int DT>
int launch_fwd(const void* x, const void* bias, const void* residual, const void* gamma,
               const void* beta, void* y, void* residual_out, float* mean, float* rstd, int rows,
               int N, float eps, float p, uint64_t seed, uint64_t off, int rms, hipStream_t st) {
  typedef typename IO<DT>::T T;
#define ROW_ARGS (const T*)x, (const T*)bias, (const T*)residual, (const T*)gamma, (const T*)beta, \
                 (T*)y, (T*)residual_out, mean, rstd, N, eps, p, seed, off, rms
  if (N > 4096) {  // wide rows: 512-thread workgroup per row
    switch ((N / 8 + 511) / 512) {
      case 2: hipLaunchKernelGGL((ln_fwd_row_kernel<8, 2, DT>), dim3(rows), dim3(512), 0, st, ROW_ARGS); break;
      case 3: hipLaunchKernelGGL((ln_fwd_row_kernel<8, 3, DT>), dim3(rows), dim3(512), 0, st, ROW_ARGS); break;
      case 4: hipLaunchKernelGGL((ln_fwd_row_kernel<8, 4, DT>), dim3(rows), dim3(512), 0, st, ROW_ARGS); break;
      default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
  }
  // few rows (decode, batch-1 encoders): a workgroup per row — 4x the waves of the wave-per-row
  // kernel, one 16-B load per lane per operand, so the load -> reduce -> store chain is shortest
  static const int row_max = [] {
    const char* e = getenv("PIAMD_LN_ROW_MAX");
    return e ? atoi(e) : 512;
  }();
  if (rows <= row_max) {
    switch ((N / 8 + 255) / 256) {
      case 1: hipLaunchKernelGGL((ln_fwd_row_kernel<4, 1, DT>), dim3(rows), dim3(256), 0, st, ROW_ARGS); break;
      case 2: hipLaunchKernelGGL((ln_fwd_row_kernel<4, 2, DT>), dim3(rows), dim3(256), 0, st, ROW_ARGS); break;
      default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
  }
#undef ROW_ARGS
  const int nv = (N / 8 + 63) / 64;
  dim3 grid((rows + 3) / 4), block(256);
#define LNF(NVV)                                                                                  \
  hipLaunchKernelGGL((ln_fwd_kernel<NVV, DT>), grid, block, 0, st, (const T*)x, (const T*)bias, \
                     (const T*)residual, (const T*)gamma, (const T*)beta, (T*)y,               \
                     (T*)residual_out, mean, rstd, rows, N, eps, p, seed, off, rms);           \
  break;
  switch (nv) {
    case 1: LNF(1)
    case 2: LNF(2)
    case 3: LNF(3)
    case 4: LNF(4)
    case 5: case 6: LNF(6)
    case 7: case 8: LNF(8)
    default: return (int)hipErrorInvalidValue;
  }
#undef LNF
  return (int)hipGetLastError();
}

// 1024 < N <= 2048 on the two-waves-per-row kernel (PIAMD_LN_BWD_PAIR=0: the wave-per-row one)
static inline bool bwd_pair(int N) {
  static const bool on = [] {
    const char* e = getenv("PIAMD_LN_BWD_PAIR");
    return !(e && e[0] == '0');
  }();
  return on && N > 1024 && N <= 2048;
}

// Workgroups of the backward (= rows of the partial slab).
static inline int bwd_grid(int rows, int N) {
  if (bwd_pair(N)) {  // 2 rows per workgroup; ~160 VGPRs = 3 workgroups per CU, all resident
    const int g = (rows + 1) / 2;
    return g > 768 ? 768 : (g < 1 ? 1 : g);
  }
  const int g = N > 2048 ? rows : (rows + 3) / 4;
  return g > 512 ? 512 : (g < 1 ? 1 : g);
}

template <int DT>
int launch_bwd(const void* dy, const void* h, const void* gamma, const float* mean,
               const float* rstd, const void* dres_in, void* dres, void* dx, float* acc_dg,
               float* acc_db, float* acc_dbias, int rows, int N, float p, uint64_t seed,
               uint64_t off, int rms, hipStream_t st) {
  typedef typename IO<DT>::T T;
#define BWD_ARGS (const T*)dy, (const T*)h, (const T*)gamma, mean, rstd, (const T*)dres_in, \
                 (T*)dres, (T*)dx, acc_dg, acc_db, acc_dbias, rows, N, p, seed, off, rms
  if (N > 2048) {
    // 512-thread workgroup per row, grid-stride rows; 2 workgroups per CU
    dim3 grid(bwd_grid(rows, N)), block(512);
    switch ((N / 8 + 511) / 512) {
      case 1: hipLaunchKernelGGL((ln_bwd_wide_kernel<1, DT>), grid, block, 0, st, BWD_ARGS); break;
      case 2: hipLaunchKernelGGL((ln_bwd_wide_kernel<2, DT>), grid, block, 0, st, BWD_ARGS); break;
      case 3: hipLaunchKernelGGL((ln_bwd_wide_kernel<3, DT>), grid, block, 0, st, BWD_ARGS); break;
      case 4: hipLaunchKernelGGL((ln_bwd_wide_kernel<4, DT>), grid, block, 0, st, BWD_ARGS); break;
      default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
  }
  dim3 grid(bwd_grid(rows, N)), block(256);
  if (bwd_pair(N)) {
    if constexpr (DT == 0)
      hipLaunchKernelGGL((ln_bwd_pair_kernel_f32<DT>), grid, block, 0, st, BWD_ARGS);
    else
      hipLaunchKernelGGL((ln_bwd_pair_kernel<DT>), grid, block, 0, st, BWD_ARGS);
    return (int)hipGetLastError();
  }
  switch ((N / 8 + 63) / 64) {
    case 1: hipLaunchKernelGGL((ln_bwd_kernel<1, DT>), grid, block, 0, st, BWD_ARGS); break;
    case 2: hipLaunchKernelGGL((ln_bwd_kernel<2, DT>), grid, block, 0, st, BWD_ARGS); break;
    case 3: hipLaunchKernelGGL((ln_bwd_kernel<3, DT>), grid, block, 0, st, BWD_ARGS); break;
    case 4: hipLaunchKernelGGL((ln_bwd_kernel<4, DT>), grid, block, 0, st, BWD_ARGS); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef BWD_ARGS
  return (int)hipGetLastError();
}

// Many partial rows (G ≥ 64: the rowsum / dact-epilogue column-sum planes, 256-768 rows): 32
// columns per workgroup as 8 float4 lanes × 32 row groups, so each thread sums G / 32 rows (the
// 4-row-group kernel left ~N/64 workgroups each walking G / 4 rows serially: latency-bound,
// ≈ 17 µs per bias gradient in the GPT step). Fixed summation order: deterministic.
template <int DT>
__global__ __launch_bounds__(256) void col_sum4_kernel(const float* __restrict__ part, int G, int N,
                                                      typename IO<DT>::T* __restrict__ out,
                                                      int accumulate) {
  const int q = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int col = blockIdx.x * 32 + 4 * q;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (col < N) {
#pragma unroll 4
    for (int g = rg; g < G; g += 32) s += *reinterpret_cast<const f32x4*>(part + (size_t)g * N + col);
  }
  __shared__ f32x4 red[32][9];
  red[rg][q] = s;
  __syncthreads();
  if (threadIdx.x < 32) {  // thread (qq, j): column 4·qq + j of the block
    const int qq = threadIdx.x >> 2, j = threadIdx.x & 3, c = blockIdx.x * 32 + threadIdx.x;
    if (c < N) {
      float t = 0.f;
#pragma unroll 8
      for (int r = 0; r < 32; ++r) t += red[r][qq][j];
      if (accumulate) t += IO<DT>::load1(out + c);
      IO<DT>::store1(out + c, t);
    }
  }
}

template <int DT>
void launch_colsum_out(const float* part, int G, int N, void* out, int acc, hipStream_t st) {
  if (G >= 64 && N % 4 == 0 && ((uintptr_t)part & 15) == 0) {
    hipLaunchKernelGGL((col_sum4_kernel<DT>), dim3((N + 31) / 32), dim3(256), 0, st, part, G, N,
                       (typename IO<DT>::T*)out, acc);
    return;
  }
  hipLaunchKernelGGL((col_sum_kernel<DT>), dim3((N + 63) / 64), dim3(256), 0, st, part, G, N,
                     (typename IO<DT>::T*)out, acc);
}

}  // namespace

// dtype: 0 = f32, 1 = bf16, 2 = fp16. flags bit 0: RMSNorm. Any of bias / residual /
// residual_out / gamma / beta / mean / rstd may be null. N % 8 == 0, N <= 16384.
PIAMD_EXPORT int piamd_layernorm_fwd(int dtype, const void* x, const void* bias,
                                     const void* residual, const void* gamma, const void* beta,
                                     void* y, void* residual_out, float* mean, float* rstd,
                                     int rows, int N, float eps, float p_drop, uint64_t seed,
                                     uint64_t offset, int flags, hipStream_t stream) {
  if (N % 8 != 0 || N > 16384 || dtype < 0 || dtype > 2) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  const int rms = flags & 1;
#define FWD(D) launch_fwd<D>(x, bias, residual, gamma, beta, y, residual_out, mean, rstd, rows, N, \
                             eps, p_drop, seed, offset, rms, stream)
  return dtype == DT_BF16 ? FWD(DT_BF16) : (dtype == DT_F16 ? FWD(DT_F16) : FWD(DT_F32));
#undef FWD
}

// Floats of workspace piamd_layernorm_bwd needs: three [G][N] partial slabs + three [N] sums.
PIAMD_EXPORT long long piamd_layernorm_bwd_ws(int rows, int N) {
  return 3LL * ((long long)bwd_grid(rows, N) * N + N);
}

// Backward. ws: piamd_layernorm_bwd_ws(rows, N) floats. dgamma / dbeta / dbias outputs (same
// dtype as the activations) are written from the column sums, or added into per accum_mask bit.
PIAMD_EXPORT int piamd_layernorm_bwd(int dtype, const void* dy, const void* h, const void* gamma,
                                     const float* mean, const float* rstd, const void* dres_in,
                                     void* dres, void* dx, void* dgamma, void* dbeta, void* dbias,
                                     float* ws, int rows, int N, float p_drop, uint64_t seed,
                                     uint64_t offset, int accum_mask, int flags,
                                     hipStream_t stream) {
  if (N % 8 != 0 || N > 16384 || dtype < 0 || dtype > 2) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  const int rms = flags & 1;
  const int G = bwd_grid(rows, N);
  void* outs[3] = {dgamma, dbeta, dbias};
  float *slab[3], *acc[3];
  for (int q = 0; q < 3; ++q) {
    slab[q] = outs[q] ? ws + (size_t)q * G * N : nullptr;
    acc[q] = outs[q] ? ws + (size_t)3 * G * N + (size_t)q * N : nullptr;
    if (outs[q]) (void)hipMemsetAsync(acc[q], 0, sizeof(float) * N, stream);
  }
#define BWD(D) launch_bwd<D>(dy, h, gamma, mean, rstd, dres_in, dres, dx, slab[0], slab[1], slab[2], \
                             rows, N, p_drop, seed, offset, rms, stream)
  int e = dtype == DT_BF16 ? BWD(DT_BF16) : (dtype == DT_F16 ? BWD(DT_F16) : BWD(DT_F32));
#undef BWD
  if (e) return e;
  if (dgamma || dbeta || dbias)
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((N + 1023) / 1024, (G + 15) / 16, 3), dim3(256), 0,
                       stream, slab[0], slab[1], slab[2], acc[0], acc[1], acc[2], G, N);
  for (int q = 0; q < 3; ++q) {
    if (!outs[q]) continue;
    const int a = (accum_mask >> q) & 1;  // add into an existing grad (e.g. a flat main_grad view)
    if (dtype == DT_BF16) launch_colsum_out<DT_BF16>(acc[q], 1, N, outs[q], a, stream);
    else if (dtype == DT_F16) launch_colsum_out<DT_F16>(acc[q], 1, N, outs[q], a, stream);
    else launch_colsum_out<DT_F32>(acc[q], 1, N, outs[q], a, stream);
  }
  return (int)hipGetLastError();
}

// Column sum of a [rows][N] matrix into out[N] (bias gradients). Uses the same partial scheme.
template <int DT>
__global__ __launch_bounds__(256) void rowsum_partial_kernel(const typename IO<DT>::T* __restrict__ x,
                                                            int rows, int N,
                                                            float* __restrict__ part) {
  // block handles 256 columns (one per thread) over a grid-stride set of rows
  const int col = blockIdx.y * 256 + threadIdx.x;
  if (col >= N) return;
  float s = 0.f;
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    s += IO<DT>::load1(x + (size_t)r * N + col);
  }
  part[(size_t)blockIdx.x * N + col] = s;
}

// bf16 variant: 8 columns per thread (16-B loads), 4 rows in flight; block = 2048 columns.
__global__ __launch_bounds__(256) void rowsum_partial_bf16x8_kernel(const bf16_t* __restrict__ x,
                                                                    int rows, int N,
                                                                    float* __restrict__ part) {
  const int c8 = blockIdx.y * 256 + threadIdx.x;
  if (c8 * 8 >= N) return;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  constexpr int U = 4;
  for (int r0 = blockIdx.x; r0 < rows; r0 += U * gridDim.x) {
    u16x8 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = min(r0 + u * (int)gridDim.x, rows - 1);
      v[u] = reinterpret_cast<const u16x8*>(x + (size_t)r * N)[c8];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (r0 + u * (int)gridDim.x < rows)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += bf2f(v[u][j]);
  }
  float* p = part + (size_t)blockIdx.x * N + c8 * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) p[j] = s[j];
}

PIAMD_EXPORT int piamd_colsum(int dtype, const void* x, void* out, float* part, int G, int rows,
                              int N, int accumulate, hipStream_t stream) {
  if (rows == 0) return 0;
  if (dtype < 0 || dtype > 2) return (int)hipErrorInvalidValue;
  dim3 grid(G, (N + 255) / 256), block(256);
  if (dtype == DT_BF16 && N % 8 == 0)
    hipLaunchKernelGGL(rowsum_partial_bf16x8_kernel, dim3(G, (N / 8 + 255) / 256), block, 0, stream,
                       (const bf16_t*)x, rows, N, part);
  else if (dtype == DT_BF16)
    hipLaunchKernelGGL((rowsum_partial_kernel<DT_BF16>), grid, block, 0, stream, (const bf16_t*)x,
                       rows, N, part);
  else if (dtype == DT_F16)
    hipLaunchKernelGGL((rowsum_partial_kernel<DT_F16>), grid, block, 0, stream,
                       (const unsigned short*)x, rows, N, part);
  else
    hipLaunchKernelGGL((rowsum_partial_kernel<DT_F32>), grid, block, 0, stream, (const float*)x,
                       rows, N, part);
  if (dtype == DT_BF16) launch_colsum_out<DT_BF16>(part, G, N, out, accumulate, stream);
  else if (dtype == DT_F16) launch_colsum_out<DT_F16>(part, G, N, out, accumulate, stream);
  else launch_colsum_out<DT_F32>(part, G, N, out, accumulate, stream);
  return (int)hipGetLastError();
}

// out[N] (+)= Σ_g part[g][N] (f32 partial rows — e.g. the column-sum planes the assembly GEMM's
// dact epilogue writes, piamd_agemm2 colsum): the bias gradient without a pass over the activation.
PIAMD_EXPORT int piamd_colsum_parts(int dtype, const float* part, int G, int N, void* out, int accumulate,
                                    hipStream_t stream) {
  if (G <= 0 || N <= 0) return 0;
  if (dtype == DT_BF16) launch_colsum_out<DT_BF16>(part, G, N, out, accumulate, stream);
  else if (dtype == DT_F16) launch_colsum_out<DT_F16>(part, G, N, out, accumulate, stream);
  else if (dtype == DT_F32) launch_colsum_out<DT_F32>(part, G, N, out, accumulate, stream);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
