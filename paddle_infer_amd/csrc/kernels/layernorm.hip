// LayerNorm forward / backward with optional fused bias + dropout + residual-add prologue.
//
// Parity: reference `paddle/phi/kernels/gpu/layer_norm_kernel.cu`,
// `paddle/fluid/operators/fused/fused_layernorm_residual_dropout_bias.h` and
// `fused_bias_dropout_residual_layer_norm_op.cu` (the `fused_bias_dropout_residual_layer_norm`
// op: out = LN(residual + dropout(x + bias))).
//
// MI355X design: one wave64 per row for rows of up to 8192 elements, the whole row held in
// registers (16 B/lane loads: each vector instruction moves 1 KiB contiguous), exact two-pass
// mean/variance from registers (no Welford, no second HBM read). 4 rows per 256-thread block so a
// 8192×2048 activation gets 2048 blocks (≫ 256 CUs). Backward fuses dgamma/dbeta: every wave
// accumulates its columns across a grid-stride set of rows in registers, the block reduces them
// in LDS and adds one f32 atomic per column (no [blocks x N] partial slab, no second pass). Dropout masks are regenerated from a stateless hash in
// backward (no mask tensor in HBM).
#include "common.h"

namespace {

template <bool BF16>
struct IO;
template <>
struct IO<true> {
  typedef bf16_t T;
  typedef u16x8 Raw;  // 8 elements held in 4 VGPRs until used
  static __device__ __forceinline__ Raw ldraw(const T* p) { return *reinterpret_cast<const Raw*>(p); }
  static __device__ __forceinline__ float el(const Raw& r, int j) { return bf2f(r[j]); }
  static __device__ __forceinline__ void load8(const T* p, float* v) {
    u16x8 r = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f(r[j]);
  }
  static __device__ __forceinline__ void store8(T* p, const float* v) {
    u16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = f2bf(v[j]);
    *reinterpret_cast<u16x8*>(p) = r;
  }
};
template <>
struct IO<false> {
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
};

// NV = max 8-element vectors per lane (ceil(N / 512)).
template <int NV, bool BF16>
__global__ __launch_bounds__(256) void ln_fwd_kernel(
    const typename IO<BF16>::T* __restrict__ x, const typename IO<BF16>::T* __restrict__ bias,
    const typename IO<BF16>::T* __restrict__ residual, const typename IO<BF16>::T* __restrict__ gamma,
    const typename IO<BF16>::T* __restrict__ beta, typename IO<BF16>::T* __restrict__ y,
    typename IO<BF16>::T* __restrict__ residual_out, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int rows, int N, float eps, float p_drop, uint64_t seed,
    uint64_t offset) {
  typedef IO<BF16> io;
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
      if (bias) {
        float b[8];
        io::load8(bias + vi * 8, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += b[j];
      }
      if (p_drop > 0.f) {
        float u[8];
        hash_uniform8(seed, offset, base + vi * 8, u);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[i][j] = u[j] >= p_drop ? v[i][j] * keep_scale : 0.f;
        }
      }
      if (residual) {
        float r[8];
        io::load8(residual + base + vi * 8, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
      }
      if (residual_out) io::store8(residual_out + base + vi * 8, v[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)N;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * 64 + lane;
    if (vi < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { float d = v[i][j] - mean; ss += d * d; }
    }
  }
  const float var = wave_sum(ss) / (float)N;
  const float rstd = rsqrtf(var + eps);
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

// Few-row variant (decode: rows = batch): one 256-thread workgroup per row so every operand of
// the row (x, bias, residual, gamma, beta) is fetched in ONE round of 16 B loads issued up front;
// the latency chain is load → block reduce ×2 → store instead of NV dependent wave iterations.
template <int NV, bool BF16>
__global__ __launch_bounds__(256) void ln_fwd_row_kernel(
    const typename IO<BF16>::T* __restrict__ x, const typename IO<BF16>::T* __restrict__ bias,
    const typename IO<BF16>::T* __restrict__ residual, const typename IO<BF16>::T* __restrict__ gamma,
    const typename IO<BF16>::T* __restrict__ beta, typename IO<BF16>::T* __restrict__ y,
    typename IO<BF16>::T* __restrict__ residual_out, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int N, float eps, float p_drop, uint64_t seed, uint64_t offset) {
  typedef IO<BF16> io;
  __shared__ float red[4];
  const int row = blockIdx.x, t = threadIdx.x;
  const int nvec = N >> 3;
  const size_t base = (size_t)row * N;
  float v[NV][8], g[NV][8], bb[NV][8];
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * 256 + t;
    if (vi < nvec) {
      io::load8(x + base + vi * 8, v[i]);
      if (gamma) io::load8(gamma + vi * 8, g[i]); else for (int j = 0; j < 8; ++j) g[i][j] = 1.f;
      if (beta) io::load8(beta + vi * 8, bb[i]); else for (int j = 0; j < 8; ++j) bb[i][j] = 0.f;
      float b[8], r[8];
      if (bias) io::load8(bias + vi * 8, b);
      if (residual) io::load8(residual + base + vi * 8, r);
      float u[8];
      if (p_drop > 0.f) hash_uniform8(seed, offset, base + vi * 8, u);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = v[i][j] + (bias ? b[j] : 0.f);
        if (p_drop > 0.f) a = u[j] >= p_drop ? a * keep_scale : 0.f;
        v[i][j] = a + (residual ? r[j] : 0.f);
      }
      if (residual_out) io::store8(residual_out + base + vi * 8, v[i]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[i][j];
  const float mean = block_sum<4>(s, red) / (float)N;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (i * 256 + t < nvec)
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mean; ss += d * d; }
  const float rstd = rsqrtf(block_sum<4>(ss, red) / (float)N + eps);
  if (t == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = i * 256 + t;
    if (vi < nvec) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * g[i][j] + bb[i][j];
      io::store8(y + base + vi * 8, o);
    }
  }
}

// Backward. x_hat is recomputed from the saved pre-norm input `h` (= residual_out of forward, or x
// when no prologue) and mean/rstd. Outputs:
//   dh = LN_bwd(dy) (+ d_res_in if given)      -> written to dres (grad of residual input)
//   dx = dropout_bwd(dh)                        -> written to dx (grad of x / of x+bias), if dx
//   per-block partial dgamma/dbeta (+ dbias partial = column sums of dx) -> partials
template <int NV, bool BF16>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const typename IO<BF16>::T* __restrict__ dy, const typename IO<BF16>::T* __restrict__ h,
    const typename IO<BF16>::T* __restrict__ gamma, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const typename IO<BF16>::T* __restrict__ dres_in,
    typename IO<BF16>::T* __restrict__ dres, typename IO<BF16>::T* __restrict__ dx,
    float* __restrict__ part_dg, float* __restrict__ part_db, float* __restrict__ part_dbias,
    int rows, int N, float p_drop, uint64_t seed, uint64_t offset) {
  typedef IO<BF16> io;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nvec = N >> 3;
  float dg[NV][8], db[NV][8], dbi[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { dg[i][j] = 0.f; db[i][j] = 0.f; dbi[i][j] = 0.f; }
  const float keep_scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  for (int row = blockIdx.x * 4 + w; row < rows; row += gridDim.x * 4) {
    const size_t base = (size_t)row * N;
    const float mean = mean_in[row], rstd = rstd_in[row];
    // h, dy and the residual gradient of the row are loaded up front as raw vectors (all three
    // streams in flight together: one memory round trip per row, not one more after the row
    // reduction) and x-hat / gamma*dy are recomputed in the second pass instead of being held in
    // f32 registers: 2 waves/SIMD at N = 2048.
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
    const float m1 = wave_sum(s1) / (float)N, m2 = wave_sum(s2) / (float)N;
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
            for (int j = 0; j < 8; ++j) {
              o[j] = u[j] >= p_drop ? o[j] * keep_scale : 0.f;
            }
          }
          io::store8(dx + base + vi * 8, o);
#pragma unroll
          for (int j = 0; j < 8; ++j) dbi[i][j] += o[j];
        }
      }
    }
  }
  // Block-reduce the 4 waves' column partials through LDS, then ONE f32 atomic add per column
  // per block into acc[N] (zeroed by the launcher): G x N x 4 B of atomics, spread over the
  // kernel, instead of a [G][N] partial slab and a second column-sum pass.
  __shared__ float red[4][512];
  float* outs[3] = {part_dg, part_db, part_dbias};
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
        if (col < N) atomicAdd(outs[q] + col, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
      }
      __syncthreads();
    }
  }
}

// partials [G][N] -> out[N] (f32 or bf16)
template <bool BF16>
__global__ __launch_bounds__(256) void col_sum_kernel(const float* __restrict__ part, int G, int N,
                                                     typename IO<BF16>::T* __restrict__ out,
                                                     float* __restrict__ out_f32, int accumulate) {
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
    if (out_f32) {
      out_f32[col] = accumulate ? out_f32[col] + t : t;
    } else if (BF16) {
      if (accumulate) t += bf2f(((const bf16_t*)out)[col]);
      ((bf16_t*)out)[col] = f2bf(t);
    } else {
      if (accumulate) t += ((float*)out)[col];
      ((float*)out)[col] = t;
    }
  }
}

template <bool BF16>
int launch_fwd(const void* x, const void* bias, const void* residual, const void* gamma,
               const void* beta, void* y, void* residual_out, float* mean, float* rstd, int rows,
               int N, float eps, float p, uint64_t seed, uint64_t off, hipStream_t st) {
  typedef typename IO<BF16>::T T;
  if (rows <= 64) {  // few rows (decode): a workgroup per row
    const int nv2 = (N / 8 + 255) / 256;
#define LNR(NVV)                                                                                \
  case NVV:                                                                                     \
    hipLaunchKernelGGL((ln_fwd_row_kernel<NVV, BF16>), dim3(rows), dim3(256), 0, st,           \
                       (const T*)x, (const T*)bias, (const T*)residual, (const T*)gamma,       \
                       (const T*)beta, (T*)y, (T*)residual_out, mean, rstd, N, eps, p, seed, off); \
    return (int)hipGetLastError();
    switch (nv2) { LNR(1) LNR(2) LNR(3) LNR(4) default: break; }
#undef LNR
  }
  const int nv = (N / 8 + 63) / 64;
  dim3 grid((rows + 3) / 4), block(256);
#define LNF(NVV)                                                                              \
  case NVV:                                                                                     \
    hipLaunchKernelGGL((ln_fwd_kernel<NVV, BF16>), grid, block, 0, st, (const T*)x,            \
                       (const T*)bias, (const T*)residual, (const T*)gamma, (const T*)beta,    \
                       (T*)y, (T*)residual_out, mean, rstd, rows, N, eps, p, seed, off);       \
    break;
  switch (nv) {
    LNF(1) LNF(2) LNF(3) LNF(4) LNF(5) LNF(6) LNF(8) LNF(10) LNF(12) LNF(16)
    case 7: hipLaunchKernelGGL((ln_fwd_kernel<8, BF16>), grid, block, 0, st, (const T*)x, (const T*)bias, (const T*)residual, (const T*)gamma, (const T*)beta, (T*)y, (T*)residual_out, mean, rstd, rows, N, eps, p, seed, off); break;
    case 9: hipLaunchKernelGGL((ln_fwd_kernel<10, BF16>), grid, block, 0, st, (const T*)x, (const T*)bias, (const T*)residual, (const T*)gamma, (const T*)beta, (T*)y, (T*)residual_out, mean, rstd, rows, N, eps, p, seed, off); break;
    case 11: hipLaunchKernelGGL((ln_fwd_kernel<12, BF16>), grid, block, 0, st, (const T*)x, (const T*)bias, (const T*)residual, (const T*)gamma, (const T*)beta, (T*)y, (T*)residual_out, mean, rstd, rows, N, eps, p, seed, off); break;
    case 13: case 14: case 15: hipLaunchKernelGGL((ln_fwd_kernel<16, BF16>), grid, block, 0, st, (const T*)x, (const T*)bias, (const T*)residual, (const T*)gamma, (const T*)beta, (T*)y, (T*)residual_out, mean, rstd, rows, N, eps, p, seed, off); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef LNF
  return (int)hipGetLastError();
}

template <bool BF16>
int launch_bwd(const void* dy, const void* h, const void* gamma, const float* mean,
               const float* rstd, const void* dres_in, void* dres, void* dx, float* part_dg,
               float* part_db, float* part_dbias, int G, int rows, int N, float p, uint64_t seed,
               uint64_t off, hipStream_t st) {
  typedef typename IO<BF16>::T T;
  const int nv = (N / 8 + 63) / 64;
  dim3 grid(G), block(256);
#define LNB(NVV)                                                                               \
  case NVV:                                                                                    \
    hipLaunchKernelGGL((ln_bwd_kernel<NVV, BF16>), grid, block, 0, st, (const T*)dy,          \
                       (const T*)h, (const T*)gamma, mean, rstd, (const T*)dres_in, (T*)dres, \
                       (T*)dx, part_dg, part_db, part_dbias, rows, N, p, seed, off);          \
    break;
  switch (nv) {
    LNB(1) LNB(2) LNB(3) LNB(4) LNB(5) LNB(6) LNB(8)
    case 7: hipLaunchKernelGGL((ln_bwd_kernel<8, BF16>), grid, block, 0, st, (const T*)dy, (const T*)h, (const T*)gamma, mean, rstd, (const T*)dres_in, (T*)dres, (T*)dx, part_dg, part_db, part_dbias, rows, N, p, seed, off); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef LNB
  return (int)hipGetLastError();
}

}  // namespace

// dtype: 0 = f32, 1 = bf16. Any of bias/residual/residual_out/gamma/beta/mean/rstd may be null.
PIAMD_EXPORT int piamd_layernorm_fwd(int dtype, const void* x, const void* bias,
                                     const void* residual, const void* gamma, const void* beta,
                                     void* y, void* residual_out, float* mean, float* rstd,
                                     int rows, int N, float eps, float p_drop, uint64_t seed,
                                     uint64_t offset, hipStream_t stream) {
  if (N % 8 != 0 || N > 8192) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  return dtype ? launch_fwd<true>(x, bias, residual, gamma, beta, y, residual_out, mean, rstd,
                                  rows, N, eps, p_drop, seed, offset, stream)
               : launch_fwd<false>(x, bias, residual, gamma, beta, y, residual_out, mean, rstd,
                                   rows, N, eps, p_drop, seed, offset, stream);
}

// Number of partial rows the backward uses (caller allocates partials [G][N] f32).
PIAMD_EXPORT int piamd_layernorm_bwd_grid(int rows) {
  int g = (rows + 3) / 4;
  return g > 512 ? 512 : (g < 1 ? 1 : g);
}

// Backward. part_* are f32 [N] accumulators (zeroed here); dgamma/dbeta/dbias outputs (dtype of
// the params) are converted from them; each may be null.
PIAMD_EXPORT int piamd_layernorm_bwd(int dtype, const void* dy, const void* h, const void* gamma,
                                     const float* mean, const float* rstd, const void* dres_in,
                                     void* dres, void* dx, void* dgamma, void* dbeta, void* dbias,
                                     float* part_dg, float* part_db, float* part_dbias, int rows,
                                     int N, float p_drop, uint64_t seed, uint64_t offset,
                                     int accum_mask, hipStream_t stream) {
  if (N % 8 != 0 || N > 4096) return (int)hipErrorInvalidValue;
  if (rows == 0) return 0;
  const int G = piamd_layernorm_bwd_grid(rows);
  if (dgamma) (void)hipMemsetAsync(part_dg, 0, sizeof(float) * N, stream);
  if (dbeta) (void)hipMemsetAsync(part_db, 0, sizeof(float) * N, stream);
  if (dbias) (void)hipMemsetAsync(part_dbias, 0, sizeof(float) * N, stream);
  int e = dtype ? launch_bwd<true>(dy, h, gamma, mean, rstd, dres_in, dres, dx,
                                   dgamma ? part_dg : nullptr, dbeta ? part_db : nullptr,
                                   dbias ? part_dbias : nullptr, G, rows, N, p_drop, seed, offset,
                                   stream)
                : launch_bwd<false>(dy, h, gamma, mean, rstd, dres_in, dres, dx,
                                    dgamma ? part_dg : nullptr, dbeta ? part_db : nullptr,
                                    dbias ? part_dbias : nullptr, G, rows, N, p_drop, seed,
                                    offset, stream);
  if (e) return e;
  void* outs[3] = {dgamma, dbeta, dbias};
  float* parts[3] = {part_dg, part_db, part_dbias};
  for (int q = 0; q < 3; ++q) {
    if (!outs[q]) continue;
    dim3 grid((N + 63) / 64), block(256);
    const int acc = (accum_mask >> q) & 1;  // add into an existing grad (e.g. a flat main_grad view)
    if (dtype)
      hipLaunchKernelGGL((col_sum_kernel<true>), grid, block, 0, stream, parts[q], 1, N,
                         (bf16_t*)outs[q], (float*)nullptr, acc);
    else
      hipLaunchKernelGGL((col_sum_kernel<false>), grid, block, 0, stream, parts[q], 1, N,
                         (float*)outs[q], (float*)nullptr, acc);
  }
  return (int)hipGetLastError();
}

// Column sum of a [rows][N] matrix into out[N] (bias gradients). Uses the same partial scheme.
template <bool BF16>
__global__ __launch_bounds__(256) void rowsum_partial_kernel(const typename IO<BF16>::T* __restrict__ x,
                                                            int rows, int N,
                                                            float* __restrict__ part) {
  // block handles 256 columns (one per thread) over a grid-stride set of rows
  const int col = blockIdx.y * 256 + threadIdx.x;
  if (col >= N) return;
  float s = 0.f;
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    if (BF16) s += bf2f(((const bf16_t*)x)[(size_t)r * N + col]);
    else s += ((const float*)x)[(size_t)r * N + col];
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
  dim3 grid(G, (N + 255) / 256), block(256);
  if (dtype && N % 8 == 0)
    hipLaunchKernelGGL(rowsum_partial_bf16x8_kernel, dim3(G, (N / 8 + 255) / 256), block, 0, stream,
                       (const bf16_t*)x, rows, N, part);
  else if (dtype)
    hipLaunchKernelGGL((rowsum_partial_kernel<true>), grid, block, 0, stream, (const bf16_t*)x,
                       rows, N, part);
  else
    hipLaunchKernelGGL((rowsum_partial_kernel<false>), grid, block, 0, stream, (const float*)x,
                       rows, N, part);
  dim3 g2((N + 63) / 64);
  if (dtype)
    hipLaunchKernelGGL((col_sum_kernel<true>), g2, dim3(256), 0, stream, part, G, N, (bf16_t*)out,
                       (float*)nullptr, accumulate);
  else
    hipLaunchKernelGGL((col_sum_kernel<false>), g2, dim3(256), 0, stream, part, G, N,
                       (float*)out, (float*)nullptr, accumulate);
  return (int)hipGetLastError();
}
