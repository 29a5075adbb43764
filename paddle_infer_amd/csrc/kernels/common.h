// Shared device helpers for the paddle_infer_amd CDNA4 (gfx950) kernel library.
//
// Conventions (all kernels):
//   * wave64: every reduction / shuffle idiom is written for 64 lanes.
//   * bf16 is carried as raw `unsigned short` bits in memory and widened to f32 in registers;
//     narrowing uses the hardware `v_cvt_pk_bf16_f32` (plain `__bf16` cast at -O3), which keeps NaN.
//   * global loads are 16 B/lane (`u16x8`) wherever the row length allows (guide G13).
//   * every exported launcher is `extern "C" int piamd_<name>(..., hipStream_t)` returning the
//     hipError_t of the launch, so the Python side can raise loudly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PIAMD_EXPORT extern "C" __attribute__((visibility("default")))

typedef unsigned short bf16_t;
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// 16-bit float storage (bf16 or IEEE fp16) <-> f32, selected at compile time.
template <bool F16>
__device__ __forceinline__ float h2f(unsigned short v) {
  if (F16) return (float)__builtin_bit_cast(_Float16, v);
  return bf2f(v);
}
template <bool F16>
__device__ __forceinline__ unsigned short f2h(float f) {
  if (F16) return __builtin_bit_cast(unsigned short, (_Float16)f);
  return f2bf(f);
}

// pack two floats into one dword of 2 x bf16 (lo in bits 0..15)
__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == 64 * NW; `red` must hold NW floats.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  __syncthreads();
  return t;
}
template <int NW>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

// Counter-based dropout RNG (stateless, so backward and recompute regenerate the mask instead of
// storing it). One 32-bit integer hash (lowbias32: 2 multiplies) per PAIR of elements, split into
// two 16-bit uniforms: the former per-element 64-bit splitmix (3 64-bit = 9 quarter-rate 32-bit
// multiplies per element) made the LayerNorm passes VALU-bound. The value of element `idx` depends
// only on (seed, offset, idx); (seed, offset) are folded into a per-call key (uniform across the
// grid, hoisted by the compiler). p granularity 2^-16.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t rng_key(uint64_t seed, uint64_t offset) {
  uint32_t k = lowbias32((uint32_t)(offset >> 32) + 0x9E3779B9u);
  k = lowbias32((uint32_t)offset ^ k);
  k = lowbias32((uint32_t)(seed >> 32) ^ k);
  return lowbias32((uint32_t)seed ^ k);
}
// u[j] = uniform [0,1) of element idx + j, j < 8; idx must be a multiple of 8.
// Two keyed rounds: h = lowbias32(lowbias32(pair + k_lo) ^ k_hi). With a single round keyed by
// XOR, two launches whose keys differ by a small d read the same hash stream shifted by d, i.e.
// one dropout mask is an index-permuted copy of the other; the second (non-linear) round makes
// every launch's stream a different function of the element index.
__device__ __forceinline__ void hash_uniform8(uint64_t seed, uint64_t offset, uint64_t idx,
                                              float* u) {
  const uint64_t pair = idx >> 1;
  const uint32_t k_lo = rng_key(seed, offset) ^ ((uint32_t)(pair >> 32) * 0x85EBCA6Bu);
  const uint32_t k_hi = lowbias32(k_lo ^ 0x632BE5ABu);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t h = lowbias32(lowbias32((uint32_t)pair + t + k_lo) ^ k_hi);
    u[2 * t] = (float)(h & 0xFFFFu) * (1.0f / 65536.0f);
    u[2 * t + 1] = (float)(h >> 16) * (1.0f / 65536.0f);
  }
}

// tanh(u) = 1 - 2 / (1 + e^{2u}) on one v_exp_f32 + one v_rcp_f32 (≈6 VALU ops instead of libm
// tanhf's ≈40): the [tokens x 4h] bias+GELU passes were VALU-bound on tanhf, not HBM-bound.
// Saturates cleanly (e^{2u} -> inf gives 1, -> 0 gives -1); absolute error ≈1e-7, far below the
// bf16 output rounding.
__device__ __forceinline__ float fast_tanh(float u) {
  const float e = __builtin_amdgcn_exp2f(u * 2.8853900817779268f);  // 2u * log2(e)
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + e);
}
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.f + fast_tanh(u));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float x2 = x * x;
  float u = k0 * (x + k1 * x2 * x);
  float t = fast_tanh(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x2);
}
__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.7071067811865476f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

// Cross-workgroup hand-off inside one kernel (split-K fixups) WITHOUT __threadfence(): on gfx950 a
// device-scope release fence writes back the whole (per-XCD) L2, which costs more than the work.
// Device-scope atomics are performed memory-side, coherent across the 8 XCD L2s, so partials are
// published with returning atomics (the return forces completion), then `xcd_drain()` waits for
// them before the arrival counter is bumped; the consumer reads with `xcd_take` (read + clear).
__device__ __forceinline__ float xcd_put(float* p, float v) { return atomicExch(p, v); }
__device__ __forceinline__ float xcd_add(float* p, float v) { return atomicAdd(p, v); }
__device__ __forceinline__ float xcd_take(float* p) { return atomicExch(p, 0.f); }
__device__ __forceinline__ void xcd_drain(float sink) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("" ::"v"(sink));
}

// Grid size for grid-stride memory-bound kernels (guide G11): ≤ 256 CUs × 8 blocks.
static inline int stride_grid(long long work_items, int block) {
  long long g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}
