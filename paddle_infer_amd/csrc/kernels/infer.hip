// Inference kernels for the fused multi-transformer (serving) path on CDNA4 (gfx950).
//
//   qkv_prep      : QKV bias add + rotary embedding (NeoX rotate-half or GPT-J interleaved,
//                   partial rotary) + KV-cache write, in place on the packed QKV GEMM output.
//                   Parity: the bias/rotary/cache-write prologue of the reference's
//                   `fluid/operators/fused/fused_multi_transformer_op.cu.h` (write_cache_kv,
//                   add_fusedQKV_bias_transpose, rotary_qk).
//   decode_attn   : single-token attention over the KV cache ("masked multihead attention",
//                   reference `fused_multi_transformer_op.cu.h:masked_multihead_attention_kernel`),
//                   re-designed as split-K (flash-decoding): grid = (key splits, kv heads, batch),
//                   each workgroup streams a chunk of K then V once (HBM-bound) for ALL query heads
//                   of its GQA group, partials merged by decode_combine. Lengths come from device
//                   memory so a captured hipGraph replays every decode step unchanged.
//   wo_gemm       : weight-only int8 / int4 GEMM y = act((x·Wᵀ)·scale + bias) on MFMA
//                   (`v_mfma_f32_32x32x16_bf16`; int→bf16 is exact for |q| ≤ 127) over an
//                   MI355X-native pre-packed weight layout: one 1 KB fully-coalesced load per wave
//                   per 32 (int8) / 64 (int4) k. Parity: reference `cutlass_kernels/fpA_intB_gemm`
//                   (weight_only_linear, FusedMultiTransformerWeightOnly).
//   wo_dequant    : packed int8/int4 → bf16 [N, K] (weight_dequantize; large-M GEMMs).
#include "common.h"

// =====================================================================================
// qkv_prep
// =====================================================================================
// qkv   : [B*S rows, (Hq + 2*Hk) * D] bf16, row stride `ld` (elements); modified in place
// cache : k_cache / v_cache [B, Hk, maxS, D] bf16 (either may be null → no cache write)
// pos0  : [B] int32 start position per batch (null → 0); token s of batch b sits at pos0[b]+s
template <int D>
__global__ __launch_bounds__(256) void qkv_prep_kernel(
    bf16_t* __restrict__ qkv, long long ld, const bf16_t* __restrict__ bias,
    bf16_t* __restrict__ kc, bf16_t* __restrict__ vc, const int* __restrict__ pos0, int B, int S,
    int Hq, int Hk, int maxS, int rot, int neox, float log2_base) {
  constexpr int E = D / 64;
  const int H = Hq + 2 * Hk;
  const long long wid = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= (long long)B * S * H) return;
  const int lane = threadIdx.x & 63;
  const int h = (int)(wid % H);
  const long long tok = wid / H;
  const int b = (int)(tok / S), s = (int)(tok % S);
  const int pos = (pos0 ? pos0[b] : 0) + s;
  bf16_t* row = qkv + tok * ld + (long long)h * D;
  const bf16_t* brow = bias ? bias + (long long)h * D : nullptr;
  float y[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane + 64 * e;
    float x = bf2f(row[i]) + (brow ? bf2f(brow[i]) : 0.f);
    if (h < Hq + Hk && i < rot) {
      const int half = rot >> 1;
      int p, f;
      float sgn;
      if (neox) {
        p = i < half ? i + half : i - half;
        f = i < half ? i : i - half;
        sgn = i < half ? -1.f : 1.f;
      } else {
        p = i ^ 1;
        f = i >> 1;
        sgn = (i & 1) ? 1.f : -1.f;
      }
      const float xp = bf2f(row[p]) + (brow ? bf2f(brow[p]) : 0.f);
      const float inv_freq = exp2f(-(2.f * f / (float)rot) * log2_base);
      float sn, cs;
      sincosf((float)pos * inv_freq, &sn, &cs);
      x = x * cs + sgn * xp * sn;
    }
    y[e] = x;
  }
  // every lane's loads (incl. rotary partners) precede any store in the single wave stream
  bf16_t* dst = nullptr;
  if (h >= Hq && pos < maxS) {
    const bool is_v = h >= Hq + Hk;
    const int kvh = is_v ? h - Hq - Hk : h - Hq;
    bf16_t* c = is_v ? vc : kc;
    if (c) dst = c + (((long long)b * Hk + kvh) * maxS + pos) * D;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = lane + 64 * e;
    const bf16_t v = f2bf(y[e]);
    row[i] = v;
    if (dst) dst[i] = v;
  }
}

PIAMD_EXPORT int piamd_qkv_prep(void* qkv, long long ld, const void* bias, void* kc, void* vc,
                                const int* pos0, int B, int S, int Hq, int Hk, int D, int maxS,
                                int rot, int neox, float base, hipStream_t st) {
  const long long waves = (long long)B * S * (Hq + 2 * Hk);
  dim3 grid((unsigned)((waves + 3) / 4)), block(256);
  const float l2b = log2f(base);
  if (D == 128)
    hipLaunchKernelGGL(qkv_prep_kernel<128>, grid, block, 0, st, (bf16_t*)qkv, ld,
                       (const bf16_t*)bias, (bf16_t*)kc, (bf16_t*)vc, pos0, B, S, Hq, Hk, maxS, rot,
                       neox, l2b);
  else if (D == 64)
    hipLaunchKernelGGL(qkv_prep_kernel<64>, grid, block, 0, st, (bf16_t*)qkv, ld,
                       (const bf16_t*)bias, (bf16_t*)kc, (bf16_t*)vc, pos0, B, S, Hq, Hk, maxS, rot,
                       neox, l2b);
  else if (D == 256)
    hipLaunchKernelGGL(qkv_prep_kernel<256>, grid, block, 0, st, (bf16_t*)qkv, ld,
                       (const bf16_t*)bias, (bf16_t*)kc, (bf16_t*)vc, pos0, B, S, Hq, Hk, maxS, rot,
                       neox, l2b);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// =====================================================================================
// decode attention (split-K, fused prologue, in-kernel combine)
// =====================================================================================
// qkv   : row b at qkv + b*ldq: [Hq q-heads | Hk k-heads | Hk v-heads] × D
//         prep == 0: q already prepared (bias/RoPE applied), k/v of the new token already cached
//         prep == 1: raw QKV GEMM output of the new token; the kernel adds `bias`, applies RoPE
//                    (rot ∈ {0, D}) to q and k, and the workgroup whose key range holds the new
//                    position writes k/v into the cache before scoring
// kc,vc : [B, Hk, maxS, D]; keys [0, lens[b]) are attended; the new token sits at lens[b]-1
// mask  : optional additive bf16 mask, element (b, key) at mask[b*ldm + key]
// part  : [B, Hq, nsplit, D + 2] f32 partials (acc, m, l) when nsplit > 1; `cnt` [B*Hk] int
//         arrival counters (zero on entry, restored to zero by the combining workgroup)
// out   : element (b, head, d) at out[b*ldo + head*D + d]
constexpr int DA_CHUNK_MAX = 512;

// U: K/V rows in flight per lane per pass (4; 16 = the short-context single-pass variant: a
// 256-key chunk (D = 128) needs no split, partials, counters or combine — one global round trip
// for K and V each)
template <int D, int G, int U = 4>
__global__ __launch_bounds__(256) void decode_attn_kernel(
    const bf16_t* __restrict__ qkv, long long ldq, const bf16_t* __restrict__ bias, int prep,
    int rot, int neox, float log2_base, bf16_t* __restrict__ kc, bf16_t* __restrict__ vc,
    const int* __restrict__ lens, int Hk, int maxS, int chunk, int nsplit,
    const bf16_t* __restrict__ mask, long long ldm, float scale_log2, float* __restrict__ part,
    int* __restrict__ cnt, bf16_t* __restrict__ out, long long ldo) {
  constexpr int LPK = D / 8;        // lanes per key row (16 B per lane)
  constexpr int KPW = 64 / LPK;     // keys per wave per step
  constexpr int KPI = KPW * 4;      // keys per workgroup per step
  __shared__ float sc[G][DA_CHUNK_MAX];
  __shared__ float red[4][G * D];
  __shared__ float stat[2][G];
  __shared__ float wred[8];
  __shared__ int s_last;

  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int Hq = Hk * G;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int sub = lane % LPK, kslot = w * KPW + lane / LPK;
  const int len = lens[b], pos = len - 1;
  const int k0 = split * chunk, k1 = min(len, k0 + chunk);
  const long long kvbase = ((long long)b * Hk + hk) * maxS * D;
  const bf16_t* row = qkv + (long long)b * ldq;

  // ---- prologue: q (and the new k/v) with bias + rotary, in registers ----
  float rc[8], rs[8];  // rotary cos/sin for this lane's 8 elements
  const bool rope = prep && rot == D;
  if (rope) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = sub * 8 + j;
      const int f = neox ? (i % (D / 2)) : (i >> 1);
      const float inv = exp2f(-(2.f * f / (float)D) * log2_base);
      sincosf((float)pos * inv, &rs[j], &rc[j]);
    }
  }
  auto load_vec = [&](int head, float* v) {
    const u16x8 x = *(const u16x8*)(row + (long long)head * D + sub * 8);
    u16x8 bb;
    if (prep && bias) bb = *(const u16x8*)(bias + (long long)head * D + sub * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f(x[j]) + ((prep && bias) ? bf2f(bb[j]) : 0.f);
  };
  auto rotate = [&](float* v) {
    if (!rope) return;
    float pr[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (neox) {
        pr[j] = __shfl_xor(v[j], LPK / 2, 64);
        const float sg = sub < LPK / 2 ? -1.f : 1.f;
        pr[j] *= sg;
      } else {
        pr[j] = (j & 1) ? v[j - 1] : -v[j + 1];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = v[j] * rc[j] + pr[j] * rs[j];
  };

  float qf[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    load_vec(hk * G + g, qf[g]);
    rotate(qf[g]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[g][j] *= scale_log2;
  }
  if (prep) {
    // k/v of the new token: only the workgroup owning position `pos` stores them (every lane of
    // the wave evaluates the shuffles; waves 1..3 skip the store)
    float kn[8], vn[8];
    load_vec(Hq + hk, kn);
    rotate(kn);
    load_vec(Hq + Hk + hk, vn);
    if (w == 0 && lane < LPK && pos >= k0 && pos < k1 && pos < maxS) {
      u16x8 ko, vo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ko[j] = f2bf(kn[j]);
        vo[j] = f2bf(vn[j]);
      }
      *(u16x8*)(kc + kvbase + (long long)pos * D + sub * 8) = ko;
      *(u16x8*)(vc + kvbase + (long long)pos * D + sub * 8) = vo;
    }
    __threadfence_block();
    __syncthreads();
  }

  const int n = k1 - k0;
  if (n <= 0) {  // workgroup-uniform: empty split
    if (nsplit > 1 && tid < G) {
      float* p = part + (((long long)b * Hq + hk * G + tid) * nsplit + split) * (D + 2);
      xcd_drain(xcd_put(p + D, -INFINITY) + xcd_put(p + D + 1, 0.f));
    }
  } else {
    // ---- scores: s = (q·k) * scale * log2(e) (+ mask * log2(e)) ----
    for (int base = kslot; base < n; base += KPI * U) {
      u16x8 kr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = min(base + u * KPI, n - 1);  // clamped: every load is issued
        kr[u] = *(const u16x8*)(kc + kvbase + (long long)(k0 + kk) * D + sub * 8);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = base + u * KPI;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          float d = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) d += qf[g][j] * bf2f(kr[u][j]);
#pragma unroll
          for (int o = LPK / 2; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
          if (sub == 0 && kk < n) {
            if (mask) d += bf2f(mask[(long long)b * ldm + k0 + kk]) * 1.4426950408889634f;
            sc[g][kk] = d;
          }
        }
      }
    }
    // V rows of the first P·V pass requested now: their latency hides under the softmax
    u16x8 vpre[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      vpre[u] = *(const u16x8*)(vc + kvbase + (long long)(k0 + min(kslot + u * KPI, n - 1)) * D + sub * 8);
    __syncthreads();

    // ---- softmax statistics over the chunk (base-2 domain) ----
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float m = -INFINITY;
      for (int i = tid; i < n; i += 256) m = fmaxf(m, sc[g][i]);
      m = block_max<4>(m, wred);
      float l = 0.f;
      for (int i = tid; i < n; i += 256) {
        const float p = exp2f(sc[g][i] - m);
        sc[g][i] = p;
        l += p;
      }
      l = block_sum<4>(l, wred);
      if (tid == 0) {
        stat[0][g] = m;
        stat[1][g] = l;
      }
    }
    __syncthreads();

    // ---- P·V ----
    float acc[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
    for (int base = kslot; base < n; base += KPI * U) {
      u16x8 vr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = min(base + u * KPI, n - 1);
        vr[u] = base == kslot ? vpre[u] : *(const u16x8*)(vc + kvbase + (long long)(k0 + kk) * D + sub * 8);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = base + u * KPI;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float p = kk < n ? sc[g][min(kk, n - 1)] : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[g][j] += p * bf2f(vr[u][j]);
        }
      }
    }
    // reduce over the KPW key slots of the wave (lanes with equal `sub`)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = acc[g][j];
#pragma unroll
        for (int o = LPK; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
        acc[g][j] = v;
      }
    if (lane < LPK) {
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int j = 0; j < 8; ++j) red[w][g * D + sub * 8 + j] = acc[g][j];
    }
    __syncthreads();
    float sink = 0.f;
    for (int i = tid; i < G * D; i += 256) {
      const int g = i / D, d = i % D;
      const float v = red[0][i] + red[1][i] + red[2][i] + red[3][i];
      const int head = hk * G + g;
      if (nsplit == 1) {
        out[(long long)b * ldo + (long long)head * D + d] = f2bf(v / stat[1][g]);
      } else {
        float* p = part + (((long long)b * Hq + head) * nsplit + split) * (D + 2);
        sink += xcd_put(p + d, v);
        if (d == 0) {
          sink += xcd_put(p + D, stat[0][g]);
          sink += xcd_put(p + D + 1, stat[1][g]);
        }
      }
    }
    if (nsplit > 1) xcd_drain(sink);
  }
  if (nsplit == 1) return;

  // ---- the last-arriving split of (b, hk) merges all partials (no combine launch) ----
  __syncthreads();  // every thread's partial stores have completed (xcd_drain)
  if (tid == 0) s_last = atomicAdd(&cnt[b * Hk + hk], 1) == nsplit - 1;
  __syncthreads();
  if (!s_last) return;
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i % D;
    const int head = hk * G + g;
    float* p = part + ((long long)b * Hq + head) * nsplit * (D + 2);
    float m = -INFINITY;
    for (int s2 = 0; s2 < nsplit; ++s2)
      m = fmaxf(m, __hip_atomic_load(p + s2 * (D + 2) + D, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    float l = 0.f, a = 0.f;
    for (int s2 = 0; s2 < nsplit; ++s2) {
      const float ms = __hip_atomic_load(p + s2 * (D + 2) + D, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ms == -INFINITY) continue;  // empty split: its acc slots hold stale data
      const float wgt = exp2f(ms - m);
      l += wgt * __hip_atomic_load(p + s2 * (D + 2) + D + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a += wgt * __hip_atomic_load(p + s2 * (D + 2) + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    out[(long long)b * ldo + (long long)head * D + d] = f2bf(a / l);
  }
  if (tid == 0) atomicExch(&cnt[b * Hk + hk], 0);
}

template <int D, int G>
static void launch_decode(dim3 grid, hipStream_t st, const void* qkv, long long ldq,
                          const void* bias, int prep, int rot, int neox, float l2b, void* kc,
                          void* vc, const int* lens, int Hk, int maxS, int chunk, int nsplit,
                          const void* mask, long long ldm, float sl2, float* part, int* cnt,
                          void* out, long long ldo) {
  constexpr int KPI = (64 / (D / 8)) * 4;
  if (G <= 2 && nsplit == 1 && chunk > 4 * KPI && chunk <= 16 * KPI) {
    hipLaunchKernelGGL((decode_attn_kernel<D, (G <= 2 ? G : 1), 16>), grid, dim3(256), 0, st,
                       (const bf16_t*)qkv, ldq, (const bf16_t*)bias, prep, rot, neox, l2b,
                       (bf16_t*)kc, (bf16_t*)vc, lens, Hk, maxS, chunk, nsplit,
                       (const bf16_t*)mask, ldm, sl2, part, cnt, (bf16_t*)out, ldo);
    return;
  }
  hipLaunchKernelGGL((decode_attn_kernel<D, G>), grid, dim3(256), 0, st, (const bf16_t*)qkv, ldq,
                     (const bf16_t*)bias, prep, rot, neox, l2b, (bf16_t*)kc, (bf16_t*)vc, lens,
                     Hk, maxS, chunk, nsplit, (const bf16_t*)mask, ldm, sl2, part, cnt,
                     (bf16_t*)out, ldo);
}

#define PIAMD_DECODE_ARGS grid, st, qkv, ldq, bias, prep, rot, neox, l2b, kc, vc, lens, Hk, maxS, \
                          chunk, nsplit, mask, ldm, sl2, part, cnt, out, ldo
template <int D>
static int dispatch_decode_g(int G, dim3 grid, hipStream_t st, const void* qkv, long long ldq,
                             const void* bias, int prep, int rot, int neox, float l2b, void* kc,
                             void* vc, const int* lens, int Hk, int maxS, int chunk, int nsplit,
                             const void* mask, long long ldm, float sl2, float* part, int* cnt,
                             void* out, long long ldo) {
  switch (G) {
    case 1: launch_decode<D, 1>(PIAMD_DECODE_ARGS); break;
    case 2: launch_decode<D, 2>(PIAMD_DECODE_ARGS); break;
    case 4: launch_decode<D, 4>(PIAMD_DECODE_ARGS); break;
    case 8: launch_decode<D, 8>(PIAMD_DECODE_ARGS); break;
    default: return (int)hipErrorInvalidValue;
  }
  return 0;
}

// chunk ≤ 512 keys per split; nsplit * chunk ≥ max length; part/cnt may be null iff nsplit == 1.
// rot must be 0 or D when prep == 1 (partial rotary: run piamd_qkv_prep first, prep = 0).
PIAMD_EXPORT int piamd_decode_attn(const void* qkv, long long ldq, const void* bias, int prep,
                                   int rot, int neox, float base, void* kc, void* vc,
                                   const int* lens, int B, int Hq, int Hk, int D, int maxS,
                                   int chunk, int nsplit, const void* mask, long long ldm,
                                   float scale, float* part, int* cnt, void* out, long long ldo,
                                   hipStream_t st) {
  if (Hk <= 0 || Hq % Hk || chunk <= 0 || chunk > DA_CHUNK_MAX ||
      (nsplit > 1 && (!part || !cnt)) || (prep && rot != 0 && rot != D))
    return (int)hipErrorInvalidValue;
  const int G = Hq / Hk;
  dim3 grid(nsplit, Hk, B);
  const float sl2 = scale * 1.4426950408889634f;
  const float l2b = log2f(base);
  int rc;
  if (D == 128)
    rc = dispatch_decode_g<128>(G, PIAMD_DECODE_ARGS);
  else if (D == 64)
    rc = dispatch_decode_g<64>(G, PIAMD_DECODE_ARGS);
  else
    return (int)hipErrorInvalidValue;
  if (rc) return rc;
  return (int)hipGetLastError();
}
#undef PIAMD_DECODE_ARGS

// =====================================================================================
// weight-only GEMM
// =====================================================================================
// Packed layout (produced by piamd_wo_pack / nn.quant.weight_quantize), n-tiles of 32 rows:
//   int8: byte(n,k) at (((n/32)*(K/32) + k/32)*64 + (n%32) + 32*((k%32)/16))*16 + k%16
//   int4: nibble(n,k) in byte (((n/32)*(K/64) + k/64)*64 + (n%32) + 32*((k%64)/32))*16 + (k%32)/2,
//         low nibble for even k, two's complement in [-8, 7]
//   bf16: element(n,k) at (((n/32)*(K/16) + k/16)*64 + (n%32) + 32*((k%16)/8))*8 + k%8
//         (the same tiling for unquantized serving weights: one MFMA B operand per 16 B load)
// so each wave reads one contiguous 1 KB block per k-block: lane l holds row n0+(l&31), k-run
// [kb*KB + (KB/2)*(l>>5), +KB/2) — exactly the bf16x8 B-operand runs of consecutive MFMAs.
__device__ __forceinline__ bf16x8 i8x8_to_bf16(unsigned lo, unsigned hi) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (__bf16)(float)((int)(lo << (24 - 8 * j)) >> 24);
    r[4 + j] = (__bf16)(float)((int)(hi << (24 - 8 * j)) >> 24);
  }
  return r;
}
__device__ __forceinline__ bf16x8 i4x8_to_bf16(unsigned d) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)(float)((int)(d << (28 - 4 * j)) >> 28);
  return r;
}
__device__ __forceinline__ float act_apply(float v, int act) {
  switch (act) {
    case 1: return gelu_tanh(v);
    case 2: return gelu_erf(v);
    case 3: return fmaxf(v, 0.f);
    case 4: return v / (1.f + __expf(-v));
    default: return v;
  }
}

// grid (N/32, ceil(M/32), KS); 256 threads = 4 waves splitting the k-blocks of this WG's K range.
#ifndef WO_NT
#define WO_NT 1
#endif
#ifndef WO_UNROLL
#define WO_UNROLL 8  // k-blocks per wave per iteration: 8 x 16 B weight loads in flight per lane (16: no gain, profiles/rocprof_decode_gpt1.3b_b1_r3_nt.txt)
#endif
// LNP (decode, KS == 1, M ≤ 8): the workgroup LayerNorms its input rows into LDS first (shifted-sum
// statistics in one pass over registers, then γ/β), so the pre-LN of a transformer layer needs no
// launch of its own. `resid` (nullable): y = act(acc·scale + bias) + resid — the residual add of
// the out-proj / FFN2 projection folded into the epilogue.
template <int BITS, bool LNP>
__global__ __launch_bounds__(256) void wo_gemm_kernel(
    const bf16_t* __restrict__ x, long long ldx, const unsigned char* __restrict__ wp,
    const float* __restrict__ scale, const bf16_t* __restrict__ bias, bf16_t* __restrict__ y,
    long long ldy, float* __restrict__ ws, int* __restrict__ cnt, int M, int N, int K, int act,
    const int* __restrict__ offs, int E, long long wstride, const bf16_t* __restrict__ ln_g,
    const bf16_t* __restrict__ ln_b, float eps, const bf16_t* __restrict__ resid, long long ldr) {
  constexpr int KB = BITS == 16 ? 16 : (BITS == 8 ? 32 : 64);  // k per block (16 B lane load)
  constexpr int NMF = KB / 16;               // MFMAs per block
  __shared__ float red[3][16][64];
  extern __shared__ __attribute__((aligned(16))) char xln[];  // LNP: [rows][K] bf16, row pitch K*2+16
  const int nt = blockIdx.x, kz = blockIdx.z, KS = gridDim.z;
  int mt = blockIdx.y, mbase = 0;
  if (offs) {
    // grouped (MoE experts): global 32-row tile → (expert, tile); rows [offs[e], offs[e+1])
    int acc_t = 0, e = -1;
    for (int i = 0; i < E; ++i) {
      const int nt_e = (offs[i + 1] - offs[i] + 31) / 32;
      if (mt < acc_t + nt_e) { e = i; break; }
      acc_t += nt_e;
    }
    if (e < 0) return;  // surplus tile of the worst-case grid
    mbase = offs[e] + (mt - acc_t) * 32;
    M = offs[e + 1];
    mt = 0;
    wp += e * wstride;
    if (scale) scale += (long long)e * N;
    if (bias) bias += (long long)e * N;
  }
  mbase += mt * 32;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nkb = K / KB;
  const int kb_beg = (int)((long long)nkb * kz / KS), kb_end = (int)((long long)nkb * (kz + 1) / KS);
  const int m = min(mbase + (lane & 31), M - 1);  // rows ≥ M compute duplicates, never stored
  const bf16_t* xr = x + (long long)m * ldx + (KB / 2) * (lane >> 5);
  const uint4* wt = (const uint4*)wp + (long long)nt * nkb * 64 + lane;
  const long long pitch = (long long)K * 2 + 16;  // LDS row pitch: +16 B keeps row reads conflict-free
  const char* xl = xln + (long long)(m - mbase) * pitch + (KB / 2) * (lane >> 5) * 2;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  constexpr int U = BITS == 16 ? WO_UNROLL : (BITS == 8 ? WO_UNROLL / 2 : WO_UNROLL / 4);
  // software pipeline: the next group's weight / activation loads are issued before this group's
  // MFMAs, so each lane keeps 2·U 16-B weight loads in flight (the GEMV is an HBM stream)
  uint4 wv[U];
  bf16x8 xa[U][NMF];
  auto load_w = [&](int kb0, uint4 (&wd)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // weights are streamed exactly once per step: non-temporal loads keep them from evicting
      // the activations / KV cache the other kernels of the step re-read from L2 / MALL
      const uint4* src = wt + (long long)min(kb0 + 4 * u, kb_end - 1) * 64;
#if WO_NT
      typedef unsigned u32x4_nt __attribute__((ext_vector_type(4)));
      const u32x4_nt t = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(src));
      wd[u] = make_uint4(t[0], t[1], t[2], t[3]);
#else
      wd[u] = *src;
#endif
    }
  };
  auto load_x = [&](int kb0, bf16x8 (&xd)[U][NMF]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kb = min(kb0 + 4 * u, kb_end - 1);
#pragma unroll
      for (int i = 0; i < NMF; ++i)
        xd[u][i] = LNP ? *(const bf16x8*)(xl + ((long long)kb * KB + 8 * i) * 2)
                       : *(const bf16x8*)(xr + (long long)kb * KB + 8 * i);
    }
  };
  // the first weight group is requested BEFORE the LayerNorm prologue: its HBM latency covers the
  // prologue's L2 round trip
  if (kb_beg + w < kb_end) load_w(kb_beg + w, wv);
  if (LNP) {
    // ≤ 8 rows (M ≤ 8), K % 512 == 0, K ≤ 2048: thread t holds chunk t of each row (16 B), each
    // wave's 64 chunks lie in one row → wave sums + ≤ 4 LDS atomics per row
    __shared__ float st[2][8];
    const int rows_t = min(8, M - mbase);
    const int cpr = K >> 3;  // 16-B chunks per row
    if (threadIdx.x < 16) st[threadIdx.x / 8][threadIdx.x % 8] = 0.f;
    u16x8 v[8], g[8], b[8];
    float sh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (c < rows_t * cpr) {
        const int rr = c / cpr, cc = c % cpr;
        const bf16_t* row = x + (long long)(mbase + rr) * ldx;
        v[i] = *reinterpret_cast<const u16x8*>(row + 8 * cc);
        g[i] = *reinterpret_cast<const u16x8*>(ln_g + 8 * cc);
        b[i] = *reinterpret_cast<const u16x8*>(ln_b + 8 * cc);
        sh[i] = bf2f(row[0]);  // shifted sums: a stable single-pass variance
      }
    }
    __syncthreads();  // st zeroed
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c0 = (threadIdx.x & ~63) + 256 * i;  // wave-uniform
      if (c0 < rows_t * cpr) {
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = bf2f(v[i][j]) - sh[i]; s1 += d; s2 += d * d; }
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        if (lane == 0) {
          atomicAdd(&st[0][c0 / cpr], s1);
          atomicAdd(&st[1][c0 / cpr], s2);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (c < rows_t * cpr) {
        const int rr = c / cpr, cc = c % cpr;
        const float dm = st[0][rr] / K;  // mean − shift
        const float mu = sh[i] + dm;
        const float rs = rsqrtf(fmaxf(st[1][rr] / K - dm * dm, 0.f) + eps);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf((bf2f(v[i][j]) - mu) * rs * bf2f(g[i][j]) + bf2f(b[i][j]));
        *reinterpret_cast<u16x8*>(xln + (long long)rr * pitch + 16 * cc) = o;
      }
    }
    __syncthreads();
  }
  if (kb_beg + w < kb_end) load_x(kb_beg + w, xa);
  for (int kb0 = kb_beg + w; kb0 < kb_end; kb0 += 4 * U) {
    uint4 wn[U];
    bf16x8 xn[U][NMF];
    const bool more = kb0 + 4 * U < kb_end;
    if (more) {
      load_w(kb0 + 4 * U, wn);
      load_x(kb0 + 4 * U, xn);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (kb0 + 4 * u >= kb_end) {  // zero the weight operand: the MFMA then adds nothing
        wv[u] = make_uint4(0, 0, 0, 0);
      }
      if (BITS == 16) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[u][0], __builtin_bit_cast(bf16x8, wv[u]), acc, 0, 0, 0);
      } else if (BITS == 8) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[u][0], i8x8_to_bf16(wv[u].x, wv[u].y), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[u][1], i8x8_to_bf16(wv[u].z, wv[u].w), acc, 0, 0, 0);
      } else {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[u][0], i4x8_to_bf16(wv[u].x), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[u][1], i4x8_to_bf16(wv[u].y), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[u][2], i4x8_to_bf16(wv[u].z), acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[u][3], i4x8_to_bf16(wv[u].w), acc, 0, 0, 0);
      }
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        wv[u] = wn[u];
#pragma unroll
        for (int i = 0; i < NMF; ++i) xa[u][i] = xn[u][i];
      }
    }
  }
  if (w > 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[w - 1][r][lane] = acc[r];
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] += red[0][r][lane] + red[1][r][lane] + red[2][r][lane];
  // D layout: column (n) = lane & 31, row (m) = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int n = nt * 32 + (lane & 31);
  const float sc = scale ? scale[n] : 1.f;
  const float bs = bias ? bf2f(bias[n]) : 0.f;
  if (KS == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = mbase + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (mm < M)
        y[(long long)mm * ldy + n] = f2bf(act_apply(acc[r] * sc + bs, act) +
                                          (resid ? bf2f(resid[(long long)mm * ldr + n]) : 0.f));
    }
    return;
  }
  // split-K: every slice adds its partial into the zeroed f32 tile with memory-side atomics; the
  // last-arriving slice takes (reads + re-zeroes) the sums and runs the epilogue — a stream-K
  // style fixup with no second launch and no L2-flushing fence (see xcd_* in common.h)
  if (cnt == nullptr) {  // slice mode (larger M): plain partial slices + wo_finalize_kernel
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = mbase + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (mm < M) ws[((long long)kz * M + mm) * N + n] = acc[r];
    }
    return;
  }
  float sink = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int mm = mbase + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (mm < M) sink += xcd_add(ws + (long long)mm * N + n, acc[r]);
  }
  xcd_drain(sink);
  int last = 0;
  if (lane == 0) last = atomicAdd(&cnt[mt * gridDim.x + nt], 1) == KS - 1;
  last = __shfl(last, 0, 64);
  if (!last) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int mm = mbase + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (mm < M) {
      const float v = xcd_take(ws + (long long)mm * N + n);
      y[(long long)mm * ldy + n] = f2bf(act_apply(v * sc + bs, act) +
                                        (resid ? bf2f(resid[(long long)mm * ldr + n]) : 0.f));
    }
  }
  if (lane == 0) atomicExch(&cnt[mt * gridDim.x + nt], 0);
}

__global__ void wo_finalize_kernel(const float* __restrict__ ws, int KS, const float* __restrict__ scale,
                                   const bf16_t* __restrict__ bias, bf16_t* __restrict__ y, long long ldy,
                                   int M, int N, int act, const bf16_t* __restrict__ resid,
                                   long long ldr) {
  const long long total = (long long)M * N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(i % N);
    float v = 0.f;
    for (int z = 0; z < KS; ++z) v += ws[(long long)z * total + i];
    v = v * (scale ? scale[n] : 1.f) + (bias ? bf2f(bias[n]) : 0.f);
    y[(i / N) * ldy + n] = f2bf(act_apply(v, act) + (resid ? bf2f(resid[(i / N) * ldr + n]) : 0.f));
  }
}

// KS > 1, fixup mode (cnt != null): ws = M*N zeroed f32, cnt = ceil(M/32)*(N/32) zeroed ints
// (both left zeroed) — one launch. Slice mode (cnt == null): ws = KS*M*N f32, plus a finalize
// launch (cheaper than memory-side atomics once M is large).
// Requires N % 32 == 0 and K % KB == 0 (KB = 16 / 32 / 64 for bits = 16 / 8 / 4).
// bits = 16: packed bf16 weights, scale may be null.
static void wo_launch(int bits, dim3 grid, hipStream_t st, const void* x, long long ldx,
                      const void* wp, const float* scale, const void* bias, void* y, long long ldy,
                      float* ws, int* cnt, int M, int N, int K, int act, const int* offs, int E,
                      long long wstride, const void* ln_g = nullptr, const void* ln_b = nullptr,
                      float eps = 0.f, const void* resid = nullptr, long long ldr = 0) {
  const size_t lds = ln_g ? (size_t)min(M, 32) * ((size_t)K * 2 + 16) : 0;
#define WO_LAUNCH(B, L)                                                                           \
  hipLaunchKernelGGL((wo_gemm_kernel<B, L>), grid, dim3(256), lds, st, (const bf16_t*)x, ldx,    \
                     (const unsigned char*)wp, scale, (const bf16_t*)bias, (bf16_t*)y, ldy, ws,   \
                     cnt, M, N, K, act, offs, E, wstride, (const bf16_t*)ln_g,                    \
                     (const bf16_t*)ln_b, eps, (const bf16_t*)resid, ldr)
  if (ln_g) {
    if (bits == 16) WO_LAUNCH(16, true);
    else if (bits == 8) WO_LAUNCH(8, true);
    else WO_LAUNCH(4, true);
  } else {
    if (bits == 16) WO_LAUNCH(16, false);
    else if (bits == 8) WO_LAUNCH(8, false);
    else WO_LAUNCH(4, false);
  }
#undef WO_LAUNCH
}

// Extended form: ln_g/ln_b (nullable, bf16 [K]): y = act(LN(x)·Wᵀ·scale + bias) with the
// LayerNorm (ε = eps) computed in the prologue — requires KS == 1, M ≤ 8, K % 512 == 0, K ≤ 2048;
// resid (nullable, bf16 rows of pitch ldr): + resid[m, n] after the activation.
PIAMD_EXPORT int piamd_wo_gemm_ex(int bits, const void* x, long long ldx, const void* wp,
                                  const float* scale, const void* bias, void* y, long long ldy,
                                  float* ws, int* cnt, int M, int N, int K, int KS, int act,
                                  const void* ln_g, const void* ln_b, float eps, const void* resid,
                                  long long ldr, hipStream_t st) {
  const int KB = bits == 16 ? 16 : (bits == 8 ? 32 : 64);
  if ((bits != 16 && bits != 8 && bits != 4) || N % 32 || K % KB || KS < 1 ||
      (KS > 1 && !ws) || M < 1 || (ln_g && (!ln_b || KS != 1 || K % 512 || K > 2048 || M > 8)))
    return (int)hipErrorInvalidValue;
  wo_launch(bits, dim3(N / 32, (M + 31) / 32, KS), st, x, ldx, wp, scale, bias, y, ldy, ws, cnt,
            M, N, K, act, nullptr, 0, 0, ln_g, ln_b, eps, resid, ldr);
  if (KS > 1 && !cnt)
    hipLaunchKernelGGL(wo_finalize_kernel, dim3(stride_grid((long long)M * N, 256)), dim3(256), 0,
                       st, ws, KS, scale, (const bf16_t*)bias, (bf16_t*)y, ldy, M, N, act,
                       (const bf16_t*)resid, ldr);
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_wo_gemm(int bits, const void* x, long long ldx, const void* wp,
                               const float* scale, const void* bias, void* y, long long ldy,
                               float* ws, int* cnt, int M, int N, int K, int KS, int act,
                               hipStream_t st) {
  return piamd_wo_gemm_ex(bits, x, ldx, wp, scale, bias, y, ldy, ws, cnt, M, N, K, KS, act,
                          nullptr, nullptr, 0.f, nullptr, 0, st);
}

// Grouped weight-only expert GEMM (the decode / small-batch MoE path of
// fused_multi_transformer_moe_weight_only): x [rows][K] expert-sorted with device offsets
// offs[E+1]; expert e's packed weights at wp + e*wstride bytes, scale/bias [E][N]. 32-row tiles,
// worst-case grid ceil(rows_cap/32) + E, surplus tiles exit. bits 16 (packed bf16) / 8 / 4.
PIAMD_EXPORT int piamd_wo_moe_gemm(int bits, const void* x, long long ldx, const void* wp,
                                   long long wstride, const float* scale, const void* bias,
                                   const int* offs, int E, int rows_cap, void* y, long long ldy,
                                   int N, int K, int act, hipStream_t st) {
  const int KB = bits == 16 ? 16 : (bits == 8 ? 32 : 64);
  if ((bits != 16 && bits != 8 && bits != 4) || N % 32 || K % KB || E < 1 || rows_cap < 0)
    return (int)hipErrorInvalidValue;
  wo_launch(bits, dim3(N / 32, (rows_cap + 31) / 32 + E, 1), st, x, ldx, wp, scale, bias, y, ldy,
            nullptr, nullptr, rows_cap, N, K, act, offs, E, wstride);
  return (int)hipGetLastError();
}

// packed → bf16 [N, K] (row-major, no scale when scale == null)
// One thread per packed 16-B chunk (the lane load of the GEMV layout): coalesced 16-B reads; the
// 4 waves of a workgroup cover 4 consecutive k-blocks of one 32-row tile, so each output row gets
// 4 adjacent 32-B (int8) / 64-B (int4) pieces — whole cache lines per workgroup.
template <int BITS>
__global__ __launch_bounds__(256) void wo_dequant_kernel(const uint4* __restrict__ wp,
                                                         const float* __restrict__ scale,
                                                         bf16_t* __restrict__ out, int N, int K) {
  constexpr int KB = BITS == 8 ? 32 : 64;
  const int nkb = K / KB;
  const long long chunks = (long long)(N / 32) * nkb * 64;
  for (long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x; c < chunks;
       c += (long long)gridDim.x * blockDim.x) {
    const int lane = (int)(c & 63);
    const long long blk = c >> 6;
    const int nt = (int)(blk / nkb), kb = (int)(blk % nkb);
    const int n = nt * 32 + (lane & 31);
    const int k0 = kb * KB + (lane >> 5) * (KB / 2);
    const uint4 v = wp[c];
    const float sc = scale ? scale[n] : 1.f;
    uint4* dst = reinterpret_cast<uint4*>(out + (long long)n * K + k0);
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
    if (BITS == 8) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // 8 values per 16-B store
        unsigned o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned word = w[2 * h + j / 2];
          const int q0 = (int)(signed char)(word >> (16 * (j & 1)));
          const int q1 = (int)(signed char)(word >> (16 * (j & 1) + 8));
          o[j] = (unsigned)f2bf(q0 * sc) | ((unsigned)f2bf(q1 * sc) << 16);
        }
        dst[h] = make_uint4(o[0], o[1], o[2], o[3]);
      }
    } else {
#pragma unroll
      for (int h = 0; h < 4; ++h) {  // one 32-bit word = 8 nibbles = 8 values, low nibble first
        unsigned o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q0 = (int)(w[h] << (28 - 8 * j)) >> 28;
          const int q1 = (int)(w[h] << (24 - 8 * j)) >> 28;
          o[j] = (unsigned)f2bf(q0 * sc) | ((unsigned)f2bf(q1 * sc) << 16);
        }
        dst[h] = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  }
}

PIAMD_EXPORT int piamd_wo_dequant(int bits, const void* wp, const float* scale, void* out, int N,
                                  int K, hipStream_t st) {
  const int KB = bits == 8 ? 32 : 64;
  if ((bits != 8 && bits != 4) || N % 32 || K % KB) return (int)hipErrorInvalidValue;
  const dim3 grid(stride_grid((long long)(N / 32) * (K / KB) * 64, 256));
  if (bits == 8)
    hipLaunchKernelGGL(wo_dequant_kernel<8>, grid, dim3(256), 0, st, (const uint4*)wp, scale,
                       (bf16_t*)out, N, K);
  else
    hipLaunchKernelGGL(wo_dequant_kernel<4>, grid, dim3(256), 0, st, (const uint4*)wp, scale,
                       (bf16_t*)out, N, K);
  return (int)hipGetLastError();
}
