// Host side of the hand-scheduled assembly GEMM (`csrc/asm/gemm_gen.py` → _lib/piamd_agemm.hsaco):
// code-object loading, the kernel-argument block, work decomposition (tile grid, group-M order,
// split-K) and the deterministic split-K reduction.
//
// Parity: reference `paddle/phi/kernels/funcs/blas/blas_impl.cu.h` (GEMM behind matmul / linear
// and their gradients), `paddle/fluid/operators/fused/fused_gemm_epilogue_op.cu` (epilogues).
#include "common.h"

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

namespace {

// mirror of gemm_gen.ARGS (byte offsets noted)
struct __attribute__((packed)) AgemmArgs {
  const void* a;               // 0
  const void* b;               // 8
  unsigned long long a_bytes;  // 16
  unsigned long long b_bytes;  // 24
  unsigned lda_b, ldb_b;       // 32, 36
  unsigned M, N;               // 40, 44
  unsigned nk, tiles_n;        // 48, 52
  unsigned nwg, ksplit;        // 56, 60
  unsigned tiles_m, ntiles;    // 64, 68
  float rcp_ntiles;            // 72
  unsigned per_group;          // 76
  float rcp_per_group;         // 80
  unsigned gm, act, grid;      // 84, 88, 92
  void* c;                     // 96
  unsigned long long c_bytes;  // 104
  unsigned ldc_b, ldaux_b;     // 112, 116
  unsigned long long c_part;   // 120
  void* aux;                   // 128
  unsigned long long aux_bytes;// 136
  const void* bias;            // 144
  unsigned kmul, pad0;         // 152: K start = part·kmul (split-K), 0 when batched
  unsigned long long a_bstride, b_bstride;  // 160, 168: operand base += part·bstride (batched)
  void* colsum;                // 176: dact epilogue column sums, f32 [ceil(M/128)][N] (*cs kernels)
  unsigned colsum_bytes, pad1; // 184, 188
};
static_assert(sizeof(AgemmArgs) == 192, "AgemmArgs layout");

std::mutex g_mu;
hipModule_t g_mod = nullptr;
std::map<std::string, hipFunction_t> g_fn;

hipFunction_t get_fn(const std::string& name) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_mod) return nullptr;
  auto it = g_fn.find(name);
  if (it != g_fn.end()) return it->second;
  hipFunction_t f = nullptr;
  if (hipModuleGetFunction(&f, g_mod, name.c_str()) != hipSuccess) f = nullptr;
  g_fn[name] = f;
  return f;
}

constexpr int GROUP_M = 8;

int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// C (+)= Σ_p ws[p] in a fixed order (deterministic); 4 columns per thread; 16-bit C is bf16 or
// (F16) IEEE fp16
template <bool F16>
__global__ __launch_bounds__(256) void agemm_reduce_kernel(const float* __restrict__ ws, int ksplit,
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
      const u16x4 old = accumulate ? *pc : u16x4{0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2h<F16>(v[j] + (accumulate ? h2f<F16>(old[j]) : 0.f));
      *pc = o;
    }
  }
}

}  // namespace

// Load the assembled code object (once per process; later calls are no-ops).
PIAMD_EXPORT int piamd_agemm_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_mod) return 0;
  return (int)hipModuleLoad(&g_mod, path);
}

PIAMD_EXPORT int piamd_agemm_loaded() { return g_mod != nullptr; }

// C[M][N] (+)= op(A) · op(B), same contract as piamd_gemm_pipe:
// trans_a: A stored [K][M] (else [M][K]); trans_b: B stored [N][K] (else [K][N]).
// K % (64·ksplit) == 0 with K/ksplit ≥ 128; N % 4 == 0; leading dims % 8 == 0 and < 2^22;
// M % 8 == 0 when A is [K][M]; N % 8 == 0 when B is [K][N]; 16-byte aligned pointers.
// c_f32 / accumulate: bf16 or f32 C, stored or accumulated (C += A·B).
// ksplit > 1: f32 partial planes in ws [ksplit][M][N], reduced in a fixed order.
// f16: IEEE fp16 operands (and fp16 where a bf16 kernel writes 16-bit values).
// batch > 1: C[i] (+)= op(A[i])·op(B[i]) for i < batch, operand i at base + i·s{a,b,c} elements
// (a stride may be 0: broadcast); no split-K, no fused epilogue.
// colsum (nullable, epi == 2 only): the data-gradient epilogue also writes the column sums of C per
// 128-row band into colsum f32 [ceil(M/128)][N] (the bias gradient of the activation's producer,
// reduced over the bands by the caller: no separate pass over C).
PIAMD_EXPORT int piamd_agemm2(const void* a, long long lda, int trans_a, const void* b, long long ldb,
                              int trans_b, void* c, long long ldc, int c_f32, int accumulate, int M,
                              int N, int K, int epi, int act, const void* bias, void* aux,
                              long long ldaux, int ksplit, void* ws, int f16, int batch,
                              long long sa, long long sb, long long sc, void* colsum,
                              hipStream_t st) {
  const bool a_kc = !trans_a, b_kc = trans_b;
  if (batch < 1 || (batch > 1 && (ksplit != 1 || epi != 0 || sa < 0 || sb < 0 || sc <= 0)))
    return (int)hipErrorInvalidValue;
  if (M <= 0 || N <= 0 || K <= 0 || ksplit < 1 || K % (64 * ksplit) || K / ksplit < 128 || N % 4 ||
      (!a_kc && M % 8) || (!b_kc && N % 8) || lda % 8 || ldb % 8 || ldc % 4 ||
      lda >= (1 << 22) || ldb >= (1 << 22) || ldc >= (1 << 26) || epi < 0 || epi > 2 ||
      (epi != 0 && (!a_kc || !b_kc || c_f32 || accumulate || ksplit > 1 || ldaux % 4 ||
                    (epi == 2 && !aux) || !(act == 0 || act == 1 || act == 3 || (act == 2 && epi == 1)) ||
                    (epi == 2 && act == 0))) ||
      (ksplit > 1 && !ws) ||
      ((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) % 16)
    return (int)hipErrorInvalidValue;
  const char* lay = a_kc ? (b_kc ? "nt" : "nn") : (b_kc ? "tt" : "tn");
  const char* ek;
  AgemmArgs g;
  std::memset(&g, 0, sizeof(g));
  if (epi != 0) {
    static const char* const kFused[2][4] = {{"bias", "biasgelu", "biasgeluerf", "biasrelu"},
                                             {"", "dgelu", "", "drelu"}};
    ek = (epi == 1 && act == 0 && !aux) ? "biasnx" : kFused[epi - 1][act];
    if (colsum) {
      if (epi != 2 || (act != 1 && act != 3)) return (int)hipErrorInvalidValue;
      ek = act == 1 ? "dgelucs" : "drelucs";
      g.colsum = colsum;
      g.colsum_bytes = (unsigned)((unsigned long long)((M + 127) / 128) * N * 4);
    }
    g.c = c;
    g.ldc_b = (unsigned)(ldc * 2);
    g.c_bytes = ((unsigned long long)(M - 1) * ldc + N) * 2;
    g.aux_bytes = aux ? ((unsigned long long)(M - 1) * ldaux + N) * 2 : 0;
  } else if (ksplit > 1) {
    ek = "f32";
    g.c = ws;
    g.ldc_b = (unsigned)N * 4;
    g.c_part = (unsigned long long)M * N * 4;
    g.c_bytes = g.c_part * ksplit;
  } else {
    ek = c_f32 ? (accumulate ? "f32acc" : "f32") : (accumulate ? "bf16acc" : "bf16");
    const int es = c_f32 ? 4 : 2;
    g.c = c;
    g.ldc_b = (unsigned)(ldc * es);
    g.c_bytes = ((unsigned long long)(M - 1) * ldc + N) * es;
    if (batch > 1) {
      g.c_part = (unsigned long long)sc * es;
      g.c_bytes += (unsigned long long)(batch - 1) * sc * es;
    }
  }
  // persistent kernel (work units chained through the LDS-DMA stream) when every unit has an
  // even K-block count >= 4; otherwise one tile per workgroup
  const int nk = K / ksplit / 64;
  const bool persistent = nk % 2 == 0 && nk >= 4 && !getenv("PIAMD_AGEMM_NO_PERSIST");
  std::string name = std::string("piamd_agemm_") + (persistent ? "p_" : "") + lay + "_" + ek + (f16 ? "_f16" : "");
  hipFunction_t f = get_fn(name);
  if (!f) return (int)hipErrorInvalidDeviceFunction;
  g.a = a;
  g.b = b;
  g.a_bytes = (a_kc ? (unsigned long long)(M - 1) * lda + K : (unsigned long long)(K - 1) * lda + M) * 2;
  g.b_bytes = (b_kc ? (unsigned long long)(N - 1) * ldb + K : (unsigned long long)(K - 1) * ldb + N) * 2;
  if (batch > 1) {
    g.a_bytes += (unsigned long long)(batch - 1) * sa * 2;
    g.b_bytes += (unsigned long long)(batch - 1) * sb * 2;
    g.a_bstride = (unsigned long long)sa * 2;
    g.b_bstride = (unsigned long long)sb * 2;
  }
  g.lda_b = (unsigned)(lda * 2);
  g.ldb_b = (unsigned)(ldb * 2);
  g.M = M;
  g.N = N;
  g.nk = K / ksplit / 64;
  g.tiles_m = (M + 255) / 256;
  g.tiles_n = (N + 255) / 256;
  g.ntiles = g.tiles_m * g.tiles_n;
  g.ksplit = ksplit;
  g.kmul = batch > 1 ? 0u : (unsigned)(K / ksplit);
  const long long nwg = (long long)g.ntiles * (batch > 1 ? batch : ksplit);
  if (nwg >= (1 << 24)) return (int)hipErrorInvalidValue;
  g.nwg = (unsigned)nwg;
  g.grid = persistent ? (unsigned)std::min<long long>(nwg, num_cus()) : (unsigned)nwg;
  g.rcp_ntiles = 1.0f / (float)g.ntiles;
  static const int group_m = [] {  // PIAMD_AGEMM_GM: m-tiles per tile group (A/B experiments)
    const char* e = getenv("PIAMD_AGEMM_GM");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : GROUP_M;
  }();
  g.gm = group_m;
  g.per_group = group_m * g.tiles_n;
  g.rcp_per_group = 1.0f / (float)g.per_group;
  g.act = act;
  g.aux = aux;
  g.ldaux_b = (unsigned)(ldaux * 2);
  g.bias = bias;
  size_t sz = sizeof(g);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &g, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                 HIP_LAUNCH_PARAM_END};
  hipError_t err = hipModuleLaunchKernel(f, g.grid, 1, 1, 256, 1, 1, 0, st, nullptr, cfg);
  if (err != hipSuccess || ksplit == 1) return (int)err;
  const long long q = (long long)M * N / 4;
  const int grid = (int)std::min<long long>(2048, (q + 255) / 256);
  if (f16)
    hipLaunchKernelGGL(agemm_reduce_kernel<true>, dim3(grid), dim3(256), 0, st, (const float*)ws, ksplit,
                       M, N, c, ldc, c_f32, accumulate);
  else
    hipLaunchKernelGGL(agemm_reduce_kernel<false>, dim3(grid), dim3(256), 0, st, (const float*)ws, ksplit,
                       M, N, c, ldc, c_f32, accumulate);
  return (int)hipGetLastError();
}

PIAMD_EXPORT int piamd_agemm(const void* a, long long lda, int trans_a, const void* b, long long ldb,
                             int trans_b, void* c, long long ldc, int c_f32, int accumulate, int M,
                             int N, int K, int epi, int act, const void* bias, void* aux,
                             long long ldaux, int ksplit, void* ws, int f16, int batch,
                             long long sa, long long sb, long long sc, hipStream_t st) {
  return piamd_agemm2(a, lda, trans_a, b, ldb, trans_b, c, ldc, c_f32, accumulate, M, N, K, epi, act,
                      bias, aux, ldaux, ksplit, ws, f16, batch, sa, sb, sc, nullptr, st);
}
