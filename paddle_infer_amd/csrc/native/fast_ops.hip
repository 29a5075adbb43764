// bf16 / fp16 GPU ops of the native engine on the FRAMEWORK's kernels (libpiamd_kernels.so and the
// hand-scheduled assembly GEMM code object): the same kernels the Python Predictor runs, called
// through their C entry points with no Python in the process.
//
// * GEMMs: a port of ops/gemm.py `gemm_nt` — the skinny MFMA kernel (piamd_small_gemm, tuned
//   configs + heuristic) for few rows, the assembly GEMM (piamd_agemm: persistent, split-K, fused
//   bias / bias+GELU(erf|tanh) / bias+ReLU epilogues) otherwise. Weights stored [in, out] are
//   transposed once to K-contiguous [out, in] copies (piamd_transpose_bf16) and cached.
// * Fused transformer ops of an IR-optimised program (the Python Predictor's passes, saved with
//   `Predictor.save_optimized_model`): multihead_matmul (QKV GEMM + bias, packed flash attention
//   with the BiasQK mask), fc (+ activation), fused_fc_elementwise_layernorm, skip_layernorm,
//   fused_embedding_eltwise_layernorm, layer_norm, softmax, matmul / matmul_v2, lookup_table_v2,
//   and fused_multi_transformer (GPT context + cached decode: flash attention, the split-K decode
//   attention and the packed weight-stream GEMVs).
//
// Parity: reference `paddle/fluid/inference/api/analysis_predictor.cc` running the fused GPU ops
// (`operators/fused/multihead_matmul_op.cu`, `fc_op`, `fused_fc_elementwise_layernorm_op.cu`,
// `skip_layernorm_op.cu`, `fused_embedding_eltwise_layernorm_op.cu`).
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <numeric>
#include <string>
#include <tuple>

#include "../kernels/fa_args.h"
#include "kernels.h"

extern "C" {
int piamd_agemm_load(const char* path);
int piamd_agemm(const void* a, long long lda, int trans_a, const void* b, long long ldb, int trans_b,
                void* c, long long ldc, int c_f32, int accumulate, int M, int N, int K, int epi, int act,
                const void* bias, void* aux, long long ldaux, int ksplit, void* ws, int f16, int batch,
                long long sa, long long sb, long long sc, hipStream_t st);
int piamd_small_gemm(int f16, const void* a, long long lda, const void* b, long long ldb, void* c,
                     long long ldc, int c_f32, int M, int N, int K, int mb, int nb, int wn, int depth,
                     int ks, float alpha, const void* bias, int act, const void* resid, long long ldr,
                     float* ws, int* cnt, hipStream_t st);
int piamd_bias_act_fwd(int f16, int act, const void* x, const void* bias, void* y, void* pre, long long n,
                       int N, hipStream_t stream);
int piamd_layernorm_fwd(int dtype, const void* x, const void* bias, const void* residual, const void* gamma,
                        const void* beta, void* y, void* residual_out, float* mean, float* rstd, int rows,
                        int N, float eps, float p_drop, uint64_t seed, uint64_t offset, int flags,
                        hipStream_t stream);
int piamd_fa_fwd(const FaArgs* args, int f16, hipStream_t stream);
int piamd_embedding_fwd(const long long* ids, const void* w, long long start, int vlocal, const void* p,
                        const long long* pos, int S, void* out, long long T, int H, hipStream_t st);
int piamd_transpose_bf16(const void* src, void* dst, int R, int C, hipStream_t stream);
int piamd_softmax_fwd(int f16, const void* x, const void* mask, int mask_rows, int causal_q, void* y,
                      int rows, int N, float scale, hipStream_t stream);
int piamd_qkv_prep(void* qkv, long long ld, const void* bias, void* kc, void* vc, const int* pos0, int B, int S,
                   int Hq, int Hk, int D, int maxS, int rot, int neox, float base, hipStream_t st);
int piamd_decode_attn(const void* qkv, long long ldq, const void* bias, int prep, int rot, int neox, float base,
                      void* kc, void* vc, const int* lens, int B, int Hq, int Hk, int D, int maxS, int chunk,
                      int nsplit, const void* mask, long long ldm, float scale, float* part, int* cnt, void* out,
                      long long ldo, hipStream_t st);
int piamd_wo_gemm_ex(int bits, const void* x, long long ldx, const void* wp, const float* scale, const void* bias,
                     void* y, long long ldy, float* ws, int* cnt, int M, int N, int K, int KS, int act,
                     const void* ln_g, const void* ln_b, float eps, const void* resid, long long ldr, hipStream_t st);
}

#define FCHK(call, what)                                                                      \
  do {                                                                                        \
    int e_ = (call);                                                                          \
    if (e_ != 0) throw std::runtime_error(std::string(what) + ": framework kernel error " +   \
                                          std::to_string(e_));                                \
  } while (0)

namespace pdn {

// activation codes of the framework kernels (ops/activation.py ACTS)
enum { A_NONE = 0, A_GELU_TANH = 1, A_GELU = 2, A_RELU = 3, A_SILU = 4 };

struct FastState {
  std::map<const void*, DTensor> wt;      // [out, in] K-contiguous copies of [in, out] weights
  std::shared_ptr<Buffer> sg_ws, sg_cnt;  // skinny-GEMM split-K fixup (left zeroed by the kernel)
  size_t sg_ws_n = 0, sg_cnt_n = 0;
  std::shared_ptr<Buffer> ks_ws;          // assembly split-K f32 planes
  size_t ks_ws_n = 0;
  std::map<const void*, DTensor> b16;     // bf16 copies of fp32 parameters (fused_multi_transformer)
  std::map<const void*, DTensor> packed;  // MFMA-tile packed decode weights, keyed by the [N, K] copy
  std::map<std::string, std::shared_ptr<Buffer>> scratch;  // zero-initialised, kept zeroed by the kernels
};

namespace {

hipStream_t S(Ctx& c) { return (hipStream_t)c.stream; }

FastState& state(Ctx& c) {
  if (!c.fast) c.fast = std::make_shared<FastState>();
  return *c.fast;
}

void load_agemm() {
  static std::once_flag once;
  static int err = 0;
  std::call_once(once, [] {
    std::string path;
    if (const char* e = std::getenv("PIAMD_AGEMM_HSACO")) path = e;
    if (path.empty()) {
      Dl_info info;
      if (dladdr((void*)&load_agemm, &info) && info.dli_fname) {
        path = info.dli_fname;
        path = path.substr(0, path.rfind('/') + 1) + "piamd_agemm.hsaco";
      }
    }
    err = piamd_agemm_load(path.c_str());
  });
  if (err) throw std::runtime_error("native engine: cannot load the assembly GEMM code object");
}

DTensor make(Ctx& c, int dtype, std::vector<int64_t> dims) {
  DTensor t;
  t.dtype = dtype;
  t.dims = std::move(dims);
  t.buf = alloc_buffer(t.nbytes(), c.gpu);
  return t;
}

DTensor& get(Ctx& c, Scope& s, const std::string& n) {
  auto it = s.find(n);
  if (it == s.end()) throw std::runtime_error("variable '" + n + "' is not set");
  if (!it->second.on_dev()) it->second = to_device(it->second, c);
  return it->second;
}

int64_t prod(const std::vector<int64_t>& d, size_t b, size_t e) {
  int64_t p = 1;
  for (size_t i = b; i < e && i < d.size(); ++i) p *= d[i];
  return p;
}

int h16(const DTensor& t) { return t.dtype == VT_FP16 ? 1 : 0; }

// ------------------------------------------------------------------------- GEMM dispatcher
// ops/gemm.py small_cfg / use_small / pick_ksplit (measured: profiles/small_gemm_tune_r4.jsonl,
// small_gemm_bdeep_r6.jsonl; depth = A depth | B depth << 4)
const int kShapes[][2] = {{1, 1}, {1, 2}, {1, 4}, {2, 1}, {2, 2}, {2, 4}, {4, 1}, {4, 2}, {4, 4}, {8, 1}, {8, 2}};

struct SgCfg { int mb, nb, wn, depth, ks; };

SgCfg small_cfg(int M, int N, int K) {
  static const std::map<std::tuple<int, int, int>, SgCfg> tuned = {
      {{16, 3072, 1024}, {1, 1, 1, 1, 1}}, {{16, 1024, 4096}, {1, 1, 1, 1, 4}},
      {{32, 3072, 1024}, {1, 2, 1, 1, 1}}, {{32, 1024, 4096}, {1, 1, 1, 1, 2}},
      {{64, 3072, 1024}, {2, 2, 1, 1, 1}}, {{64, 1024, 4096}, {1, 1, 1, 1, 1}},
      {{128, 3072, 1024}, {2, 4, 1, 0x41, 1}}, {{128, 1024, 1024}, {1, 2, 1, 0x81, 1}},
      {{128, 4096, 1024}, {2, 4, 1, 0x41, 1}}, {{128, 1024, 4096}, {2, 1, 1, 0x81, 1}},
      {{128, 6144, 2048}, {4, 4, 1, 2, 1}}, {{128, 2048, 2048}, {2, 2, 1, 1, 1}},
      {{128, 8192, 2048}, {4, 4, 1, 2, 1}}, {{256, 3072, 1024}, {4, 4, 1, 1, 1}},
      {{256, 1024, 4096}, {2, 2, 1, 2, 1}}, {{256, 2048, 2048}, {4, 2, 1, 1, 1}},
      {{512, 2048, 2048}, {4, 4, 1, 1, 1}}};
  auto it = tuned.find({M, N, K});
  if (it != tuned.end()) return it->second;
  const int nkb = K / 64;
  int best_mb = 0, best_nb = 0, best_wgs = 0;
  std::tuple<int, int, int> best_key{-1, 0, 0};
  for (auto& sh : kShapes) {
    const int mb = sh[0], nb = sh[1];
    if (mb > 1 && 16 * mb > M) continue;
    const int wgs = ((M + 16 * mb - 1) / (16 * mb)) * ((N + 16 * nb - 1) / (16 * nb));
    if (wgs < 192) continue;
    std::tuple<int, int, int> key{mb * nb, -std::abs(mb - nb), nb};
    if (key > best_key) best_key = key, best_mb = mb, best_nb = nb, best_wgs = wgs;
  }
  if (!best_mb) {
    const int wgs = ((M + 15) / 16) * ((N + 15) / 16);
    int ks = 1;
    while (wgs * ks < 192 && ks * 2 <= nkb / 4) ks *= 2;
    return {1, 1, 1, 1, ks};
  }
  const int depth = (best_mb * best_nb >= 16 && K >= 2048 && best_wgs <= 256) ? 2 : 1;
  return {best_mb, best_nb, 1, depth, 1};
}

bool use_small(int M, int N, int K) {
  if (M <= 64) return true;
  if (M <= 128 && K < 8192) return true;
  return M <= 512 && (int64_t)N * K <= 2048LL * 2048;
}

int pick_ksplit(int M, int N, int K) {  // ops/gemm.py pick_ksplit
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const int nk = K / 64;
  if (tiles >= 512 || nk < 16) return 1;
  int best = 1;
  double best_t = -1;
  for (int ks = 1; ks <= std::min(256, nk / 8); ++ks) {
    if (nk % ks) continue;
    const int waves = (tiles * ks + 255) / 256;
    const double t = (double)waves / ks;
    if (best_t < 0 || t < best_t - 1e-9) best = ks, best_t = t;
  }
  return best;
}

void zero_dev(Ctx& c, void* p, size_t bytes) {
  if (hipMemsetAsync(p, 0, bytes, S(c)) != hipSuccess) throw std::runtime_error("hipMemsetAsync");
}

// C[M, N] (ldc) = act(A[M, K] (lda) · B[N, K]ᵀ (ldb) + bias); 16-bit A / B / C of one dtype;
// K % 64 == 0, N % 4 == 0 (the callers' shapes; checked).
void gemm_nt(Ctx& c, int f16, const void* a, int64_t lda, const void* b, int64_t ldb, void* out,
             int64_t ldc, int M, int N, int K, const void* bias, int act, const std::string& who) {
  if (M == 0) return;
  if (K % 64 || N % 4 || K < 64)
    throw std::runtime_error(who + ": native GEMM needs K % 64 == 0 and N % 4 == 0 (got N=" +
                             std::to_string(N) + ", K=" + std::to_string(K) + ")");
  FastState& st = state(c);
  if (use_small(M, N, K)) {
    const SgCfg g = small_cfg(M, N, K);
    float* ws = nullptr;
    int* cnt = nullptr;
    if (g.ks > 1) {
      const size_t tiles = (size_t)((M + 16 * g.mb - 1) / (16 * g.mb)) * ((N + 16 * g.nb * g.wn - 1) / (16 * g.nb * g.wn));
      const size_t need = (size_t)M * N;
      if (st.sg_ws_n < need) {
        st.sg_ws = alloc_buffer(need * 4, true);
        st.sg_ws_n = need;
        zero_dev(c, st.sg_ws->p, need * 4);
      }
      if (st.sg_cnt_n < std::max<size_t>(tiles, 4096)) {
        st.sg_cnt_n = std::max<size_t>(tiles, 4096);
        st.sg_cnt = alloc_buffer(st.sg_cnt_n * 4, true);
        zero_dev(c, st.sg_cnt->p, st.sg_cnt_n * 4);
      }
      ws = (float*)st.sg_ws->p;
      cnt = (int*)st.sg_cnt->p;
    }
    FCHK(piamd_small_gemm(f16, a, lda, b, ldb, out, ldc, 0, M, N, K, g.mb, g.nb, g.wn, g.depth, g.ks, 1.f,
                          bias, act, nullptr, 0, ws, cnt, S(c)),
         who + " (skinny GEMM)");
    return;
  }
  if (K < 128) throw std::runtime_error(who + ": assembly GEMM needs K >= 128");
  load_agemm();
  int ks = pick_ksplit(M, N, K);
  if (K % (64 * ks) || K / ks < 128) ks = 1;
  const bool fused = ks == 1 && (act == A_NONE || act == A_GELU_TANH || act == A_GELU || act == A_RELU) &&
                     (bias || act != A_NONE);
  if (fused) {
    FCHK(piamd_agemm(a, lda, 0, b, ldb, 1, out, ldc, 0, 0, M, N, K, 1, act, bias, nullptr, 0, 1, nullptr, f16,
                     1, 0, 0, 1, S(c)),
         who + " (assembly GEMM)");
    return;
  }
  void* ws = nullptr;
  if (ks > 1) {
    const size_t need = (size_t)ks * M * N;
    if (st.ks_ws_n < need) {
      st.ks_ws = alloc_buffer(need * 4, true);
      st.ks_ws_n = need;
    }
    ws = st.ks_ws->p;
  }
  FCHK(piamd_agemm(a, lda, 0, b, ldb, 1, out, ldc, 0, 0, M, N, K, 0, 0, nullptr, nullptr, 0, ks, ws, f16, 1,
                   0, 0, 1, S(c)),
       who + " (assembly GEMM)");
  if (bias || act != A_NONE) {
    if (ldc != N) throw std::runtime_error(who + ": strided output with an unfused epilogue");
    FCHK(piamd_bias_act_fwd(f16, act, out, bias, out, nullptr, (long long)M * N, N, S(c)), who + " (bias_act)");
  }
}

// Caches keyed by a source buffer hold only derivatives of persistent buffers (the loaded
// parameters and earlier cache products, `Ctx::persist`): an activation's address can be handed
// back by the allocator to a different tensor in a later Run, so its derivatives are recomputed.
bool persistent(const Ctx& c, const DTensor& t) { return c.persist && t.buf && c.persist->count(t.buf.get()); }
void keep_persistent(Ctx& c, const DTensor& t) {
  if (c.persist && t.buf) c.persist->insert(t.buf.get());
}

// K-contiguous [out, in] copy of a [in, out] weight (cached per persistent source buffer)
DTensor transposed(Ctx& c, const DTensor& w, const std::string& who) {
  FastState& st = state(c);
  const bool cache = persistent(c, w);
  if (cache) {
    auto it = st.wt.find(w.buf->p);
    if (it != st.wt.end()) return it->second;
  }
  if (w.dims.size() != 2) throw std::runtime_error(who + ": weight must be 2-D");
  const int R = (int)w.dims[0], C = (int)w.dims[1];
  DTensor t = make(c, w.dtype, {w.dims[1], w.dims[0]});
  FCHK(piamd_transpose_bf16(w.buf->p, t.buf->p, R, C, S(c)), who + " (transpose)");
  if (!cache) return t;
  keep_persistent(c, t);
  return st.wt[w.buf->p] = t;
}

int act_code(const std::string& a, bool* tanh_after) {
  *tanh_after = false;
  if (a.empty() || a == "identity") return A_NONE;
  if (a == "relu") return A_RELU;
  if (a == "gelu") return A_GELU;
  if (a == "gelu_tanh") return A_GELU_TANH;
  if (a == "silu" || a == "swish") return A_SILU;
  if (a == "tanh") { *tanh_after = true; return A_NONE; }
  throw std::runtime_error("native fc: activation '" + a + "' not supported");
}

// y[rows, N] = x[rows, K] · W[K, N] + bias (act), x flattened at num_col_dims
DTensor linear(Ctx& c, const DTensor& x, int ncol, const DTensor& w, const DTensor* bias, int act,
               bool tanh_after, const std::string& who) {
  const int64_t rows = prod(x.dims, 0, ncol), K = prod(x.dims, ncol, x.dims.size());
  if (w.dims.size() != 2 || w.dims[0] != K) throw std::runtime_error(who + ": weight shape mismatch");
  const int64_t N = w.dims[1];
  std::vector<int64_t> od(x.dims.begin(), x.dims.begin() + ncol);
  od.push_back(N);
  DTensor y = make(c, x.dtype, od);
  const DTensor& wt = transposed(c, w, who);
  gemm_nt(c, h16(x), x.buf->p, K, wt.buf->p, K, y.buf->p, N, (int)rows, (int)N, (int)K,
          bias ? bias->buf->p : nullptr, act, who);
  if (tanh_after) gpu::unary16(c, U_TANH, h16(x), y.buf->p, y.buf->p, y.numel(), 0.f, 0.f);
  return y;
}

void layer_norm16(Ctx& c, const DTensor& x, const DTensor* resid, const DTensor* g, const DTensor* b, DTensor& y,
                  int64_t rows, int64_t N, float eps, const std::string& who) {
  if (N % 8) throw std::runtime_error(who + ": width must be a multiple of 8");
  FCHK(piamd_layernorm_fwd(x.dtype == VT_FP16 ? 2 : 1, x.buf->p, nullptr, resid ? resid->buf->p : nullptr,
                           g ? g->buf->p : nullptr, b ? b->buf->p : nullptr, y.buf->p, nullptr, nullptr, nullptr,
                           (int)rows, (int)N, eps, 0.f, 0, 0, 0, S(c)),
       who);
}

const DTensor* opt_in(Ctx& c, Scope& s, const OpDesc& op, const std::string& slot) {
  if (!op.has_in(slot)) return nullptr;
  return &get(c, s, op.in(slot));
}

void need16(const DTensor& t, int dt, const std::string& who) {
  if (t.dtype != dt) throw std::runtime_error(who + ": mixed tensor dtypes");
}

// ---------------------------------------------------------------------------------- ops
void op_fc(Ctx& c, const OpDesc& op, Scope& s) {
  const DTensor& x = get(c, s, op.in("Input"));
  const DTensor& w = get(c, s, op.in("W"));
  const DTensor* bias = opt_in(c, s, op, "Bias");
  need16(w, x.dtype, "fc");
  bool ta;
  const int act = act_code(op.as("activation_type", ""), &ta);
  const int ncol = (int)op.ai("in_num_col_dims", (int64_t)x.dims.size() - 1);
  s[op.out("Out")] = linear(c, x, ncol, w, bias, act, ta, "fc");
}

void op_fc_eltwise_ln(Ctx& c, const OpDesc& op, Scope& s) {
  const DTensor& x = get(c, s, op.in("X"));
  const DTensor& w = get(c, s, op.in("W"));
  const DTensor& y = get(c, s, op.in("Y"));
  const DTensor* b0 = opt_in(c, s, op, "Bias0");
  const int ncol = (int)op.ai("x_num_col_dims", (int64_t)x.dims.size() - 1);
  const int act = op.as("activation_type", "") == "relu" ? A_RELU : A_NONE;
  DTensor h = linear(c, x, ncol, w, b0, act, false, "fused_fc_elementwise_layernorm");
  DTensor out = make(c, x.dtype, h.dims);
  const int64_t N = h.dims.back(), rows = h.numel() / N;
  layer_norm16(c, h, &y, opt_in(c, s, op, "Scale"), opt_in(c, s, op, "Bias1"), out, rows, N,
               op.af("epsilon", 1e-5f), "fused_fc_elementwise_layernorm");
  s[op.out("Out")] = out;
}

void op_skip_ln(Ctx& c, const OpDesc& op, Scope& s) {
  const DTensor& x = get(c, s, op.in("X"));
  const DTensor& y = get(c, s, op.in("Y"));
  DTensor out = make(c, x.dtype, x.dims);
  const int64_t N = x.dims.back(), rows = x.numel() / N;
  layer_norm16(c, x, &y, opt_in(c, s, op, "Scale"), opt_in(c, s, op, "Bias"), out, rows, N,
               op.af("epsilon", 1e-5f), "skip_layernorm");
  s[op.out("Out")] = out;
}

void op_layer_norm(Ctx& c, const OpDesc& op, Scope& s) {
  const DTensor& x = get(c, s, op.in("X"));
  const int64_t bna = op.ai("begin_norm_axis", 1);
  const int64_t rows = prod(x.dims, 0, (size_t)bna), N = x.numel() / std::max<int64_t>(rows, 1);
  DTensor out = make(c, x.dtype, x.dims);
  layer_norm16(c, x, nullptr, opt_in(c, s, op, "Scale"), opt_in(c, s, op, "Bias"), out, rows, N,
               op.af("epsilon", 1e-5f), "layer_norm");
  s[op.out("Y")] = out;
}

void op_mha(Ctx& c, const OpDesc& op, Scope& s) {
  const DTensor& x = get(c, s, op.in("Input"));
  const DTensor& w = get(c, s, op.in("W"));
  const DTensor& bias = get(c, s, op.in("Bias"));
  const DTensor* mask = opt_in(c, s, op, "BiasQK");
  if (x.dims.size() != 3) throw std::runtime_error("multihead_matmul: Input must be [B, S, E]");
  const int64_t B = x.dims[0], S_ = x.dims[1], E = x.dims[2];
  const int H = (int)op.ai("head_number", 1);
  const int D = (int)(E / H);
  // W [E, 3, E] (or [E, 3E]) viewed [E, 3E]
  DTensor w2 = w;
  w2.dims = {E, 3 * E};
  DTensor b2 = bias;
  b2.dims = {3 * E};
  DTensor qkv = linear(c, x, 2, w2, &b2, A_NONE, false, "multihead_matmul");
  DTensor o = make(c, x.dtype, {B, S_, E});
  FaArgs a;
  std::memset(&a, 0, sizeof(a));
  const char* base = (const char*)qkv.buf->p;
  const size_t es = 2;
  a.q = base;
  a.k = base + (size_t)E * es;
  a.v = base + (size_t)2 * E * es;
  a.o = o.buf->p;
  a.lse = nullptr;
  a.B = (int)B, a.Sq = (int)S_, a.Sk = (int)S_, a.Hq = H, a.Hk = H, a.D = D, a.causal = 0;
  a.sqb = a.skb = a.svb = S_ * 3 * E;
  a.sqs = a.sks = a.svs = 3 * E;
  a.sqh = a.skh = a.svh = D;
  a.sob = S_ * E, a.sos = E, a.soh = D;
  if (mask) {
    const auto& md = mask->dims;  // [B|1, H|1, Sq|1, Sk]
    if (md.size() != 4 || md[3] != S_) throw std::runtime_error("multihead_matmul: BiasQK must be [B, H, S, S]");
    need16(*mask, x.dtype, "multihead_matmul BiasQK");
    a.mask = mask->buf->p;
    a.smb = md[0] > 1 ? md[1] * md[2] * md[3] : 0;
    a.smh = md[1] > 1 ? md[2] * md[3] : 0;
    a.smq = md[2] > 1 ? md[3] : 0;
  }
  a.scale = op.af("alpha", 1.f / std::sqrt((float)D));
  FCHK(piamd_fa_fwd(&a, h16(x), S(c)), "multihead_matmul (flash attention)");
  s[op.out("Out")] = o;
}

void op_lookup(Ctx& c, const OpDesc& op, Scope& s) {
  const DTensor& ids = get(c, s, op.in("Ids"));
  const DTensor& w = get(c, s, op.in("W"));
  const int64_t pad = op.ai("padding_idx", -1);
  if (ids.dtype != VT_INT64) throw std::runtime_error("lookup_table_v2: int64 ids");
  if (pad >= 0) throw std::runtime_error("lookup_table_v2: padding_idx is not supported by the 16-bit path");
  std::vector<int64_t> od = ids.dims;
  if (op.type == "lookup_table" && !od.empty() && od.back() == 1) od.pop_back();
  const int64_t H = w.dims[1];
  od.push_back(H);
  DTensor o = make(c, w.dtype, od);
  FCHK(piamd_embedding_fwd((const long long*)ids.buf->p, w.buf->p, 0, (int)w.dims[0], nullptr, nullptr, 1,
                           o.buf->p, ids.numel(), (int)H, S(c)),
       "lookup_table_v2");
  s[op.out("Out")] = o;
}

void op_emb_eltwise_ln(Ctx& c, const OpDesc& op, Scope& s) {
  // Σ_i Embs[i][Ids[i]] → LayerNorm(Scale, Bias)
  const auto& idn = op.inputs.at("Ids");
  const auto& emn = op.inputs.at("Embs");
  if (idn.size() != emn.size() || idn.empty()) throw std::runtime_error("fused_embedding_eltwise_layernorm: Ids/Embs");
  DTensor acc;
  for (size_t i = 0; i < idn.size(); ++i) {
    const DTensor& ids = get(c, s, idn[i]);
    const DTensor& w = get(c, s, emn[i]);
    std::vector<int64_t> od = ids.dims;
    if (!od.empty() && od.back() == 1) od.pop_back();
    od.push_back(w.dims[1]);
    DTensor e = make(c, w.dtype, od);
    FCHK(piamd_embedding_fwd((const long long*)ids.buf->p, w.buf->p, 0, (int)w.dims[0], nullptr, nullptr, 1,
                             e.buf->p, ids.numel(), (int)w.dims[1], S(c)),
         "fused_embedding_eltwise_layernorm");
    if (i == 0) {
      acc = e;
    } else {
      Bcast bc;
      bc.nd = 1;
      bc.dims[0] = e.numel();
      bc.sa[0] = bc.sb[0] = 1;
      bc.n = e.numel();
      gpu::binary16(c, B_ADD, h16(e), acc.buf->p, e.buf->p, acc.buf->p, bc);
    }
  }
  DTensor out = make(c, acc.dtype, acc.dims);
  const int64_t N = acc.dims.back(), rows = acc.numel() / N;
  layer_norm16(c, acc, nullptr, opt_in(c, s, op, "Scale"), opt_in(c, s, op, "Bias"), out, rows, N,
               op.af("epsilon", 1e-5f), "fused_embedding_eltwise_layernorm");
  s[op.out("Out")] = out;
}

void op_softmax(Ctx& c, const OpDesc& op, Scope& s) {
  const DTensor& x = get(c, s, op.in("X"));
  const int64_t axis = op.ai("axis", -1);
  if (axis != -1 && axis != (int64_t)x.dims.size() - 1)
    throw std::runtime_error("softmax: the 16-bit path takes the last axis");
  const int64_t N = x.dims.back(), rows = x.numel() / N;
  DTensor o = make(c, x.dtype, x.dims);
  FCHK(piamd_softmax_fwd(h16(x), x.buf->p, nullptr, 0, 0, o.buf->p, (int)rows, (int)N, 1.f, S(c)), "softmax");
  s[op.out("Out")] = o;
}

// matmul / matmul_v2 with a 2-D weight-like Y (the projections of exported models)
void op_matmul(Ctx& c, const OpDesc& op, Scope& s) {
  const DTensor& x = get(c, s, op.in("X"));
  const DTensor& y = get(c, s, op.in("Y"));
  const bool v2 = op.type == "matmul_v2";
  const bool tx = v2 ? op.ab("trans_x", false) : op.ab("transpose_X", false);
  const bool ty = v2 ? op.ab("trans_y", false) : op.ab("transpose_Y", false);
  const float alpha = v2 ? 1.f : op.af("alpha", 1.f);
  if (tx || y.dims.size() != 2 || x.dims.size() < 2 || alpha != 1.f)
    throw std::runtime_error(op.type + ": the 16-bit native path takes X[.., K] · Y[K, N] (or Yᵀ)");
  const int64_t K = x.dims.back(), rows = x.numel() / K;
  const int64_t N = ty ? y.dims[0] : y.dims[1];
  std::vector<int64_t> od(x.dims.begin(), x.dims.end() - 1);
  od.push_back(N);
  DTensor o = make(c, x.dtype, od);
  const DTensor& wt = ty ? y : transposed(c, y, op.type);
  gemm_nt(c, h16(x), x.buf->p, K, wt.buf->p, K, o.buf->p, N, (int)rows, (int)N, (int)K, nullptr, A_NONE, op.type);
  s[op.out("Out")] = o;
}

// ------------------------------------------------------------------ fused_multi_transformer
// Parity: reference `operators/fused/fused_multi_transformer_op.cu` (pre-LN GPT blocks with a
// [2, B, H, max_seq, D] CacheKV per layer: context pass without TimeStep, one-token decode with it)
// and the Python Predictor's path (incubate/nn/functional.py multi_transformer_forward): context =
// LN → QKV GEMM → qkv_prep (bias, cache write) → flash attention → out GEMM → add+LN → FFN1(+act) →
// FFN2, the residual adds folded into the next LayerNorm; decode = per layer four weight-stream
// GEMVs on MFMA-tile packed weights (pre-LN in the GEMV prologue at ≤ 2 rows, residual adds in the
// epilogues) around the split-K decode attention that also adds the QKV bias and writes the cache.
// bf16 compute (fp32 models need PrecisionType::kBf16); caches updated in place.
__global__ void fmt_pack_kernel(const unsigned short* __restrict__ w, unsigned short* __restrict__ p, int N, int K) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)N * K) return;
  const int n = (int)(i / K), k = (int)(i % K);
  p[(((long long)(n / 32) * (K / 16) + k / 16) * 64 + (n % 32) + 32 * ((k % 16) / 8)) * 8 + k % 8] = w[i];
}

__global__ void fmt_lens_kernel(const int* __restrict__ ts, int* __restrict__ lens, int B) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b < B) lens[b] = ts[0] + 1;
}

// zero-initialised scratch, one buffer per key (the kernels that use it leave it zeroed again)
void* zscratch(Ctx& c, const std::string& key, size_t bytes) {
  FastState& st = state(c);
  auto& b = st.scratch[key];
  if (!b) {
    b = alloc_buffer(std::max<size_t>(bytes, 4), true);
    zero_dev(c, b->p, std::max<size_t>(bytes, 4));
  }
  return b->p;
}

// bf16 view of a floating tensor: bf16 as is; fp32 cast (cached per source buffer when `cache`)
DTensor as_bf16(Ctx& c, const DTensor& t, bool cache, const std::string& who) {
  if (t.dtype == VT_BF16) return t;
  if (t.dtype != VT_FP32) throw std::runtime_error(who + ": bf16 or fp32 tensors only (fp16 model)");
  FastState& st = state(c);
  cache = cache && persistent(c, t);
  if (cache) {
    auto it = st.b16.find(t.buf->p);
    if (it != st.b16.end()) return it->second;
  }
  DTensor o = make(c, VT_BF16, t.dims);
  gpu::cast(c, t.buf->p, VT_FP32, o.buf->p, VT_BF16, t.numel());
  if (cache) {
    keep_persistent(c, o);
    st.b16[t.buf->p] = o;
  }
  return o;
}

DTensor packed_of(Ctx& c, const DTensor& nk, const std::string& who) {
  FastState& st = state(c);
  const bool cache = persistent(c, nk);
  if (cache) {
    auto it = st.packed.find(nk.buf->p);
    if (it != st.packed.end()) return it->second;
  }
  const int N = (int)nk.dims[0], K = (int)nk.dims[1];
  if (N % 32 || K % 16) throw std::runtime_error(who + ": decode weights need N % 32 == 0 and K % 16 == 0");
  DTensor p = make(c, VT_BF16, nk.dims);
  const long long n = (long long)N * K;
  hipLaunchKernelGGL(fmt_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(c),
                     (const unsigned short*)nk.buf->p, (unsigned short*)p.buf->p, N, K);
  if (!cache) return p;
  keep_persistent(c, p);
  return st.packed[nk.buf->p] = p;
}

// y[M, N] = act(LN?(x) · W + bias) (+ resid) on the packed weight-stream GEMV (ops/inference.py
// packed_linear: LN in the prologue at ≤ 2 rows, split-K to ~192 workgroups otherwise)
DTensor fmt_gemv(Ctx& c, const DTensor& x, int M, int K, const DTensor& wp, int N, const DTensor* bias, int act,
                 const DTensor* lng, const DTensor* lnb, float eps, const DTensor* resid, const std::string& who) {
  DTensor y = make(c, VT_BF16, {M, N});
  const void* xin = x.buf->p;
  DTensor xn;
  const bool fuse_ln = lng && lnb && M <= 2 && K % 512 == 0 && K <= 2048;
  if (lng && !fuse_ln) {
    xn = make(c, VT_BF16, {M, K});
    layer_norm16(c, x, nullptr, lng, lnb, xn, M, K, eps, who);
    xin = xn.buf->p;
  }
  const int tiles = (N / 32) * ((M + 31) / 32);
  int KS = 1;
  if (!fuse_ln)
    while (tiles * KS < 192 && (K / 16) / (KS * 2) >= 16) KS *= 2;
  float* ws = nullptr;
  int* cnt = nullptr;
  if (KS > 1) {
    const std::string k = std::to_string(M) + "x" + std::to_string(N);
    if (M <= 8) {  // in-kernel fixup: zeroed partials + arrival counters
      ws = (float*)zscratch(c, "wo_ws" + k, (size_t)M * N * 4);
      cnt = (int*)zscratch(c, "wo_cnt" + k, (size_t)tiles * 4);
    } else {
      ws = (float*)zscratch(c, "wo_ks" + k + "x" + std::to_string(KS), (size_t)KS * M * N * 4);
    }
  }
  FCHK(piamd_wo_gemm_ex(16, xin, K, wp.buf->p, nullptr, bias ? bias->buf->p : nullptr, y.buf->p, N, ws, cnt, M, N,
                        K, KS, act, fuse_ln ? lng->buf->p : nullptr, fuse_ln ? lnb->buf->p : nullptr, eps,
                        resid ? resid->buf->p : nullptr, resid ? N : 0, S(c)),
       who + " (weight-stream GEMV)");
  return y;
}

void op_fmt(Ctx& c, const OpDesc& op, Scope& s) {
  const std::string who = "fused_multi_transformer";
  auto reject = [&](const std::string& what) {
    throw std::runtime_error(who + " (native engine): " + what + " is not supported (use the Python Predictor)");
  };
  if (!op.ab("pre_layer_norm", true)) reject("post-LayerNorm");
  if (!op.ab("trans_qkvw", true)) reject("trans_qkvw = false");
  if (op.has_in("PreCaches") || op.has_in("RotaryPosEmb") || op.ai("rotary_emb_dims", 0) != 0) reject("RoPE / PreCaches");
  if (op.has_in("SeqLengths") || op.has_in("BeamCacheOffset")) reject("SeqLengths / BeamCacheOffset");
  if (op.ai("ring_id", -1) >= 0) reject("a tensor-parallel ring");
  const std::string actn = op.as("act_method", "gelu");
  const int act = actn == "gelu" ? A_GELU : actn == "relu" ? A_RELU : -1;
  if (act < 0) reject("act_method " + actn);
  const float eps = op.af("epsilon", 1e-5f);
  const DTensor& x0 = get(c, s, op.in("X"));
  if (x0.dtype == VT_FP32 && c.prec16 != VT_BF16)
    throw std::runtime_error(who + ": fp32 models run natively in bf16 (EnableUseGpu(..., PrecisionType::kBf16))");
  const DTensor x = as_bf16(c, x0, false, who);
  if (x.dims.size() != 3) throw std::runtime_error(who + ": X must be [B, S, E]");
  const int B = (int)x.dims[0], S_ = (int)x.dims[1], E = (int)x.dims[2], T = B * S_;
  const int L = (int)op.inputs.at("QKVW").size();
  std::vector<DTensor> W[12];
  const char* slots[12] = {"LnScale", "LnBias", "QKVW", "QKVBias", "OutLinearW", "OutLinearBias",
                           "FFNLnScale", "FFNLnBias", "FFN1Weight", "FFN1Bias", "FFN2Weight", "FFN2Bias"};
  for (int k = 0; k < 12; ++k) {
    const bool required = k == 0 || k == 2 || k == 4 || k == 6 || k == 8 || k == 10;
    if (!op.has_in(slots[k])) {
      if (required) throw std::runtime_error(who + ": missing " + slots[k]);
      W[k].assign(L, DTensor());
      continue;
    }
    const auto& names = op.inputs.at(slots[k]);
    if ((int)names.size() != L) throw std::runtime_error(who + ": " + slots[k] + " needs one entry per layer");
    for (const auto& n : names) W[k].push_back(as_bf16(c, get(c, s, n), true, who));
  }
  auto opt = [&](int k, int l) -> const DTensor* { return W[k][l].buf ? &W[k][l] : nullptr; };
  // QKVW [3, H, D, E] or [Hq + 2Hk, D, E] (trans_qkvw): already the K-contiguous [N, E] operand
  const auto& qd = W[2][0].dims;
  if (qd.back() != E || (qd.size() != 4 && qd.size() != 3)) throw std::runtime_error(who + ": QKVW shape");
  const int D = (int)qd[qd.size() - 2];
  const int nh = (int)(W[2][0].numel() / ((int64_t)D * E));
  const int Hk = op.ai("num_kv_heads", -1) > 0 ? (int)op.ai("num_kv_heads", -1) : nh / 3;
  const int Hq = nh - 2 * Hk, HQD = Hq * D, NQKV = nh * D;
  const int F = (int)W[8][0].dims[1];
  // caches: per layer [2, B, Hk, maxS, D], bf16 in place (an fp32 feed is converted once and kept)
  std::vector<DTensor*> caches;
  if (op.has_in("CacheKV")) {
    for (const auto& n : op.inputs.at("CacheKV")) {
      DTensor& ct = get(c, s, n);
      if (ct.dtype != VT_BF16) ct = as_bf16(c, ct, false, who);
      if (ct.dims.size() != 5 || ct.dims[0] != 2 || ct.dims[1] != B || ct.dims[2] != Hk || ct.dims[4] != D)
        throw std::runtime_error(who + ": CacheKV must be [2, B, Hk, max_seq, D]");
      caches.push_back(&ct);
    }
    if ((int)caches.size() != L) throw std::runtime_error(who + ": one CacheKV per layer");
  }
  const int maxS = caches.empty() ? 0 : (int)caches[0]->dims[3];
  auto kv = [&](int l, int which) -> void* {
    if (caches.empty()) return nullptr;
    return (char*)caches[l]->buf->p + (size_t)which * B * Hk * maxS * D * 2;
  };
  const DTensor* mask = nullptr;
  DTensor maskb;
  if (op.has_in("SrcMask")) {
    maskb = as_bf16(c, get(c, s, op.in("SrcMask")), false, who);
    mask = &maskb;
  }
  const bool decode = op.has_in("TimeStep");
  DTensor res = x;
  res.dims = {T, E};
  if (decode) {
    if (S_ != 1 || caches.empty()) throw std::runtime_error(who + ": decode (TimeStep) needs one token and CacheKV");
    if (Hq % Hk || (Hq / Hk != 1 && Hq / Hk != 2 && Hq / Hk != 4 && Hq / Hk != 8) || (D != 64 && D != 128))
      reject("this head geometry in decode");
    const DTensor& ts = get(c, s, op.in("TimeStep"));
    if (ts.dtype != VT_INT32) throw std::runtime_error(who + ": TimeStep must be int32");
    int* lens = (int*)zscratch(c, "fmt_lens" + std::to_string(B), (size_t)B * 4);
    hipLaunchKernelGGL(fmt_lens_kernel, dim3((B + 63) / 64), dim3(64), 0, S(c), (const int*)ts.buf->p, lens, B);
    int chunk = maxS <= 256 ? std::max(16, maxS) : maxS <= 1024 ? 64 : maxS <= 4096 ? 128 : 256;
    chunk = std::max(16, std::min(512, chunk));
    const int ns = std::max(1, (maxS + chunk - 1) / chunk);
    float* part = nullptr;
    int* cnt = nullptr;
    if (ns > 1) {
      part = (float*)zscratch(c, "fmt_part" + std::to_string(B * Hq * ns * (D + 2)), (size_t)B * Hq * ns * (D + 2) * 4);
      cnt = (int*)zscratch(c, "fmt_cnt" + std::to_string(B * Hk), (size_t)B * Hk * 4);
    }
    const long long ldm = mask ? mask->numel() / B : 0;
    for (int l = 0; l < L; ++l) {
      DTensor q2 = W[2][l];
      q2.dims = {NQKV, E};
      const DTensor& wq = packed_of(c, q2, who);
      const DTensor& wo = packed_of(c, transposed(c, W[4][l], who), who);
      const DTensor& w1 = packed_of(c, transposed(c, W[8][l], who), who);
      const DTensor& w2 = packed_of(c, transposed(c, W[10][l], who), who);
      DTensor qkv = fmt_gemv(c, res, B, E, wq, NQKV, nullptr, A_NONE, &W[0][l], opt(1, l), eps, nullptr, who);
      DTensor att = make(c, VT_BF16, {B, HQD});
      FCHK(piamd_decode_attn(qkv.buf->p, NQKV, opt(3, l) ? W[3][l].buf->p : nullptr, 1, 0, 1, 10000.f, kv(l, 0),
                             kv(l, 1), lens, B, Hq, Hk, D, maxS, chunk, ns, mask ? mask->buf->p : nullptr, ldm,
                             1.f / std::sqrt((float)D), part, cnt, att.buf->p, HQD, S(c)),
           who + " (decode attention)");
      res = fmt_gemv(c, att, B, HQD, wo, E, opt(5, l), A_NONE, nullptr, nullptr, eps, &res, who);
      DTensor h = fmt_gemv(c, res, B, E, w1, F, opt(9, l), act, &W[6][l], opt(7, l), eps, nullptr, who);
      res = fmt_gemv(c, h, B, F, w2, E, opt(11, l), A_NONE, nullptr, nullptr, eps, &res, who);
    }
  } else {
    int* pos0 = (int*)zscratch(c, "fmt_pos0_" + std::to_string(B), (size_t)B * 4);
    DTensor pend;
    const DTensor* pend_b = nullptr;
    for (int l = 0; l < L; ++l) {
      DTensor xn = make(c, VT_BF16, {T, E});
      if (!pend.buf) {
        layer_norm16(c, res, nullptr, &W[0][l], opt(1, l), xn, T, E, eps, who);
      } else {  // LN(residual + ffn2 + bias) of the previous block, its sum kept as the residual
        DTensor nr = make(c, VT_BF16, {T, E});
        FCHK(piamd_layernorm_fwd(1, pend.buf->p, pend_b ? pend_b->buf->p : nullptr, res.buf->p, W[0][l].buf->p,
                                 opt(1, l) ? W[1][l].buf->p : nullptr, xn.buf->p, nr.buf->p, nullptr, nullptr, T, E,
                                 eps, 0.f, 0, 0, 0, S(c)),
             who + " (add + LayerNorm)");
        res = nr;
      }
      DTensor qkv = make(c, VT_BF16, {T, NQKV});
      gemm_nt(c, 0, xn.buf->p, E, W[2][l].buf->p, E, qkv.buf->p, NQKV, T, NQKV, E, nullptr, A_NONE, who);
      FCHK(piamd_qkv_prep(qkv.buf->p, NQKV, opt(3, l) ? W[3][l].buf->p : nullptr, kv(l, 0), kv(l, 1), pos0, B, S_,
                          Hq, Hk, D, maxS, 0, 1, 10000.f, S(c)),
           who + " (qkv bias + cache write)");
      DTensor att = make(c, VT_BF16, {T, HQD});
      FaArgs a;
      std::memset(&a, 0, sizeof(a));
      const char* base = (const char*)qkv.buf->p;
      a.q = base;
      a.k = base + (size_t)HQD * 2;
      a.v = base + (size_t)(Hq + Hk) * D * 2;
      a.o = att.buf->p;
      a.B = B, a.Sq = S_, a.Sk = S_, a.Hq = Hq, a.Hk = Hk, a.D = D;
      a.causal = (!mask && op.ab("causal", false)) ? 1 : 0;
      a.sqb = a.skb = a.svb = (long long)S_ * NQKV;
      a.sqs = a.sks = a.svs = NQKV;
      a.sqh = a.skh = a.svh = D;
      a.sob = (long long)S_ * HQD, a.sos = HQD, a.soh = D;
      if (mask) {
        const auto& md = mask->dims;  // [B|1, H|1, S|1, S]
        if (md.size() != 4 || md[3] != S_ || S_ % 4) reject("this SrcMask shape");
        a.mask = mask->buf->p;
        a.smb = md[0] > 1 ? md[1] * md[2] * md[3] : 0;
        a.smh = md[1] > 1 ? md[2] * md[3] : 0;
        a.smq = md[2] > 1 ? md[3] : 0;
      }
      a.scale = 1.f / std::sqrt((float)D);
      FCHK(piamd_fa_fwd(&a, 0, S(c)), who + " (flash attention)");
      DTensor o = make(c, VT_BF16, {T, E});
      const DTensor& wo = transposed(c, W[4][l], who);
      gemm_nt(c, 0, att.buf->p, HQD, wo.buf->p, HQD, o.buf->p, E, T, E, HQD, nullptr, A_NONE, who);
      DTensor yn = make(c, VT_BF16, {T, E}), nr = make(c, VT_BF16, {T, E});
      FCHK(piamd_layernorm_fwd(1, o.buf->p, opt(5, l) ? W[5][l].buf->p : nullptr, res.buf->p, W[6][l].buf->p,
                               opt(7, l) ? W[7][l].buf->p : nullptr, yn.buf->p, nr.buf->p, nullptr, nullptr, T, E, eps,
                               0.f, 0, 0, 0, S(c)),
           who + " (add + LayerNorm)");
      res = nr;
      DTensor h = make(c, VT_BF16, {T, F});
      const DTensor& w1 = transposed(c, W[8][l], who);
      gemm_nt(c, 0, yn.buf->p, E, w1.buf->p, E, h.buf->p, F, T, F, E, opt(9, l) ? W[9][l].buf->p : nullptr, act, who);
      pend = make(c, VT_BF16, {T, E});
      const DTensor& w2 = transposed(c, W[10][l], who);
      gemm_nt(c, 0, h.buf->p, F, w2.buf->p, F, pend.buf->p, E, T, E, F, nullptr, A_NONE, who);
      pend_b = opt(11, l);
    }
    // out = residual + ffn2 (+ bias)
    DTensor out = make(c, VT_BF16, {T, E});
    Bcast bc;
    bc.nd = 1;
    bc.dims[0] = (int64_t)T * E;
    bc.sa[0] = bc.sb[0] = 1;
    bc.n = (int64_t)T * E;
    gpu::binary16(c, B_ADD, 0, res.buf->p, pend.buf->p, out.buf->p, bc);
    if (pend_b) {
      Bcast bb;
      bb.nd = 2;
      bb.dims[0] = T, bb.dims[1] = E;
      bb.sa[0] = E, bb.sa[1] = 1;
      bb.sb[0] = 0, bb.sb[1] = 1;
      bb.n = (int64_t)T * E;
      gpu::binary16(c, B_ADD, 0, out.buf->p, pend_b->buf->p, out.buf->p, bb);
    }
    res = out;
  }
  res.dims = {B, S_, E};
  s[op.out("Out")] = res;
  if (op.has_out("CacheKVOut")) {
    const auto& outs = op.outputs.at("CacheKVOut");
    for (size_t i = 0; i < outs.size() && i < caches.size(); ++i) s[outs[i]] = *caches[i];
  }
}

using FastFn = void (*)(Ctx&, const OpDesc&, Scope&);

const std::map<std::string, FastFn>& fast_ops() {
  static const std::map<std::string, FastFn> m = {
      {"fc", op_fc},
      {"fused_fc_elementwise_layernorm", op_fc_eltwise_ln},
      {"skip_layernorm", op_skip_ln},
      {"layer_norm", op_layer_norm},
      {"multihead_matmul", op_mha},
      {"lookup_table_v2", op_lookup},
      {"lookup_table", op_lookup},
      {"fused_embedding_eltwise_layernorm", op_emb_eltwise_ln},
      {"softmax", op_softmax},
      {"matmul", op_matmul},
      {"matmul_v2", op_matmul},
      {"fused_multi_transformer", op_fmt},
  };
  return m;
}

// the dtype that decides the path: the first floating input of the op
int float_dtype(Ctx& c, const OpDesc& op, Scope& s) {
  for (const auto& kv : op.inputs)
    for (const auto& n : kv.second) {
      auto it = s.find(n);
      if (it == s.end()) continue;
      const int dt = it->second.dtype;
      if (dt == VT_FP32 || dt == VT_FP16 || dt == VT_BF16 || dt == VT_FP64) return dt;
    }
  return -1;
}

}  // namespace

bool fast_knows(const std::string& type) { return fast_ops().count(type) > 0; }

bool fast_run(Ctx& c, const OpDesc& op, Scope& s) {
  if (!c.gpu) return false;
  auto it = fast_ops().find(op.type);
  if (it == fast_ops().end()) return false;
  const int dt = float_dtype(c, op, s);
  // fused_multi_transformer has no generic implementation: it always runs here (bf16)
  if (!is16(dt) && op.type != "fused_multi_transformer") return false;
  it->second(c, op, s);
  return true;
}

void fast_release(Ctx& c) { c.fast.reset(); }

}  // namespace pdn
