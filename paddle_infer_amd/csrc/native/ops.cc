// Op implementations of the native engine: shape logic on the host, the arithmetic through
// kern:: (CPU loops or HIP kernels / rocBLAS, by the predictor's place). Semantics follow the
// reference op definitions (`paddle/phi/ops/compat/*`, `paddle/fluid/operators/*_op.cc`): the
// elementwise `axis` broadcast, matmul(_v2) batch broadcast and transposes, reshape2's 0 / -1,
// lookup_table's padding_idx, layer_norm's begin_norm_axis, slice's decrease_axis.
#include <algorithm>
#include <cmath>
#include <numeric>

#include "kernels.h"

namespace pdn {

namespace {

DTensor make(Ctx& c, int dtype, std::vector<int64_t> dims) {
  DTensor t;
  t.dtype = dtype;
  t.dims = std::move(dims);
  t.buf = alloc_buffer(t.nbytes(), c.gpu);
  return t;
}

const DTensor& get(Scope& s, const std::string& n) {
  auto it = s.find(n);
  if (it == s.end()) throw std::runtime_error("variable '" + n + "' is not set");
  return it->second;
}

DTensor ensure_place(const DTensor& t, Ctx& c) { return c.gpu ? to_device(t, c) : to_host(t, c); }

const DTensor& in(Ctx& c, Scope& s, const OpDesc& op, const std::string& slot, size_t i = 0) {
  const std::string& n = op.in(slot, i);
  DTensor& t = const_cast<DTensor&>(get(s, n));
  if (t.on_dev() != c.gpu) t = ensure_place(t, c);
  return t;
}

void need_f32(const DTensor& t, const OpDesc& op) {
  if (t.dtype != VT_FP32)
    throw std::runtime_error(op.type + ": the native engine computes float32 (got dtype " +
                             std::to_string(t.dtype) + ")");
}

int64_t norm_axis(int64_t a, size_t nd) { return a < 0 ? a + (int64_t)nd : a; }

std::vector<int64_t> host_ints(Ctx& c, const DTensor& t) {
  DTensor h = to_host(t, c);
  std::vector<int64_t> v((size_t)h.numel());
  for (int64_t i = 0; i < h.numel(); ++i)
    v[i] = h.dtype == VT_INT64 ? h.data<int64_t>()[i] : h.data<int32_t>()[i];
  return v;
}

// ------------------------------------------------------------------------------ elementwise
void elementwise(Ctx& c, const OpDesc& op, Scope& s, int bop) {
  const DTensor& x = in(c, s, op, "X");
  const DTensor& y = in(c, s, op, "Y");
  const bool h16 = c.gpu && is16(x.dtype) && x.dtype == y.dtype;
  if (!h16) {
    need_f32(x, op);
    need_f32(y, op);
  }
  // Paddle axis broadcast: Y's dims align with X's starting at `axis` (-1: trailing)
  std::vector<int64_t> xd = x.dims, yd = y.dims;
  if (yd.size() > xd.size()) {
    if (bop != B_ADD && bop != B_MUL && bop != B_MAX && bop != B_MIN)
      throw std::runtime_error(op.type + ": Y of higher rank than X");
  }
  const size_t nd = std::max(xd.size(), yd.size());
  int64_t axis = op.ai("axis", -1);
  std::vector<int64_t> xa(nd, 1), ya(nd, 1);
  if (xd.size() >= yd.size()) {
    std::copy(xd.begin(), xd.end(), xa.begin());
    const int64_t off = axis < 0 ? (int64_t)(nd - yd.size()) : axis;
    for (size_t i = 0; i < yd.size(); ++i) ya[off + i] = yd[i];
  } else {
    std::copy(yd.begin(), yd.end(), ya.begin());
    const int64_t off = axis < 0 ? (int64_t)(nd - xd.size()) : axis;
    for (size_t i = 0; i < xd.size(); ++i) xa[off + i] = xd[i];
  }
  std::vector<int64_t> od(nd);
  for (size_t i = 0; i < nd; ++i) {
    if (xa[i] != ya[i] && xa[i] != 1 && ya[i] != 1)
      throw std::runtime_error(op.type + ": shapes do not broadcast");
    od[i] = std::max(xa[i], ya[i]);
  }
  if (nd > (size_t)kMaxDims) throw std::runtime_error(op.type + ": too many dims");
  Bcast bc;
  bc.nd = (int)nd;
  int64_t sx = 1, sy = 1;
  for (int i = (int)nd - 1; i >= 0; --i) {
    bc.dims[i] = od[i];
    bc.sa[i] = xa[i] == 1 ? 0 : sx;
    bc.sb[i] = ya[i] == 1 ? 0 : sy;
    sx *= xa[i];
    sy *= ya[i];
  }
  DTensor o = make(c, h16 ? x.dtype : VT_FP32, od);
  bc.n = o.numel();
  if (h16) gpu::binary16(c, bop, x.dtype == VT_FP16, x.buf->p, y.buf->p, o.buf->p, bc);
  else kern::binary(c, bop, x.data<float>(), y.data<float>(), o.data<float>(), bc);
  s[op.out("Out")] = o;
}

void unary_op(Ctx& c, const OpDesc& op, Scope& s, int uop, float p0 = 0.f, float p1 = 0.f) {
  const DTensor& x = in(c, s, op, "X");
  if (c.gpu && is16(x.dtype)) {
    DTensor o = make(c, x.dtype, x.dims);
    gpu::unary16(c, uop, x.dtype == VT_FP16, x.buf->p, o.buf->p, x.numel(), p0, p1);
    s[op.out("Out")] = o;
    return;
  }
  need_f32(x, op);
  DTensor o = make(c, VT_FP32, x.dims);
  kern::unary(c, uop, x.data<float>(), o.data<float>(), x.numel(), p0, p1);
  s[op.out("Out")] = o;
}

// ------------------------------------------------------------------------------ matmul
// out = op(X)·op(Y) with batch broadcast; X [.., M, K], Y [.., K, N] (before transposes)
DTensor matmul(Ctx& c, const DTensor& x0, const DTensor& y0, bool tx, bool ty, float alpha,
               const std::string& name) {
  DTensor x = x0, y = y0;
  bool x1d = false, y1d = false;
  if (x.dims.size() == 1) { x.dims.insert(x.dims.begin(), 1); x1d = true; tx = false; }
  if (y.dims.size() == 1) { y.dims.push_back(1); y1d = true; ty = false; }
  const size_t xn = x.dims.size(), yn = y.dims.size();
  const int64_t M = tx ? x.dims[xn - 1] : x.dims[xn - 2];
  const int64_t Kx = tx ? x.dims[xn - 2] : x.dims[xn - 1];
  const int64_t Ky = ty ? y.dims[yn - 1] : y.dims[yn - 2];
  const int64_t N = ty ? y.dims[yn - 2] : y.dims[yn - 1];
  if (Kx != Ky) throw std::runtime_error(name + ": inner dims differ");
  std::vector<int64_t> xb(x.dims.begin(), x.dims.end() - 2), yb(y.dims.begin(), y.dims.end() - 2);
  const int64_t nxb = std::accumulate(xb.begin(), xb.end(), (int64_t)1, std::multiplies<int64_t>());
  const int64_t nyb = std::accumulate(yb.begin(), yb.end(), (int64_t)1, std::multiplies<int64_t>());
  std::vector<int64_t> od;
  int64_t batch, sA, sB;
  int64_t Mg = M;
  if (nyb == 1 && !tx) {  // weights-like Y: fold X's batch into the rows — one GEMM
    od = xb;
    Mg = M * nxb;
    batch = 1;
    sA = sB = 0;
  } else if (nxb == nyb || nxb == 1 || nyb == 1) {
    od = nxb >= nyb ? xb : yb;
    batch = std::max(nxb, nyb);
    sA = nxb == 1 ? 0 : M * Kx;
    sB = nyb == 1 ? 0 : Kx * N;
  } else {
    throw std::runtime_error(name + ": unsupported batch broadcast");
  }
  od.push_back(M);
  od.push_back(N);
  DTensor o = make(c, VT_FP32, od);
  const int64_t lda = tx ? M : Kx, ldb = ty ? Kx : N;
  kern::gemm(c, tx, ty, Mg, N, Kx, alpha, x.data<float>(), lda, sA, y.data<float>(), ldb, sB, 0.f,
             o.data<float>(), N, Mg * N, batch);
  if (x1d) o.dims.erase(o.dims.end() - 2);
  if (y1d) o.dims.pop_back();
  return o;
}

DTensor flatten2(const DTensor& t, int64_t ncol) {
  DTensor r = t;
  int64_t a = 1, b = 1;
  for (size_t i = 0; i < t.dims.size(); ++i) (i < (size_t)ncol ? a : b) *= t.dims[i];
  r.dims = {a, b};
  return r;
}

void act_inplace(Ctx& c, DTensor& t, const std::string& act) {
  if (act.empty() || act == "identity") return;
  int u = act == "relu" ? U_RELU : act == "gelu" ? U_GELU : act == "tanh" ? U_TANH
        : act == "sigmoid" ? U_SIGMOID : (act == "silu" || act == "swish") ? U_SILU : -1;
  if (u < 0) throw std::runtime_error("fc: unsupported activation_type " + act);
  kern::unary(c, u, t.data<float>(), t.data<float>(), t.numel(), 0.f, 0.f);
}

void add_bias_rows(Ctx& c, DTensor& o, const DTensor& bias) {
  Bcast bc;
  bc.nd = 2;
  bc.dims[0] = o.numel() / o.dims.back();
  bc.dims[1] = o.dims.back();
  bc.sa[0] = bc.dims[1];
  bc.sa[1] = 1;
  bc.sb[0] = 0;
  bc.sb[1] = 1;
  bc.n = o.numel();
  kern::binary(c, B_ADD, o.data<float>(), bias.data<float>(), o.data<float>(), bc);
}

// ------------------------------------------------------------------------------ layout
Strided contiguous_view(const std::vector<int64_t>& dims) {
  Strided s;
  s.nd = (int)dims.size();
  int64_t st = 1;
  for (int i = s.nd - 1; i >= 0; --i) {
    s.dims[i] = dims[i];
    s.stride[i] = st;
    st *= dims[i];
  }
  s.n = st;
  return s;
}

std::vector<int64_t> strides_of(const std::vector<int64_t>& d) {
  std::vector<int64_t> s(d.size());
  int64_t st = 1;
  for (int i = (int)d.size() - 1; i >= 0; --i) {
    s[i] = st;
    st *= d[i];
  }
  return s;
}

DTensor transpose(Ctx& c, const DTensor& x, const std::vector<int64_t>& perm) {
  if (perm.size() != x.dims.size() || perm.size() > (size_t)kMaxDims)
    throw std::runtime_error("transpose: bad axis");
  const auto xs = strides_of(x.dims);
  Strided s;
  s.nd = (int)perm.size();
  std::vector<int64_t> od(perm.size());
  for (size_t i = 0; i < perm.size(); ++i) {
    od[i] = x.dims[perm[i]];
    s.dims[i] = od[i];
    s.stride[i] = xs[perm[i]];
  }
  DTensor o = make(c, x.dtype, od);
  s.n = o.numel();
  kern::strided_copy(c, x.buf->p, o.buf->p, (int)vt_size(x.dtype), s);
  return o;
}

DTensor reshaped(const DTensor& x, std::vector<int64_t> shape) {
  int64_t known = 1, neg = -1;
  for (size_t i = 0; i < shape.size(); ++i) {
    if (shape[i] == 0) shape[i] = x.dims.at(i);
    if (shape[i] == -1) neg = (int64_t)i;
    else known *= shape[i];
  }
  if (neg >= 0) shape[neg] = known ? x.numel() / known : 0;
  DTensor r = x;
  r.dims = shape;
  if (r.numel() != x.numel()) throw std::runtime_error("reshape: element count changes");
  return r;
}


// ------------------------------------------------------------------------------ conv / pool
// Paddle padding resolution (`conv_op.h UpdatePaddingAndDilation`): paddings [p] x2 or [lo, hi]
// per spatial dim; SAME → out = ceil(in / st), VALID → no padding.
void resolve_pad(int64_t in, int64_t k_eff, int64_t st, const std::string& algo, int64_t lo_in,
                 int64_t hi_in, bool ceil_mode, int64_t& lo, int64_t& out) {
  if (algo == "SAME") {
    out = (in + st - 1) / st;
    const int64_t total = std::max<int64_t>((out - 1) * st + k_eff - in, 0);
    lo = total / 2;
  } else if (algo == "VALID") {
    lo = 0;
    out = (in - k_eff) / st + 1;
  } else {
    lo = lo_in;
    const int64_t span = in + lo_in + hi_in - k_eff;
    out = (ceil_mode ? span + st - 1 : span) / st + 1;
  }
  if (out < 1) throw std::runtime_error("conv/pool: empty output");
}

void pads4(const std::vector<int64_t>& p, int64_t (&q)[4]) {  // → top, bottom, left, right
  if (p.size() == 4) { q[0] = p[0]; q[1] = p[1]; q[2] = p[2]; q[3] = p[3]; }
  else if (p.size() == 2) { q[0] = q[1] = p[0]; q[2] = q[3] = p[1]; }
  else q[0] = q[1] = q[2] = q[3] = 0;
}

bool nhwc_layout(const OpDesc& o, const char* key) { return o.as(key, "NCHW") == "NHWC"; }

void conv2d_op(Ctx& c, const OpDesc& o, Scope& s) {
  DTensor x = in(c, s, o, "Input");
  const DTensor& w = in(c, s, o, "Filter");
  need_f32(x, o);
  need_f32(w, o);
  const bool nhwc = nhwc_layout(o, "data_format");
  if (nhwc) x = transpose(c, x, {0, 3, 1, 2});
  if (x.dims.size() != 4 || w.dims.size() != 4) throw std::runtime_error(o.type + ": 4-D input/filter");
  const int64_t N = x.dims[0], Cin = x.dims[1], H = x.dims[2], W = x.dims[3];
  const int64_t K = w.dims[0], cg = w.dims[1], R = w.dims[2], S = w.dims[3];
  const int64_t G = std::max<int64_t>(o.ai("groups", 1), 1);
  if (cg * G != Cin || K % G) throw std::runtime_error(o.type + ": groups do not match the channels");
  std::vector<int64_t> st = o.aints("strides"), dl = o.aints("dilations");
  if (st.size() < 2) st = {1, 1};
  if (dl.size() < 2) dl = {1, 1};
  int64_t p4[4];
  pads4(o.aints("paddings"), p4);
  const std::string algo = o.as("padding_algorithm", "EXPLICIT");
  ConvG g{cg, H, W, R, S, 0, 0, st[0], st[1], 0, 0, dl[0], dl[1]};
  resolve_pad(H, dl[0] * (R - 1) + 1, st[0], algo, p4[0], p4[1], false, g.ph, g.OH);
  resolve_pad(W, dl[1] * (S - 1) + 1, st[1], algo, p4[2], p4[3], false, g.pw, g.OW);
  DTensor y = make(c, VT_FP32, {N, K, g.OH, g.OW});
  const int64_t P = g.OH * g.OW, kg = K / G;
  if (cg == 1 && G == Cin) {  // depthwise (channel multiplier K / Cin): direct kernel
    g.C = Cin;
    kern::dwconv(c, x.data<float>(), w.data<float>(), nullptr, y.data<float>(), N, K / Cin, g);
  } else {
    const bool direct = R == 1 && S == 1 && st[0] == 1 && st[1] == 1 && g.ph == 0 && g.pw == 0 &&
                        g.OH == H && g.OW == W;  // 1×1: the image itself is the column matrix
    DTensor col;
    if (!direct) col = make(c, VT_FP32, {N, cg * R * S, P});
    for (int64_t gi = 0; gi < G; ++gi) {
      const float* xg = x.data<float>() + gi * cg * H * W;
      const float* B = xg;
      int64_t sB = Cin * H * W;
      if (!direct) {
        kern::im2col(c, xg, Cin * H * W, col.data<float>(), N, g);
        B = col.data<float>();
        sB = cg * R * S * P;
      }
      kern::gemm(c, false, false, kg, P, cg * R * S, 1.f, w.data<float>() + gi * kg * cg * R * S,
                 cg * R * S, 0, B, P, sB, 0.f, y.data<float>() + gi * kg * P, P, K * P, N);
    }
  }
  if (o.has_in("Bias")) {  // conv2d_fusion-style bias [K]
    const DTensor& b = in(c, s, o, "Bias");
    DTensor one = make(c, VT_FP32, {K});
    kern::fill(c, one.buf->p, VT_FP32, K, 1.0);
    kern::channel_affine(c, y.data<float>(), one.data<float>(), b.data<float>(), y.data<float>(), N, K, P, U_IDENT, 0.f);
  }
  s[o.out("Output")] = nhwc ? transpose(c, y, {0, 2, 3, 1}) : y;
}

void pool2d_op(Ctx& c, const OpDesc& o, Scope& s) {
  DTensor x = in(c, s, o, "X");
  need_f32(x, o);
  const bool nhwc = nhwc_layout(o, "data_format");
  if (nhwc) x = transpose(c, x, {0, 3, 1, 2});
  if (x.dims.size() != 4) throw std::runtime_error("pool2d: 4-D input");
  const int64_t N = x.dims[0], C = x.dims[1], H = x.dims[2], W = x.dims[3];
  std::vector<int64_t> k = o.aints("ksize"), st = o.aints("strides");
  if (k.size() < 2) throw std::runtime_error("pool2d: ksize");
  if (st.size() < 2) st = {1, 1};
  PoolG p{H, W, 0, 0, k[0], k[1], st[0], st[1], 0, 0, o.as("pooling_type", "max") == "max",
          o.ab("exclusive", true), o.ab("adaptive", false)};
  if (o.ab("global_pooling", false)) {
    p.kh = H; p.kw = W; p.OH = p.OW = 1; p.adaptive = 0; p.sh = p.sw = 1;
  } else if (p.adaptive) {
    p.OH = k[0]; p.OW = k[1];
  } else {
    int64_t p4[4];
    pads4(o.aints("paddings"), p4);
    const std::string algo = o.as("padding_algorithm", "EXPLICIT");
    const bool ceil = o.ab("ceil_mode", false);
    resolve_pad(H, p.kh, p.sh, algo, p4[0], p4[1], ceil, p.ph, p.OH);
    resolve_pad(W, p.kw, p.sw, algo, p4[2], p4[3], ceil, p.pw, p.OW);
  }
  DTensor y = make(c, VT_FP32, {N, C, p.OH, p.OW});
  kern::pool2d(c, x.data<float>(), y.data<float>(), N * C, p);
  s[o.out("Out")] = nhwc ? transpose(c, y, {0, 2, 3, 1}) : y;
}

// inference batch norm: y = x · γ/√(σ²+ε) + (β − μ·γ/√(σ²+ε)) per channel. The fold runs once on
// the host (the first Run: eager, before any hipGraph capture) and is kept on the device while its
// inputs are loaded parameters, so a captured Run never reads device data back.
void batch_norm_op(Ctx& c, const OpDesc& o, Scope& s) {
  const DTensor& x = in(c, s, o, "X");
  need_f32(x, o);
  const DTensor &g0 = in(c, s, o, "Scale"), &b0 = in(c, s, o, "Bias");
  const DTensor &m0 = in(c, s, o, "Mean"), &v0 = in(c, s, o, "Variance");
  auto is_param = [&](const DTensor& t) { return c.persist && t.buf && c.persist->count(t.buf.get()); };
  const bool cacheable = c.consts && is_param(g0) && is_param(b0) && is_param(m0) && is_param(v0);
  const std::string key = "bn_fold:" + o.out("Y");
  DTensor sc, sh;
  if (cacheable && c.consts->count(key + ":sc")) {
    sc = c.consts->at(key + ":sc");
    sh = c.consts->at(key + ":sh");
  } else {
    const DTensor g = to_host(g0, c), b = to_host(b0, c), m = to_host(m0, c), v = to_host(v0, c);
    const int64_t C = g.numel();
    const float eps = o.af("epsilon", 1e-5f);
    sc.dtype = sh.dtype = VT_FP32;
    sc.dims = sh.dims = {C};
    sc.buf = alloc_buffer(C * 4, false);
    sh.buf = alloc_buffer(C * 4, false);
    for (int64_t i = 0; i < C; ++i) {
      const float a = g.data<float>()[i] / std::sqrt(v.data<float>()[i] + eps);
      sc.data<float>()[i] = a;
      sh.data<float>()[i] = b.data<float>()[i] - m.data<float>()[i] * a;
    }
    if (c.gpu) {
      sc = to_device(sc, c);
      sh = to_device(sh, c);
      dev_sync(c);  // the host staging buffers die at the end of this scope
    }
    if (cacheable) {
      (*c.consts)[key + ":sc"] = sc;
      (*c.consts)[key + ":sh"] = sh;
    }
  }
  const int64_t C = sc.numel();
  const bool nhwc = nhwc_layout(o, "data_layout");
  const int64_t N = x.dims.at(0);
  const int64_t inner = nhwc ? 1 : x.numel() / (N * C);
  const int64_t outer = nhwc ? x.numel() / C : N;
  DTensor y = make(c, VT_FP32, x.dims);
  kern::channel_affine(c, x.data<float>(), sc.data<float>(), sh.data<float>(), y.data<float>(), outer, C, inner, U_IDENT, 0.f);
  s[o.out("Y")] = y;
}

}  // namespace

const std::unordered_map<std::string, OpFn>& op_registry() {
  static const std::unordered_map<std::string, OpFn> R = [] {
    std::unordered_map<std::string, OpFn> r;
    r["elementwise_add"] = [](Ctx& c, const OpDesc& o, Scope& s) { elementwise(c, o, s, B_ADD); };
    r["elementwise_sub"] = [](Ctx& c, const OpDesc& o, Scope& s) { elementwise(c, o, s, B_SUB); };
    r["elementwise_mul"] = [](Ctx& c, const OpDesc& o, Scope& s) { elementwise(c, o, s, B_MUL); };
    r["elementwise_div"] = [](Ctx& c, const OpDesc& o, Scope& s) { elementwise(c, o, s, B_DIV); };
    r["elementwise_max"] = [](Ctx& c, const OpDesc& o, Scope& s) { elementwise(c, o, s, B_MAX); };
    r["elementwise_min"] = [](Ctx& c, const OpDesc& o, Scope& s) { elementwise(c, o, s, B_MIN); };
    r["elementwise_pow"] = [](Ctx& c, const OpDesc& o, Scope& s) { elementwise(c, o, s, B_POW); };
    r["relu"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_RELU); };
    r["gelu"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      unary_op(c, o, s, o.ab("approximate", false) ? U_GELU_TANH : U_GELU);
    };
    r["tanh"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_TANH); };
    r["sigmoid"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_SIGMOID); };
    r["silu"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_SILU); };
    r["swish"] = r["silu"];
    r["exp"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_EXP); };
    r["sqrt"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_SQRT); };
    r["rsqrt"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_RSQRT); };
    r["abs"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_ABS); };
    r["scale"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const float sc = o.af("scale", 1.f), b = o.af("bias", 0.f);
      unary_op(c, o, s, o.ab("bias_after_scale", true) ? U_SCALE : U_SCALE_PRE, sc, b);
    };
    r["dropout"] = [](Ctx& c, const OpDesc& o, Scope& s) {  // inference
      const bool up = o.as("dropout_implementation", "downgrade_in_infer") == "upscale_in_train";
      unary_op(c, o, s, U_SCALE, up ? 1.f : 1.f - o.af("dropout_prob", 0.5f), 0.f);
    };
    r["assign"] = [](Ctx& c, const OpDesc& o, Scope& s) { s[o.out("Out")] = in(c, s, o, "X"); };
    r["softmax"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      need_f32(x, o);
      const int64_t ax = norm_axis(o.ai("axis", -1), x.dims.size());
      int64_t outer = 1, inner = 1;
      for (int64_t i = 0; i < ax; ++i) outer *= x.dims[i];
      for (size_t i = ax + 1; i < x.dims.size(); ++i) inner *= x.dims[i];
      DTensor out = make(c, VT_FP32, x.dims);
      kern::softmax(c, x.data<float>(), out.data<float>(), outer, x.dims[ax], inner);
      s[o.out("Out")] = out;
    };
    r["layer_norm"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      need_f32(x, o);
      const int64_t b = o.ai("begin_norm_axis", 1);
      int64_t rows = 1, cols = 1;
      for (size_t i = 0; i < x.dims.size(); ++i) ((int64_t)i < b ? rows : cols) *= x.dims[i];
      const float* g = o.has_in("Scale") ? in(c, s, o, "Scale").data<float>() : nullptr;
      const float* bb = o.has_in("Bias") ? in(c, s, o, "Bias").data<float>() : nullptr;
      DTensor out = make(c, VT_FP32, x.dims);
      kern::layernorm(c, x.data<float>(), g, bb, out.data<float>(), rows, cols, o.af("epsilon", 1e-5f));
      s[o.out("Y")] = out;
    };
    auto lookup = [](Ctx& c, const OpDesc& o, Scope& s, bool v1) {
      const DTensor& ids = in(c, s, o, "Ids");
      const DTensor& w = in(c, s, o, "W");
      need_f32(w, o);
      std::vector<int64_t> od = ids.dims;
      if (v1 && !od.empty() && od.back() == 1) od.pop_back();
      const int64_t width = w.dims.at(1);
      od.push_back(width);
      DTensor out = make(c, VT_FP32, od);
      if (ids.dtype != VT_INT64 && ids.dtype != VT_INT32) throw std::runtime_error(o.type + ": ids dtype");
      kern::gather_rows(c, w.data<float>(), ids.buf->p, ids.dtype == VT_INT64, out.data<float>(),
                        ids.numel(), width, w.dims[0], o.ai("padding_idx", -1));
      s[o.out("Out")] = out;
    };
    r["lookup_table_v2"] = [lookup](Ctx& c, const OpDesc& o, Scope& s) { lookup(c, o, s, false); };
    r["lookup_table"] = [lookup](Ctx& c, const OpDesc& o, Scope& s) { lookup(c, o, s, true); };
    r["matmul_v2"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      const DTensor& y = in(c, s, o, "Y");
      need_f32(x, o);
      need_f32(y, o);
      s[o.out("Out")] = matmul(c, x, y, o.ab("trans_x", false), o.ab("trans_y", false), 1.f, o.type);
    };
    r["matmul"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      const DTensor& y = in(c, s, o, "Y");
      need_f32(x, o);
      need_f32(y, o);
      s[o.out("Out")] = matmul(c, x, y, o.ab("transpose_X", false), o.ab("transpose_Y", false),
                               o.af("alpha", 1.f), o.type);
    };
    r["mul"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      const DTensor& y = in(c, s, o, "Y");
      const int64_t xc = o.ai("x_num_col_dims", 1), yc = o.ai("y_num_col_dims", 1);
      DTensor out = matmul(c, flatten2(x, xc), flatten2(y, yc), false, false, 1.f, o.type);
      std::vector<int64_t> od(x.dims.begin(), x.dims.begin() + xc);
      od.insert(od.end(), y.dims.begin() + yc, y.dims.end());
      out.dims = od;
      s[o.out("Out")] = out;
    };
    r["fc"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "Input");
      const DTensor& w = in(c, s, o, "W");
      const int64_t nc = o.ai("in_num_col_dims", 1);
      DTensor out = matmul(c, flatten2(x, nc), w, false, false, 1.f, o.type);
      if (o.has_in("Bias")) add_bias_rows(c, out, in(c, s, o, "Bias"));
      act_inplace(c, out, o.as("activation_type", ""));
      std::vector<int64_t> od(x.dims.begin(), x.dims.begin() + nc);
      od.push_back(w.dims[1]);
      out.dims = od;
      s[o.out("Out")] = out;
    };
    auto tr = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      s[o.out("Out")] = transpose(c, x, o.aints("axis"));
    };
    r["transpose2"] = tr;
    r["transpose"] = tr;
    auto rs = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      std::vector<int64_t> shape = o.aints("shape");
      if (o.has_in("Shape")) shape = host_ints(c, in(c, s, o, "Shape"));
      s[o.out("Out")] = reshaped(x, shape);
    };
    r["reshape2"] = rs;
    r["reshape"] = rs;
    auto unsq = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      std::vector<int64_t> d = x.dims;
      for (int64_t a : o.aints("axes")) {
        const int64_t ax = a < 0 ? a + (int64_t)d.size() + 1 : a;
        d.insert(d.begin() + ax, 1);
      }
      DTensor r2 = x;
      r2.dims = d;
      s[o.out("Out")] = r2;
    };
    r["unsqueeze2"] = unsq;
    r["unsqueeze"] = unsq;
    auto sq = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      std::vector<int64_t> axes = o.aints("axes"), d;
      for (auto& a : axes) a = norm_axis(a, x.dims.size());
      for (size_t i = 0; i < x.dims.size(); ++i) {
        const bool drop = x.dims[i] == 1 && (axes.empty() || std::count(axes.begin(), axes.end(), (int64_t)i));
        if (!drop) d.push_back(x.dims[i]);
      }
      DTensor r2 = x;
      r2.dims = d;
      s[o.out("Out")] = r2;
    };
    r["squeeze2"] = sq;
    r["squeeze"] = sq;
    r["flatten_contiguous_range"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      const int64_t a = norm_axis(o.ai("start_axis", 1), x.dims.size());
      const int64_t b = norm_axis(o.ai("stop_axis", -1), x.dims.size());
      std::vector<int64_t> d(x.dims.begin(), x.dims.begin() + a);
      int64_t m = 1;
      for (int64_t i = a; i <= b; ++i) m *= x.dims[i];
      d.push_back(m);
      d.insert(d.end(), x.dims.begin() + b + 1, x.dims.end());
      DTensor r2 = x;
      r2.dims = d;
      s[o.out("Out")] = r2;
    };
    r["concat"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const auto& names = o.inputs.at("X");
      std::vector<DTensor> xs;
      for (size_t i = 0; i < names.size(); ++i) xs.push_back(in(c, s, o, "X", i));
      const int64_t ax = norm_axis(o.ai("axis", 0), xs[0].dims.size());
      std::vector<int64_t> od = xs[0].dims;
      od[ax] = 0;
      for (auto& t : xs) od[ax] += t.dims[ax];
      DTensor out = make(c, xs[0].dtype, od);
      int64_t outer = 1, inner = 1;
      for (int64_t i = 0; i < ax; ++i) outer *= od[i];
      for (size_t i = ax + 1; i < od.size(); ++i) inner *= od[i];
      const int elem = (int)vt_size(out.dtype);
      int64_t col = 0;
      for (auto& t : xs) {  // each input is a column band of the output's [outer, od[ax]·inner] view
        const int64_t w = t.dims[ax] * inner;
        kern::copy2d(c, t.buf->p, w, (char*)out.buf->p + col * elem, od[ax] * inner, outer, w, elem);
        col += w;
      }
      s[o.out("Out")] = out;
    };
    r["split"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      const int64_t ax = norm_axis(o.ai("axis", 0), x.dims.size());
      const auto& outs = o.outputs.at("Out");
      std::vector<int64_t> secs = o.aints("sections");
      if (secs.empty()) secs.assign(outs.size(), x.dims[ax] / (int64_t)outs.size());
      int64_t known = 0, neg = -1;
      for (size_t i = 0; i < secs.size(); ++i) (secs[i] < 0 ? neg = (int64_t)i : known += secs[i]);
      if (neg >= 0) secs[neg] = x.dims[ax] - known;
      const auto xs = strides_of(x.dims);
      int64_t start = 0;
      for (size_t k = 0; k < outs.size(); ++k) {
        std::vector<int64_t> od = x.dims;
        od[ax] = secs[k];
        DTensor out = make(c, x.dtype, od);
        Strided st;
        st.nd = (int)od.size();
        for (int i = 0; i < st.nd; ++i) {
          st.dims[i] = od[i];
          st.stride[i] = xs[i];
        }
        st.offset = start * xs[ax];
        st.n = out.numel();
        kern::strided_copy(c, x.buf->p, out.buf->p, (int)vt_size(x.dtype), st);
        s[outs[k]] = out;
        start += secs[k];
      }
    };
    r["slice"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "Input");
      const auto axes = o.aints("axes"), starts = o.aints("starts"), ends = o.aints("ends");
      std::vector<int64_t> od = x.dims, lo(x.dims.size(), 0);
      for (size_t i = 0; i < axes.size(); ++i) {
        const int64_t a = norm_axis(axes[i], x.dims.size()), n = x.dims[a];
        int64_t b = starts[i] < 0 ? starts[i] + n : starts[i];
        int64_t e = ends[i] < 0 ? ends[i] + n : std::min(ends[i], n);
        b = std::max<int64_t>(0, std::min(b, n));
        e = std::max(b, std::min(e, n));
        lo[a] = b;
        od[a] = e - b;
      }
      const auto xs = strides_of(x.dims);
      DTensor out = make(c, x.dtype, od);
      Strided st;
      st.nd = (int)od.size();
      for (int i = 0; i < st.nd; ++i) {
        st.dims[i] = od[i];
        st.stride[i] = xs[i];
        st.offset += lo[i] * xs[i];
      }
      st.n = out.numel();
      kern::strided_copy(c, x.buf->p, out.buf->p, (int)vt_size(x.dtype), st);
      std::vector<int64_t> dec = o.aints("decrease_axis"), fd;
      for (auto& a : dec) a = norm_axis(a, od.size());
      for (size_t i = 0; i < od.size(); ++i)
        if (!std::count(dec.begin(), dec.end(), (int64_t)i)) fd.push_back(od[i]);
      out.dims = fd.empty() && !od.empty() ? std::vector<int64_t>{1} : fd;
      s[o.out("Out")] = out;
    };
    r["cast"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      const int odt = (int)o.ai("out_dtype", VT_FP32);
      DTensor out = make(c, odt, x.dims);
      kern::cast(c, x.buf->p, x.dtype, out.buf->p, odt, x.numel());
      s[o.out("Out")] = out;
    };
    r["fill_any_like"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      int dt = (int)o.ai("dtype", -1);
      if (dt < 0) dt = x.dtype;  // -1: the input's dtype
      DTensor out = make(c, dt, x.dims);
      kern::fill(c, out.buf->p, dt, out.numel(), (double)o.af("value", 0.f));
      s[o.out("Out")] = out;
    };
    r["fill_zeros_like"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const DTensor& x = in(c, s, o, "X");
      DTensor out = make(c, x.dtype, x.dims);
      kern::fill(c, out.buf->p, x.dtype, out.numel(), 0.0);
      s[o.out("Out")] = out;
    };
    r["fill_constant"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      std::vector<int64_t> shape = o.aints("shape");
      const int dt = (int)o.ai("dtype", VT_FP32);
      const std::string sv = o.as("str_value", "");
      const double v = sv.empty() ? (double)o.af("value", 0.f) : std::stod(sv);
      DTensor out = make(c, dt, shape);
      kern::fill(c, out.buf->p, dt, out.numel(), v);
      s[o.out("Out")] = out;
    };
    auto red = [](Ctx& c, const OpDesc& o, Scope& s, bool mean) {
      const DTensor& x = in(c, s, o, "X");
      need_f32(x, o);
      std::vector<int64_t> dims = o.aints("dim");
      const bool all = o.ab("reduce_all", false) || dims.empty();
      const bool keep = o.ab("keep_dim", false);
      DTensor cur = x;
      std::vector<int64_t> axes;
      if (all) for (size_t i = 0; i < x.dims.size(); ++i) axes.push_back((int64_t)i);
      else for (auto d : dims) axes.push_back(norm_axis(d, x.dims.size()));
      std::sort(axes.rbegin(), axes.rend());
      for (int64_t a : axes) {  // one axis at a time, innermost first
        int64_t outer = 1, inner = 1;
        for (int64_t i = 0; i < a; ++i) outer *= cur.dims[i];
        for (size_t i = a + 1; i < cur.dims.size(); ++i) inner *= cur.dims[i];
        std::vector<int64_t> nd = cur.dims;
        nd[a] = 1;
        DTensor out = make(c, VT_FP32, nd);
        kern::reduce(c, cur.data<float>(), out.data<float>(), outer, cur.dims[a], inner, mean);
        cur = out;
      }
      if (!keep) {
        std::vector<int64_t> nd;
        for (size_t i = 0; i < cur.dims.size(); ++i)
          if (!std::count(axes.begin(), axes.end(), (int64_t)i)) nd.push_back(cur.dims[i]);
        cur.dims = nd.empty() ? std::vector<int64_t>{1} : nd;
      }
      s[o.out("Out")] = cur;
    };
    r["conv2d"] = conv2d_op;
    r["depthwise_conv2d"] = conv2d_op;
    r["pool2d"] = pool2d_op;
    r["batch_norm"] = batch_norm_op;
    r["relu6"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_RELU6, o.af("threshold", 6.f)); };
    r["hard_swish"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      const float th = o.af("threshold", 6.f), sc = o.af("scale", 6.f), off = o.af("offset", 3.f);
      if (sc != th) throw std::runtime_error("hard_swish: scale != threshold is not supported");
      unary_op(c, o, s, U_HSWISH, th, off);
    };
    r["hard_sigmoid"] = [](Ctx& c, const OpDesc& o, Scope& s) {
      unary_op(c, o, s, U_HSIGMOID, o.af("slope", 0.2f), o.af("offset", 0.5f));
    };
    r["leaky_relu"] = [](Ctx& c, const OpDesc& o, Scope& s) { unary_op(c, o, s, U_LEAKY, o.af("alpha", 0.02f)); };
    r["reduce_mean"] = [red](Ctx& c, const OpDesc& o, Scope& s) { red(c, o, s, true); };
    r["reduce_sum"] = [red](Ctx& c, const OpDesc& o, Scope& s) { red(c, o, s, false); };
    return r;
  }();
  return R;
}

}  // namespace pdn
