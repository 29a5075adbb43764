// CPU reference kernels of the native engine (plain C++; the GEMM is blocked over K for cache
// reuse and parallelised over rows with std::thread when Config::SetCpuMathLibraryNumThreads > 1).
#include <algorithm>
#include <cmath>
#include <thread>

#include "kernels.h"

namespace pdn {
namespace cpu {

namespace {

inline float unary_f(int op, float x, float p0, float p1) {
  switch (op) {
    case U_IDENT: return x;
    case U_RELU: return x > 0.f ? x : 0.f;
    case U_GELU: return 0.5f * x * (1.f + std::erf(x * 0.70710678118654752f));
    case U_GELU_TANH: return 0.5f * x * (1.f + std::tanh(0.7978845608028654f * (x + 0.044715f * x * x * x)));
    case U_TANH: return std::tanh(x);
    case U_SIGMOID: return 1.f / (1.f + std::exp(-x));
    case U_SILU: return x / (1.f + std::exp(-x));
    case U_EXP: return std::exp(x);
    case U_SQRT: return std::sqrt(x);
    case U_RSQRT: return 1.f / std::sqrt(x);
    case U_ABS: return std::fabs(x);
    case U_SCALE: return x * p0 + p1;
    case U_SCALE_PRE: return (x + p1) * p0;
    case U_RELU6: return std::min(std::max(x, 0.f), p0);
    case U_HSWISH: return x * std::min(std::max(x + p1, 0.f), p0) / p0;
    case U_HSIGMOID: return std::min(std::max(x * p0 + p1, 0.f), 1.f);
    case U_LEAKY: return x > 0.f ? x : p0 * x;
  }
  return x;
}

inline float binary_f(int op, float a, float b) {
  switch (op) {
    case B_ADD: return a + b;
    case B_SUB: return a - b;
    case B_MUL: return a * b;
    case B_DIV: return a / b;
    case B_MAX: return a > b ? a : b;
    case B_MIN: return a < b ? a : b;
    case B_POW: return std::pow(a, b);
  }
  return a;
}

template <typename F>
void parallel_rows(int threads, int64_t rows, F&& f) {
  if (threads <= 1 || rows < 2) {
    f(0, rows);
    return;
  }
  const int nt = (int)std::min<int64_t>(threads, rows);
  std::vector<std::thread> ts;
  for (int t = 0; t < nt; ++t) {
    const int64_t a = rows * t / nt, b = rows * (t + 1) / nt;
    ts.emplace_back([&, a, b] { f(a, b); });
  }
  for (auto& t : ts) t.join();
}

}  // namespace

void unary(Ctx&, int op, const float* x, float* y, int64_t n, float p0, float p1) {
  for (int64_t i = 0; i < n; ++i) y[i] = unary_f(op, x[i], p0, p1);
}

void binary(Ctx&, int op, const float* a, const float* b, float* y, const Bcast& bc) {
  int64_t idx[kMaxDims] = {0};
  int64_t oa = 0, ob = 0;
  for (int64_t i = 0; i < bc.n; ++i) {
    y[i] = binary_f(op, a[oa], b[ob]);
    for (int d = bc.nd - 1; d >= 0; --d) {  // odometer increment
      ++idx[d];
      oa += bc.sa[d];
      ob += bc.sb[d];
      if (idx[d] < bc.dims[d]) break;
      oa -= bc.sa[d] * idx[d];
      ob -= bc.sb[d] * idx[d];
      idx[d] = 0;
    }
  }
}

void softmax(Ctx&, const float* x, float* y, int64_t outer, int64_t n, int64_t inner) {
  for (int64_t o = 0; o < outer; ++o)
    for (int64_t j = 0; j < inner; ++j) {
      const float* xr = x + o * n * inner + j;
      float* yr = y + o * n * inner + j;
      float m = -INFINITY;
      for (int64_t i = 0; i < n; ++i) m = std::max(m, xr[i * inner]);
      double s = 0.0;
      for (int64_t i = 0; i < n; ++i) {
        const float e = std::exp(xr[i * inner] - m);
        yr[i * inner] = e;
        s += e;
      }
      const float inv = (float)(1.0 / s);
      for (int64_t i = 0; i < n; ++i) yr[i * inner] *= inv;
    }
}

void layernorm(Ctx&, const float* x, const float* g, const float* b, float* y, int64_t rows,
               int64_t cols, float eps) {
  for (int64_t r = 0; r < rows; ++r) {
    const float* xr = x + r * cols;
    float* yr = y + r * cols;
    double s = 0.0, s2 = 0.0;
    for (int64_t c = 0; c < cols; ++c) s += xr[c];
    const double mu = s / cols;
    for (int64_t c = 0; c < cols; ++c) s2 += (xr[c] - mu) * (xr[c] - mu);
    const float rs = (float)(1.0 / std::sqrt(s2 / cols + eps));
    for (int64_t c = 0; c < cols; ++c)
      yr[c] = (float)(xr[c] - mu) * rs * (g ? g[c] : 1.f) + (b ? b[c] : 0.f);
  }
}

void strided_copy(Ctx&, const void* src, void* dst, int elem, const Strided& s) {
  int64_t idx[kMaxDims] = {0};
  int64_t off = s.offset;
  const char* sp = (const char*)src;
  char* dp = (char*)dst;
  for (int64_t i = 0; i < s.n; ++i) {
    std::memcpy(dp + i * elem, sp + off * elem, elem);
    for (int d = s.nd - 1; d >= 0; --d) {
      ++idx[d];
      off += s.stride[d];
      if (idx[d] < s.dims[d]) break;
      off -= s.stride[d] * idx[d];
      idx[d] = 0;
    }
  }
}

void gather_rows(Ctx&, const float* table, const void* ids, int ids_i64, float* y, int64_t n,
                 int64_t width, int64_t rows, int64_t padding_idx) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t id = ids_i64 ? ((const int64_t*)ids)[i] : ((const int32_t*)ids)[i];
    float* yr = y + i * width;
    if (id == padding_idx || id < 0 || id >= rows) {
      std::fill(yr, yr + width, 0.f);
    } else {
      std::memcpy(yr, table + id * width, width * sizeof(float));
    }
  }
}

void gemm(Ctx& c, bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
          int64_t lda, int64_t sA, const float* B, int64_t ldb, int64_t sB, float beta, float* C,
          int64_t ldc, int64_t sC, int64_t batch) {
  for (int64_t bi = 0; bi < batch; ++bi) {
    const float* Ab = A + bi * sA;
    const float* Bb = B + bi * sB;
    float* Cb = C + bi * sC;
    parallel_rows(c.threads, M, [&](int64_t m0, int64_t m1) {
      std::vector<float> acc(N);
      for (int64_t m = m0; m < m1; ++m) {
        std::fill(acc.begin(), acc.end(), 0.f);
        for (int64_t k = 0; k < K; ++k) {
          const float av = ta ? Ab[k * lda + m] : Ab[m * lda + k];
          if (av == 0.f) continue;
          if (!tb) {
            const float* br = Bb + k * ldb;
            for (int64_t n = 0; n < N; ++n) acc[n] += av * br[n];
          } else {
            for (int64_t n = 0; n < N; ++n) acc[n] += av * Bb[n * ldb + k];
          }
        }
        float* cr = Cb + m * ldc;
        for (int64_t n = 0; n < N; ++n) cr[n] = alpha * acc[n] + (beta != 0.f ? beta * cr[n] : 0.f);
      }
    });
  }
}

namespace {
template <typename T>
double ld(const void* p, int64_t i) { return (double)((const T*)p)[i]; }
template <typename T>
void st(void* p, int64_t i, double v) { ((T*)p)[i] = (T)v; }
double load_any(const void* p, int dt, int64_t i) {
  switch (dt) {
    case VT_FP32: return ld<float>(p, i);
    case VT_FP64: return ld<double>(p, i);
    case VT_INT64: return ld<int64_t>(p, i);
    case VT_INT32: return ld<int32_t>(p, i);
    case VT_INT16: return ld<int16_t>(p, i);
    case VT_INT8: return ld<int8_t>(p, i);
    case VT_UINT8: return ld<uint8_t>(p, i);
    case VT_BOOL: return ((const uint8_t*)p)[i] ? 1.0 : 0.0;
  }
  throw std::runtime_error("cast: unsupported source dtype " + std::to_string(dt));
}
void store_any(void* p, int dt, int64_t i, double v) {
  switch (dt) {
    case VT_FP32: return st<float>(p, i, v);
    case VT_FP64: return st<double>(p, i, v);
    case VT_INT64: return st<int64_t>(p, i, v);
    case VT_INT32: return st<int32_t>(p, i, v);
    case VT_INT16: return st<int16_t>(p, i, v);
    case VT_INT8: return st<int8_t>(p, i, v);
    case VT_UINT8: return st<uint8_t>(p, i, v);
    case VT_BOOL: ((uint8_t*)p)[i] = v != 0.0; return;
  }
  throw std::runtime_error("cast: unsupported target dtype " + std::to_string(dt));
}
}  // namespace

void cast(Ctx&, const void* x, int dtx, void* y, int dty, int64_t n) {
  for (int64_t i = 0; i < n; ++i) store_any(y, dty, i, load_any(x, dtx, i));
}

void fill(Ctx&, void* y, int dt, int64_t n, double v) {
  for (int64_t i = 0; i < n; ++i) store_any(y, dt, i, v);
}

void reduce(Ctx&, const float* x, float* y, int64_t outer, int64_t n, int64_t inner, bool mean) {
  for (int64_t o = 0; o < outer; ++o)
    for (int64_t j = 0; j < inner; ++j) {
      double s = 0.0;
      for (int64_t i = 0; i < n; ++i) s += x[(o * n + i) * inner + j];
      y[o * inner + j] = (float)(mean ? s / n : s);
    }
}

void copy2d(Ctx&, const void* src, int64_t spitch, void* dst, int64_t dpitch, int64_t rows,
            int64_t cols, int elem) {
  for (int64_t r = 0; r < rows; ++r)
    std::memcpy((char*)dst + r * dpitch * elem, (const char*)src + r * spitch * elem, (size_t)(cols * elem));
}


void im2col(Ctx&, const float* x, int64_t x_img, float* col, int64_t N, const ConvG& g) {
  const int64_t P = g.OH * g.OW, rows = g.C * g.R * g.S;
  for (int64_t n = 0; n < N; ++n)
    for (int64_t q = 0; q < rows; ++q) {
      const int64_t c = q / (g.R * g.S), r = (q / g.S) % g.R, s = q % g.S;
      const float* xp = x + n * x_img + c * g.H * g.W;
      float* cp = col + (n * rows + q) * P;
      for (int64_t oh = 0; oh < g.OH; ++oh) {
        const int64_t ih = oh * g.sh - g.ph + r * g.dh;
        for (int64_t ow = 0; ow < g.OW; ++ow) {
          const int64_t iw = ow * g.sw - g.pw + s * g.dw;
          cp[oh * g.OW + ow] = (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) ? xp[ih * g.W + iw] : 0.f;
        }
      }
    }
}

void dwconv(Ctx& c, const float* x, const float* w, const float* bias, float* y, int64_t N,
            int64_t mult, const ConvG& g) {
  const int64_t K = g.C * mult;
  parallel_rows(c.threads, N * K, [&](int64_t a, int64_t b) {
    for (int64_t nk = a; nk < b; ++nk) {
      const int64_t n = nk / K, k = nk % K, ci = k / mult;
      const float* xp = x + (n * g.C + ci) * g.H * g.W;
      const float* wp = w + k * g.R * g.S;
      float* yp = y + nk * g.OH * g.OW;
      for (int64_t oh = 0; oh < g.OH; ++oh)
        for (int64_t ow = 0; ow < g.OW; ++ow) {
          float acc = bias ? bias[k] : 0.f;
          for (int64_t r = 0; r < g.R; ++r) {
            const int64_t ih = oh * g.sh - g.ph + r * g.dh;
            if (ih < 0 || ih >= g.H) continue;
            for (int64_t s = 0; s < g.S; ++s) {
              const int64_t iw = ow * g.sw - g.pw + s * g.dw;
              if (iw >= 0 && iw < g.W) acc += xp[ih * g.W + iw] * wp[r * g.S + s];
            }
          }
          yp[oh * g.OW + ow] = acc;
        }
    }
  });
}

void pool2d(Ctx& c, const float* x, float* y, int64_t planes, const PoolG& p) {
  parallel_rows(c.threads, planes, [&](int64_t a, int64_t b) {
    for (int64_t pl = a; pl < b; ++pl) {
      const float* xp = x + pl * p.H * p.W;
      for (int64_t oh = 0; oh < p.OH; ++oh)
        for (int64_t ow = 0; ow < p.OW; ++ow) {
          int64_t h0, h1, w0, w1;
          if (p.adaptive) {
            h0 = oh * p.H / p.OH; h1 = ((oh + 1) * p.H + p.OH - 1) / p.OH;
            w0 = ow * p.W / p.OW; w1 = ((ow + 1) * p.W + p.OW - 1) / p.OW;
          } else {
            h0 = oh * p.sh - p.ph; h1 = h0 + p.kh;
            w0 = ow * p.sw - p.pw; w1 = w0 + p.kw;
          }
          const int64_t area = (h1 - h0) * (w1 - w0);
          h0 = std::max<int64_t>(h0, 0); h1 = std::min(h1, p.H);
          w0 = std::max<int64_t>(w0, 0); w1 = std::min(w1, p.W);
          float acc = p.max ? -INFINITY : 0.f;
          for (int64_t ih = h0; ih < h1; ++ih)
            for (int64_t iw = w0; iw < w1; ++iw)
              acc = p.max ? std::max(acc, xp[ih * p.W + iw]) : acc + xp[ih * p.W + iw];
          if (!p.max) acc /= (float)((p.exclusive || p.adaptive) ? std::max<int64_t>((h1 - h0) * (w1 - w0), 1) : area);
          y[(pl * p.OH + oh) * p.OW + ow] = acc;
        }
    }
  });
}

void channel_affine(Ctx&, const float* x, const float* sc, const float* sh, float* y, int64_t outer,
                    int64_t C, int64_t inner, int act, float p0) {
  for (int64_t o = 0; o < outer; ++o)
    for (int64_t ch = 0; ch < C; ++ch) {
      const float a = sc[ch], b = sh[ch];
      const int64_t base = (o * C + ch) * inner;
      for (int64_t i = 0; i < inner; ++i) y[base + i] = unary_f(act, x[base + i] * a + b, p0, 0.f);
    }
}

}  // namespace cpu
}  // namespace pdn
