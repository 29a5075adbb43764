// Direct NHWC grouped / depthwise convolution: forward, data gradient, weight gradient.
//
// Parity: reference `phi/kernels/gpu/depthwise_conv_kernel.cu` / `depthwise_conv_grad_kernel.cu`
// (`math/depthwise_conv.cu`) and the grouped path of `gpudnn/conv_kernel.cu`. A depthwise or
// narrow-group convolution has ≤ a few dozen MACs per loaded element, so it is an HBM-streaming
// problem, not an MFMA one: every lane owns V consecutive channels of one output pixel (16-byte
// loads: 8 × bf16/fp16 or 4 × f32) and walks the R × S taps with f32 accumulation; a wave covers
// 64·V contiguous channels of NHWC rows, so every tap reads whole 128-byte lines and neighbouring
// pixels' taps hit the same lines in L2.
//
// Generic form (one kernel for forward and data gradient):
//   out[n, p, q, o] = Σ_{i ∈ group(o), r, s} in[n, h(p, r), w(q, s), i] · W'[r·S + s][i − i0(o)][o]
// with W' = [R·S][cin_g][Cout] (output channel contiguous) and
//   * forward      : h(p, r) = p·st − pad + r·dil                        (in = x, out = y)
//   * TR (dgrad)   : h = (p + pad − r·dil) / st when divisible            (in = dY, out = dX)
// DW (cin_g == cout_g == 1): lane j's input channel is o + j (vector loads of both operands);
// otherwise the V output channels of a lane share one group and the input element is broadcast.
//
// Weight gradient (forward geometry): dW'[tap][c][o] = Σ_{n, p, q} dY[n, p, q, o] · x[n, h, w,
// i0(o) + c] — workgroups own a pixel chunk × a column block (V output channels × one c) × a chunk
// of ≤ 9 taps; the pixel lanes are reduced through LDS and each workgroup writes its f32 partial
// plane, summed in a fixed order by dconv_wgrad_finish (deterministic, no atomics).
#include "common.h"

#include <cstdlib>

namespace {

struct DGeom {
  int N, H, W, Cin;   // input [N][H][W][Cin]
  int OH, OW, Cout;   // output [N][OH][OW][Cout]
  int R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w;
  int cin_g, cout_g;  // channels per group (input / output side)
};

// DT: 0 f32, 1 bf16, 2 fp16
template <int DT>
__device__ __forceinline__ void ldv(const void* base, long long i, float* v, int n) {
  if constexpr (DT == 0) {
    const float* p = (const float*)base + i;
    if (n == 4) {
      const f32x4 t = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = t[j];
    } else {
      for (int j = 0; j < n; ++j) v[j] = p[j];
    }
  } else {
    const unsigned short* p = (const unsigned short*)base + i;
    if (n == 8) {
      const u16x8 t = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = h2f<DT == 2>(t[j]);
    } else {
      for (int j = 0; j < n; ++j) v[j] = h2f<DT == 2>(p[j]);
    }
  }
}
template <int DT>
__device__ __forceinline__ float ld1(const void* base, long long i) {
  if constexpr (DT == 0) return ((const float*)base)[i];
  else return h2f<DT == 2>(((const unsigned short*)base)[i]);
}
template <int DT>
__device__ __forceinline__ void stv(void* base, long long i, const float* v, int n) {
  if constexpr (DT == 0) {
    float* p = (float*)base + i;
    if (n == 4) {
      *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    } else {
      for (int j = 0; j < n; ++j) p[j] = v[j];
    }
  } else {
    unsigned short* p = (unsigned short*)base + i;
    if (n == 8) {
      u16x8 t;
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = f2h<DT == 2>(v[j]);
      *reinterpret_cast<u16x8*>(p) = t;
    } else {
      for (int j = 0; j < n; ++j) p[j] = f2h<DT == 2>(v[j]);
    }
  }
}

// input row / column a tap reads, or -1 when outside (or, TR, not on the stride lattice)
template <bool TR>
__device__ __forceinline__ int tap_src(int p, int r, int st, int pad, int dil, int lim) {
  if (!TR) {
    const int h = p * st - pad + r * dil;
    return (h >= 0 && h < lim) ? h : -1;
  }
  const int t = p + pad - r * dil;
  if (t < 0 || t % st) return -1;
  const int h = t / st;
  return h < lim ? h : -1;
}

template <int DT, int V, bool DW, bool TR>
__global__ __launch_bounds__(256) void dconv_kernel(const void* __restrict__ x,
                                                    const void* __restrict__ w,
                                                    const void* __restrict__ bias,
                                                    void* __restrict__ y, DGeom g, long long total) {
  // 32-bit index math (total < 2^31, checked by the launcher)
  const unsigned idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= (unsigned)total) return;
  const unsigned cvec = (unsigned)(g.Cout / V);
  const int cv = (int)(idx % cvec);
  const unsigned pixu = idx / cvec;
  const long long pix = pixu;
  const int q = (int)(pixu % (unsigned)g.OW);
  const unsigned t = pixu / (unsigned)g.OW;
  const int p = (int)(t % (unsigned)g.OH), n = (int)(t / (unsigned)g.OH);
  const int o0 = cv * V;
  const int ci0 = DW ? o0 : (o0 / g.cout_g) * g.cin_g;
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  for (int r = 0; r < g.R; ++r) {
    const int ih = tap_src<TR>(p, r, g.st_h, g.pad_h, g.dil_h, g.H);
    if (ih < 0) continue;
    for (int s = 0; s < g.S; ++s) {
      const int iw = tap_src<TR>(q, s, g.st_w, g.pad_w, g.dil_w, g.W);
      if (iw < 0) continue;
      const long long xo = (((long long)n * g.H + ih) * g.W + iw) * g.Cin + ci0;
      const long long wo = (long long)(r * g.S + s) * g.cin_g * g.Cout + o0;
      float wv[V];
      if (DW) {
        float xv[V];
        ldv<DT>(x, xo, xv, V);
        ldv<DT>(w, wo, wv, V);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = fmaf(xv[j], wv[j], acc[j]);
      } else {
        for (int c = 0; c < g.cin_g; ++c) {
          const float xs = ld1<DT>(x, xo + c);
          ldv<DT>(w, wo + (long long)c * g.Cout, wv, V);
#pragma unroll
          for (int j = 0; j < V; ++j) acc[j] = fmaf(xs, wv[j], acc[j]);
        }
      }
    }
  }
  if (bias) {
    float bv[V];
    ldv<DT>(bias, o0, bv, V);
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] += bv[j];
  }
  stv<DT>(y, pix * g.Cout + o0, acc, V);
}

constexpr int WG_TAPS = 9;  // taps per weight-gradient launch slice (accumulators 9·V floats)

// grid: x = pixel chunks (pixels [chunk·per, (chunk+1)·per)), y = column blocks of CB columns,
// z = tap slices. Column = (output-channel vector kv, input channel c of the group).
template <int DT, int V, bool DW>
__global__ __launch_bounds__(256) void dconv_wgrad_kernel(const void* __restrict__ x,
                                                          const void* __restrict__ dy,
                                                          float* __restrict__ ws, DGeom g,
                                                          int cb_log2, long long per,
                                                          long long M) {
  __shared__ float red[256 * WG_TAPS * V / 2 + 1];  // holds half the lanes' partials per round
  const int CB = 1 << cb_log2, PL = 256 / CB;
  const int tid = threadIdx.x, cb = tid & (CB - 1), pl = tid >> cb_log2;
  const int kvn = g.Cout / V, ncol = kvn * g.cin_g;
  const int col = blockIdx.y * CB + cb;
  const bool live = col < ncol;
  const int kv = live ? col % kvn : 0, c = live ? col / kvn : 0;
  const int o0 = kv * V;
  const int ci = DW ? o0 : (o0 / g.cout_g) * g.cin_g + c;
  const int T = g.R * g.S, t0 = blockIdx.z * WG_TAPS;
  const int nt = min(WG_TAPS, T - t0);
  float acc[WG_TAPS][V];
#pragma unroll
  for (int a = 0; a < WG_TAPS; ++a)
#pragma unroll
    for (int j = 0; j < V; ++j) acc[a][j] = 0.f;
  const long long m0 = (long long)blockIdx.x * per;
  const long long m1 = min(M, m0 + per);
  if (live) {
    for (long long m = m0 + pl; m < m1; m += PL) {
      const unsigned mu = (unsigned)m;  // M < 2^31 (launcher)
      const int q = (int)(mu % (unsigned)g.OW);
      const unsigned tt = mu / (unsigned)g.OW;
      const int p = (int)(tt % (unsigned)g.OH), n = (int)(tt / (unsigned)g.OH);
      float dv[V];
      ldv<DT>(dy, m * g.Cout + o0, dv, V);
#pragma unroll
      for (int a = 0; a < WG_TAPS; ++a) {
        const int tap = t0 + a, r = tap / g.S, s = tap - r * g.S;
        const int ih = p * g.st_h - g.pad_h + r * g.dil_h, iw = q * g.st_w - g.pad_w + s * g.dil_w;
        if (a >= nt || ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) continue;
        const long long xo = (((long long)n * g.H + ih) * g.W + iw) * g.Cin + ci;
        if (DW) {
          float xv[V];
          ldv<DT>(x, xo, xv, V);
#pragma unroll
          for (int j = 0; j < V; ++j) acc[a][j] = fmaf(dv[j], xv[j], acc[a][j]);
        } else {
          const float xs = ld1<DT>(x, xo);
#pragma unroll
          for (int j = 0; j < V; ++j) acc[a][j] = fmaf(dv[j], xs, acc[a][j]);
        }
      }
    }
  }
  // reduce the PL pixel lanes of each column: two rounds through LDS (half the lanes each), the
  // first half adds the second half's partials, then a tree over what remains in LDS.
  constexpr int A = WG_TAPS * V;
  float* out = ws + (long long)blockIdx.x * T * g.cin_g * g.Cout;
  if (PL == 1) {
    if (live)
      for (int a = 0; a < nt; ++a)
        for (int j = 0; j < V; ++j) out[((long long)(t0 + a) * g.cin_g + c) * g.Cout + o0 + j] = acc[a][j];
    return;
  }
  const int half = PL / 2;
  if (pl >= half) {
    float* d = red + ((pl - half) * CB + cb) * A;
#pragma unroll
    for (int a = 0; a < WG_TAPS; ++a)
#pragma unroll
      for (int j = 0; j < V; ++j) d[a * V + j] = acc[a][j];
  }
  __syncthreads();
  if (pl < half) {
    float* d = red + (pl * CB + cb) * A;
#pragma unroll
    for (int a = 0; a < WG_TAPS; ++a)
#pragma unroll
      for (int j = 0; j < V; ++j) d[a * V + j] += acc[a][j];
  }
  __syncthreads();
  for (int h = half / 2; h >= 1; h >>= 1) {
    for (int e = tid; e < h * CB * A; e += 256) red[e] += red[e + h * CB * A];
    __syncthreads();
  }
  for (int e = tid; e < CB * A; e += 256) {
    const int cc = e / A, a = (e % A) / V, j = e % V;
    const int col2 = blockIdx.y * CB + cc;
    if (col2 >= ncol || a >= nt) continue;
    const int kv2 = col2 % kvn, c2 = col2 / kvn;
    out[((long long)(t0 + a) * g.cin_g + c2) * g.Cout + kv2 * V + j] = red[e];
  }
}

__global__ __launch_bounds__(256) void dconv_wgrad_finish(const float* __restrict__ ws, int parts,
                                                          long long n, float* __restrict__ d) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float v = 0.f;
  for (int p = 0; p < parts; ++p) v += ws[p * n + i];
  d[i] = v;
}

// First level of the partial-plane sum when there are many planes (a depthwise plane is only
// 9·C floats, so one thread per weight walking every plane left a handful of workgroups each
// serially loading thousands of values): grid (column blocks of 64, slices of the planes); the 4
// lane rows of a block take interleaved planes of the slice, reduced in LDS in a fixed order;
// out[slice][i]. Deterministic (fixed assignment and order); dconv_wgrad_finish sums the slices.
constexpr int FIN_SLICES = 64;
__global__ __launch_bounds__(256) void dconv_wgrad_reduce(const float* __restrict__ ws, int parts,
                                                          long long n, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const long long i = (long long)blockIdx.x * 64 + tx;
  const int per = (parts + gridDim.y - 1) / gridDim.y;
  const int p0 = blockIdx.y * per, p1 = min(parts, p0 + per);
  float v = 0.f;
  if (i < n) {
    int p = p0 + ty;
    for (; p + 12 < p1; p += 16) {  // 4 independent loads in flight per lane
      const float a = ws[(long long)p * n + i], b = ws[(long long)(p + 4) * n + i];
      const float c = ws[(long long)(p + 8) * n + i], e = ws[(long long)(p + 12) * n + i];
      v += (a + b) + (c + e);
    }
    for (; p < p1; p += 4) v += ws[(long long)p * n + i];
  }
  red[ty][tx] = v;
  __syncthreads();
  if (ty == 0 && i < n) out[(long long)blockIdx.y * n + i] = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
}

// Depthwise 3×3 weight gradient (pad 1, dilation 1, stride ST ∈ {1, 2}; 16-bit NHWC, C % 8 == 0):
// the generic kernel above reloads x for every tap (10 loads per output pixel) and walks pixels
// in a scattered order, ~0.2-0.6 TB/s at MobileNetV2 shapes (tools/bench_dwconv.py). Here a thread
// owns 8 channels of one segment of an output row and slides a 3×3 window of x along it: per
// output pixel 1 (stride 1) or 2 (stride 2) new x columns of 3 rows + one dy vector, 72 FMAs into
// 72 f32 accumulators. Thread → (channel vector cv = tid mod NCVP, work slot = (n, p, segment));
// the SL = 256 / NCVP slots of a workgroup are reduced through LDS in a fixed tree and each
// workgroup writes one partial plane [9][C] (summed in a fixed order by dconv_wgrad_reduce /
// finish): deterministic, no atomics.
template <int V> struct DwVec;
template <> struct DwVec<8> { typedef u16x8 T; };
template <> struct DwVec<4> { typedef u16x4 T; };

template <int DT, int ST, int V>
__global__ __launch_bounds__(256) void dw3_wgrad_kernel(const unsigned short* __restrict__ x,
                                                        const unsigned short* __restrict__ dy,
                                                        float* __restrict__ ws, DGeom g, int ncv_log2,
                                                        int segs, int qs) {
  typedef typename DwVec<V>::T VT;
  constexpr int A = 9 * V;
  __shared__ float red[128 * A];  // half of the slots' partials
  const int NCVP = 1 << ncv_log2, SL = 256 >> ncv_log2;
  const int tid = threadIdx.x, cv = tid & (NCVP - 1), sl = tid >> ncv_log2;
  const int C = g.Cout, ncv = C / V;
  const long long wi = (long long)blockIdx.x * SL + sl;
  const long long nwork = (long long)g.N * g.OH * segs;
  float acc[9][V];
#pragma unroll
  for (int a = 0; a < 9; ++a)
#pragma unroll
    for (int j = 0; j < V; ++j) acc[a][j] = 0.f;
  if (cv < ncv && wi < nwork) {
    const int seg = (int)(wi % segs);
    const long long np = wi / segs;
    const int p = (int)(np % g.OH), n = (int)(np / g.OH);
    const int q0 = seg * qs, q1 = min(g.OW, q0 + qs);
    const int c0 = cv * V;
    const unsigned short* xr[3];
    bool rv[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int ih = p * ST - 1 + r;
      rv[r] = ih >= 0 && ih < g.H;
      xr[r] = x + ((long long)n * g.H + (rv[r] ? ih : 0)) * g.W * C + c0;
    }
    auto ldx = [&](int r, int iw) {
      VT v = {};
      if (rv[r] && iw >= 0 && iw < g.W) v = *reinterpret_cast<const VT*>(xr[r] + (long long)iw * C);
      return v;
    };
    const unsigned short* dyr = dy + (((long long)n * g.OH + p) * g.OW) * C + c0;
    VT w0[3], w1[3], w2[3], nw1[3], nw2[3], nd;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      w0[r] = ldx(r, q0 * ST - 1);
      w1[r] = ldx(r, q0 * ST);
      nw2[r] = ldx(r, q0 * ST + 1);
    }
    nd = *reinterpret_cast<const VT*>(dyr + (long long)q0 * C);
    for (int q = q0; q < q1; ++q) {
      // this column's operands were requested one iteration ahead; request the next column's
      const VT d = nd;
#pragma unroll
      for (int r = 0; r < 3; ++r) w2[r] = nw2[r];
      if (q + 1 < q1) {
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          if (ST == 2) nw1[r] = ldx(r, (q + 1) * ST);
          nw2[r] = ldx(r, (q + 1) * ST + 1);
        }
        nd = *reinterpret_cast<const VT*>(dyr + (long long)(q + 1) * C);
      }
      float dv[V];
#pragma unroll
      for (int j = 0; j < V; ++j) dv[j] = h2f<DT == 2>(d[j]);
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          acc[r * 3][j] = fmaf(dv[j], h2f<DT == 2>(w0[r][j]), acc[r * 3][j]);
          acc[r * 3 + 1][j] = fmaf(dv[j], h2f<DT == 2>(w1[r][j]), acc[r * 3 + 1][j]);
          acc[r * 3 + 2][j] = fmaf(dv[j], h2f<DT == 2>(w2[r][j]), acc[r * 3 + 2][j]);
        }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        if (ST == 1) {
          w0[r] = w1[r];
          w1[r] = w2[r];
        } else {  // next window: columns 2q+1 (= this w2), 2q+2, 2q+3
          w0[r] = w2[r];
          w1[r] = nw1[r];
        }
      }
    }
  }
  float* out = ws + (long long)blockIdx.x * 9 * C;
  auto store = [&](int cvv, int a, float v) {
    if (cvv < ncv) out[(long long)(a / V) * C + cvv * V + (a % V)] = v;
  };
  if (SL == 1) {
#pragma unroll
    for (int a = 0; a < A; ++a) store(cv, a, acc[a / V][a % V]);
    return;
  }
  const int half = SL / 2;
  if (sl >= half) {
    float* d = red + ((sl - half) * NCVP + cv) * A;
#pragma unroll
    for (int a = 0; a < A; ++a) d[a] = acc[a / V][a % V];
  }
  __syncthreads();
  if (sl < half) {
    float* d = red + (sl * NCVP + cv) * A;
#pragma unroll
    for (int a = 0; a < A; ++a) d[a] += acc[a / V][a % V];
  }
  __syncthreads();
  for (int h = half / 2; h >= 1; h >>= 1) {
    for (int e = tid; e < h * NCVP * A; e += 256) red[e] += red[e + h * NCVP * A];
    __syncthreads();
  }
  for (int e = tid; e < NCVP * A; e += 256) store(e / A, e % A, red[e]);
}

// channels per thread of dw3_wgrad_kernel (PIAMD_DW3_V = 4 or 8; 4 by default: half the
// accumulators, more waves in flight)
static int dw3_v() {
  static const int v = [] {
    const char* e = getenv("PIAMD_DW3_V");
    return e && atoi(e) == 8 ? 8 : 4;
  }();
  return v;
}

// Depthwise 3×3 forward (and the stride-1 data gradient, TR: the same window with the taps
// flipped), pad 1, dilation 1, 16-bit NHWC: a thread owns V channels of one segment of an output
// row, keeps the 9·V weights in registers and slides the 3×3 x window along the row — 1 (stride
// 1) or 2 (stride 2) new x columns of 3 rows per output pixel instead of 9 gathered taps.
template <int DT, int ST, int V, bool TR>
__global__ __launch_bounds__(256) void dw3_fwd_kernel(const unsigned short* __restrict__ x,
                                                      const unsigned short* __restrict__ w,
                                                      const unsigned short* __restrict__ bias,
                                                      unsigned short* __restrict__ y, DGeom g, int segs,
                                                      int qs, long long items) {
  typedef typename DwVec<V>::T VT;
  const int C = g.Cout, ncv = C / V;
  for (long long it = (long long)blockIdx.x * 256 + threadIdx.x; it < items; it += (long long)gridDim.x * 256) {
    const int cv = (int)(it % ncv);
    long long rest = it / ncv;
    const int seg = (int)(rest % segs);
    rest /= segs;
    const int p = (int)(rest % g.OH), n = (int)(rest / g.OH);
    const int c0 = cv * V, q0 = seg * qs, q1 = min(g.OW, q0 + qs);
    float wt[9][V], b[V];
#pragma unroll
    for (int a = 0; a < 9; ++a) {
      const VT u = *reinterpret_cast<const VT*>(w + (long long)(TR ? 8 - a : a) * C + c0);
#pragma unroll
      for (int j = 0; j < V; ++j) wt[a][j] = h2f<DT == 2>(u[j]);
    }
    if (bias) {
      const VT u = *reinterpret_cast<const VT*>(bias + c0);
#pragma unroll
      for (int j = 0; j < V; ++j) b[j] = h2f<DT == 2>(u[j]);
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) b[j] = 0.f;
    }
    const unsigned short* xr[3];
    bool rv[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int ih = p * ST - 1 + r;
      rv[r] = ih >= 0 && ih < g.H;
      xr[r] = x + ((long long)n * g.H + (rv[r] ? ih : 0)) * g.W * C + c0;
    }
    auto ldx = [&](int r, int iw) {
      VT v = {};
      if (rv[r] && iw >= 0 && iw < g.W) v = *reinterpret_cast<const VT*>(xr[r] + (long long)iw * C);
      return v;
    };
    VT w0[3], w1[3], w2[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      w0[r] = ldx(r, q0 * ST - 1);
      w1[r] = ldx(r, q0 * ST);
    }
    unsigned short* yr = y + (((long long)n * g.OH + p) * g.OW) * C + c0;
    for (int q = q0; q < q1; ++q) {
#pragma unroll
      for (int r = 0; r < 3; ++r) w2[r] = ldx(r, q * ST + 1);
      float o[V];
#pragma unroll
      for (int j = 0; j < V; ++j) o[j] = b[j];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          o[j] = fmaf(wt[r * 3][j], h2f<DT == 2>(w0[r][j]), o[j]);
          o[j] = fmaf(wt[r * 3 + 1][j], h2f<DT == 2>(w1[r][j]), o[j]);
          o[j] = fmaf(wt[r * 3 + 2][j], h2f<DT == 2>(w2[r][j]), o[j]);
        }
      VT ov;
#pragma unroll
      for (int j = 0; j < V; ++j) ov[j] = f2h<DT == 2>(o[j]);
      *reinterpret_cast<VT*>(yr + (long long)q * C) = ov;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        if (ST == 1) {
          w0[r] = w1[r];
          w1[r] = w2[r];
        } else {
          w0[r] = w2[r];
          w1[r] = ldx(r, (q + 1) * ST);
        }
      }
    }
  }
}

// Work split of dw3_wgrad_kernel: row segments of ≤ 16 output columns; parts = workgroups.
static void dw3_split(const DGeom& g, int& ncv_log2, int& segs, int& qs, long long& parts) {
  const int ncv = g.Cout / dw3_v();
  ncv_log2 = 0;
  while ((1 << ncv_log2) < ncv) ++ncv_log2;
  segs = (g.OW + 15) / 16;
  qs = (g.OW + segs - 1) / segs;
  const long long nwork = (long long)g.N * g.OH * segs;
  const int SL = 256 >> ncv_log2;
  parts = (nwork + SL - 1) / SL;
}

static bool dw3_ok(const DGeom& g, int dtype) {
  return dtype != 0 && g.cin_g == 1 && g.cout_g == 1 && g.R == 3 && g.S == 3 && g.pad_h == 1 &&
         g.pad_w == 1 && g.dil_h == 1 && g.dil_w == 1 && g.st_h == g.st_w && (g.st_h == 1 || g.st_h == 2) &&
         g.Cout % dw3_v() == 0 && g.Cout / dw3_v() <= 256;
}

template <int DT, int V, bool DW, bool TR>
void launch_fwd(const void* x, const void* w, const void* b, void* y, const DGeom& g,
                hipStream_t st) {
  const long long total = (long long)g.N * g.OH * g.OW * (g.Cout / V);
  hipLaunchKernelGGL((dconv_kernel<DT, V, DW, TR>), dim3((unsigned)((total + 255) / 256)),
                     dim3(256), 0, st, x, w, b, y, g, total);
}

template <int DT, int V>
void dispatch_fwd(bool dw, bool tr, const void* x, const void* w, const void* b, void* y,
                  const DGeom& g, hipStream_t st) {
  if (dw) {
    if (tr) launch_fwd<DT, V, true, true>(x, w, b, y, g, st);
    else launch_fwd<DT, V, true, false>(x, w, b, y, g, st);
  } else {
    if (tr) launch_fwd<DT, V, false, true>(x, w, b, y, g, st);
    else launch_fwd<DT, V, false, false>(x, w, b, y, g, st);
  }
}

bool geom_ok(const DGeom& g) {
  return g.N > 0 && g.H > 0 && g.W > 0 && g.OH > 0 && g.OW > 0 && g.R > 0 && g.S > 0 &&
         g.st_h > 0 && g.st_w > 0 && g.dil_h > 0 && g.dil_w > 0 && g.cin_g > 0 && g.cout_g > 0 &&
         g.Cin % g.cin_g == 0 && g.Cout % g.cout_g == 0 && g.Cin / g.cin_g == g.Cout / g.cout_g;
}

// lane width: 16-byte vectors when every lane's V channels stay in one group (or DW)
int pick_v(int dt, const DGeom& g, bool dw) {
  const int vmax = dt == 0 ? 4 : 8;
  if (g.Cout % vmax == 0 && (dw || g.cout_g % vmax == 0)) return vmax;
  return 1;
}

}  // namespace

// out [N][OH][OW][Cout] = grouped conv of in [N][H][W][Cin] with W' [R·S][cin_g][Cout] (+ bias
// [Cout], nullable); transposed = 1: data-gradient geometry (see the header). dtype 0 f32, 1 bf16,
// 2 fp16 (all operands one dtype; f32 accumulation).
PIAMD_EXPORT int piamd_dconv2d(const void* in, const void* w, const void* bias, void* out, int N,
                               int H, int W, int Cin, int OH, int OW, int Cout, int R, int S,
                               int st_h, int st_w, int pad_h, int pad_w, int dil_h, int dil_w,
                               int cin_g, int cout_g, int transposed, int dtype, hipStream_t st) {
  const DGeom g{N, H, W, Cin, OH, OW, Cout, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w, cin_g, cout_g};
  if (!geom_ok(g) || dtype < 0 || dtype > 2) return (int)hipErrorInvalidValue;
  const bool dw = cin_g == 1 && cout_g == 1, tr = transposed != 0;
  // depthwise 3×3 pad 1: the sliding-window kernel (forward at stride 1 / 2, data gradient at
  // stride 1, where the transposed geometry is the forward one with flipped taps)
  if (dw3_ok(g, dtype) && (!tr || st_h == 1) && OW > 0) {
    const int segs = (OW + 15) / 16, qs = (OW + segs - 1) / segs;
    const int V = dw3_v();
    const long long items = (long long)N * OH * segs * (Cout / V);
    const long long nb = (items + 255) / 256;
    const unsigned grid = (unsigned)(nb < (1 << 20) ? nb : (1 << 20));
#define DWF(DT, ST, VV, TRV)                                                                        \
  hipLaunchKernelGGL((dw3_fwd_kernel<DT, ST, VV, TRV>), dim3(grid), dim3(256), 0, st,                \
                     (const unsigned short*)in, (const unsigned short*)w, (const unsigned short*)bias, \
                     (unsigned short*)out, g, segs, qs, items)
#define DWF_V(DT, ST, TRV) do { if (V == 8) DWF(DT, ST, 8, TRV); else DWF(DT, ST, 4, TRV); } while (0)
    if (dtype == 1) {
      if (tr) DWF_V(1, 1, true); else if (st_h == 1) DWF_V(1, 1, false); else DWF_V(1, 2, false);
    } else {
      if (tr) DWF_V(2, 1, true); else if (st_h == 1) DWF_V(2, 1, false); else DWF_V(2, 2, false);
    }
#undef DWF_V
#undef DWF
    return (int)hipGetLastError();
  }
  const int v = pick_v(dtype, g, dw);
  if ((long long)N * OH * OW * (Cout / v) >= 0x7fffffffLL) return (int)hipErrorInvalidValue;
  if (dtype == 0) {
    if (v == 4) dispatch_fwd<0, 4>(dw, tr, in, w, bias, out, g, st);
    else dispatch_fwd<0, 1>(dw, tr, in, w, bias, out, g, st);
  } else if (dtype == 1) {
    if (v == 8) dispatch_fwd<1, 8>(dw, tr, in, w, bias, out, g, st);
    else dispatch_fwd<1, 1>(dw, tr, in, w, bias, out, g, st);
  } else {
    if (v == 8) dispatch_fwd<2, 8>(dw, tr, in, w, bias, out, g, st);
    else dispatch_fwd<2, 1>(dw, tr, in, w, bias, out, g, st);
  }
  return (int)hipGetLastError();
}

template <int DT, int V, bool DW>
static void launch_wg(const void* x, const void* dy, float* ws, const DGeom& g, dim3 grid,
                      int cb_log2, long long per, long long M, hipStream_t st) {
  hipLaunchKernelGGL((dconv_wgrad_kernel<DT, V, DW>), grid, dim3(256), 0, st, x, dy, ws, g,
                     cb_log2, per, M);
}

// Partial planes the depthwise-3×3 weight-gradient path needs for this geometry (0: the generic
// kernel serves it and takes any `parts`).
PIAMD_EXPORT long long piamd_dconv2d_wgrad_parts(int N, int H, int W, int C, int OH, int OW, int K, int R,
                                                 int S, int st_h, int st_w, int pad_h, int pad_w, int dil_h,
                                                 int dil_w, int cin_g, int cout_g, int dtype) {
  const DGeom g{N, H, W, C, OH, OW, K, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w, cin_g, cout_g};
  if (!geom_ok(g) || !dw3_ok(g, dtype) || (long long)N * H * W * C >= (1LL << 40)) return 0;
  int l2, segs, qs;
  long long parts;
  dw3_split(g, l2, segs, qs, parts);
  return parts;
}

// dW' [R·S][cin_g][Cout] f32 of the forward conv (x [N][H][W][Cin], dy [N][OH][OW][Cout]);
// ws: (parts + 64) · R·S·cin_g·Cout floats: the partial planes (parts ≥ 1 pixel chunks), then
// room for the 64 slice sums of the two-level finish (used when parts > 128).
PIAMD_EXPORT int piamd_dconv2d_wgrad(const void* x, const void* dy, float* d, float* ws, int parts,
                                     int N, int H, int W, int Cin, int OH, int OW, int Cout, int R,
                                     int S, int st_h, int st_w, int pad_h, int pad_w, int dil_h,
                                     int dil_w, int cin_g, int cout_g, int dtype, hipStream_t st) {
  const DGeom g{N, H, W, Cin, OH, OW, Cout, R, S, st_h, st_w, pad_h, pad_w, dil_h, dil_w, cin_g, cout_g};
  if (!geom_ok(g) || dtype < 0 || dtype > 2 || parts < 1 || !ws || !d) return (int)hipErrorInvalidValue;
  const bool dw = cin_g == 1 && cout_g == 1;
  if (dw3_ok(g, dtype)) {
    int l2, segs, qs;
    long long np;
    dw3_split(g, l2, segs, qs, np);
    if (np != parts) return (int)hipErrorInvalidValue;  // ws sized by piamd_dconv2d_wgrad_parts
#define DW3(DT, ST, VV)                                                                           \
  hipLaunchKernelGGL((dw3_wgrad_kernel<DT, ST, VV>), dim3((unsigned)np), dim3(256), 0, st,          \
                     (const unsigned short*)x, (const unsigned short*)dy, ws, g, l2, segs, qs)
    const bool v8 = dw3_v() == 8;
    if (dtype == 1) {
      if (st_h == 1) { if (v8) DW3(1, 1, 8); else DW3(1, 1, 4); }
      else { if (v8) DW3(1, 2, 8); else DW3(1, 2, 4); }
    } else {
      if (st_h == 1) { if (v8) DW3(2, 1, 8); else DW3(2, 1, 4); }
      else { if (v8) DW3(2, 2, 8); else DW3(2, 2, 4); }
    }
#undef DW3
  }
  const int v = pick_v(dtype, g, dw);
  const int ncol = (Cout / v) * cin_g;
  int cb_log2 = 0;
  while ((1 << cb_log2) < ncol && cb_log2 < 6) ++cb_log2;  // ≤ 64 columns, ≥ 4 pixel lanes
  const long long M = (long long)N * OH * OW;
  if (M >= 0x7fffffffLL) return (int)hipErrorInvalidValue;
  const long long per = (M + parts - 1) / parts;
  const dim3 grid((unsigned)parts, (unsigned)((ncol + (1 << cb_log2) - 1) >> cb_log2),
                  (unsigned)((R * S + WG_TAPS - 1) / WG_TAPS));
  if (!dw3_ok(g, dtype)) {
#define WG(DT, VV)                                                                                \
  do {                                                                                            \
    if (dw) launch_wg<DT, VV, true>(x, dy, ws, g, grid, cb_log2, per, M, st);                     \
    else launch_wg<DT, VV, false>(x, dy, ws, g, grid, cb_log2, per, M, st);                       \
  } while (0)
  if (dtype == 0) {
    if (v == 4) WG(0, 4); else WG(0, 1);
  } else if (dtype == 1) {
    if (v == 8) WG(1, 8); else WG(1, 1);
  } else {
    if (v == 8) WG(2, 8); else WG(2, 1);
  }
#undef WG
  }
  const long long n = (long long)R * S * cin_g * Cout;
  if (parts > 2 * FIN_SLICES) {
    // two-level sum: the planes into FIN_SLICES slice sums (after the planes in ws), then those
    float* slices = ws + (long long)parts * n;  // caller sized ws for parts + FIN_SLICES planes
    hipLaunchKernelGGL(dconv_wgrad_reduce, dim3((unsigned)((n + 63) / 64), FIN_SLICES), dim3(256), 0, st,
                       (const float*)ws, parts, n, slices);
    hipLaunchKernelGGL(dconv_wgrad_finish, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const float*)slices, FIN_SLICES, n, d);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(dconv_wgrad_finish, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (const float*)ws, parts, n, d);
  return (int)hipGetLastError();
}
