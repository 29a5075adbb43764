// Host side of the hand-scheduled assembly flash-attention backward (`csrc/asm/fa_gen.py` →
// _lib/piamd_fa.hsaco): code-object loading, the kernel-argument block and the launch contract.
// `launch_bwd` (flash_attn.h) asks fa_dkdv_asm() first and runs the HIP dK/dV kernel when the
// assembly kernel does not take the shape.
//
// Parity: reference `paddle/phi/kernels/gpu/flash_attn_grad_kernel.cu` (dK / dV of
// flash_attn_grad).
#include "common.h"
#include "fa_args.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <mutex>

namespace {

// mirror of fa_gen.ARGS (byte offsets noted)
struct __attribute__((packed)) FaDkdvArgs {
  const void *q, *k, *v, *dout;  // 0, 8, 16, 24
  void *dk, *dv;                 // 32, 40
  const float *nl, *nd;          // 48, 56: −lse/scale, −δ rows
  unsigned q_bytes, k_bytes, v_bytes, o_bytes, st_bytes;  // 64 .. 80 (descriptor ranges)
  unsigned sqs, sqh, sqb;        // 84 ..: byte strides
  unsigned sks, skh, skb;
  unsigned svs, svh, svb;
  unsigned sos, soh, sob;        // .. 128
  unsigned Hq, Hk, group, Sq;    // 132 ..
  int coff;                      // 148
  unsigned nqt, npair, nkb1;     // 152, 156, 160: key blocks nkb = Sk/128 = 2·npair
  float c, scale, rcp_npair, rcp_Hk;  // 164 .. 176
  unsigned nitems, G, G2m1;      // 180: items (= nkb·Hk·B), grid (multiple of 8), 2G − 1
};
static_assert(sizeof(FaDkdvArgs) == 192, "FaDkdvArgs layout");

// mirror of fa_gen.DQ_ARGS
struct __attribute__((packed)) FaDqArgs {
  const void *q, *k, *v, *dout;  // 0 ..
  void* dq;                      // 32
  unsigned long long pad0;       // 40
  const float *nl, *nd;          // 48, 56
  unsigned q_bytes, k_bytes, v_bytes, o_bytes, st_bytes;  // 64 .. 80
  unsigned sqs, sqh, sqb, sks, skh, skb, svs, svh, svb, sos, soh, sob;  // 84 .. 128
  unsigned Hq, group;            // 132, 136
  float rcp_group;               // 140
  unsigned Sq, nkt, npair, nqb1; // 144 .. 156
  float rcp_npair, c, scale, rcp_Hq;  // 160 .. 172
  unsigned pad1, nitems, G, G2m1;     // 176 .. 188
};
static_assert(sizeof(FaDqArgs) == 192, "FaDqArgs layout");

std::mutex g_mu;
hipModule_t g_mod = nullptr;
hipFunction_t g_fn[8] = {};
int g_enabled = -1;  // bit 0: dK/dV kernel, bit 1: dQ kernel, bit 2: forward kernel
int g_fwd_nw = -1;   // forward variant: 4 or 8 waves per workgroup

// PIAMD_FA_ASM: unset / 1 = every assembly kernel, 0 = none, "dkdv" / "dq" / "fwd" / "bwd" = those
int enabled_mask() {
  if (g_enabled < 0) {
    const char* e = getenv("PIAMD_FA_ASM");
    g_enabled = !e ? 7 : e[0] == '0' ? 0 : !strcmp(e, "dkdv") ? 1 : !strcmp(e, "dq") ? 2
              : !strcmp(e, "fwd") ? 4 : !strcmp(e, "bwd") ? 3 : 7;
  }
  return g_enabled;
}

// byte extent of a [B, S, H, 128] view from its base (last byte + 1), 0 on overflow past 2^31
unsigned long long extent(long long sb, long long ss, long long sh, int B, int S, int H) {
  if (sb < 0 || ss < 0 || sh < 0) return 0;
  const unsigned long long e = ((unsigned long long)(B - 1) * sb + (unsigned long long)(S - 1) * ss +
                                (unsigned long long)(H - 1) * sh + 128) * 2ull;
  return e < (1ull << 31) ? e : 0;
}

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

bool stride_ok(long long s) { return s > 0 && (s * 2) % 16 == 0 && s * 2 < (1ll << 24); }

}  // namespace

PIAMD_EXPORT int piamd_fa_asm_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_mod) return 0;
  hipModule_t m = nullptr;
  int err = (int)hipModuleLoad(&m, path);
  if (err) return err;
  if (hipModuleGetFunction(&g_fn[0], m, "piamd_fa_dkdv_d128") != hipSuccess ||
      hipModuleGetFunction(&g_fn[1], m, "piamd_fa_dkdv_d128_causal") != hipSuccess ||
      hipModuleGetFunction(&g_fn[2], m, "piamd_fa_dq_d128") != hipSuccess ||
      hipModuleGetFunction(&g_fn[3], m, "piamd_fa_dq_d128_causal") != hipSuccess ||
      hipModuleGetFunction(&g_fn[4], m, "piamd_fa_fwd_d128") != hipSuccess ||
      hipModuleGetFunction(&g_fn[5], m, "piamd_fa_fwd_d128_causal") != hipSuccess ||
      hipModuleGetFunction(&g_fn[6], m, "piamd_fa_fwd8_d128") != hipSuccess ||
      hipModuleGetFunction(&g_fn[7], m, "piamd_fa_fwd8_d128_causal") != hipSuccess)
    return (int)hipErrorNotFound;
  g_mod = m;
  return 0;
}

PIAMD_EXPORT int piamd_fa_asm_loaded() { return g_mod != nullptr; }

// bit mask of the assembly kernels to use where they apply: 1 = dK/dV, 2 = dQ, 4 = forward
// (default 7; env PIAMD_FA_ASM)
PIAMD_EXPORT int piamd_fa_asm_enable(int mask) {
  g_enabled = mask & 7;
  return 0;
}

// forward kernel variant (4 or 8 waves per workgroup; tests / A-B)
PIAMD_EXPORT int piamd_fa_fwd_nw(int nw) {
  g_fwd_nw = nw;
  return 0;
}

// Would the assembly kernel take this backward? (contract in fa_gen.py's docstring)
PIAMD_EXPORT int piamd_fa_asm_applies(const FaArgs* ap) {
  const FaArgs& a = *ap;
  if (!g_mod || !enabled_mask()) return 0;
  if (a.D != 128 || a.cu_q || a.mask || a.p_drop > 0.f || a.Sq != a.Sk || a.Sq % 256) return 0;
  if (a.Hk <= 0 || a.Hq % a.Hk || a.B <= 0) return 0;
  // seq strides feed 24-bit multiplies; every stride keeps 16-byte rows (LDS-DMA / dwordx4)
  for (long long s : {a.sqs, a.sks, a.svs, a.sos})
    if (!stride_ok(s)) return 0;
  for (long long s : {a.sqh, a.skh, a.svh, a.soh, a.sqb, a.skb, a.svb, a.sob})
    if (s < 0 || (s * 2) % 16) return 0;
  if (!extent(a.sqb, a.sqs, a.sqh, a.B, a.Sq, a.Hq) || !extent(a.skb, a.sks, a.skh, a.B, a.Sk, a.Hk) ||
      !extent(a.svb, a.svs, a.svh, a.B, a.Sk, a.Hk) || !extent(a.sob, a.sos, a.soh, a.B, a.Sq, a.Hq))
    return 0;
  for (const void* p : {(const void*)a.q, (const void*)a.k, (const void*)a.v, (const void*)a.dout,
                        (const void*)a.dk, (const void*)a.dv})
    if (reinterpret_cast<unsigned long long>(p) % 16) return 0;
  const long long rows = (long long)a.B * a.Hq * a.Sq;
  if (rows * 4 >= (1ll << 31) || (long long)(a.Sk / 128) * a.Hk * a.B >= (1ll << 24)) return 0;
  return 1;
}

// Launch the assembly dK/dV kernel (after bwd_pre wrote −δ / −lse/scale into a.delta). Returns
// 1 when launched, 0 when the shape is not this kernel's (caller runs the HIP kernel), < 0 on a
// launch error.
int fa_dkdv_asm(const FaArgs& a, hipStream_t st) {
  if (!(enabled_mask() & 1) || !piamd_fa_asm_applies(&a)) return 0;
  FaDkdvArgs g{};
  g.q = a.q;
  g.k = a.k;
  g.v = a.v;
  g.dout = a.dout;
  g.dk = a.dk;
  g.dv = a.dv;
  const long long rows = (long long)a.B * a.Hq * a.Sq;
  g.nd = a.delta;
  g.nl = a.delta + rows;
  g.q_bytes = (unsigned)extent(a.sqb, a.sqs, a.sqh, a.B, a.Sq, a.Hq);
  g.k_bytes = (unsigned)extent(a.skb, a.sks, a.skh, a.B, a.Sk, a.Hk);
  g.v_bytes = (unsigned)extent(a.svb, a.svs, a.svh, a.B, a.Sk, a.Hk);
  g.o_bytes = (unsigned)extent(a.sob, a.sos, a.soh, a.B, a.Sq, a.Hq);
  g.st_bytes = (unsigned)(rows * 4);
  g.sqs = (unsigned)(a.sqs * 2); g.sqh = (unsigned)(a.sqh * 2); g.sqb = (unsigned)(a.sqb * 2);
  g.sks = (unsigned)(a.sks * 2); g.skh = (unsigned)(a.skh * 2); g.skb = (unsigned)(a.skb * 2);
  g.svs = (unsigned)(a.svs * 2); g.svh = (unsigned)(a.svh * 2); g.svb = (unsigned)(a.svb * 2);
  g.sos = (unsigned)(a.sos * 2); g.soh = (unsigned)(a.soh * 2); g.sob = (unsigned)(a.sob * 2);
  g.Hq = a.Hq;
  g.Hk = a.Hk;
  g.group = a.Hq / a.Hk;
  g.Sq = a.Sq;
  g.coff = a.Sk - a.Sq;
  g.nqt = a.Sq / 64;
  const unsigned nkb = (unsigned)(a.Sk / 128);
  g.npair = nkb / 2;
  g.nkb1 = nkb - 1;
  g.c = a.scale * 1.4426950408889634f;
  g.scale = a.scale;
  g.rcp_npair = 1.f / (float)g.npair;
  g.rcp_Hk = 1.f / (float)a.Hk;
  // persistent: one workgroup per CU (LDS / register bound); workgroup v takes the key-block
  // pairs (j, nkb−1−j) of pair-members v, v + G, … (fa_gen.py decode / next_item)
  g.nitems = nkb * (unsigned)a.Hk * (unsigned)a.B;
  const unsigned members = g.nitems / 2;
  g.G = std::min<unsigned>((unsigned)num_cus() / 8 * 8, (members + 7) / 8 * 8);
  g.G2m1 = 2 * g.G - 1;
  const unsigned grid = g.G;
  size_t sz = sizeof(g);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &g, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  hipError_t err = hipModuleLaunchKernel(g_fn[a.causal ? 1 : 0], grid, 1, 1, 256, 1, 1, 0, st, nullptr, cfg);
  return err == hipSuccess ? 1 : -(int)err;
}

// the dQ / forward argument block (fa_gen.DQ_ARGS; the forward reads dq as O and nl as lse)
static FaDqArgs dq_args(const FaArgs& a, int wgs_per_cu, int qsh = 7) {
  FaDqArgs g{};
  g.q = a.q;
  g.k = a.k;
  g.v = a.v;
  g.dout = a.dout;
  g.dq = a.dq;
  const long long rows = (long long)a.B * a.Hq * a.Sq;
  g.nd = a.delta;
  g.nl = a.delta + rows;
  g.q_bytes = (unsigned)extent(a.sqb, a.sqs, a.sqh, a.B, a.Sq, a.Hq);
  g.k_bytes = (unsigned)extent(a.skb, a.sks, a.skh, a.B, a.Sk, a.Hk);
  g.v_bytes = (unsigned)extent(a.svb, a.svs, a.svh, a.B, a.Sk, a.Hk);
  g.o_bytes = (unsigned)extent(a.sob, a.sos, a.soh, a.B, a.Sq, a.Hq);
  g.st_bytes = (unsigned)(rows * 4);
  g.sqs = (unsigned)(a.sqs * 2); g.sqh = (unsigned)(a.sqh * 2); g.sqb = (unsigned)(a.sqb * 2);
  g.sks = (unsigned)(a.sks * 2); g.skh = (unsigned)(a.skh * 2); g.skb = (unsigned)(a.skb * 2);
  g.svs = (unsigned)(a.svs * 2); g.svh = (unsigned)(a.svh * 2); g.svb = (unsigned)(a.svb * 2);
  g.sos = (unsigned)(a.sos * 2); g.soh = (unsigned)(a.soh * 2); g.sob = (unsigned)(a.sob * 2);
  g.Hq = a.Hq;
  g.group = a.Hq / a.Hk;
  g.rcp_group = 1.f / (float)g.group;
  g.Sq = a.Sq;
  g.nkt = a.Sk / 64;
  const unsigned nqb = (unsigned)(a.Sq >> qsh);  // work items of 2^qsh queries
  g.npair = nqb / 2;
  g.nqb1 = nqb - 1;
  g.rcp_npair = 1.f / (float)g.npair;
  g.c = a.scale * 1.4426950408889634f;
  g.scale = a.scale;
  g.rcp_Hq = 1.f / (float)a.Hq;
  g.nitems = nqb * (unsigned)a.Hq * (unsigned)a.B;
  const unsigned members = g.nitems / 2;
  g.G = std::min<unsigned>((unsigned)(num_cus() * wgs_per_cu) / 8 * 8, (members + 7) / 8 * 8);
  g.G2m1 = 2 * g.G - 1;
  return g;
}

// Launch the assembly dQ kernel (same contract as fa_dkdv_asm).
int fa_dq_asm(const FaArgs& a, hipStream_t st) {
  if (!(enabled_mask() & 2) || !piamd_fa_asm_applies(&a)) return 0;
  FaDqArgs g = dq_args(a, 1);
  size_t sz = sizeof(g);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &g, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  hipError_t err = hipModuleLaunchKernel(g_fn[a.causal ? 3 : 2], g.G, 1, 1, 256, 1, 1, 0, st, nullptr, cfg);
  return err == hipSuccess ? 1 : -(int)err;
}

// Launch the assembly forward kernel (two workgroups per CU): O and lse (needed: lse non-null).
int fa_fwd_asm(const FaArgs& a, hipStream_t st) {
  if (!(enabled_mask() & 4) || !a.lse || reinterpret_cast<unsigned long long>(a.o) % 16 ||
      !piamd_fa_asm_applies(&a))
    return 0;
  FaArgs b = a;
  b.dq = a.o;  // output O (strides sob / sos / soh)
  b.delta = nullptr;
  // 4-wave kernel, two workgroups per CU (default); PIAMD_FA_FWD_NW=8: the 8-wave kernel (256
  // queries per workgroup, one per CU, half the K/V tile traffic per query) where the query
  // blocks pair up — measured 3 % slower at B96 S1024 H16 (695 vs 675 us, profiles/fa_asm_r6.txt)
  if (g_fwd_nw < 0) {
    const char* e = getenv("PIAMD_FA_FWD_NW");
    g_fwd_nw = e ? atoi(e) : 4;
  }
  const bool w8 = g_fwd_nw == 8 && a.Sq % 512 == 0;
  FaDqArgs g = dq_args(b, w8 ? 1 : 2, w8 ? 8 : 7);
  g.dq = a.o;
  g.nl = a.lse;
  g.nd = nullptr;
  g.dout = nullptr;
  size_t sz = sizeof(g);
  void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &g, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
  hipFunction_t f = w8 ? g_fn[a.causal ? 7 : 6] : g_fn[a.causal ? 5 : 4];
  hipError_t err = hipModuleLaunchKernel(f, g.G, 1, 1, w8 ? 512 : 256, 1, 1, 0, st, nullptr, cfg);
  return err == hipSuccess ? 1 : -(int)err;
}
