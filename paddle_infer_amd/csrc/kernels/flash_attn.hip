// Flash attention entry points + the bf16 instantiations (kernels: flash_attn.h; fp16
// instantiations: flash_attn_f16.hip, compiled in parallel).
// piamd-hipcc-flags: -mllvm -amdgpu-mfma-vgpr-form
// (MFMA results in arch VGPRs: the one-wave-per-SIMD dK/dV kernel otherwise keeps its S / dP
// accumulators in AGPRs and copies them to VGPRs for the softmax every tile)
#include "flash_attn.h"

int fa_fwd_f16(const FaArgs& a, hipStream_t st);
int fa_bwd_f16(const FaArgs& a, hipStream_t st);

// Head dims: 64 / 96 / 128 both ways; 256 (the wide forward) forward only — the backward of wider
// heads is ops/attention.py `_bwd_wide_own` (batched own-GEMM products over the forward's lse).
static int fa_check(const FaArgs& a, bool fwd) {
  if (a.Hk <= 0 || a.Hq % a.Hk || (a.cu_q && !a.cu_k)) return (int)hipErrorInvalidValue;
  if (a.D != 64 && a.D != 96 && a.D != 128 && !(fwd && a.D == 256)) return (int)hipErrorInvalidValue;
  if (a.p_drop < 0.f || a.p_drop >= 1.f) return (int)hipErrorInvalidValue;
  if (a.mask && ((a.smb | a.smh | a.smq) & 3)) return (int)hipErrorInvalidValue;  // 8-B mask reads
  return 0;
}

// Forward. q/k/v/o [B, S, H, D] (element strides b/s/h, d contiguous) or, with cu_q/cu_k (int32
// [B+1] device row offsets), packed [total, H, D] with Sq / Sk = the longest sequence.
// lse: f32 [B, Hq, Sq] (packed: [Hq, ltot]), nullable. f16: 0 = bf16, 1 = fp16.
PIAMD_EXPORT int piamd_fa_fwd(const FaArgs* args, int f16, hipStream_t stream) {
  FaArgs a = *args;
  if (int e = fa_check(a, true)) return e;
  a.map = 0;
  if (a.cu_q) a.sqb = a.skb = a.svb = a.sob = 0;
  if (a.B == 0 || a.Sq == 0) return 0;
  if (a.Sk == 0) return (int)hipErrorInvalidValue;
  if (!f16 && fa_fwd_asm(a, stream) == 1) return 0;  // hand-scheduled kernel (fa_asm_host.hip)
  return f16 ? fa_fwd_f16(a, stream) : fa::launch_fwd<false>(a, stream);
}

// Backward. q/dq share (sqb, sqs, sqh); k/dk (skb, sks, skh); v/dv (svb, svs, svh); o and dout
// share (sob, sos, soh). delta: f32 workspace shaped like lse. Same dropout seed/offset and mask
// as the forward.
PIAMD_EXPORT int piamd_fa_bwd(const FaArgs* args, int f16, hipStream_t stream) {
  FaArgs a = *args;
  if (int e = fa_check(a, false)) return e;
  a.map = fa::fa_bwd_map(a);
  if (a.cu_q) {
    a.sqb = a.skb = a.svb = a.sob = 0;
  }
  if (a.B == 0 || a.Sq == 0 || a.Sk == 0) return 0;
  return f16 ? fa_bwd_f16(a, stream) : fa::launch_bwd<false>(a, stream);
}
