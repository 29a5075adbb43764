// Argument block of the flash-attention entry points (piamd_fa_fwd / piamd_fa_bwd). Shared by
// the kernels (flash_attn.h), the Python binding (ops/_lib.py mirrors it with ctypes) and the
// native predictor (csrc/native/fast_ops.hip).
#pragma once

struct FaArgs {
  const void *q, *k, *v;
  void* o;
  float* lse;
  const void* dout;
  float* delta;  // backward scratch: 2 x rows f32 (−δ, −lse/scale)
  void *dq, *dk, *dv;
  const void* mask;  // additive, input dtype; null = none
  const int *cu_q, *cu_k;
  int B, Sq, Sk, Hq, Hk, D, ltot, causal;
  long long sqb, sqs, sqh, skb, sks, skh, svb, svs, svh, sob, sos, soh;
  long long smb, smh, smq;  // mask strides (elements; 0 = broadcast)
  float scale, p_drop;
  unsigned long long seed, offset;
  int map;  // backward grid order, bit 0 dQ / bit 1 dK-dV kernel: 0 = the blocks of one (batch,
            // head) spread over the grid, 1 = grouped on one XCD (fa_map) so they share that head's
            // K/V (dQ) or Q/dO (dK-dV) panels in L2 (set by the entry point)
  void* ds;  // reserved (ABI slot of the removed stored-dS backward; always null)
};
