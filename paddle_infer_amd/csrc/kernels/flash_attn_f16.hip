// fp16 instantiations of the flash attention kernels (flash_attn.h); entry points in flash_attn.hip.
// piamd-hipcc-flags: -mllvm -amdgpu-mfma-vgpr-form
// (MFMA results in arch VGPRs: the one-wave-per-SIMD dK/dV kernel otherwise keeps its S / dP
// accumulators in AGPRs and copies them to VGPRs for the softmax every tile)
#include "flash_attn.h"

int fa_fwd_f16(const FaArgs& a, hipStream_t st) { return fa::launch_fwd<true>(a, st); }
int fa_bwd_f16(const FaArgs& a, hipStream_t st) { return fa::launch_bwd<true>(a, st); }
