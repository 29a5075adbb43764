// fp16 instantiations of the flash attention kernels (flash_attn.h); entry points in flash_attn.hip.
#include "flash_attn.h"

int fa_fwd_f16(const FaArgs& a, hipStream_t st) { return fa::launch_fwd<true>(a, st); }
int fa_bwd_f16(const FaArgs& a, hipStream_t st) { return fa::launch_bwd<true>(a, st); }
