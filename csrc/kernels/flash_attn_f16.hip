// fp16 build of the flash-attention kernels (nanoGPT's dtype='float16'): the same source as
// flash_attn.hip with fp16 Q/K/V/O/dO/dQKV, fp16 P / dS MFMA operands
// (v_mfma_f32_32x32x16_f16, the bf16 rate on gfx950) and fp32 softmax statistics.  Entry
// points: nsa_flash_fwd_h, nsa_flash_bwd2_h, nsa_rng_advance_attn_h(_set); the kernel
// selection is the bf16 build's (nsa_flash_config_ptr).
#define NSA_FA_F16 1
#include "flash_attn.hip"
