# round 6: overlapped NT-GEMM epilogue (stores of tile t inside tile t+1's first K-tile),
# variant build vs default: bitwise check on odd shapes, then interleaved timing
scripts/gpu_session.sh \
 "r6_ovl_check|240|python -u scripts/debug/nt_alt_check.py build/variants/ovl/libnsa_kernels.so" \
 "r6_ovl_ab|400|python -u scripts/gemm_nt_ab.py --alt-lib build/variants/ovl/libnsa_kernels.so --shapes c_attn,attn.c_proj,c_fc,mlp.c_proj,c_attn.dx,c_fc.dx --rounds 7"
