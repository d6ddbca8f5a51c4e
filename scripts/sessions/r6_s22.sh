# round 6: OVL2 (rows 4-7 of the previous tile stored in the second K-tile) vs OVL vs off
V=build/variants/ovl2/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_ovl2_check|240|ALT_EPI=16384 python -u scripts/debug/nt_alt_check.py $V" \
 "r6_ovl2_ab|500|python -u scripts/gemm_nt_ab.py --alt-lib $V --alt-ovl 1 --ovls 1,2 --shapes c_attn,attn.c_proj,c_attn.dx,mlp.c_proj,c_fc.dx --rounds 9"
