# round 6: NT GEMM without the SLP vectorizer (its epilogues pack 2048 more f32 ops into v_pk_* with it)
scripts/gpu_session.sh \
 "r6_ntslp_ab|600|python -u scripts/gemm_nt_ab.py --alt-lib build/variants/nt_noslp/libnsa_kernels.so --epi --xent --shapes c_attn,mlp.c_proj,c_fc,mlp.c_proj.dx,lm_head --rounds 7 --reps 3"
