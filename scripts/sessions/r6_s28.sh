# round 6: GELU' rows 4-7 stored from the next tile's first K-tile (DDEF)
V=build/variants/ddef0/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_t_ddef|400|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_fp16_gpu.py tests/test_train_gpu.py" \
 "r6_ddef_ab|400|python -u scripts/gemm_nt_ab.py --alt-lib $V --epi --shapes mlp.c_proj.dx --rounds 9"
