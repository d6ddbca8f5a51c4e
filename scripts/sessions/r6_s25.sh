# round 6: XENT rows 4-7 stored from the next tile's first K-tile (XDEF)
V=build/variants/xdef0/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_t_xdef|400|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k 'xent or lm_head or loss'" \
 "r6_xdef_ab|400|python -u scripts/gemm_nt_ab.py --alt-lib $V --xent --shapes lm_head --rounds 8 --reps 3"
