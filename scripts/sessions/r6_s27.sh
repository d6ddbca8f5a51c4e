# round 6: XDEF with the SGPR hazard nop; NaN map, tests, A/B, plain OVL2 re-check
V=build/variants/xdef0/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_xent_nan2|200|python -u scripts/debug/xent_nan_map.py" \
 "r6_t_xdef2|400|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k 'xent or lm_head or loss or nt4'" \
 "r6_xdef_ab2|400|python -u scripts/gemm_nt_ab.py --alt-lib $V --xent --ovls 2 --shapes lm_head,c_attn --rounds 8 --reps 3"
