# round 6: XENT epilogue without the padding mask except in the edge tile's copy
scripts/gpu_session.sh \
 "r6_t_xent4|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k 'xent or lm_head or loss'" \
 "r6_xclds_ab|400|python -u scripts/gemm_nt_ab.py --alt-lib build/variants/xc0/libnsa_kernels.so --xent --shapes lm_head --rounds 8 --reps 3"
