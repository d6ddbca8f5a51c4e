# round 6: cross-entropy epilogue with the four rows' sums reduced together and the padding
# mask only in the edge tile's copy; GEMM + loss tests, XENT A/B, bench
scripts/gpu_session.sh \
 "r6_t_gemm2|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py -k 'nt4 or xent or lm_head or loss'" \
 "r6_t_fp16x|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_fp16_gpu.py -k 'lm_head or xent or loss'" \
 "r6_xent_ab|400|python -u scripts/gemm_nt_ab.py --alt-lib build/variants/growoff/libnsa_kernels.so --xent --epi --shapes lm_head,c_fc --rounds 7 --reps 3" \
 "r6_bench20e|300|python -u bench.py --steps 20 --warmup 5"
