# round 6: overlapped epilogue for fp16 outputs too; fp16 + bf16 GEMM tests, fp16 bench
scripts/gpu_session.sh \
 "r6_t_gemm5|400|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_fp16_gpu.py" \
 "r6_bench_fp16|300|python -u bench.py --dtype float16 --steps 20 --warmup 5"
