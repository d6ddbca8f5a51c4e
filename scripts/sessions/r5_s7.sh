# fp16 fused cross-entropy: numerics, fix-up rows, bf16 CE regression, fp16 / bf16 bench
scripts/gpu_session.sh \
 "t_ce|300|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_fp16_gpu.py tests/test_kernels_gpu.py tests/test_gemm_gpu.py -k 'lm_head or xent or fp16 or split'" \
 "bench_fp16b|300|python -u bench.py --steps 10 --warmup 3 --dtype float16" \
 "bench_bf16b|300|python -u bench.py --steps 10 --warmup 3"
