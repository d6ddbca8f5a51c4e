scripts/gpu_session.sh \
 "t_ce2|300|python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_fp16_gpu.py tests/test_kernels_gpu.py tests/test_gemm_gpu.py -k 'lm_head or xent or fp16 or split'" \
 "bench_fp16c|300|python -u bench.py --steps 10 --warmup 3 --dtype float16"
