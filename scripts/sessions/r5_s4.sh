# fp16 kernels: numerics, bf16 regression, bench in both dtypes
scripts/gpu_session.sh \
 "t_fp16|400|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_fp16_gpu.py" \
 "t_bf16|600|python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_optim_gpu.py" \
 "bench_bf16|300|python -u bench.py --steps 10 --warmup 3" \
 "bench_fp16|300|python -u bench.py --steps 10 --warmup 3 --dtype float16"
