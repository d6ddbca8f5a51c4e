scripts/gpu_session.sh \
 "t_fp16|400|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp16_gpu.py" \
 "bench_fp16|400|python -u bench.py --dtype float16 --steps 10 --warmup 3" \
 "bench_bf16|400|python -u bench.py --steps 10 --warmup 3" \
 "bench_fp16b|400|python -u bench.py --dtype float16 --steps 10 --warmup 3"
