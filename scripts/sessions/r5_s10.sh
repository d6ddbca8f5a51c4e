# full GPU suite (round-end tier rehearsal) + bench
scripts/gpu_session.sh \
 "t_all|900|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/" \
 "bench_fp16d|300|python -u bench.py --steps 10 --warmup 3 --dtype float16"
