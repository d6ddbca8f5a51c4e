scripts/gpu_session.sh \
 "t_all|1000|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/" \
 "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench20|300|python -u bench.py --steps 20 --warmup 5" \
 "bench_1p5b|600|python -u bench.py --model gpt2-xl --steps 2 --warmup 1"
