# round 6: full GPU test suite, smoke, bench at the headline and at 350M on the current tree
scripts/gpu_session.sh \
 "r6_pytest_gpu|900|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu" \
 "r6_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r6_bench20f|300|python -u bench.py --steps 20 --warmup 5" \
 "r6_bench_350m|400|python -u bench.py --model gpt2-medium --steps 3 --warmup 1 --calib-seconds 0"
