# round 6: last check of the final tree (after the one-walk scatter-add): full GPU suite, smoke, bench
scripts/gpu_session.sh \
 "r6_last_pytest|1000|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu" \
 "r6_last_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r6_last_bench|300|python -u bench.py --steps 20 --warmup 5"
