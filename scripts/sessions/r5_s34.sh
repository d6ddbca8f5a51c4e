# full GPU suite + smoke + headline bench on the current tree
scripts/gpu_session.sh \
 "t_all|1000|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/" \
 "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench|300|python -u bench.py"
