# round 6: step after OVL2 + XDEF + DDEF; full GPU suite; bench; per-rank 8; 1.5B
scripts/gpu_session.sh \
 "r6_pytest_gpu2|900|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu" \
 "r6_bench20h|300|python -u bench.py --steps 20 --warmup 5" \
 "r6_pr8c|300|python -u bench.py --per-rank-of 8 --steps 10 --warmup 3 --calib-seconds 0" \
 "r6_xl_res_c|600|python -u bench.py --model gpt2-xl --micro-batch 60 --steps 2 --warmup 1 --calib-seconds 0"
