# round 6: micro-batch 120 x 4 (default) vs 240 x 2 on the current tree, interleaved
scripts/gpu_session.sh \
 "r6_mb120a|300|python -u bench.py --steps 10 --warmup 3 --calib-seconds 1" \
 "r6_mb240a|300|python -u bench.py --steps 10 --warmup 3 --calib-seconds 1 --micro-batch 240" \
 "r6_mb120b|300|python -u bench.py --steps 10 --warmup 3 --calib-seconds 1" \
 "r6_mb240b|300|python -u bench.py --steps 10 --warmup 3 --calib-seconds 1 --micro-batch 240"
