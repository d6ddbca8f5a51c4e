# micro-batch size at 1 GPU: 120 x 4 (auto) vs 240 x 2 vs 480 x 1 (fewer partial CU rounds in the N = 768 GEMMs)
scripts/gpu_session.sh \
 "mb120|300|python -u bench.py --steps 6 --warmup 2" \
 "mb240|300|python -u bench.py --steps 6 --warmup 2 --micro-batch 240" \
 "mb480|400|python -u bench.py --steps 6 --warmup 2 --micro-batch 480" \
 "mb120b|300|python -u bench.py --steps 6 --warmup 2"
