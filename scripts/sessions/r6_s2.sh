scripts/gpu_session.sh \
 "r6_keysort|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'keysort or embedding or lm_head_dw_fix_sorted'" \
 "r6_hazard|400|python -u scripts/debug/overlap_hazard.py --nwg 16,32,64 --spin-us 400 --reps 6 --json gpurun_out/r6_hazard.json" \
 "r6_bench20b|300|python -u bench.py --steps 20 --warmup 5"
