scripts/gpu_session.sh \
 "r6_hazard_g1|300|python -u scripts/debug/overlap_hazard.py --grid-mult 1 --nwg 16,32,64 --reps 8 --json gpurun_out/r6_hazard_g1.json" \
 "r6_hazard_g2|300|python -u scripts/debug/overlap_hazard.py --grid-mult 2 --nwg 16,32,64 --reps 8 --json gpurun_out/r6_hazard_g2.json" \
 "r6_hazard_g4|300|python -u scripts/debug/overlap_hazard.py --grid-mult 4 --nwg 16,32,64 --reps 8 --json gpurun_out/r6_hazard_g4.json" \
 "r6_bench_g2|300|NSA_NT4_GRID_MULT=2 python -u bench.py --steps 10 --warmup 3 --calib-seconds 1" \
 "r6_bench_g1|300|NSA_NT4_GRID_MULT=1 python -u bench.py --steps 10 --warmup 3 --calib-seconds 1"
