# column-strip GEMM for N = 256 q + r: numerics, the 1.5B N = 1600 probe, 1.5B bench
scripts/gpu_session.sh \
 "t_strip|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'strip'" \
 "nt_tail|300|python -u scripts/debug/nt_tail_probe.py" \
 "bench_1p5b|600|python -u bench.py --model gpt2-xl --micro-batch 60 --steps 2 --warmup 1" \
 "bench_1p5b_nostrip|600|env NSA_NT_STRIP=0 python -u bench.py --model gpt2-xl --micro-batch 60 --steps 2 --warmup 1"
