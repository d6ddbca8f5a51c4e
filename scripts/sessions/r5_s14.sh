# fused attention backward (v4): numerics, A/B against v3, bench
scripts/gpu_session.sh \
 "t_fused|300|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'fused_matches or bwd_exact_structure'" \
 "ab_fused|300|python -u scripts/attn_ab.py --fwd 'auto:' --bwd 'v3:bwd=v3;v4:bwd=v4' --rounds 9" \
 "bench_fused|300|NSA_FLASH_BWD=v4 python -u bench.py --steps 10 --warmup 3"
