# LN split/plain bitwise after explicit FMAs; forward v4 vs v5 long A/B; round-5 step profile
scripts/gpu_session.sh \
 "t_ln|300|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'layernorm or split or exact_structure or pair_matches'" \
 "ab_fwd45|300|python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5' --bwd 'v3:bwd=v3' --rounds 15" \
 "bench_r5|300|python -u bench.py --steps 10 --warmup 3" \
 "prof_r5|400|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2"
