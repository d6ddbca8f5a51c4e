scripts/gpu_session.sh \
 "t_fused2|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'fused_matches or bwd_exact_structure'" \
 "prof_fused3|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused3 -o run -- python3 $GRAFT_REPO_ROOT/scripts/attn_ab.py --fwd auto: --bwd 'v4:bwd=v4' --rounds 2 --iters 3"
