scripts/gpu_session.sh \
 "prof_fused|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fused2 -o run -- python3 $GRAFT_REPO_ROOT/scripts/attn_ab.py --fwd auto: --bwd 'v4:bwd=v4' --rounds 2 --iters 3"
