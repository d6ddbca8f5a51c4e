scripts/gpu_session.sh \
 "bench_a|300|python -u bench.py --steps 20 --warmup 5" \
 "prof_end|300|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_end2 -o run -- python3 bench.py --steps 2 --warmup 2" \
 "bench_b|300|python -u bench.py --steps 20 --warmup 5"
