# round 6: kernel trace of the N = 8 per-rank step (emulated collectives) to find the gap to the 1-GPU per-token rate
scripts/gpu_session.sh \
 "r6_pr8b|300|python -u bench.py --per-rank-of 8 --steps 10 --warmup 3 --calib-seconds 1" \
 "r6_prof_pr8|400|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6_prof_pr8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --per-rank-of 8 --steps 4 --warmup 2 --calib-seconds 0"
