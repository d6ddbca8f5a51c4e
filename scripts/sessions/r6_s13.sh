# round 6: step kernel trace on the current tree (compare with r6_prof1 from the round start)
scripts/gpu_session.sh \
 "r6_prof_step2|400|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6_prof2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --calib-seconds 1"
