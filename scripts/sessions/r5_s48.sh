# weight-grad epilogue anatomy: kernel trace of the atomic and stored-partials forms
scripts/gpu_session.sh \
 "prof_wg|300|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_wg -o run -- python3 scripts/debug/wgrad_det_ab.py"
