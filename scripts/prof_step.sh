set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
NSA_GEMM_TUNE_VERBOSE=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_a.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof3.log 2>&1
