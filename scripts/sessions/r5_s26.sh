# fp16 step profile (fused fp16 cross-entropy on) to locate the fp16 - bf16 gap
scripts/gpu_session.sh \
 "prof_fp16|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && NSA_XENT_F16=1 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fp16 -o run -- python3 bench.py --dtype float16 --steps 2 --warmup 2" \
 "prof_bf16|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_bf16 -o run -- python3 bench.py --steps 2 --warmup 2"
