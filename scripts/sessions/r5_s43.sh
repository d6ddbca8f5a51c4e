# XENT epilogue: packed shift / row sum (default build) vs scalar (variant xent_pk0); kernel traces
scripts/gpu_session.sh \
 "t_xent|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k 'lm_head'" \
 "prof_pk1|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_pk1 -o run -- python3 bench.py --steps 3 --warmup 2" \
 "prof_pk0|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && NSA_KERNEL_LIB=build/variants/xent_pk0/libnsa_kernels.so rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_pk0 -o run -- python3 bench.py --steps 3 --warmup 2" \
 "prof_pk1b|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_pk1b -o run -- python3 bench.py --steps 3 --warmup 2"
