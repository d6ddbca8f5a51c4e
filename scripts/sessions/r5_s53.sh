scripts/gpu_session.sh \
 "t_ln|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k 'layernorm or dropout or fused_resid or checkpointing'" \
 "bench_c|300|python -u bench.py --steps 20 --warmup 5" \
 "prof_end3|300|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_end3 -o run -- python3 bench.py --steps 2 --warmup 2"
