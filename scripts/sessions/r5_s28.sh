# fp16: split-plane LN gradients, v5 forward, fused cross-entropy default; tests + bench + profile
scripts/gpu_session.sh \
 "t_fp16|400|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp16_gpu.py" \
 "t_ln|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'layernorm or split or flash_fwd_exact or deferred'" \
 "bench_fp16|400|python -u bench.py --dtype float16 --steps 10 --warmup 3" \
 "bench_bf16|400|python -u bench.py --steps 10 --warmup 3" \
 "prof_fp16|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_fp16b -o run -- python3 bench.py --dtype float16 --steps 2 --warmup 2"
