# round 6: sorted scatter-add row kernel walks each segment once for both 512-column halves; tests and same-box traces
P=$GRAFT_REPO_ROOT/gpurun_out
V=$GRAFT_REPO_ROOT/build/variants/segold/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_t_seg|400|python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_train_gpu.py" \
 "r6_prof_seg_new|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $P/r6_prof_seg_new -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --calib-seconds 0" \
 "r6_prof_seg_old|300|cd /tmp && export TMPDIR=/tmp && export NSA_KERNEL_LIB=$V && rocprofv3 --kernel-trace --stats --output-format csv -d $P/r6_prof_seg_old -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --calib-seconds 0"
