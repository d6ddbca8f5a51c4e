# sorted onehot dW term (target passed to the row loader): tests, kernel profile, deterministic char run
scripts/gpu_session.sh \
 "t_xe|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k 'lm_head or embedding or deterministic'" \
 "prof|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_xfix2 -o run -- python3 bench.py --steps 2 --warmup 2" \
 "char_prep|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "char_det|400|python -u train.py config/train_shakespeare_char.py --max_iters=200 --lr_decay_iters=200 --eval_interval=1000 --eval_iters=2 --out_dir=/tmp/out-scd --log_interval=50 --deterministic=True"
