scripts/gpu_session.sh \
 "t_lds|400|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k 'embedding or lm_head or deterministic'" \
 "char_prep|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "char_train|400|python -u train.py config/train_shakespeare_char.py --max_iters=500 --lr_decay_iters=500 --eval_interval=250 --eval_iters=20 --out_dir=/tmp/out-sc --log_interval=50" \
 "prof_char|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_char6 -o run -- python3 train.py config/train_shakespeare_char.py --max_iters=40 --lr_decay_iters=40 --eval_interval=1000 --eval_iters=2 --out_dir=/tmp/out-sc --log_interval=10"
