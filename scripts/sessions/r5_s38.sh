# sorted onehot dW term of the fused cross-entropy + embedding on segsum.h: tests, char training, GPT-2 bench
scripts/gpu_session.sh \
 "t_xe|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k 'lm_head or embedding or deterministic'" \
 "char_prep|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "char_train|400|python -u train.py config/train_shakespeare_char.py --max_iters=300 --lr_decay_iters=300 --eval_interval=1000 --eval_iters=2 --out_dir=/tmp/out-sc --log_interval=50" \
 "bench|300|python -u bench.py --steps 10 --warmup 3" \
 "bench_atomic|300|env NSA_XENT_FIX_SORTED=0 python -u bench.py --steps 10 --warmup 3" \
 "prof|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_xfix -o run -- python3 bench.py --steps 2 --warmup 2"
