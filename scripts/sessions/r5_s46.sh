# resid dropout fused into the add + LayerNorm kernel: tests, char config training + profile, GPT-2 bench
scripts/gpu_session.sh \
 "t_drop|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_train_gpu.py -k 'dropout or layernorm or split or train'" \
 "char_prep|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "char_train|400|python -u train.py config/train_shakespeare_char.py --max_iters=500 --lr_decay_iters=500 --eval_interval=250 --eval_iters=20 --out_dir=/tmp/out-sc --log_interval=50" \
 "char_train_sep|400|env NSA_LN_DROPOUT=0 python -u train.py config/train_shakespeare_char.py --max_iters=500 --lr_decay_iters=500 --eval_interval=250 --eval_iters=20 --out_dir=/tmp/out-sc2 --log_interval=50" \
 "bench|300|python -u bench.py --steps 10 --warmup 3"
