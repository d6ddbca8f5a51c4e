# the reference's own workload (char config) and long-context benches on the round-5 tree
scripts/gpu_session.sh \
 "char_prep|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "char_train|600|python -u train.py config/train_shakespeare_char.py --max_iters=2000 --lr_decay_iters=2000 --eval_interval=500 --out_dir=/tmp/out-shakespeare-char" \
 "bench_long4096|400|python -u bench.py --block-size 4096 --micro-batch 30 --steps 2 --warmup 1" \
 "bench_long8192|500|python -u bench.py --block-size 8192 --micro-batch 15 --steps 2 --warmup 1"
