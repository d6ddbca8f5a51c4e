# round-5 end-of-round verification on one fresh box
scripts/gpu_session.sh \
 "t_all|1000|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/" \
 "smoke|200|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench20|300|python -u bench.py --steps 20 --warmup 5" \
 "bench_fp16|300|python -u bench.py --dtype float16 --steps 10 --warmup 3" \
 "bench_350m|400|python -u bench.py --model gpt2-medium --steps 3 --warmup 1" \
 "bench_1p5b|600|python -u bench.py --model gpt2-xl --steps 2 --warmup 1" \
 "char_prep|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "char_train|600|python -u train.py config/train_shakespeare_char.py --max_iters=2000 --lr_decay_iters=2000 --eval_interval=500 --out_dir=/tmp/out-shakespeare-char"
