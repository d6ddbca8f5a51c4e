# round 6: final verification — full GPU suite, smoke, bf16 bench 20/5, fp16 bench, per-rank N=8 projection, char config
CH="python -u train.py config/train_shakespeare_char.py --max_iters=300 --lr_decay_iters=300 --eval_interval=1000 --eval_iters=2 --log_interval=50 --out_dir=/tmp/ofin"
scripts/gpu_session.sh \
 "r6_fin_pytest|1000|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu" \
 "r6_fin_smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r6_fin_bench|300|python -u bench.py --steps 20 --warmup 5" \
 "r6_fin_fp16|300|python -u bench.py --steps 10 --warmup 3 --dtype float16" \
 "r6_fin_pr8|300|python -u bench.py --per-rank-of 8 --steps 10 --warmup 3" \
 "r6_fin_char_prep|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "r6_fin_char|300|$CH"
