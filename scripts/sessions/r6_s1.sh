scripts/gpu_session.sh \
 "r6_bench20|300|python -u bench.py --steps 20 --warmup 5" \
 "r6_prof_step|400|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6_prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2" \
 "r6_char|300|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char && python -u train.py config/train_shakespeare_char.py --max_iters=300 --lr_decay_iters=300 --eval_interval=1000 --log_interval=50 --compile=False"
