# round 6: end-of-round step trace (OVL2 + XDEF + DDEF default) and the char config, timed and traced
P=$GRAFT_REPO_ROOT/gpurun_out
scripts/gpu_session.sh \
 "r6_prof3|400|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $P/r6_prof3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --calib-seconds 1" \
 "r6_char_prep|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "r6_char_train|400|python -u train.py config/train_shakespeare_char.py --max_iters=500 --lr_decay_iters=500 --eval_interval=250 --eval_iters=20 --out_dir=/tmp/out-sc --log_interval=50" \
 "r6_prof_char|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $P/r6_prof_char -o run -- python3 train.py config/train_shakespeare_char.py --max_iters=40 --lr_decay_iters=40 --eval_interval=1000 --eval_iters=2 --out_dir=/tmp/out-sc2 --log_interval=10"
