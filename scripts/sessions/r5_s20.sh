# profile the reference's own workload (char config, 6L/384C, 64 x 256 tokens, dropout 0.2)
scripts/gpu_session.sh \
 "char_prep|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "prof_char|400|cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_char -o run -- python3 train.py config/train_shakespeare_char.py --max_iters=40 --lr_decay_iters=40 --eval_interval=1000 --eval_iters=2 --out_dir=/tmp/out-sc --log_interval=10"
