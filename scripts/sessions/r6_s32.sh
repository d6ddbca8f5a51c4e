# round 6: weight gradients on a second stream for small models (wgrad_stream): trainer tests, char config on / off
CH="python -u train.py config/train_shakespeare_char.py --max_iters=300 --lr_decay_iters=300 --eval_interval=1000 --eval_iters=2 --log_interval=50"
scripts/gpu_session.sh \
 "r6_t_wgs|600|python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_train_gpu.py" \
 "r6_char_prep2|200|python -u -m nanosandbox_amd.data.prepare char --out data/shakespeare_char" \
 "r6_char_wgs_on|300|$CH --out_dir=/tmp/o1 --wgrad_stream=on" \
 "r6_char_wgs_off|300|$CH --out_dir=/tmp/o2 --wgrad_stream=off" \
 "r6_char_wgs_on2|300|$CH --out_dir=/tmp/o3 --wgrad_stream=on" \
 "r6_char_wgs_off2|300|$CH --out_dir=/tmp/o4 --wgrad_stream=off"
