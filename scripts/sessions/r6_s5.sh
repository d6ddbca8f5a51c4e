scripts/gpu_session.sh \
 "r6_pr8|300|python -u bench.py --per-rank-of 8 --steps 10 --warmup 3 --calib-seconds 1" \
 "r6_pr8_nocomm|300|python -u bench.py --per-rank-of 8 --steps 10 --warmup 3 --emu-busbw 1e9 --calib-seconds 0" \
 "r6_pr4|300|python -u bench.py --per-rank-of 4 --steps 6 --warmup 2 --calib-seconds 0" \
 "r6_pr2|300|python -u bench.py --per-rank-of 2 --steps 4 --warmup 2 --calib-seconds 0" \
 "r6_xl_res|600|python -u bench.py --model gpt2-xl --micro-batch 60 --steps 2 --warmup 1 --calib-seconds 1" \
 "r6_xl_ckpt60|600|python -u bench.py --model gpt2-xl --grad-ckpt --micro-batch 60 --steps 2 --warmup 1 --calib-seconds 0" \
 "r6_xl_ckpt120|600|python -u bench.py --model gpt2-xl --grad-ckpt --micro-batch 120 --steps 2 --warmup 1 --calib-seconds 0"
