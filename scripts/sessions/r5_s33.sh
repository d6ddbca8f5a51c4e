# long context: v5 (auto) vs v4 forward, same box
scripts/gpu_session.sh \
 "long4096_v5|400|python -u bench.py --block-size 4096 --micro-batch 30 --steps 2 --warmup 1" \
 "long4096_v4|400|env NSA_FLASH_FWD=v4 python -u bench.py --block-size 4096 --micro-batch 30 --steps 2 --warmup 1" \
 "long8192_v5|500|python -u bench.py --block-size 8192 --micro-batch 15 --steps 2 --warmup 1" \
 "long8192_v4|500|env NSA_FLASH_FWD=v4 python -u bench.py --block-size 8192 --micro-batch 15 --steps 2 --warmup 1"
