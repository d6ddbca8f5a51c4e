# round 6: end-of-round larger models (no-regression check): 350M and 1.5B resident
scripts/gpu_session.sh \
 "r6_fin_350m|400|python -u bench.py --model gpt2-medium --steps 3 --warmup 1" \
 "r6_fin_xl|600|python -u bench.py --model gpt2-xl --micro-batch 60 --steps 2 --warmup 1"
