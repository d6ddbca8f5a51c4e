# full GPU suite; loss parity bf16 / fp16 vs fp32 HF; 350M / 1.5B benches on the round-5 tree
scripts/gpu_session.sh \
 "t_all|900|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/" \
 "parity_bf16|900|python -u scripts/loss_parity.py --steps 300 --batch 16 --out gpurun_out/r5_loss_parity_bf16.jsonl" \
 "parity_fp16|900|python -u scripts/loss_parity.py --steps 300 --batch 16 --dtype float16 --out gpurun_out/r5_loss_parity_fp16.jsonl" \
 "bench_350m|400|python -u bench.py --model gpt2-medium --steps 3 --warmup 1" \
 "bench_1p5b|600|python -u bench.py --model gpt2-xl --steps 2 --warmup 1"
