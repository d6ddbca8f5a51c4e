# loss parity vs fp32 HF GPT-2 on the current tree (fp16: fused cross-entropy, split8h gradients, v5 forward)
scripts/gpu_session.sh \
 "parity_fp16|900|python -u scripts/loss_parity.py --steps 300 --batch 16 --dtype float16 --out gpurun_out/r5_loss_parity_fp16b.jsonl" \
 "parity_bf16|900|python -u scripts/loss_parity.py --steps 300 --batch 16 --out gpurun_out/r5_loss_parity_bf16b.jsonl"
