# GPT-2 XL (1.5B) bf16 DDP=8 (BASELINE.json config 5).
# fp32 params + grads + 2 Adam moments = 23.2 GiB; the activations of a 12 x 1024-token
# micro-step are ~35 GiB and of a 60 x 1024 one ~170 GiB: both stay resident in the
# 288 GB of HBM3E, so activation checkpointing is left to the HBM planner
# (hbm_plan=True: utils/memory.py turns it on only when the estimate exceeds free
# memory, e.g. at 120 x 1024 tokens per micro-step).  Checkpointing when it is not
# needed costs a third of the forward: 5043 vs 6750 ms/step at 60 x 1024.
# grad_ckpt = True forces it.
wandb_run_name = 'gpt2-1.5B'
n_layer = 48
n_head = 25
n_embd = 1600
batch_size = 12
block_size = 1024
gradient_accumulation_steps = 5 * 8
grad_ckpt = False
max_iters = 600000
lr_decay_iters = 600000
learning_rate = 2e-4
min_lr = 2e-5
eval_interval = 1000
eval_iters = 100
log_interval = 10
weight_decay = 1e-1
