# GPT-2 XL (1.5B) bf16 DDP=8 with activation checkpointing (BASELINE.json config 5).
# fp32 params+grads+2 Adam moments = 23.2 GiB; activations at B=12,T=1024 are tens
# of GB: both fit in 288 GB HBM3E, grad_ckpt buys headroom for larger micro-batches.
wandb_run_name = 'gpt2-1.5B'
n_layer = 48
n_head = 25
n_embd = 1600
batch_size = 12
block_size = 1024
gradient_accumulation_steps = 5 * 8
grad_ckpt = True
max_iters = 600000
lr_decay_iters = 600000
learning_rate = 2e-4
min_lr = 2e-5
eval_interval = 1000
eval_iters = 100
log_interval = 10
weight_decay = 1e-1
