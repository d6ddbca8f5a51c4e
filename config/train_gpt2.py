# GPT-2 (124M) training; the benchmark config of this repo (BASELINE.json).
# 12 batch size * 1024 block size * 5 gradaccum * 8 GPUs = 491,520 tokens/iter
# (nanoGPT config/train_gpt2.py semantics)

wandb_log = False
wandb_project = 'owt'
wandb_run_name = 'gpt2-124M'

batch_size = 12
block_size = 1024
gradient_accumulation_steps = 5 * 8

# this makes total number of tokens be 300B
max_iters = 600000
lr_decay_iters = 600000

# eval stuff
eval_interval = 1000
eval_iters = 200
log_interval = 10

# weight decay
weight_decay = 1e-1
