# GPT-2 medium (350M): the multi-Pod StatefulSet config of BASELINE.json
# (nnodes=8 x 1 GPU, c10d rendezvous through the headless Service).
wandb_run_name = 'gpt2-350M'
n_layer = 24
n_head = 16
n_embd = 1024
batch_size = 12
block_size = 1024
gradient_accumulation_steps = 5 * 8
max_iters = 600000
lr_decay_iters = 600000
learning_rate = 3e-4
min_lr = 3e-5
eval_interval = 1000
eval_iters = 200
log_interval = 10
weight_decay = 1e-1
