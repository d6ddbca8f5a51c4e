# The reference's CPU smoke test (notebooks/colab_nanoGPT_companion.ipynb:70-79):
# tiny 2L/2H/64C char model, 50 iterations, gloo/CPU.
out_dir = 'out-smoke-cpu'
dataset = 'shakespeare_char'
eval_interval = 50
log_interval = 1
block_size = 128
batch_size = 16
n_layer = 2
n_head = 2
n_embd = 64
max_iters = 50
lr_decay_iters = 50
dropout = 0.0
device = 'cpu'
compile = False
backend = 'gloo'
eval_iters = 20
gradient_accumulation_steps = 1
always_save_checkpoint = False
learning_rate = 1e-3
min_lr = 1e-4
warmup_iters = 5
