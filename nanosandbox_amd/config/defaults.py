"""Default training configuration.

The nanoGPT keys and defaults are the contract of SURVEY.md §2.9.1 (upstream
``train.py`` globals, driven by reference ``notebooks/colab_nanoGPT_companion.ipynb:70-79``).
Keys added by this framework are typed so that the configurator's strict type
check keeps working (``--ddp_bucket_mb=128`` is an int, ``--data_dir=/data/x``
a str, ...).
"""

from __future__ import annotations

TRAIN_DEFAULTS = dict(
    # I/O
    out_dir="out",
    eval_interval=2000,
    log_interval=1,
    eval_iters=200,
    eval_only=False,
    always_save_checkpoint=True,
    init_from="scratch",  # 'scratch' | 'resume' | 'gpt2*' (needs local HF weights)
    # wandb logging (kept for CLI compatibility; wandb is not installed -> no-op with a warning)
    wandb_log=False,
    wandb_project="owt",
    wandb_run_name="gpt2",
    # data
    dataset="openwebtext",
    gradient_accumulation_steps=5 * 8,
    batch_size=12,
    block_size=1024,
    # model
    n_layer=12,
    n_head=12,
    n_embd=768,
    dropout=0.0,
    bias=False,
    # adamw optimizer
    learning_rate=6e-4,
    max_iters=600000,
    weight_decay=1e-1,
    beta1=0.9,
    beta2=0.95,
    grad_clip=1.0,
    # learning rate decay settings
    decay_lr=True,
    warmup_iters=2000,
    lr_decay_iters=600000,
    min_lr=6e-5,
    # DDP settings
    backend="nccl",  # 'nccl' binds to RCCL on ROCm; 'gloo' for CPU
    # system
    device="cuda",
    dtype="bfloat16",
    compile=True,  # no Triton/Inductor here: True = capture the fwd+bwd micro-step as a HIP graph
    # ---- keys added by nanosandbox_amd (all typed) ----
    data_dir="",  # root holding <dataset>/train.bin; '' -> ./data (nanoGPT) ; k8s: /data/datasets
    seed=1337,
    ddp_impl="flat",  # 'flat' (our bucketed RCCL reducer) | 'torch' (torch DDP)
    ddp_bucket_mb=64,  # gradient bucket cap; 64 MiB suits ring all-reduce over 7 xGMI links
    grad_reduce_dtype="float32",  # 'float32' | 'bfloat16' (compressed all-reduce)
    rccl_report=True,  # at DDP start: per-peer RCCL transport (P2P/SHM/NET) + 64 MiB all-reduce bus bandwidth
    grad_ckpt=False,  # recompute each Block in backward (activation checkpointing)
    recompute_mlp=False,  # selective recomputation: MLPs keep only their input, redo c_fc + GELU in backward
    hbm_plan=True,  # grad_ckpt=False: turn checkpointing on only if the activation estimate exceeds free HBM
    fp32_residual=True,  # residual stream + its gradient in fp32 (nanoGPT autocast contract); False: bf16
    deterministic=False,  # bitwise-reproducible steps: no fp32 atomics (fixed-order split-K, sorted embedding bwd)
    metrics_jsonl=True,  # write <out_dir>/metrics.jsonl
    tensorboard_dir="",  # '' disables; else tfevents written to <tensorboard_dir>/<run>
    auto_resume=False,  # resume from <out_dir>/ckpt.pt if it exists (elastic restarts)
    fault_inject_iter=-1,  # >=0: rank fault_inject_rank raises at that iteration (tests)
    fault_inject_rank=-1,
    profile=False,  # torch.profiler trace around a few iterations into <out_dir>/trace
)
