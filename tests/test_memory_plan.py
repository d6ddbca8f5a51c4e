"""HBM planner (utils/memory.py): activation estimate and the grad-checkpointing decision."""

from nanosandbox_amd.utils.memory import GiB, activation_bytes, layer_bytes_per_token, plan_grad_ckpt

XL = dict(n_layer=48, n_embd=1600, n_head=25, vocab_size=50304)


def test_layer_bytes_match_the_saved_tensors():
    # fp32 residual: 2x4C ln inputs + 2x2C ln outputs + 6C qkv + 2C attn out + 8C + 8C mlp
    C, H = 768, 12
    assert layer_bytes_per_token(C, H) == 36 * C + 4 * H + 16
    assert layer_bytes_per_token(C, H, fp32_residual=False) == 32 * C + 4 * H + 16


def test_estimate_scales_with_tokens_and_checkpointing_saves():
    a = activation_bytes(tokens=12 * 1024, **XL)
    b = activation_bytes(tokens=60 * 1024, **XL)
    assert abs(b / a - 5.0) < 1e-6
    assert activation_bytes(tokens=60 * 1024, grad_ckpt=True, **XL) < 0.3 * b


def test_plan_keeps_resident_when_it_fits_in_hbm():
    free = 255 * GiB  # MI355X after the 1.5B model's parameters, grads and Adam state
    p = plan_grad_ckpt(tokens=60 * 1024, free_bytes=free, **XL)
    assert not p.grad_ckpt and p.reason == "fits resident"
    # 120 x 1024 no longer fits resident; the MLP-recompute tier does (one c_fc GEMM per
    # layer recomputed instead of a whole extra forward)
    p = plan_grad_ckpt(tokens=120 * 1024, free_bytes=free, **XL)
    assert not p.grad_ckpt and p.recompute_mlp and p.mlp_recompute_bytes <= p.budget_bytes < p.resident_bytes
    assert "recompute_mlp=True" in p.describe()
    p = plan_grad_ckpt(tokens=240 * 1024, free_bytes=free, **XL)
    assert p.grad_ckpt and not p.recompute_mlp and p.ckpt_bytes <= p.budget_bytes
    assert "grad_ckpt=True" in p.describe()


def test_mlp_recompute_drops_the_mlp_activations():
    C, H = 1600, 25
    assert layer_bytes_per_token(C, H) - layer_bytes_per_token(C, H, recompute_mlp=True) == 16 * C
    p = plan_grad_ckpt(tokens=1024, free_bytes=255 * GiB, recompute_mlp=True, **XL)
    assert p.recompute_mlp and not p.grad_ckpt


def test_plan_honours_request_and_unknown_memory():
    assert plan_grad_ckpt(tokens=1024, free_bytes=255 * GiB, requested=True, **XL).grad_ckpt
    assert not plan_grad_ckpt(tokens=10 ** 7, free_bytes=0, **XL).grad_ckpt


def test_trainer_reports_no_plan_on_cpu(tmp_path):
    from nanosandbox_amd.config import TRAIN_DEFAULTS
    from nanosandbox_amd.train import Trainer

    c = dict(TRAIN_DEFAULTS)
    c.update(dataset="synthetic", out_dir=str(tmp_path), n_layer=1, n_head=2, n_embd=32, block_size=32,
             batch_size=2, gradient_accumulation_steps=1, device="cpu", compile=False, dtype="float32",
             metrics_jsonl=False)
    tr = Trainer(c)
    assert tr.activation_plan is None and not tr.raw_model.grad_ckpt


def test_choose_micro_batch_prefers_resident_over_checkpointing():
    from nanosandbox_amd.utils.memory import choose_micro_batch

    hbm = 288 * GiB  # what the MI355X reports as total memory (309e9 bytes)
    # GPT-2 124M / 350M: the whole 120-sequence micro-step stays resident
    assert choose_micro_batch(12, 768, 12, 50304, 1024, 480, hbm) == (120, False)
    assert choose_micro_batch(24, 1024, 16, 50304, 1024, 480, hbm) == (120, False)
    # 1.5B: 120 would need checkpointing, 60 fits resident (round 3: 4592 resident; round 2: 6779 checkpointed)
    assert choose_micro_batch(48, 1600, 25, 50304, 1024, 480, hbm) == (60, False)
    # eight ranks: 60 sequences per rank, one resident micro-step
    assert choose_micro_batch(48, 1600, 25, 50304, 1024, 60, hbm) == (60, False)
    # a small device shrinks the micro-step first ...
    assert choose_micro_batch(48, 1600, 25, 50304, 1024, 480, 48 * 10 ** 9) == (2, False)
    # ... and checkpoints only when not even one resident sequence fits
    mb, ck = choose_micro_batch(48, 1600, 25, 50304, 1024, 480, 33 * 10 ** 9)
    assert ck and 480 % mb == 0
