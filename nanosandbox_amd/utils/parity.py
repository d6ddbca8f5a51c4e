"""Training-curve parity: our bf16 stack against an independent fp32 PyTorch GPT-2.

The reference is HuggingFace ``GPT2LMHeadModel`` (exact-erf GELU, no dropout, fp32 on the
same GPU, ``torch.optim.AdamW``), started from a copy of our model's fp32 master weights
and fed the same batches with the same learning-rate schedule, weight-decay groups and
gradient clipping as nanoGPT's ``train.py``.  Our side is the production path: bf16 HIP
kernels (flash attention, NT / split-K GEMMs, fused add+LayerNorm, fused cross-entropy),
fp32 residual stream, fp32 master weights in a flat buffer, the fused flat AdamW.

The two runs share nothing but the initial weights and the token stream, so the per-step
loss difference measures the whole stack's numerics (bf16 rounding included) over a real
optimisation trajectory, not one forward pass.  Used by ``scripts/loss_parity.py``
(GPT-2 124M shape) and ``tests/test_parity_gpu.py`` (a small shape).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# ours (nn.Linear [out, in]) -> HF (Conv1D [in, out])
_TRANSPOSED = ("attn.c_attn.weight", "attn.c_proj.weight", "mlp.c_fc.weight", "mlp.c_proj.weight")


def hf_reference(model, device):
    """An fp32 ``GPT2LMHeadModel`` holding ``model``'s current weights.  Bias-free configs
    (nanoGPT ``bias=False``) keep HF's bias / LayerNorm-bias tensors at zero, frozen."""
    from transformers import GPT2Config, GPT2LMHeadModel

    c = model.config
    hc = GPT2Config(vocab_size=c.vocab_size, n_positions=c.block_size, n_embd=c.n_embd, n_layer=c.n_layer,
                    n_head=c.n_head, activation_function="gelu", resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0,
                    layer_norm_epsilon=1e-5, tie_word_embeddings=True)
    ref = GPT2LMHeadModel(hc).to(device=device, dtype=torch.float32)
    ref.config.use_cache = False
    ours = {k: v for k, v in model.state_dict().items() if not k.endswith(".attn.bias")}
    hsd = ref.state_dict()
    with torch.no_grad():
        for k, t in hsd.items():
            if k.endswith(".attn.masked_bias") or k.endswith(".attn.bias") and t.dim() > 1:
                continue
            if k in ours:
                src = ours[k].float()
                t.copy_(src.t() if k.endswith(_TRANSPOSED) else src)
            elif k.endswith(".bias"):
                t.zero_()  # bias=False on our side
            else:
                raise KeyError(f"no source for HF parameter {k}")
    for name, p in ref.named_parameters():
        if name.endswith(".bias") and name not in ours:
            p.requires_grad_(False)
    return ref


def reference_optimizer(ref, lr, weight_decay, betas):
    decay = [p for p in ref.parameters() if p.requires_grad and p.dim() >= 2]
    nodecay = [p for p in ref.parameters() if p.requires_grad and p.dim() < 2]
    return torch.optim.AdamW([{"params": decay, "weight_decay": weight_decay},
                              {"params": nodecay, "weight_decay": 0.0}], lr=lr, betas=betas, eps=1e-8)


def nanogpt_lr(it, lr, warmup, decay_iters, min_lr):
    if it < warmup:
        return lr * (it + 1) / (warmup + 1)
    if it > decay_iters:
        return min_lr
    r = (it - warmup) / (decay_iters - warmup)
    return min_lr + 0.5 * (1.0 + math.cos(math.pi * r)) * (lr - min_lr)


def run_parity(cfg, batches, lr=6e-4, min_lr=6e-5, warmup=10, weight_decay=0.1, betas=(0.9, 0.95), grad_clip=1.0,
               seed=1337, device="cuda", log=None, dtype=torch.bfloat16):
    """Train our model and the fp32 reference side by side; returns per-step records
    {step, loss, loss_ref, lr}.  ``batches``: list of (X, Y) int64 CPU tensors.  ``dtype``:
    the compute dtype of our side (bf16, or fp16 with the dynamic loss scale as train.py
    runs it: the loss times the device-resident scale, unscale / inf check / skip in the
    optimizer's kernels)."""
    from ..models import GPT
    from ..optim import FlatParamStore
    from ..optim.loss_scale import DynamicLossScale

    torch.manual_seed(seed)
    model = GPT(cfg).to(device).set_compute_dtype(dtype, residual_dtype=torch.float32)
    store = FlatParamStore(model, device, compute_dtype=dtype)
    opt = model.configure_optimizers(weight_decay, lr, betas, "cuda", store=store)
    scaler = None
    if dtype == torch.float16:
        scaler = DynamicLossScale(device=device)
        opt.attach_loss_scale(scaler)
    ref = hf_reference(model, device)
    ropt = reference_optimizer(ref, lr, weight_decay, betas)
    steps = len(batches)
    out = []
    for it, (X, Y) in enumerate(batches):
        cur = nanogpt_lr(it, lr, warmup, steps, min_lr)
        for g in opt.param_groups:
            g["lr"] = cur
        for g in ropt.param_groups:
            g["lr"] = cur
        X, Y = X.to(device), Y.to(device)
        _, loss = model(X, Y)
        (loss * scaler.scale_t if scaler is not None else loss).backward()
        if grad_clip:
            opt.clip_grad_norm_(grad_clip)
        opt.step()
        opt.zero_grad(set_to_none=True)
        logits = ref(X).logits
        rloss = F.cross_entropy(logits.view(-1, logits.size(-1)), Y.view(-1))
        rloss.backward()
        if grad_clip:
            torch.nn.utils.clip_grad_norm_([p for p in ref.parameters() if p.requires_grad], grad_clip)
        ropt.step()
        ropt.zero_grad(set_to_none=True)
        rec = {"step": it, "loss": loss.item(), "loss_ref": rloss.item(), "lr": cur}
        out.append(rec)
        if log is not None:
            log(rec)
    return out
