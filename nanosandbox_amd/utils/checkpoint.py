"""nanoGPT-compatible checkpoints (``<out_dir>/ckpt.pt``).

Layout (upstream nanoGPT ``train.py``)::

    {'model': state_dict, 'optimizer': torch-AdamW-format state dict,
     'model_args': {n_layer, n_head, n_embd, block_size, bias, vocab_size, dropout},
     'iter_num': int, 'best_val_loss': float, 'config': {...}}

Writes are atomic (temp file + ``os.replace``) so a pod killed mid-save never
leaves a truncated ``ckpt.pt`` on the PVC — the elastic auto-resume path
relies on that.  Loading always uses ``torch.load(weights_only=True)``.
"""

from __future__ import annotations

import os

import torch

UNWANTED_PREFIX = "_orig_mod."


def strip_compile_prefix(state_dict: dict) -> dict:
    """Checkpoints of ``torch.compile``d models carry ``_orig_mod.`` in every key."""
    sd = dict(state_dict)
    for k in list(sd.keys()):
        if k.startswith(UNWANTED_PREFIX):
            sd[k[len(UNWANTED_PREFIX):]] = sd.pop(k)
    return sd


def model_state_dict(model: torch.nn.Module) -> dict:
    # clone: parameters are views into the flat master buffer; saving the views
    # would serialize the whole shared storage under every key's metadata
    return {k: v.detach().clone().cpu() for k, v in model.state_dict().items()}


def save_checkpoint(path: str, model, optimizer, model_args: dict, iter_num: int, best_val_loss, config: dict):
    ckpt = {
        "model": model_state_dict(model),
        "optimizer": _to_cpu(optimizer.state_dict()),
        "model_args": dict(model_args),
        "iter_num": int(iter_num),
        "best_val_loss": float(best_val_loss),
        "config": dict(config),
    }
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(ckpt, tmp)
    os.replace(tmp, path)


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_to_cpu(v) for v in obj]
    return obj


def load_checkpoint(path: str, map_location="cpu") -> dict:
    return torch.load(path, map_location=map_location, weights_only=True)


def load_model_state(model: torch.nn.Module, state_dict: dict):
    """Copy a nanoGPT state dict into the model *in place* (keeps flat-buffer views)."""
    sd = strip_compile_prefix(state_dict)
    own = model.state_dict()
    missing = [k for k in own if k not in sd and not k.endswith(".attn.bias")]
    unexpected = [k for k in sd if k not in own and not k.endswith(".attn.bias")]
    if missing or unexpected:
        raise KeyError(f"state dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
    with torch.no_grad():
        for k, v in own.items():
            if k in sd:
                v.copy_(sd[k].to(v.device, v.dtype))
