"""Offline loading of HuggingFace GPT-2 weights for ``init_from='gpt2*'``.

nanoGPT downloads ``GPT2LMHeadModel.from_pretrained``.
There is no network here, so we only read a local snapshot: a directory given
by ``NSA_HF_GPT2_DIR`` (or the HF cache) holding ``model.safetensors``.
safetensors never executes code from the file.
"""

from __future__ import annotations

import glob
import os


def _find_snapshot(model_type: str) -> str:
    root = os.environ.get("NSA_HF_GPT2_DIR")
    cands = []
    if root:
        cands += [os.path.join(root, model_type), root]
    hub = os.path.expanduser(os.environ.get("HF_HOME", "~/.cache/huggingface"))
    cands += glob.glob(os.path.join(hub, "hub", f"models--{model_type}", "snapshots", "*"))
    cands += glob.glob(os.path.join(hub, "hub", f"models--openai-community--{model_type}", "snapshots", "*"))
    for c in cands:
        if os.path.exists(os.path.join(c, "model.safetensors")):
            return c
    raise FileNotFoundError(
        f"no local HuggingFace snapshot for {model_type!r} (set NSA_HF_GPT2_DIR); "
        "this environment has no network access to download it")


def load_hf_gpt2_state_dict(model_type: str) -> dict:
    from safetensors.torch import load_file
    sd = load_file(os.path.join(_find_snapshot(model_type), "model.safetensors"))
    out = {}
    for k, v in sd.items():
        key = k if k.startswith("transformer.") or k.startswith("lm_head.") else "transformer." + k
        out[key] = v
    if "lm_head.weight" not in out:
        out["lm_head.weight"] = out["transformer.wte.weight"]
    return out
