"""Sampling CLI (nanoGPT ``sample.py`` contract).

    python sample.py --out_dir=out-shakespeare-char --start="ROMEO:" --num_samples=3 --max_new_tokens=200

Loads ``<out_dir>/ckpt.pt`` (``init_from='resume'``) or GPT-2 weights from a
local HF snapshot (``init_from='gpt2*'``).  Text codec: the dataset's
``meta.json``/``meta.pkl`` for char models, else tiktoken / a local HF GPT-2
tokenizer when available, else raw token ids (``--start="11,42,7"``).
On MI355X the forward runs the same HIP kernels as training; with ``kv_cache=True``
(default) each new token runs one position through the model against per-layer
KV caches, replayed as a HIP graph (``runtime/decode.py``).
"""

from __future__ import annotations

import os
import sys

import torch

from .config import parse_argv
from .data import load_meta, resolve_data_dir
from .models import GPT, GPTConfig
from .utils import load_checkpoint, load_model_state

SAMPLE_DEFAULTS = dict(
    init_from="resume",  # 'resume' (from out_dir) or a gpt2 variant (e.g. 'gpt2-xl')
    out_dir="out",
    start="\n",  # or "<|endoftext|>" or etc. Can also specify a file, use as: "FILE:prompt.txt"
    num_samples=10,
    max_new_tokens=500,
    temperature=0.8,
    top_k=200,
    seed=1337,
    device="cuda",
    dtype="bfloat16",
    compile=False,
    data_dir="",
    kv_cache=True,  # per-layer KV caches + a replayed HIP-graph decode step (runtime/decode.py); False: nanoGPT's recompute loop
)


def _codec(checkpoint, data_dir):
    meta = None
    if checkpoint is not None and "config" in checkpoint and "dataset" in checkpoint["config"]:
        meta = load_meta(resolve_data_dir(checkpoint["config"]["dataset"], data_dir or
                                          checkpoint["config"].get("data_dir", "")))
    if meta is not None:
        print("Loading meta for char codec")
        stoi, itos = meta["stoi"], meta["itos"]
        return (lambda s: [stoi[c] for c in s]), (lambda ids: "".join(itos[i] for i in ids))
    try:
        import tiktoken
        enc = tiktoken.get_encoding("gpt2")
        return (lambda s: enc.encode(s, allowed_special={"<|endoftext|>"})), enc.decode
    except Exception:
        pass
    try:
        from transformers import GPT2TokenizerFast
        tok = GPT2TokenizerFast.from_pretrained(os.environ.get("NSA_HF_GPT2_DIR", "gpt2"), local_files_only=True)
        return tok.encode, tok.decode
    except Exception:
        print("no GPT-2 tokenizer available offline: prompts/outputs are raw token ids")
        return (lambda s: [int(t) for t in s.split(",") if t.strip()]), (lambda ids: ",".join(map(str, ids)))


def main(argv=None):
    c = parse_argv(SAMPLE_DEFAULTS, sys.argv[1:] if argv is None else argv)
    torch.manual_seed(c["seed"])
    device = c["device"]
    if device.startswith("cuda") and not torch.cuda.is_available():
        device = "cpu"
    checkpoint = None
    if c["init_from"] == "resume":
        checkpoint = load_checkpoint(os.path.join(c["out_dir"], "ckpt.pt"), map_location="cpu")
        model = GPT(GPTConfig(**checkpoint["model_args"]))
        load_model_state(model, checkpoint["model"])
    elif c["init_from"].startswith("gpt2"):
        model = GPT.from_pretrained(c["init_from"], dict(dropout=0.0))
    else:
        raise ValueError(c["init_from"])
    model.eval().to(device)
    if device.startswith("cuda"):
        model.set_compute_dtype(torch.bfloat16)
    encode, decode = _codec(checkpoint, c["data_dir"])
    start = c["start"]
    if start.startswith("FILE:"):
        with open(start[5:], "r", encoding="utf-8") as f:
            start = f.read()
    x = torch.tensor(encode(start), dtype=torch.long, device=device)[None, ...]
    outs = []
    dec = None
    if c["kv_cache"]:
        # one decoder for all samples: weight shadows and the captured step graph are
        # built once, not per sample
        from .runtime.decode import Decoder
        dec = Decoder(model, x.shape[0], max_len=model.config.block_size)
    try:
        with torch.no_grad():
            for _ in range(c["num_samples"]):
                if dec is not None:
                    y = model.generate_cached(x, c["max_new_tokens"], temperature=c["temperature"], top_k=c["top_k"],
                                              decoder=dec)
                else:
                    y = model.generate(x, c["max_new_tokens"], temperature=c["temperature"], top_k=c["top_k"])
                text = decode(y[0].tolist())
                outs.append(text)
                print(text)
                print("---------------")
    finally:
        if dec is not None:
            dec.release()
    return outs


if __name__ == "__main__":
    main()
