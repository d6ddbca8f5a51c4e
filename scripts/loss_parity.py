"""Loss-curve parity of the production bf16 stack against an fp32 PyTorch GPT-2
(HuggingFace GPT2LMHeadModel) over a real optimisation trajectory
(nanosandbox_amd/utils/parity.py).  GPT-2 124M shape by default, learnable synthetic
char text (no network), identical initial weights and batches.

    python scripts/loss_parity.py [--steps 300] [--batch 16] [--out gpurun_out/loss_parity.jsonl]
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.data.prepare import synthetic_corpus  # noqa: E402
from nanosandbox_amd.models import GPTConfig  # noqa: E402
from nanosandbox_amd.utils.parity import run_parity  # noqa: E402


def char_batches(steps, batch, block, seed=7):
    text = synthetic_corpus(2_000_000)
    chars = sorted(set(text))
    ids = torch.from_numpy(np.array([chars.index(c) for c in text], dtype=np.int64))
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(steps):
        ix = torch.randint(len(ids) - block - 1, (batch,), generator=g)
        x = torch.stack([ids[i:i + block] for i in ix])
        y = torch.stack([ids[i + 1:i + 1 + block] for i in ix])
        out.append((x, y))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--embd", type=int, default=768)
    ap.add_argument("--block", type=int, default=1024)
    ap.add_argument("--lr", type=float, default=6e-4)
    ap.add_argument("--out", default="gpurun_out/loss_parity.jsonl")
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float16"])
    a = ap.parse_args()
    cfg = GPTConfig(block_size=a.block, vocab_size=50304, n_layer=a.layers, n_head=a.heads, n_embd=a.embd,
                    dropout=0.0, bias=False)
    batches = char_batches(a.steps, a.batch, a.block)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    f = open(a.out, "w")

    def log(rec):
        f.write(json.dumps(rec) + "\n")
        f.flush()
        if rec["step"] % 25 == 0:
            print(json.dumps(rec), flush=True)

    recs = run_parity(cfg, batches, lr=a.lr, min_lr=a.lr / 10, warmup=max(1, a.steps // 30), log=log,
                      dtype=getattr(torch, a.dtype))
    rel = [abs(r["loss"] - r["loss_ref"]) / r["loss_ref"] for r in recs]
    tail = recs[-20:]
    print(json.dumps({"summary": True, "dtype": a.dtype, "steps": a.steps, "tokens_per_step": a.batch * a.block,
                      "first": [round(recs[0]["loss"], 4), round(recs[0]["loss_ref"], 4)],
                      "last20_mean": [round(sum(r["loss"] for r in tail) / len(tail), 4),
                                      round(sum(r["loss_ref"] for r in tail) / len(tail), 4)],
                      "max_rel_diff": round(max(rel), 4), "mean_rel_diff": round(sum(rel) / len(rel), 5)}),
          flush=True)


if __name__ == "__main__":
    main()
