"""Cost of the fused cross-entropy's exact fix-up as the share of flagged rows grows.

fp16 E = exp(logit - target logit) saturates when a row's largest logit passes its target's by
more than ~11 nats (E > 65504); such rows, and rows whose sum falls outside the kept range, are
recomputed exactly by nsa_xent_fixup.  This times the lm_head loss forward (GPT-2 124M shapes:
122880 x 768 against 50304 x 768) with a chosen fraction of rows pushed far past that edge
(their hidden state scaled up), and reports how many rows the combine pass flagged.

    python scripts/debug/xent_f16_cliff.py [--dtype float16] [--fracs 0,0.001,0.01,0.05]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd.ops import functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="float16")
    ap.add_argument("--fracs", default="0,0.001,0.01,0.05")
    ap.add_argument("--n", type=int, default=122880)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dt = getattr(torch, a.dtype)
    N, C, V = a.n, 768, 50304
    g = torch.Generator(device="cuda").manual_seed(0)
    w = (torch.randn(V, C, device="cuda", generator=g) * 0.02).to(dt)
    t = torch.randint(0, 50257, (N,), device="cuda", generator=g)
    base = torch.randn(N, C, device="cuda", generator=g) * 2.0  # logits ~ N(0, 1.2^2): no row past the edge
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for frac in [float(f) for f in a.fracs.split(",")]:
        x = base.clone()
        k = int(round(frac * N))
        if k:
            rows = torch.randperm(N, device="cuda", generator=g)[:k]
            x[rows] *= 6.0  # logits ~ N(0, 7^2): the row max passes the target by far more than 11 nats
        x = x.to(dt)
        with torch.no_grad():
            loss = F.lm_head_loss(x, w, t)
            torch.cuda.synchronize()
            ts = []
            for _ in range(a.reps):
                e0.record()
                loss = F.lm_head_loss(x, w, t)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
        ts.sort()
        ref = None
        if k:  # the flagged rows' loss against fp32 (a sample)
            rs = rows[:64]
            lf = torch.log_softmax(x[rs].float() @ w.float().t(), -1)
            ref = (-lf.gather(1, t[rs, None])).mean().item()
        print(json.dumps({"dtype": a.dtype, "flag_frac": frac, "rows_pushed": k, "fwd_ms_median": round(ts[len(ts) // 2], 3),
                          "loss": round(loss.item(), 4), "fp32_loss_of_pushed_sample": ref}), flush=True)


if __name__ == "__main__":
    main()
