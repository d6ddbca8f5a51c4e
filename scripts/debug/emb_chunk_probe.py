"""Probe: sorted (chunked) vs atomic embedding backward, with and without dropout, on the
char shape with Zipf-distributed ids; each against the index_add reference built from the
forward's dropout mask."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd import ops  # noqa: E402
from nanosandbox_amd.ops import functional as Fn  # noqa: E402


def run(idx, dx, V, p, sorted_path):
    B, T, C = dx.shape
    Fn._EMB_SORTED_MIN_TOKENS = 0 if sorted_path else 1 << 40
    wte = torch.nn.Parameter(torch.randn(V, C, device="cuda") * 0.02)
    wte.main_grad = torch.zeros(V, C, device="cuda")
    wte.compute = wte.detach().bfloat16()
    wpe = torch.nn.Parameter(torch.randn(T, C, device="cuda") * 0.02)
    wpe.main_grad = torch.zeros(T, C, device="cuda")
    wpe.compute = wpe.detach().bfloat16()
    torch.manual_seed(3)
    x = ops.embedding(idx, wte, wpe, p, True, dtype=torch.float32)
    x.backward(dx)
    return x, wte.main_grad.clone(), wpe.main_grad.clone()


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


torch.manual_seed(2)
B, T, V, C = 64, 256, 56, 384
w = 1.0 / torch.arange(1, V + 1, dtype=torch.float32) ** 1.2
idx = torch.multinomial(w, B * T, replacement=True).view(B, T).cuda()
dx = torch.randn(B, T, C, device="cuda")
for p in (0.0, 0.2):
    xs, gs, ps = run(idx, dx, V, p, True)
    xa, ga, pa = run(idx, dx, V, p, False)
    keep = (xs != 0).float() / (1 - p) if p > 0 else torch.ones_like(dx)
    ref = torch.zeros(V, C, device="cuda").index_add_(0, idx.reshape(-1), (dx * keep).reshape(-1, C))
    refp = (dx * keep).sum(0)
    per_row = ((gs - ref).norm(dim=1) / ref.norm(dim=1)).tolist()
    print(json.dumps({"p": p, "x_same": torch.equal(xs, xa), "sorted_vs_ref": rel(gs, ref),
                      "atomic_vs_ref": rel(ga, ref), "sorted_vs_atomic": rel(gs, ga),
                      "wpe_sorted": rel(ps, refp), "wpe_atomic": rel(pa, refp),
                      "worst_rows": sorted(range(V), key=lambda v: -per_row[v])[:5],
                      "worst_err": sorted(per_row)[-5:],
                      "counts": torch.bincount(idx.reshape(-1), minlength=V)[:8].tolist()}), flush=True)
