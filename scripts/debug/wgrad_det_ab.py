"""GPT-2 124M weight-gradient GEMMs (122880 tokens): the split-K kernel's fp32 atomic epilogue
against storing per-split partials plus one ordered reduction pass (the deterministic form),
at the rule's split count and around it.  Medians of interleaved rounds, us."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd.ops import gemm as G  # noqa: E402

T = 122880
for n_out, n_in in [(2304, 768), (768, 768), (3072, 768), (768, 3072), (50304, 768)]:
    torch.manual_seed(0)
    dy = (torch.randn(T, n_out, device="cuda") * 0.1).bfloat16()
    x = (torch.randn(T, n_in, device="cuda") * 0.1).bfloat16()
    g = torch.zeros(n_out, n_in, device="cuda")
    s0 = G.wgrad_splits(n_out, n_in, T)
    cands = sorted({s0, max(1, s0 // 2), s0 * 2} if n_out < 50000 else {s0, 2, 4})
    fns = {}
    for s in cands:
        fns[f"atomic_s{s}"] = (lambda s=s: G.wgrad_acc(dy, x, g, splits=s))
        fns[f"stored_s{s}"] = (lambda s=s: G.wgrad_acc(dy, x, g, splits=s, deterministic=True))
    res = {k: [] for k in fns}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        for k, fn in fns.items():
            e0.record()
            for _ in range(3):
                fn()
            e1.record()
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) / 3 * 1e3)
    print(json.dumps({"shape": [n_out, n_in, T], "rule": s0,
                      "us": {k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}}), flush=True)
