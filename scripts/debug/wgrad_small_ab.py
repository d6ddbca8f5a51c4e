"""Weight-gradient GEMMs of the shakespeare_char config (n_embd 384, 64 x 256 tokens): the
four-wave split-K kernel (256 x 256 tiles, fp32 atomic epilogue) and the ring64 kernel
(64 x 64 tiles) at several split counts.  Medians of interleaved rounds, us."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd.ops import gemm as G  # noqa: E402

T = 64 * 256
shapes = [(1152, 384), (384, 384), (1536, 384), (384, 1536), (64, 384)]
splits = [1, 2, 4, 8, 12, 16, 24, 32, 48, 64]
for n_out, n_in in shapes:
    torch.manual_seed(0)
    dy = (torch.randn(T, n_out, device="cuda") * 0.1).bfloat16()
    x = (torch.randn(T, n_in, device="cuda") * 0.1).bfloat16()
    g = torch.zeros(n_out, n_in, device="cuda")
    ref = dy.float().t() @ x.float()
    fns = {}
    four_ok = G.wgrad4_supported(n_out, n_in, T)
    for s in splits:
        if four_ok:
            fns[f"wg4_s{s}"] = (lambda s=s: G.wgrad_acc(dy, x, g, splits=s))
        fns[f"ring64_s{s}"] = (lambda s=s: _ring(dy, x, g, s))

    def _ring(dy, x, g, s):
        orig = G.wgrad4_supported
        G.wgrad4_supported = lambda *a: False
        try:
            G.wgrad_acc(dy, x, g, splits=s)
        finally:
            G.wgrad4_supported = orig

    errs = {}
    for k, fn in fns.items():
        g.zero_()
        fn()
        torch.cuda.synchronize()
        errs[k] = ((g - ref).norm() / ref.norm()).item()
    res = {k: [] for k in fns}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        for k, fn in fns.items():
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) / 10 * 1e3)
    med = {k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}
    best = min(med, key=med.get)
    print(json.dumps({"shape": [n_out, n_in, T], "rule_splits": G.wgrad_splits(n_out, n_in, T),
                      "rule_kernel": "wgrad4" if four_ok else "ring64", "best": best, "us": med,
                      "max_rel_err": max(errs.values())}), flush=True)
