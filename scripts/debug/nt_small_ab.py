"""Forward / input-gradient GEMMs of the shakespeare_char config (M = 64 x 256 tokens,
n_embd 384): the persistent four-wave kernel against the small-tile kernel.  Medians, us."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd.ops import gemm as G  # noqa: E402

M = 64 * 256
for N, K in [(1152, 384), (384, 384), (1536, 384), (384, 1536), (384, 1152), (64, 384), (384, 64)]:
    torch.manual_seed(0)
    a = (torch.randn(M, K, device="cuda") * 0.1).bfloat16()
    b = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    fns = {"small": lambda: G.small(a, b)}
    if G.nt_supported(M, N, K):
        fns["nt4"] = lambda: G.nt(a, b)
    if G.nt_supported(M, N, K) or K % 64 == 0:
        pass
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
    print(json.dumps({"shape": [M, N, K], "us": {k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}}),
          flush=True)
