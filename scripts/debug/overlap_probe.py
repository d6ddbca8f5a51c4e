"""Probe: a layer's input-gradient GEMM (persistent four-wave kernel, N = 768: 5.6 CU rounds)
and its weight-gradient GEMM (split-K kernel) back to back on one stream against the
weight-gradient GEMM on a second stream launched right after (filling the CUs the persistent
kernel's last partial round leaves idle, if the dispatcher places it there).  Medians, us."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd.ops import gemm as G  # noqa: E402

T = 122880
side = torch.cuda.Stream()
for name, n_out, n_in in [("attn.c_proj", 768, 768), ("c_fc", 3072, 768), ("c_attn", 2304, 768)]:
    torch.manual_seed(0)
    dy = (torch.randn(T, n_out, device="cuda") * 0.1).bfloat16()
    x = (torch.randn(T, n_in, device="cuda") * 0.1).bfloat16()
    wt = (torch.randn(n_in, n_out, device="cuda") * 0.1).bfloat16()  # W^T, K-contiguous for dX = dY W
    g = torch.zeros(n_out, n_in, device="cuda")

    def dgrad():
        return G.nt(dy, wt)

    def wgrad():
        G.wgrad_acc(dy, x, g)

    def seq():
        dgrad()
        wgrad()

    def par():
        ev = torch.cuda.Event()
        ev.record()
        dgrad()
        with torch.cuda.stream(side):
            side.wait_event(ev)
            wgrad()
        torch.cuda.current_stream().wait_stream(side)

    def par_wfirst():
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(side):
            side.wait_event(ev)
            wgrad()
        dgrad()
        torch.cuda.current_stream().wait_stream(side)

    fns = {"dgrad": dgrad, "wgrad": wgrad, "seq": seq, "par": par, "par_wfirst": par_wfirst}
    for fn in fns.values():
        fn()
    torch.cuda.synchronize()
    res = {k: [] for k in fns}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(7):
        for k, fn in fns.items():
            e0.record()
            for _ in range(3):
                fn()
            e1.record()
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) / 3 * 1e3)
    print(json.dumps({"shape": name, **{k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}}), flush=True)
