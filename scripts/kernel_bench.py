"""Micro-benchmarks of the HIP kernels at GPT-2 training shapes.

Reports time, achieved TFLOP/s (attention) or effective HBM bandwidth
(memory-bound kernels) so kernel changes can be A/B'd in one process
(cdna_hip_programming.md §5.4 rule 24: interleaved rounds, report median).

    python scripts/kernel_bench.py [--B 12] [--T 1024] [--C 768] [--H 12] [--only attn,ln,...]
"""

import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nanosandbox_amd import ops  # noqa: E402
from nanosandbox_amd.ops import _lib  # noqa: E402

BF = torch.bfloat16


def timeit(fn, iters=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / iters * 1e-3)
    return statistics.median(res)


def param(t):
    p = torch.nn.Parameter(t.float())
    p.main_grad = torch.zeros_like(p)
    p.compute = p.detach().to(BF)
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=12)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--C", type=int, default=768)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--V", type=int, default=50304)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else None
    B, T, C, H, V = a.B, a.T, a.C, a.H, a.V
    D = C // H
    N = B * T
    dev = "cuda"
    out = {}
    st = _lib.stream

    if only is None or "attn" in only:
        qkv = torch.randn(B, T, 3 * C, device=dev).to(BF)
        y = torch.empty(B, T, C, device=dev, dtype=BF)
        lse = torch.empty(B, H, T, device=dev)
        dy = torch.randn(B, T, C, device=dev).to(BF)
        dqkv = torch.empty_like(qkv)
        sc = 1.0 / math.sqrt(D)

        def fwd():
            _lib.call("nsa_flash_fwd", qkv.data_ptr(), y.data_ptr(), lse.data_ptr(), B, T, H, D, sc, 0.0, 0, st())

        ws = torch.empty(2, B, H, T, device=dev)

        def bwd():
            _lib.call("nsa_flash_bwd2", qkv.data_ptr(), y.data_ptr(), dy.data_ptr(), lse.data_ptr(), ws.data_ptr(),
                      dqkv.data_ptr(), B, T, H, D, sc, 0.0, 0, st())

        flops = 4.0 * B * H * T * T * D / 2  # causal
        tf = timeit(fwd)
        tb = timeit(bwd)
        out["attn_fwd"] = {"us": tf * 1e6, "TFLOPs": flops / tf / 1e12}
        out["attn_bwd"] = {"us": tb * 1e6, "TFLOPs": 2.5 * flops / tb / 1e12}

    if only is None or "ln" in only:
        x = torch.randn(N, C, device=dev).to(BF).requires_grad_(True)
        r = torch.randn(N, C, device=dev).to(BF).requires_grad_(True)
        w = param(torch.ones(C, device=dev))
        b = param(torch.zeros(C, device=dev))
        s, h = ops.add_layer_norm(x, r, w, b)
        dh = torch.randn_like(h)
        ds = torch.randn_like(s)
        t = timeit(lambda: ops.add_layer_norm(x, r, w, b))
        out["add_ln_fwd"] = {"us": t * 1e6, "GBps": 5 * N * C * 2 / t / 1e9}

        def lnb():
            s2, h2 = ops.add_layer_norm(x, r, w, b)
            torch.autograd.backward([s2, h2], [ds, dh])

        t2 = timeit(lnb)
        out["add_ln_fwd_bwd"] = {"us": t2 * 1e6, "GBps": (5 + 4) * N * C * 2 / t2 / 1e9}

    if only is None or "gelu" in only:
        u = torch.randn(N, 4 * C, device=dev).to(BF).requires_grad_(True)
        g = ops.gelu(u)
        dg = torch.randn_like(g)
        t = timeit(lambda: ops.gelu(u))
        out["gelu_fwd"] = {"us": t * 1e6, "GBps": 2 * u.numel() * 2 / t / 1e9}
        t2 = timeit(lambda: torch.autograd.backward([ops.gelu(u)], [dg]))
        out["gelu_fwd_bwd"] = {"us": t2 * 1e6, "GBps": 5 * u.numel() * 2 / t2 / 1e9}
        du = torch.empty_like(dg)
        t3 = timeit(lambda: _lib.call("nsa_gelu_bwd", dg.data_ptr(), u.data_ptr(), du.data_ptr(), u.numel(), st()))
        out["gelu_bwd"] = {"us": t3 * 1e6, "GBps": 3 * u.numel() * 2 / t3 / 1e9}

    if only is None or "xent" in only:
        logits = torch.randn(N, V, device=dev).to(BF)
        tg = torch.randint(0, V, (N,), device=dev)
        rl = torch.empty(N, device=dev)
        base = logits.clone()

        def xe():
            _lib.call("nsa_xent_fwd", logits.data_ptr(), tg.data_ptr(), rl.data_ptr(), N, V, 1, st())

        t = timeit(xe, iters=5, rounds=3)
        out["xent"] = {"us": t * 1e6, "GBps": 3 * N * V * 2 / t / 1e9}
        del logits, base

    if only is None or "emb" in only:
        idx = torch.randint(0, V, (B, T), device=dev)
        wte = param(torch.randn(V, C, device=dev) * 0.02)
        wpe = param(torch.randn(T, C, device=dev) * 0.02)
        xx = ops.embedding(idx, wte, wpe, 0.0, True, dtype=BF)
        dx = torch.randn_like(xx)
        t = timeit(lambda: ops.embedding(idx, wte, wpe, 0.0, True, dtype=BF))
        out["emb_fwd"] = {"us": t * 1e6}
        t2 = timeit(lambda: torch.autograd.backward([ops.embedding(idx, wte, wpe, 0.0, True, dtype=BF)], [dx]))
        out["emb_fwd_bwd"] = {"us": t2 * 1e6}

    if only is None or "adamw" in only:
        n = 124_373_760
        p = torch.randn(n, device=dev)
        g = torch.randn(n, device=dev)
        m = torch.zeros(n, device=dev)
        v = torch.zeros(n, device=dev)
        pb = torch.empty(n, device=dev, dtype=BF)
        mask = torch.ones(n // 64, device=dev, dtype=torch.uint8)
        coef = torch.ones(1, device=dev)

        def step():
            _lib.call("nsa_adamw_step", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), pb.data_ptr(),
                      mask.data_ptr(), n, 6e-4, 0.9, 0.95, 1e-8, 0.1, 0.5, 0.5, coef.data_ptr(), None, st())

        t = timeit(step, iters=5, rounds=3)
        out["adamw_124M"] = {"us": t * 1e6, "GBps": 30 * n / t / 1e9}

    for k, v in out.items():
        print(json.dumps({"kernel": k, "shape": f"B{B} T{T} C{C} H{H}", **{kk: round(vv, 1) for kk, vv in v.items()}}))


if __name__ == "__main__":
    main()
