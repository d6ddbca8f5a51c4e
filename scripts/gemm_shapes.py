"""Time every GEMM shape of a GPT-2 training micro-step on hipBLASLt (via torch).

For each Linear of the model: forward (x @ W^T [+ residual]), input grad
(dy @ W) and weight grad in three forms: fp32 output accumulated in place
(addmm out_dtype=f32, beta=1), bf16 output + separate fp32 add, and fp32
output + add.  Prints TFLOP/s so the op layer can pick the fastest form.

    python scripts/gemm_shapes.py [--m 12288] [--c 768] [--v 50304]
"""

import argparse
import json

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import gemm as nsa_gemm  # noqa: E402


def bench(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=12288)
    ap.add_argument("--c", type=int, default=768)
    ap.add_argument("--v", type=int, default=50304)
    ap.add_argument("--blas", default="", help="'rocblas' or 'hipblaslt' (torch preferred_blas_library)")
    ap.add_argument("--only", default="", help="comma list of result keys to run")
    a = ap.parse_args()
    if a.blas:
        torch.backends.cuda.preferred_blas_library(a.blas)
    M, C, V = a.m, a.c, a.v
    bf = torch.bfloat16
    dev = "cuda"
    shapes = {"c_attn": (3 * C, C), "attn.c_proj": (C, C), "c_fc": (4 * C, C), "mlp.c_proj": (C, 4 * C),
              "lm_head": (V, C)}
    res = {}
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=bf)
        w = torch.randn(N, K, device=dev, dtype=bf) * 0.02
        dy = torch.randn(M, N, device=dev, dtype=bf)
        r = torch.randn(M, N, device=dev, dtype=bf)
        mg = torch.zeros(N, K, device=dev, dtype=torch.float32)
        fl = 2.0 * M * N * K
        cands = {
            "fwd": lambda: x @ w.t(),
            "fwd_residual_addmm": lambda: torch.addmm(r, x, w.t()),
            "dx": lambda: dy @ w,
            "dW_f32_inplace": lambda: torch.addmm(mg, dy.t(), x, out_dtype=torch.float32, out=mg),
            "dW_bf16": lambda: dy.t() @ x,
            "dW_bf16_then_add": lambda: mg.add_(dy.t() @ x),
            "dW_f32_then_add": lambda: mg.add_(torch.mm(dy.t(), x, out_dtype=torch.float32)),
            "ours_fwd": lambda: nsa_gemm.fwd(x, w, variant=0),
            "ours_dx": lambda: nsa_gemm.dgrad(dy, w, variant=0),
            "ours_dW_acc": lambda: nsa_gemm.wgrad_acc(dy, x, mg, variant=0),
            **{f"v{v}_{n}": f for v in (1, 2, 3, 4, 5, 6, 7, 8) for n, f in (
                ("fwd", lambda v=v: nsa_gemm.fwd(x, w, variant=v)),
                ("dx", lambda v=v: nsa_gemm.dgrad(dy, w, variant=v)),
                ("dW", lambda v=v: nsa_gemm.wgrad_acc(dy, x, mg, variant=v)))},
        }
        only = set(a.only.split(",")) if a.only else set(cands)
        t = {}
        for k, fn in cands.items():
            if k in only:
                try:
                    t[k] = bench(fn)
                except Exception as e:  # some blas backends lack a form
                    print(name, k, "failed:", str(e)[:100])
        res[name] = {k: {"us": round(v * 1e6, 1), "TFLOPs": round(fl / v / 1e12, 1)} for k, v in t.items()}
        print(f"M={M} blas={a.blas or 'default'}", name, json.dumps(res[name]), flush=True)


if __name__ == "__main__":
    main()
