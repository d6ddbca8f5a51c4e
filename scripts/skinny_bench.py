"""Per-call time of the decode linears at GPT-2 shapes: one-row GEMV, the MFMA skinny
GEMM (2..16 rows) and the library GEMM + bias (+ GELU) at the same row counts.

    python scripts/skinny_bench.py [--rows 1,4,8,16] [--iters 200]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import functional  # noqa: E402

SHAPES = {"gpt2": [("c_attn", 2304, 768), ("c_proj", 768, 768), ("c_fc", 3072, 768), ("mlp.c_proj", 768, 3072),
                   ("lm_head", 50304, 768)],
          "gpt2-xl": [("c_attn", 4800, 1600), ("c_proj", 1600, 1600), ("c_fc", 6400, 1600),
                      ("mlp.c_proj", 1600, 6400), ("lm_head", 50304, 1600)]}


def timed(fn, iters):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1,4,8,16")
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    for model, shapes in SHAPES.items():
        for op, N, K in shapes:
            w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
            b = None if op == "lm_head" else torch.zeros(N, device="cuda", dtype=torch.bfloat16)
            gelu = op == "c_fc"
            f32 = op == "lm_head"
            for rows in [int(r) for r in a.rows.split(",")]:
                x = torch.randn(rows, 1, K, device="cuda").to(torch.bfloat16)
                rec = {"model": model, "op": op, "N": N, "K": K, "rows": rows}
                functional.SKINNY_MAX_ROWS = 16
                rec["ours_us"] = round(timed(lambda: functional.decode_linear(x, w, b, gelu=gelu, out_f32=f32),
                                             a.iters), 2)
                functional.SKINNY_MAX_ROWS = 1
                functional.GEMV_MAX_ROWS = 0
                rec["library_us"] = round(timed(lambda: functional.decode_linear(x, w, b, gelu=gelu, out_f32=f32),
                                                a.iters), 2)
                functional.GEMV_MAX_ROWS = 1
                rec["weight_GBps"] = round(N * K * 2 / rec["ours_us"] / 1e3, 1)
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
