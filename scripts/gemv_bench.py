"""Single-row decode GEMV timings (the batch-1 serving kernels) on the GPU.

For every decode linear shape of GPT-2 124M and 1.5B, times ``ops.decode_linear_ln``
(residual add + LayerNorm prologue), ``ops.decode_linear`` (plain) and, for c_proj, the
attention-combine prologue, each as a HIP graph of 100 back-to-back launches (the
graph-replayed decode step's launch pattern).  Prints one JSON line per shape with the
microseconds per launch and the weight bytes streamed per microsecond.  Knobs of the
kernels come from the environment (NSA_GEMV_GRID, NSA_GEMV_NC), so an A/B is one run
per setting:

    NSA_GEMV_GRID=512 python scripts/gemv_bench.py
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd import ops  # noqa: E402

BF = torch.bfloat16
DEV = "cuda"


def timed(fn, reps=100):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (5 * reps)


def main():
    torch.manual_seed(0)
    env = {k: os.environ.get(k) for k in ("NSA_GEMV_GRID", "NSA_GEMV_NC")}
    for model, C, V in (("gpt2", 768, 50304), ("gpt2-xl", 1600, 50304)):
        res = torch.randn(1, 1, C, device=DEV)
        br = torch.randn(1, 1, C, device=DEV).to(BF)
        lw = torch.ones(C, device=DEV, dtype=BF)
        lb = torch.zeros(C, device=DEV, dtype=BF)
        shapes = [("c_attn", 3 * C, C, "ln", False), ("c_fc", 4 * C, C, "ln", False), ("mlp.c_proj", C, 4 * C, "plain", False),
                  ("c_proj", C, C, "attn", False), ("lm_head", V, C, "ln", True)]
        for name, N, K, kind, f32 in shapes:
            w = (torch.randn(N, K, device=DEV) * 0.02).to(BF)
            b = None if f32 else torch.zeros(N, device=DEV, dtype=BF)
            if kind == "ln":
                fn = lambda: ops.decode_linear_ln(res, br, lw, lb, w, b, gelu=name == "c_fc", out_f32=f32)  # noqa: E731
            elif kind == "plain":
                x = torch.randn(1, 1, K, device=DEV).to(BF)
                fn = lambda: ops.decode_linear(x, w, b)  # noqa: E731
            else:
                H = C // 64
                kc = torch.randn(1, H, 1024, 64, device=DEV).to(BF)
                vc = torch.randn(1, H, 1024, 64, device=DEV).to(BF)
                qkv = torch.randn(1, 1, 3 * C, device=DEV).to(BF)
                pos = torch.tensor([383], device=DEV)
                part = ops.decode_attention(qkv, kc, vc, pos, H, append=False, combine=False)
                fn = lambda: ops.decode_linear(part, w, b)  # noqa: E731
                us_att = timed(lambda: ops.decode_attention(qkv, kc, vc, pos, H, append=False, combine=False))
                print(json.dumps({"model": model, "op": "decode_attn_partial", "pos": 383, "us": round(us_att, 2)}),
                      flush=True)
            us = timed(fn)
            print(json.dumps({"model": model, "op": name, "N": N, "K": K, "us": round(us, 2),
                              "GBps": round(N * K * 2 / us / 1e3, 1), **env}), flush=True)
    logits = torch.randn(1, 50304, device=DEV) * 3
    tok = torch.zeros(1, 1, dtype=torch.int64, device=DEV)
    gen = torch.zeros(1, 2, dtype=torch.int64, device=DEV)
    p = torch.zeros(1, dtype=torch.int64, device=DEV)
    us = timed(lambda: ops.sample_topk_(logits, 0.8, 200, 1, p, tok, gen))
    print(json.dumps({"op": "sample_topk", "V": 50304, "top_k": 200, "us": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
