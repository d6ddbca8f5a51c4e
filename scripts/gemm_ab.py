"""A/B timing of GEMM backends on the GPT-2 training shapes (interleaved rounds, random data).

For every Linear of a micro-step (M tokens): forward Y = X W^T and input grad
dX = dY W on hipBLASLt (torch) and on our kernel variants, plus the fused GELU
epilogues (c_fc forward, mlp.c_proj input grad).  Candidates are interleaved
inside each round so they share the same clock / thermal state
(cdna_hip_programming.md §5.4 rule 24); operands are uniform [-1, 1) (rule 25).

    python scripts/gemm_ab.py [--m 122880] [--variants 7,9,10] [--rounds 5]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import gemm  # noqa: E402


def uni(*shape, scale=1.0):
    return (torch.rand(*shape, device="cuda").mul_(2).sub_(1) * scale).to(torch.bfloat16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=122880)
    ap.add_argument("--c", type=int, default=768)
    ap.add_argument("--v", type=int, default=50304)
    ap.add_argument("--variants", default="7,9,10")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ops", default="fwd,dx,fwd_gelu,dx_dgelu")
    ap.add_argument("--shapes", default="c_attn,attn.c_proj,c_fc,mlp.c_proj,lm_head")
    ap.add_argument("--check", action="store_true", help="also compare each variant against hipBLASLt")
    a = ap.parse_args()
    M, C, V = a.m, a.c, a.v
    variants = [int(v) for v in a.variants.split(",") if v]
    shapes = {"c_attn": (3 * C, C), "attn.c_proj": (C, C), "c_fc": (4 * C, C), "mlp.c_proj": (C, 4 * C),
              "lm_head": (V, C)}
    ops = a.ops.split(",")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name in a.shapes.split(","):
        N, K = shapes[name]
        fl = 2.0 * M * N * K
        x = uni(M, K)
        w = uni(N, K, scale=0.05)
        dy = uni(M, N)
        cands = {}
        if "fwd" in ops:
            cands["fwd/hipblaslt"] = lambda: x @ w.t()
            for v in variants:
                cands[f"fwd/v{v}"] = lambda v=v: gemm.fwd(x, w, variant=v)
        if "fwd_gelu" in ops and name == "c_fc":
            for v in variants:
                cands[f"fwd_gelu/v{v}"] = lambda v=v: gemm.fwd_gelu(x, w, variant=v)
        if "dx" in ops:
            cands["dx/hipblaslt"] = lambda: dy @ w
            for v in variants:
                cands[f"dx/v{v}"] = lambda v=v: gemm.dgrad(dy, w, variant=v)
        if "dx_dgelu" in ops and name == "mlp.c_proj":
            # (dY [M, C] @ W [C, 4C]) * gelu'(u [M, 4C])
            u4 = uni(M, K)
            for v in variants:
                cands[f"dx_dgelu/v{v}"] = lambda v=v: gemm.dgrad(dy, w, u=u4, variant=v)
        if a.check:
            ref_f = (x @ w.t()).float()
            ref_d = (dy @ w).float()
            for v in variants:
                for tag, got, ref in (("fwd", gemm.fwd(x, w, variant=v), ref_f),
                                      ("dx", gemm.dgrad(dy, w, variant=v), ref_d)):
                    err = ((got.float() - ref).norm() / ref.norm()).item()
                    print(json.dumps({"check": f"{name}/{tag}/v{v}", "rel_err": err}), flush=True)
        for fn in cands.values():  # first launch, cache state
            fn()
        torch.cuda.synchronize()
        samples = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, fn in cands.items():
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                e1.synchronize()
                samples[k].append(e0.elapsed_time(e1) / a.reps)
        out = {}
        for k, s in samples.items():
            s = sorted(s)
            med = s[len(s) // 2]
            out[k] = {"ms": round(med, 4), "TF": round(fl / (med * 1e-3) / 1e12, 1),
                      "TF_best": round(fl / (s[0] * 1e-3) / 1e12, 1)}
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "res": out}), flush=True)


if __name__ == "__main__":
    main()
