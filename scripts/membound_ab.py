"""A/B timing of the memory-bound kernels on GPT-2 124M micro-step shapes (M = 120 x 1024 rows).

Reports achieved HBM bandwidth (algorithmic bytes / time) per variant, variants
interleaved inside each round (cdna_hip_programming.md §5.4 rule 24):
  * LayerNorm backward (fused residual): pipelined / non-pipelined body x grid size
  * cross-entropy (register-resident): 256 x 25, 512 x 13, 1024 x 7 geometries
  * GELU forward / backward

    python scripts/membound_ab.py [--rows 122880] [--rounds 5]
"""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import _lib  # noqa: E402

BF, F32 = torch.bfloat16, torch.float32


def run(cands, rounds, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for fn, _ in cands.values():
        fn()
    torch.cuda.synchronize()
    samples = {k: [] for k in cands}
    for _ in range(rounds):
        for k, (fn, _) in cands.items():
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            samples[k].append(e0.elapsed_time(e1) / reps)
    out = {}
    for k, s in samples.items():
        med = sorted(s)[len(s) // 2]
        out[k] = {"us": round(med * 1e3, 1), "TB/s": round(cands[k][1] / (med * 1e-3) / 1e12, 2)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=122880)
    ap.add_argument("--c", type=int, default=768)
    ap.add_argument("--v", type=int, default=50304)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="ln,xent,gelu")
    a = ap.parse_args()
    N, C, V = a.rows, a.c, a.v
    only = a.only.split(",")
    dev = "cuda"
    S = _lib.stream
    if "ln" in only:
        x = torch.randn(N, C, device=dev).to(BF)
        dy = torch.randn(N, C, device=dev).to(BF)
        dres = torch.randn(N, C, device=dev).to(BF)
        w = torch.randn(C, device=dev).to(BF)
        mean = torch.randn(N, device=dev)
        rstd = torch.rand(N, device=dev) + 0.5
        dx = torch.empty_like(x)
        part = torch.empty(4096, C, device=dev, dtype=F32)
        partb = torch.empty(4096, C, device=dev, dtype=F32)
        byts = 4 * N * C * 2
        cands = {}
        for pipe in (True, False):
            for nblk in (768, 1024, 1536, 2048, 3072):
                flag = 0 if pipe else (1 << 30)
                cands[f"ln_bwd/{'pipe' if pipe else 'nopipe'}/{nblk}"] = (
                    lambda nblk=nblk, flag=flag: _lib.call(
                        "nsa_layernorm_bwd", _lib.ptr(dy), _lib.ptr(x), _lib.ptr(w), _lib.ptr(mean), _lib.ptr(rstd),
                        _lib.ptr(dres), _lib.ptr(dx), _lib.ptr(part), _lib.ptr(partb), N, C, nblk | flag, S()),
                    byts)
        print(json.dumps({"kernel": "ln_bwd", "res": run(cands, a.rounds)}), flush=True)
        del x, dy, dres, dx
    if "xent" in only:
        logits = torch.randn(N, V, device=dev).to(BF)
        tgt = torch.randint(0, V, (N,), device=dev)
        loss = torch.empty(N, device=dev, dtype=F32)
        byts = 2 * N * V * 2
        cands = {}
        for v, name in ((6, "1024x7"), (1, "256x25"), (2, "512x13"), (3, "1024x7_nt_ld_st"), (4, "1024x7_nt_st"),
                        (5, "1024x7_nt_ld"), (0, "default")):
            cands[f"xent/{name}"] = (
                lambda v=v: _lib.call("nsa_xent_fwd", _lib.ptr(logits), _lib.ptr(tgt), _lib.ptr(loss), N, V, V,
                                      1 | (v << 8), S()), byts)
        print(json.dumps({"kernel": "xent", "res": run(cands, a.rounds)}), flush=True)
        del logits
    if "gelu" in only:
        u = torch.randn(N, 4 * C, device=dev).to(BF)
        g = torch.empty_like(u)
        dg = torch.randn_like(u)
        n = u.numel()
        cands = {
            "gelu_fwd": (lambda: _lib.call("nsa_gelu_fwd", _lib.ptr(u), _lib.ptr(g), n, S()), 2 * n * 2),
            "gelu_bwd": (lambda: _lib.call("nsa_gelu_bwd", _lib.ptr(dg), _lib.ptr(u), _lib.ptr(g), n, S()), 3 * n * 2),
            "copy": (lambda: g.copy_(u), 2 * n * 2),
        }

        def plain(fn):  # same kernel without nontemporal loads / stores (nsa_ew_set_nt)
            def run_plain():
                prev = _lib.call_ret("nsa_ew_set_nt", 0)
                fn()
                _lib.call_ret("nsa_ew_set_nt", prev)
            return run_plain
        cands["gelu_fwd_plain"] = (plain(cands["gelu_fwd"][0]), cands["gelu_fwd"][1])
        cands["gelu_bwd_plain"] = (plain(cands["gelu_bwd"][0]), cands["gelu_bwd"][1])
        print(json.dumps({"kernel": "gelu", "res": run(cands, a.rounds)}), flush=True)


if __name__ == "__main__":
    main()
