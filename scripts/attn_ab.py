"""A/B of flash-attention kernel variants at the GPT-2 training shape (one process,
interleaved rounds, random data; cdna_hip_programming.md §5.4 rules 24-25).

Variants are "name:key=value,..." with keys fwd (auto / v1 / v3), bwd (v2 / v1) and
order (0 / 1), switched through ops.functional.flash_variant (the library resolves its
selection once; nsa_flash_set_variant changes it).  Also checks that every variant's
outputs match the first variant's.

    python scripts/attn_ab.py [--B 120] [--T 1024] [--H 12] [--D 64] [--rounds 7]
        [--bwd "v2:bwd=v2;v1:bwd=v1"] [--fwd "auto:;v1:fwd=v1"]
"""

import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import _lib  # noqa: E402

F32 = torch.float32


def parse(spec):
    out = []
    for item in spec.split(";"):
        if not item.strip():
            continue
        name, _, envs = item.partition(":")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if "=" in kv)
        out.append((name.strip(), env))
    return out


def with_env(env, fn):
    from nanosandbox_amd.ops.functional import flash_variant

    if any(v.isdigit() for v in env.values()):  # raw selector codes (variant libraries, NSA_KERNEL_LIB)
        from nanosandbox_amd.ops.functional import _FLASH_BWD, _FLASH_FWD
        names = {"fwd": _FLASH_FWD, "bwd": _FLASH_BWD, "order": {}}

        def code(k):
            if k not in env:
                return -1
            return int(env[k]) if env[k].isdigit() else names[k][env[k]]
        prev = _lib.call_ret("nsa_flash_set_variant", code("fwd"), code("bwd"), code("order"))
        try:
            return fn()
        finally:
            _lib.call_ret("nsa_flash_set_variant", prev & 0xF, (prev >> 4) & 0xF, (prev >> 8) & 0xF)
    with flash_variant(fwd=env.get("fwd"), bwd=env.get("bwd"),
                       order=int(env["order"]) if "order" in env else None):
        return fn()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=120)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--p", type=float, default=0.0)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--bwd", default="v2:bwd=v2;v1:bwd=v1")
    ap.add_argument("--fwd", default="auto:")
    a = ap.parse_args()
    B, T, H, D = a.B, a.T, a.H, a.D
    C = H * D
    scale = 1.0 / math.sqrt(D)
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3 * C, device="cuda").to(torch.bfloat16)
    y = torch.empty(B, T, C, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, T, device="cuda", dtype=F32)
    dy = torch.randn(B, T, C, device="cuda").to(torch.bfloat16)
    ws = torch.empty(2, B, H, T, device="cuda", dtype=F32)
    seed = 1234
    s = _lib.stream()

    def fwd():
        _lib.call("nsa_flash_fwd", _lib.ptr(qkv), _lib.ptr(y), _lib.ptr(lse), B, T, H, D, scale, a.p, seed, s)

    outs = {}

    def bwd_into(dq):
        _lib.call("nsa_flash_bwd2", _lib.ptr(qkv), _lib.ptr(y), _lib.ptr(dy), _lib.ptr(lse), _lib.ptr(ws),
                  _lib.ptr(dq), B, T, H, D, scale, a.p, seed, s)

    fwd_v = parse(a.fwd)
    bwd_v = parse(a.bwd)
    # correctness: every variant against the first one
    ref_y = None
    for name, env in fwd_v:
        with_env(env, fwd)
        torch.cuda.synchronize()
        if ref_y is None:
            ref_y = y.clone()
        else:
            err = ((y.float() - ref_y.float()).norm() / ref_y.float().norm()).item()
            print(json.dumps({"check": f"fwd/{name}", "rel_err": err}), flush=True)
    with_env(fwd_v[0][1], fwd)
    ref = None
    for name, env in bwd_v:
        dq = torch.zeros_like(qkv)
        with_env(env, lambda: bwd_into(dq))
        torch.cuda.synchronize()
        if ref is None:
            ref = dq.clone()
        else:
            for part, sl in (("dq", slice(0, C)), ("dk", slice(C, 2 * C)), ("dv", slice(2 * C, 3 * C))):
                r = ref[..., sl].float()
                err = ((dq[..., sl].float() - r).norm() / r.norm()).item()
                print(json.dumps({"check": f"bwd/{name}/{part}", "rel_err": err}), flush=True)
    dq = torch.empty_like(qkv)
    causal_flops = 4.0 * B * H * T * T * D / 2
    cands = {f"fwd/{n}": (env, fwd, causal_flops) for n, env in fwd_v}
    cands.update({f"bwd/{n}": (env, (lambda: bwd_into(dq)), 2.5 * causal_flops) for n, env in bwd_v})
    samples = {k: [] for k in cands}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for k, (env, fn, _) in cands.items():
            def run():
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                e1.synchronize()
            with_env(env, run)
            samples[k].append(e0.elapsed_time(e1) / a.iters)
    for k, v in samples.items():
        med = statistics.median(v)
        print(json.dumps({"variant": k, "median_us": round(med * 1e3, 1), "min_us": round(min(v) * 1e3, 1),
                          "TFLOPs": round(cands[k][2] / (med * 1e-3) / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
