"""A/B of the embedding backward at the training shape: fp32 atomics (the default) against the
sorted, atomic-free form the deterministic mode uses (torch.sort + searchsorted + one writer
per vocabulary row, ``nsa_embedding_bwd_det``).  Interleaved rounds in one process.

    python scripts/emb_bwd_ab.py [--B 120] [--T 1024] [--V 50304] [--C 768] [--rounds 9]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=120)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--V", type=int, default=50304)
    ap.add_argument("--C", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=9)
    a = ap.parse_args()
    B, T, V, C = a.B, a.T, a.V, a.C
    idx = torch.randint(0, V, (B, T), device="cuda")
    dx = torch.randn(B, T, C, device="cuda")
    gw = {k: torch.zeros(V, C, device="cuda") for k in ("atomic", "sorted")}
    gp = {k: torch.zeros(T, C, device="cuda") for k in ("atomic", "sorted")}

    def atomic():
        _lib.call("nsa_embedding_bwd_x32", _lib.ptr(idx), _lib.ptr(dx), _lib.ptr(gw["atomic"]), _lib.ptr(gp["atomic"]),
                  B, T, C, 0.0, 0, _lib.stream())

    def sorted_():
        ids, order = torch.sort(idx.view(-1), stable=True)
        seg = torch.searchsorted(ids, torch.arange(V + 1, device="cuda", dtype=ids.dtype))
        part = torch.empty(2 * ((B * T + 15) // 16), C, device="cuda")
        _lib.call("nsa_embedding_bwd_det", _lib.ptr(ids), _lib.ptr(order), _lib.ptr(seg), _lib.ptr(part),
                  _lib.ptr(dx), _lib.ptr(gw["sorted"]), _lib.ptr(gp["sorted"]), B, T, C, V, 1, 0.0, 0, _lib.stream())

    atomic()
    sorted_()
    torch.cuda.synchronize()
    err = ((gw["atomic"] - gw["sorted"]).norm() / gw["sorted"].norm()).item()
    print(json.dumps({"check": "wte", "rel_err": err}), flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {"atomic": [], "sorted": []}
    for _ in range(a.rounds):
        for k, fn in (("atomic", atomic), ("sorted", sorted_)):
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) / 5 * 1e3)
    for k, v in res.items():
        print(json.dumps({"variant": k, "median_us": round(sorted(v)[len(v) // 2], 1)}), flush=True)


if __name__ == "__main__":
    main()
