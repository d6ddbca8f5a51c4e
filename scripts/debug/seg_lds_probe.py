"""Embedding backward at the shakespeare_char shape (64 x 256 tokens, V = 65, C = 384, a
skewed character distribution, dropout 0.2): LDS-privatised scatter-add against the sorted
passes and per-row fp32 atomics.  Medians of interleaved rounds, us."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd.ops import _lib  # noqa: E402

B, T, V, C, p = 64, 256, 65, 384, 0.2
torch.manual_seed(0)
w = 1.0 / torch.arange(1, V + 1, dtype=torch.float64) ** 1.2
idx = torch.multinomial(w, B * T, replacement=True).view(B, T).cuda()
dx = torch.randn(B, T, C, device="cuda")
gw = {k: torch.zeros(V, C, device="cuda") for k in ("lds", "sorted", "atomic")}
gp = {k: torch.zeros(T, C, device="cuda") for k in gw}
part_lds = torch.empty(_lib.call_ret("nsa_seg_lds_parts", B * T), V * C, device="cuda")


def lds():
    _lib.call("nsa_embedding_bwd_lds", _lib.ptr(idx), _lib.ptr(dx), _lib.ptr(gw["lds"]), _lib.ptr(gp["lds"]),
              _lib.ptr(part_lds), B, T, C, V, 1, p, 7, _lib.stream())


def sorted_():
    ids, order = torch.sort(idx.view(-1), stable=True)
    seg = torch.searchsorted(ids, torch.arange(V + 1, device="cuda", dtype=ids.dtype))
    part = torch.empty(2 * ((B * T + 15) // 16), C, device="cuda")
    _lib.call("nsa_embedding_bwd_det", _lib.ptr(ids), _lib.ptr(order), _lib.ptr(seg), _lib.ptr(part),
              _lib.ptr(dx), _lib.ptr(gw["sorted"]), _lib.ptr(gp["sorted"]), B, T, C, V, 1, p, 7, _lib.stream())


def atomic():
    _lib.call("nsa_embedding_bwd_x32", _lib.ptr(idx), _lib.ptr(dx), _lib.ptr(gw["atomic"]), _lib.ptr(gp["atomic"]),
              B, T, C, p, 7, _lib.stream())


fns = {"lds": lds, "sorted": sorted_, "atomic": atomic}
for fn in fns.values():
    fn()
torch.cuda.synchronize()
for k in ("lds", "atomic"):
    err = ((gw[k] - gw["sorted"]).norm() / gw["sorted"].norm()).item()
    print(json.dumps({"check": k, "rel_err_vs_sorted": err}), flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {k: [] for k in fns}
for _ in range(9):
    for k, fn in fns.items():
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        e1.synchronize()
        res[k].append(e0.elapsed_time(e1) / 10 * 1e3)
for k, v in res.items():
    print(json.dumps({"variant": k, "median_us": round(sorted(v)[len(v) // 2], 1)}), flush=True)
