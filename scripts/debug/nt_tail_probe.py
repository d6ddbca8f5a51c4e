"""Probe: the N = 1600 GEMMs of GPT-2 1.5B (M = 61440 tokens) on the persistent nt4 kernel
(7 column tiles, the 7th 64 wide and shifted back: 1680 tiles = 6.56 rounds) against nt4 over
the first 1536 columns (1440 tiles = 5.63 rounds) plus the 64-column strip on the small-tile
kernel -- sequential, strip first, or the strip on a second stream (filling the CUs the
persistent kernel's last round leaves idle), and with the dedicated strip kernel
(gemm_strip.hip).  Interleaved rounds, medians in us."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd.ops import _lib  # noqa: E402
from nanosandbox_amd.ops import gemm as G  # noqa: E402

M, N = 61440, 1600
N0 = 1536
side = torch.cuda.Stream()


def nt4(a, b, c, n, ldc):
    _lib.call("nsa_gemm_nt4", 0, _lib.ptr(a), a.stride(0), _lib.ptr(b), b.stride(0), _lib.ptr(c), ldc, None, None,
              None, M, n, a.shape[1], G.num_cus(), _lib.stream())


def strip(a, b, c, n, ldc):
    _lib.call("nsa_gemm_strip", _lib.ptr(a), a.stride(0), _lib.ptr(b), b.stride(0), _lib.ptr(c), ldc, None, M, n,
              a.shape[1], _lib.stream())


def small(a, b, c, n, ldc):
    _lib.call("nsa_gemm_small", 0, _lib.ptr(a), a.stride(0), _lib.ptr(b), b.stride(0), _lib.ptr(c), ldc, None, None,
              None, M, n, a.shape[1], _lib.stream())


for K in (1600, 4800, 6400):
    torch.manual_seed(0)
    a = (torch.randn(M, K, device="cuda") * 0.1).bfloat16()
    b = (torch.randn(N, K, device="cuda") * 0.1).bfloat16()
    c_ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    c = torch.empty_like(c_ref)
    b0, b1 = b[:N0], b[N0:]

    def full():
        nt4(a, b, c_ref, N, N)

    def seq():
        nt4(a, b0, c, N0, N)
        small(a, b1, c[:, N0:], N - N0, N)

    def strip_first():
        small(a, b1, c[:, N0:], N - N0, N)
        nt4(a, b0, c, N0, N)

    def par():
        ev = torch.cuda.Event()
        ev.record()
        nt4(a, b0, c, N0, N)
        with torch.cuda.stream(side):
            side.wait_event(ev)
            small(a, b1, c[:, N0:], N - N0, N)
        torch.cuda.current_stream().wait_stream(side)

    def strip_only():
        small(a, b1, c[:, N0:], N - N0, N)

    def seq_strip():
        nt4(a, b0, c, N0, N)
        strip(a, b1, c[:, N0:], N - N0, N)

    def strip_kernel_only():
        strip(a, b1, c[:, N0:], N - N0, N)

    def main_only():
        nt4(a, b0, c, N0, N)

    full()
    seq()
    torch.cuda.synchronize()
    err = ((c.float() - c_ref.float()).abs().max()).item()
    c.fill_(float("nan"))
    seq_strip()
    torch.cuda.synchronize()
    err_strip = ((c.float() - c_ref.float()).abs().max()).item()
    fns = {"full": full, "seq": seq, "strip_first": strip_first, "par": par, "strip_only": strip_only,
           "nt4_1536": main_only, "seq_strip": seq_strip, "strip_kernel": strip_kernel_only}
    res = {k: [] for k in fns}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(7):
        for k, fn in fns.items():
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            e1.synchronize()
            res[k].append(e0.elapsed_time(e1) / 5 * 1e3)
    print(json.dumps({"K": K, "max_abs_diff_vs_full": err, "strip_kernel_max_abs_diff": err_strip,
                      **{k: round(sorted(v)[len(v) // 2], 1) for k, v in res.items()}}), flush=True)
