"""Per-shape GEMM backend selection (our gfx950 MFMA kernel vs hipBLASLt).

Every training GEMM shape is timed once, on first use, with both backends and
the faster one is cached (process-wide, optionally persisted to
``$NSA_GEMM_TUNE_FILE`` as JSON).  Measured on MI355X (profiles/, scripts/gemm_shapes.py):
our split-K weight-gradient kernel (fp32 accumulate straight into the flat
gradient) beats hipBLASLt's fp32-output path by 1.2-1.8x on every transformer
linear, the LDS-DMA ring kernel wins some input-gradient shapes (K-contiguous B
operand, e.g. c_attn and the 50304-wide lm_head), and hipBLASLt wins the plain
forwards — so the choice is per shape, not per op.

Weight-gradient candidates are timed into a scratch buffer so the real
accumulator is touched exactly once.  ``NSA_GEMM_BACKEND=nsa|hipblaslt`` pins a
backend (tests, A/B runs).
"""

from __future__ import annotations

import json
import os
import threading

import torch

from . import gemm as _gemm

F32 = torch.float32
_table: dict = {}
_lock = threading.Lock()
_loaded = False
FORCE = os.environ.get("NSA_GEMM_BACKEND", "")


def _load():
    global _loaded
    if _loaded:
        return
    _loaded = True
    path = os.environ.get("NSA_GEMM_TUNE_FILE")
    if path and os.path.exists(path):
        try:
            with open(path) as f:
                _table.update({tuple(json.loads(k)): v for k, v in json.load(f).items()})
        except Exception:
            pass


def _save():
    path = os.environ.get("NSA_GEMM_TUNE_FILE")
    if not path:
        return
    try:
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump({json.dumps(list(k)): v for k, v in _table.items()}, f, indent=1)
        os.replace(tmp, path)
    except OSError:
        pass


def _time(fn, reps=3):
    fn()  # warm (first launch / JIT of kernels, cache state)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def choose(key, candidates: dict) -> str:
    """Return the name of the fastest candidate for ``key`` (timed once, then cached)."""
    if FORCE:
        return FORCE if FORCE in candidates else next(iter(candidates))
    _load()
    hit = _table.get(key)
    if hit in candidates:
        return hit
    with _lock:
        times = {name: _time(fn) for name, fn in candidates.items()}
        best = min(times, key=times.get)
        _table[key] = best
        _save()
    return best


def table():
    return dict(_table)


# ------------------------------------------------------------------ ops
def _nsa_ok(*ts):
    return all(t.is_contiguous() and t.data_ptr() % 16 == 0 for t in ts)


def fwd(x2, w):
    """y = x2 @ w^T (bf16)."""
    M, K = x2.shape
    N = w.shape[0]
    if not (_nsa_ok(x2, w) and _gemm.supported(M, N, K)):
        return x2 @ w.t()
    name = choose(("fwd", M, N, K), {"hipblaslt": lambda: x2 @ w.t(), "nsa": lambda: _gemm.fwd(x2, w)})
    return _gemm.fwd(x2, w) if name == "nsa" else x2 @ w.t()


def dgrad(dy2, w):
    """dx = dy2 @ w (bf16)."""
    M, N = dy2.shape
    K = w.shape[1]
    if not (_nsa_ok(dy2, w) and _gemm.supported(M, K, N)):
        return dy2 @ w
    name = choose(("dgrad", M, N, K), {"hipblaslt": lambda: dy2 @ w, "nsa": lambda: _gemm.dgrad(dy2, w)})
    return _gemm.dgrad(dy2, w) if name == "nsa" else dy2 @ w


def _hip_wgrad(dy2, x2, g32):
    torch.addmm(g32, dy2.t(), x2, out_dtype=F32, out=g32)


def wgrad_acc(dy2, x2, g32):
    """g32 += dy2^T @ x2 in fp32."""
    T, N = dy2.shape
    K = x2.shape[1]
    ok = _nsa_ok(dy2, x2, g32) and T % 64 == 0 and N % 8 == 0 and K % 8 == 0
    if not ok:
        _hip_wgrad(dy2, x2, g32)
        return
    scratch = None

    def cand(fn):
        def run():
            nonlocal scratch
            if scratch is None:
                scratch = torch.zeros_like(g32)
            fn(dy2, x2, scratch)
        return run

    name = choose(("wgrad", T, N, K), {"hipblaslt": cand(_hip_wgrad), "nsa": cand(_gemm.wgrad_acc)})
    if name == "nsa":
        _gemm.wgrad_acc(dy2, x2, g32)
    else:
        _hip_wgrad(dy2, x2, g32)
