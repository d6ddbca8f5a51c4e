"""Fixed, shape-derived GEMM kernel selection for every training GEMM (no vendor library).

One native kernel family per op, chosen by the operand shapes alone, identical in every run,
on every box and on every DDP rank (no start-up timing race, nothing to agree on):

============================  ==============================================  ==========================
op                            shape rule                                      kernel
============================  ==============================================  ==========================
forward Y = X·W^T (+ b)       M, N >= 256, K % 64 == 0, N % 8 == 0            ``gemm_nt4.hip`` (persistent)
  (c_fc: u and gelu(u))       otherwise, K % 8 == 0                           ``gemm_small.hip``
input grad dX = dY·W          the same rules on dY · (W^T)^T, W^T cached      as above
  (mlp.c_proj: · gelu'(u))
weight grad dW += dY^T·X      both output sides >= 256                        ``gemm_wg4.hip`` (split-K)
  (fp32, into the flat grad)  otherwise (sides >= 8)                          ``gemm.hip`` ring64
bias grad db += colsum(dY)    any                                             ``optim.hip`` colsum
============================  ==============================================  ==========================

Anything outside every rule (K % 8 != 0, a side < 8, fp32 inputs) is out of the kernels'
contract and runs as a plain torch matmul — no GPT configuration in ``config/`` reaches it
(``tests/test_dispatch_cpu.py`` enumerates them).  Round 3's start-up race against the vendor
library is gone: its last library wins were 1-5 % on four shapes (docs/performance.md), and it
made the kernel set depend on the box.

Env knobs for A/B experiments only: ``NSA_WGRAD_SPLITS`` (force a weight-grad split count),
``NSA_WGRAD_FILL`` (the split rule's round-fill threshold), ``NSA_NT_STORE`` (epilogue store
policy).
"""

from __future__ import annotations

import os

import torch

from . import _lib
from . import gemm as _gemm

F32 = torch.float32
BF16 = torch.bfloat16

# Deterministic mode (config key ``deterministic``, ops.set_deterministic): weight gradients
# reduce their K splits in a fixed order (no fp32 atomics); the embedding backward and the
# lm_head loss switch to their sorted / atomic-free paths.
DETERMINISTIC = False


F16 = torch.float16

# (round 5 tried GPT-2 1.5B's N = 1600 as 1536 columns on the four-wave kernel plus a
# 64-column strip kernel: the strip re-reads all of A from HBM and the step ran slower,
# 5074 vs 4604 ms; profiles/r5_strip_v1.log, r5_strip_v2.log.  Removed in round 6.)


def _ok(*ts):
    """Operands our kernels take: CUDA, contiguous, 16-byte aligned, all bf16 or all fp16."""
    return (ts[0].dtype in (BF16, F16)
            and all(t.is_cuda and t.dtype == ts[0].dtype and t.is_contiguous() and t.data_ptr() % 16 == 0
                    for t in ts))


def kernel_for(op: str, M: int, N: int, K: int) -> str:
    """The kernel the rule picks for a GEMM of this shape ("nt4", "small", "wgrad4", "ring64",
    "torch").  ``op``: "fwd" / "dgrad" (C[M, N] = A[M, K] · B^T) or "wgrad" (M = output rows,
    N = input features, K = tokens)."""
    if op == "wgrad":
        if _gemm.wgrad4_supported(M, N, K):
            return "wgrad4"
        return "ring64" if _gemm.wgrad_supported(M, N, K) else "torch"
    if _gemm.nt_supported(M, N, K):
        return "nt4"
    return "small" if _gemm.small_supported(M, N, K) else "torch"


_used: dict = {}


def kernels_used() -> dict:
    """{(op, M, N, K): kernel} of every GEMM shape this process has run (bench / logs)."""
    return dict(_used)


def record(op: str, M: int, N: int, K: int, kernel: str) -> None:
    """Record a GEMM that bypasses the rule's front-ends (the fused cross-entropy pair
    ``gemm.nt_xent`` / ``nt_xdx``, always the four-wave kernel) so ``kernels_used`` lists
    every GEMM of the step."""
    _used.setdefault((op, M, N, K), kernel)


def _nt(a, b, epi=_gemm.NT_EPI_BF16, u=None, bias=None, op="fwd"):
    M, K = a.shape
    N = b.shape[0]
    k = kernel_for("fwd", M, N, K) if _ok(a, b, *([] if bias is None else [bias])) else "torch"
    _used.setdefault((op, M, N, K), k)
    if k == "nt4":
        return _gemm.nt(a, b, epi=epi, u=u, bias=bias)
    if k == "small":
        return _gemm.small(a, b, epi=epi, u=u, bias=bias)
    y = a @ b.t()
    if bias is not None:
        y = y + bias
    if epi == _gemm.NT_EPI_GELU:
        return _gelu_grad_torch(y.float()).to(torch.float16), _gelu_torch(y)
    if epi == _gemm.NT_EPI_DGELU:
        return (y.float() * u.float()).to(y.dtype)
    return y


def _gelu_torch(u):
    return torch.nn.functional.gelu(u.float()).to(u.dtype)


def _gelu_grad_torch(uf):
    cdf = 0.5 * (1.0 + torch.erf(uf * 0.7071067811865476))
    return cdf + uf * torch.exp(-0.5 * uf * uf) * 0.3989422804014327


def fwd(x2, w, b=None):
    """y = x2 @ w^T (+ b), bf16."""
    return _nt(x2, w, bias=b)


def fwd_gelu(x2, w, b=None):
    """(gelu'(u) in fp16, gelu(u)) with u = x2 @ w^T (+ b), both from one GEMM epilogue (the
    backward needs u only through gelu'(u); ``gemm.nt``)."""
    return _nt(x2, w, epi=_gemm.NT_EPI_GELU, bias=b, op="fwd_gelu")


def dgrad(dy2, w):
    """dx = dy2 @ w (bf16), through the cached K-contiguous w^T."""
    return _nt(dy2, _wt(w), op="dgrad")


def dgrad_dgelu(dy2, w, gp):
    """(dy2 @ w) * gp from one GEMM epilogue, gp = gelu'(u) from ``fwd_gelu``."""
    return _nt(dy2, _wt(w), epi=_gemm.NT_EPI_DGELU, u=gp, op="dgrad_dgelu")


def wgrad_acc(dy2, x2, g32, gb32=None):
    """g32 += dy2^T @ x2 in fp32 (g32: a view of the flat gradient, or a fresh buffer);
    with ``gb32`` also the bias gradient gb32 += dy2.sum(0) (fused into the weight-grad
    kernel where it can be, ``gemm.wgrad_acc``)."""
    T, N = dy2.shape
    K = x2.shape[1]
    k = kernel_for("wgrad", N, K, T) if _ok(dy2, x2) and g32.is_contiguous() else "torch"
    _used.setdefault(("wgrad", N, K, T), k if k == "torch" else f"{k}/s{_gemm.wgrad_splits(N, K, T)}")
    if k != "torch":
        if gb32 is not None and not (gb32.is_contiguous() and dy2.shape[1] % 8 == 0):
            _gemm.wgrad_acc(dy2, x2, g32, deterministic=DETERMINISTIC)
            bias_grad_acc(dy2, gb32)
            return
        _gemm.wgrad_acc(dy2, x2, g32, deterministic=DETERMINISTIC, gb32=gb32)
        return
    g32.add_(dy2.t().float() @ x2.float())
    if gb32 is not None:
        gb32.add_(dy2.float().sum(0))


def bias_grad_acc(dy2, gb32):
    """gb32 += dy2.sum(0) in fp32."""
    if _ok(dy2) and dy2.shape[1] % 8 == 0 and gb32.is_contiguous():
        _gemm.bias_grad_acc(dy2, gb32, deterministic=DETERMINISTIC)
        return
    gb32.add_(dy2.float().sum(0))


# Weight generation: bumped whenever the bf16 compute weights are rewritten outside
# torch's in-place ops (fused AdamW kernel, FlatParamStore.refresh_compute), so cached
# derived copies of a weight (its transpose, below) are rebuilt once per optimizer step.
_weight_gen = 0


def weights_changed():
    global _weight_gen
    _weight_gen += 1


def _wt(w):
    """w^T as a contiguous tensor, cached on the weight tensor for the current generation.

    The input gradient dX = dY · W runs on the NT kernel, whose B operand must be
    K-contiguous: W^T.  Transposing a weight costs microseconds and is amortised over every
    micro-step of an optimizer step.  Inside HIP-graph capture the transpose is recomputed
    (captured into the graph) instead of cached."""
    if w.is_cuda and torch.cuda.is_current_stream_capturing():
        return _transpose(w)
    key = (_weight_gen, w._version, w.data_ptr())
    hit = getattr(w, "_nsa_wt", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    t = _transpose(w, out=hit[1] if hit is not None else None)  # rebuilt in place each step
    try:
        w._nsa_wt = (key, t)
    except (AttributeError, RuntimeError):
        pass
    return t


def _transpose(w, out=None):
    """w^T, contiguous: our bf16 transpose kernel (LDS-free 8x8 register blocks) when the
    shape allows, else torch's copy."""
    R, C = w.shape
    # a 16-bit transpose: the same bit moves for bf16 and fp16
    if w.is_cuda and w.dtype in (BF16, F16) and R % 64 == 0 and C % 64 == 0 and w.is_contiguous():
        if out is None or out.shape != (C, R) or out.dtype != w.dtype or out.device != w.device:
            out = torch.empty(C, R, device=w.device, dtype=w.dtype)
        _lib.call("nsa_transpose_bf16", _lib.ptr(w), _lib.ptr(out), R, C, _lib.stream())
        return out
    return w.t().contiguous()
