"""Python front-end of our gfx950 MFMA GEMMs.

* ``nt(a, b)``             C  = A · B^T   (both K-contiguous; ``csrc/kernels/gemm_nt.hip``):
                                           every forward Y = X · W^T and, on the cached
                                           weight transpose, every input grad dX = dY · W;
                                           fused GELU / GELU' epilogues
* ``fwd``, ``dgrad``, ``fwd_gelu``         convenience wrappers over ``nt``
* ``wgrad_acc(dy, x, g)``  g += dY^T · X  (fp32; ``csrc/kernels/gemm.hip``) split over the
                                           token dim, atomically accumulated into the flat
                                           fp32 gradient (no bf16 dW)
"""

from __future__ import annotations

import os

import torch

from . import _lib

BF16 = torch.bfloat16
LAYOUT_TN = 2
EPI_ATOMIC, EPI_STORE_F32 = 1, 4
BK = 64
TILE = 256
# weight-grad variant (csrc/kernels/gemm.hip nsa_gemm): 1 = ring (32-deep slices), 7 = ring64 (default)
VARIANT = int(os.environ.get("NSA_GEMM_VARIANT", "7"))


def _check(t, name):
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.data_ptr() % 16:
        raise ValueError(f"{name} must be 16-byte aligned")


def supported(M, N, K) -> bool:
    return M % 8 == 0 and N % 8 == 0 and K % BK == 0 and M >= 8 and N >= 8


WGRAD4 = 10  # variant id of the four-wave weight-grad kernel (csrc/kernels/gemm_wg4.hip)


def _call(layout, epi, A, lda, B, ldb, C, ldc, M, N, K, splits=1, variant=None):
    v = VARIANT if variant is None else variant
    if v == WGRAD4 and M >= TILE and N >= TILE:
        _lib.call("nsa_gemm_wgrad4", epi, _lib.ptr(A), lda, _lib.ptr(B), ldb, _lib.ptr(C), ldc, M, N, K, splits,
                  _lib.stream())
        return
    epi = epi | ((7 if v == WGRAD4 else v) << 8)
    _lib.call("nsa_gemm", layout, epi, _lib.ptr(A), lda, _lib.ptr(B), ldb, _lib.ptr(C), ldc, None, None,
              M, N, K, splits, _lib.stream())


# ---------------------------------------------------------------------------------
# Persistent NT kernel (csrc/kernels/gemm_nt.hip): forward and input grads, both
# operands K-contiguous; the input grad uses the cached weight transpose.
# ---------------------------------------------------------------------------------
NT_EPI_BF16, NT_EPI_GELU, NT_EPI_DGELU = 0, 1, 2
_NCU = {}


def num_cus(device=None):
    d = torch.cuda.current_device() if device is None else torch.device(device).index or 0
    if d not in _NCU:
        _NCU[d] = torch.cuda.get_device_properties(d).multi_processor_count
    return _NCU[d]


def nt_supported(M, N, K) -> bool:
    return M >= 256 and N >= 256 and K >= BK and K % BK == 0 and N % 8 == 0


def nt4_supported(M, N, K) -> bool:
    """Shape rules of the four-wave kernel (the same as the eight-wave kernel's)."""
    return nt_supported(M, N, K)


NT_VAR = int(os.environ.get("NSA_NT_STORE", "0"))  # epilogue stores: 0 auto, 1 nontemporal, 2 plain


def _nt_call(epi, A, B, C, M, N, K, C2=None, U=None, grid=None, probe=0, var=None, gm=0, w4=False):
    var = NT_VAR if var is None else var
    _lib.call("nsa_gemm_nt4" if w4 else "nsa_gemm_nt", epi | (probe << 8) | (var << 12) | (gm << 16), _lib.ptr(A), A.stride(0), _lib.ptr(B), B.stride(0), _lib.ptr(C),
              C.stride(0), _lib.ptr(C2), _lib.ptr(U), M, N, K, grid or num_cus(A.device), _lib.stream())


def nt(a, b, epi=NT_EPI_BF16, u=None, grid=None, probe=0, var=None, gm=0, w4=False):
    """C = a @ b^T with a [M, K], b [N, K] (both K-contiguous, bf16) on the persistent kernel
    (``w4``: the four-wave kernel of gemm_nt4.hip, else the eight-wave gemm_nt.hip).

    epi NT_EPI_GELU returns (u, gelu(u)); NT_EPI_DGELU returns (a @ b^T) * gelu'(u)."""
    M, K = a.shape
    N = b.shape[0]
    _check(a, "a")
    _check(b, "b")
    out = torch.empty(M, N, device=a.device, dtype=BF16)
    if epi == NT_EPI_GELU:
        act = torch.empty_like(out)
        _nt_call(epi, a, b, out, M, N, K, C2=act, grid=grid, probe=probe, var=var, gm=gm, w4=w4)
        return out, act
    if epi == NT_EPI_DGELU:
        _check(u, "u")
        _nt_call(epi, a, b, out, M, N, K, U=u, grid=grid, probe=probe, var=var, gm=gm, w4=w4)
        return out
    _nt_call(epi, a, b, out, M, N, K, grid=grid, probe=probe, var=var, gm=gm, w4=w4)
    return out


# the fixed-kernel entry points below use the four-wave kernel (faster on every GPT-2 shape,
# docs/performance.md); the tuner (ops/gemm_tune.py) still races both against hipBLASLt
def fwd(x2, w):
    """Y = X · W^T (nn.Linear forward, bf16)."""
    return nt(x2, w, w4=True)


def fwd_gelu(x2, w):
    """(u, gelu(u)) with u = x2 @ w^T, from one GEMM pass."""
    return nt(x2, w, epi=NT_EPI_GELU, w4=True)


def dgrad(dy2, w, u=None, wt=None):
    """dX = dY · W through W^T (``wt``, K-contiguous; transposed here when not given);
    with ``u`` also multiplied by gelu'(u)."""
    wt = w.t().contiguous() if wt is None else wt
    if u is None:
        return nt(dy2, wt, w4=True)
    return nt(dy2, wt, epi=NT_EPI_DGELU, u=u, w4=True)


def wgrad_splits(n_out, n_in, tokens, cus=256):
    """Largest split count with at most two rounds of blocks (one 512-thread block per CU)."""
    tiles = -(-n_out // TILE) * -(-n_in // TILE)
    nkb = max(1, tokens // BK)
    best = 1
    for s in range(1, min(64, nkb) + 1):
        if tiles * s <= 2 * cus:
            best = s
    return best


WGRAD_MAX_ROUNDS = int(os.environ.get("NSA_WGRAD_MAX_ROUNDS", "6"))


def wgrad_splits_balanced(n_out, n_in, tokens, cus=256, max_rounds=None):
    """Split count whose block count fills whole rounds of the CUs best.

    The kernels take any split count (split z owns K blocks [z*n/S, (z+1)*n/S)),
    so e.g. 27 output tiles x 28 splits = 756 blocks = 2.95 rounds (98 % of the
    last round busy) instead of 27 x 16 = 432 = 1.69 rounds (the default rule).
    Ties go to fewer splits (fewer fp32 atomics).
    """
    if max_rounds is None:
        max_rounds = WGRAD_MAX_ROUNDS
    tiles = -(-n_out // TILE) * -(-n_in // TILE)
    nkb = max(1, tokens // BK)
    best, best_eff = 1, -1.0
    for s in range(1, min(128, nkb) + 1):
        blocks = tiles * s
        rounds = -(-blocks // cus)
        if rounds > max_rounds:
            break
        eff = blocks / (rounds * cus)
        if eff > best_eff + 1e-9:
            best, best_eff = s, eff
    return best


def wgrad_acc(dy2, x2, g32, splits=None, variant=None, deterministic=False):
    """g32 (fp32 [N_out, K_in]) += dy2^T @ x2, reduced over the token dim in-kernel.

    Default: every K split adds its partial tile into g32 with fp32 atomics (arrival
    order, so the last bits vary run to run).  ``deterministic``: each split stores
    its partial to a workspace and one pass adds the splits to g32 in split order
    (bitwise reproducible; with one split the single atomic add per element is
    already order-free)."""
    T, N_out = dy2.shape
    K_in = x2.shape[1]
    _check(dy2, "dy")
    _check(x2, "x")
    _check(g32, "grad")
    if splits is None:
        splits = wgrad_splits(N_out, K_in, T)
    if deterministic and splits > 1:
        ws = torch.empty(splits, N_out, K_in, device=g32.device, dtype=torch.float32)
        _call(LAYOUT_TN, EPI_STORE_F32, dy2, N_out, x2, K_in, ws, K_in, N_out, K_in, T, splits=splits,
              variant=variant)
        _lib.call("nsa_splitk_reduce", _lib.ptr(ws), _lib.ptr(g32), g32.numel(), splits, _lib.stream())
        return g32
    _call(LAYOUT_TN, EPI_ATOMIC, dy2, N_out, x2, K_in, g32, K_in, N_out, K_in, T, splits=splits,
          variant=variant)
    return g32
