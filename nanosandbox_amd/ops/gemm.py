"""Python front-ends of our gfx950 MFMA GEMM kernels (no vendor library on any of them).

* ``nt(a, b, ...)``        C = A · B^T, both operands K-contiguous, on the persistent four-wave
                           kernel (``csrc/kernels/gemm_nt4.hip``; M, N >= 256, K % 64 == 0,
                           N % 8 == 0): every forward Y = X · W^T and, on the cached weight
                           transpose, every input grad dX = dY · W.  Epilogues: bf16 (+ bias),
                           gelu'(u) (fp16) + gelu(u), acc · U (U = that gelu'(u)); the fused
                           cross-entropy pair
                           ``nt_xent`` / ``nt_xdx``.
* ``small(a, b, ...)``     the same contract for any M, N (K % 8 == 0) on the bounds-checked
                           64 x 64 kernel (``csrc/kernels/gemm_small.hip``): tiny models, short
                           prefills, odd widths.
* ``wgrad_acc(dy, x, g)``  g += dY^T · X in fp32, split over the token dim, accumulated straight
                           into the flat fp32 gradient: the four-wave kernel
                           (``csrc/kernels/gemm_wg4.hip``) when both output sides are >= 256,
                           else the ring64 kernel (``csrc/kernels/gemm.hip``).

Which of these runs for a given shape is a fixed rule in ``ops/gemm_dispatch.py``.
"""

from __future__ import annotations

import os

import torch

from . import _lib

BF16 = torch.bfloat16
F16 = torch.float16
LAYOUT_TN = 2


def _sym(name, t):
    """Entry point for the operand dtype: NAME (bf16) or NAME_h (fp16, nanoGPT dtype='float16';
    the same kernels with v_mfma_*_f16 and fp16 conversions)."""
    if t.dtype == F16:
        return name + "_h"
    if t.dtype != BF16:
        raise ValueError(f"GEMM kernels take bf16 or fp16 operands, got {t.dtype}")
    return name
EPI_ATOMIC, EPI_STORE_F32 = 1, 4
BK = 64
TILE = 256


def _check(t, name):
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.data_ptr() % 16:
        raise ValueError(f"{name} must be 16-byte aligned")


NT_EPI_BF16, NT_EPI_GELU, NT_EPI_DGELU = 0, 1, 2
_NCU = {}


def num_cus(device=None):
    d = torch.cuda.current_device() if device is None else (torch.device(device).index or 0)
    if d not in _NCU:
        _NCU[d] = torch.cuda.get_device_properties(d).multi_processor_count
    return _NCU[d]


def nt_supported(M, N, K) -> bool:
    """Shape rules of the persistent four-wave NT kernel."""
    return M >= TILE and N >= TILE and K >= BK and K % BK == 0 and N % 8 == 0


def small_supported(M, N, K) -> bool:
    """Shape rules of the bounds-checked small-tile NT kernel."""
    return M >= 1 and N >= 1 and K >= 8 and K % 8 == 0


def wgrad4_supported(n_out, n_in, tokens) -> bool:
    return n_out >= TILE and n_in >= TILE and n_out % 8 == 0 and n_in % 8 == 0 and tokens % BK == 0


def wgrad_supported(n_out, n_in, tokens) -> bool:
    return n_out >= 8 and n_in >= 8 and n_out % 8 == 0 and n_in % 8 == 0 and tokens % BK == 0 and tokens >= BK


NT_VAR = int(os.environ.get("NSA_NT_STORE", "0"))  # epilogue stores: 0 auto, 1 nontemporal, 2 plain
# plain bf16 outputs: a tile's stores inside the next tile's first two K-tiles (0 automatic: from
# K = 128, 1 forced on where possible, 2 never; csrc/kernels/gemm_nt4.hip OVL)
NT_OVL = int(os.environ.get("NSA_NT_OVL", "0"))


def _out(M, N, device, out, dtype=BF16):  # noqa: D401
    if out is None:
        return torch.empty(M, N, device=device, dtype=dtype)
    _check(out, "out")
    if out.dtype != dtype:
        raise ValueError(f"out must be {dtype}")
    return out


_GTAB = {}
GTAB_LO, GTAB_N = 14208, 2560  # csrc/kernels/gemm_nt4.hip Q_GTAB_*


def gelu_table(device):
    """The nt4 GELU epilogue's lookup table (cached per device): for every bf16 u with
    2^-16 <= |u| < 16 (bit pattern (GTAB_LO + i % GTAB_N) | (i >= GTAB_N) << 15), entry i =
    bf16(gelu(u)) | fp16(gelu'(u)) << 16, both from torch's exact-erf GELU in fp32 -- the
    values nanoGPT's autocast nn.GELU produces for that bf16 input."""
    key = torch.device(device)
    t = _GTAB.get(key)
    if t is None:
        i = torch.arange(2 * GTAB_N, dtype=torch.int32)
        bits = (GTAB_LO + i % GTAB_N) | ((i >= GTAB_N).to(torch.int32) << 15)
        u = (bits << 16).view(torch.float32).to(device)  # the bf16 values, exactly, in fp32
        g = torch.nn.functional.gelu(u).to(torch.bfloat16).view(torch.int16).to(torch.int32) & 0xFFFF
        cdf = 0.5 * (1.0 + torch.erf(u * 0.7071067811865476))
        gp = (cdf + u * torch.exp(-0.5 * u * u) * 0.3989422804014327).to(torch.float16)
        gp = gp.view(torch.int16).to(torch.int32) & 0xFFFF
        t = (g | (gp << 16)).contiguous()
        _GTAB[key] = t
    return t


def _check_gp(u):
    _check(u, "u")
    if u.dtype != torch.float16:
        raise ValueError("u must be gelu'(u) in fp16 (the NT_EPI_GELU epilogue's first output)")


# Persistent-grid oversubscription: the four-wave NT kernel launches NT_GRID_MULT x #CUs
# workgroups (one resident per CU).  1 = one static tile chain per CU (fastest alone); > 1 cuts
# every chain into NT_GRID_MULT pieces, so a workgroup exits -- and frees its CU for a bucket
# all-reduce's kernel, or hands the rest of the GEMM to the hardware dispatcher when a CU started
# late -- every 1 / NT_GRID_MULT of the GEMM (scripts/debug/overlap_hazard.py).
NT_GRID_MULT = int(os.environ.get("NSA_NT4_GRID_MULT", "1"))


def nt_grid(device=None) -> int:
    return num_cus(device) * max(1, NT_GRID_MULT)


def nt(a, b, epi=NT_EPI_BF16, u=None, bias=None, grid=None, probe=0, var=None, gm=0, out=None, out2=None, ovl=None):
    """C = a @ b^T with a [M, K], b [N, K] (both K-contiguous, bf16) on the four-wave kernel.

    ``bias`` [N] (bf16) is added in the epilogue (before the GELU).  epi NT_EPI_GELU returns
    (gelu'(u) as fp16, gelu(u) as bf16) for u = bf16(a @ b^T + bias): the backward's only use of
    u is gelu'(u), so the forward stores that (fp16: 2^-11 relative rounding) and the
    NT_EPI_DGELU epilogue, given it as ``u``, is a single multiply: bf16(bf16(a @ b^T) * u).
    ``probe`` needs a library built with -DNSA_PROBES (scripts/gemm_nt_ab.py).  ``ovl`` (plain bf16
    outputs): 0 automatic, 1 / 2 force the overlapped epilogue on / off (csrc/kernels/gemm_nt4.hip)."""
    M, K = a.shape
    N = b.shape[0]
    _check(a, "a")
    _check(b, "b")
    if bias is not None:
        _check(bias, "bias")
    if b.dtype != a.dtype:
        raise ValueError("a and b must have the same dtype")
    c = _out(M, N, a.device, out, torch.float16 if epi == NT_EPI_GELU else a.dtype)
    var = NT_VAR if var is None else var
    ovl = NT_OVL if ovl is None else ovl
    c2 = (_out(M, N, a.device, out2, a.dtype)) if epi == NT_EPI_GELU else None
    if epi == NT_EPI_DGELU:
        _check_gp(u)
    if epi == NT_EPI_GELU:
        # rides in the U slot; the table is indexed by bf16 bits (fp16 computes the GELU)
        u = gelu_table(a.device) if a.dtype == BF16 else None
    _lib.call(_sym("nsa_gemm_nt4", a), epi | (probe << 8) | (var << 12) | (ovl << 14) | (gm << 16), _lib.ptr(a), a.stride(0), _lib.ptr(b),
              b.stride(0), _lib.ptr(c), c.stride(0), _lib.ptr(c2), _lib.ptr(u), _lib.ptr(bias), M, N, K,
              grid or nt_grid(a.device), _lib.stream())
    return (c, c2) if epi == NT_EPI_GELU else c


def small(a, b, epi=NT_EPI_BF16, u=None, bias=None, out=None, out2=None):
    """The ``nt`` contract on the bounds-checked small-tile kernel (any M, N; K % 8 == 0)."""
    M, K = a.shape
    N = b.shape[0]
    _check(a, "a")
    _check(b, "b")
    if b.dtype != a.dtype:
        raise ValueError("a and b must have the same dtype")
    c = _out(M, N, a.device, out, torch.float16 if epi == NT_EPI_GELU else a.dtype)
    c2 = _out(M, N, a.device, out2, a.dtype) if epi == NT_EPI_GELU else None
    if epi == NT_EPI_DGELU:
        _check_gp(u)
    _lib.call(_sym("nsa_gemm_small", a), epi, _lib.ptr(a), a.stride(0), _lib.ptr(b), b.stride(0), _lib.ptr(c), c.stride(0),
              _lib.ptr(c2), _lib.ptr(u), _lib.ptr(bias), M, N, K, _lib.stream())
    return (c, c2) if epi == NT_EPI_GELU else c


def nt_xent(x, w, crow, part, nvalid, out=None):
    """Fused cross-entropy forward GEMM: E = exp(x @ w^T - crow[:, None]) (x's dtype, bf16 or
    fp16; columns >= ``nvalid`` zero) and the per-half-tile row sums into ``part``
    [2 * ceil(N / 256), M]."""
    M, K = x.shape
    N = w.shape[0]
    _check(x, "x")
    _check(w, "w")
    e = _out(M, N, x.device, out, x.dtype)
    _lib.call(_sym("nsa_gemm_nt4_xent", x), _lib.ptr(x), x.stride(0), _lib.ptr(w), w.stride(0), _lib.ptr(e), e.stride(0),
              _lib.ptr(crow), _lib.ptr(part), M, N, int(nvalid), K, nt_grid(x.device), _lib.stream())
    return e


def nt_xdx(e, wt, wrows, coef, out=None):
    """Fused cross-entropy input gradient: coef[:, 0:1] * (e @ wt^T) - coef[:, 1:2] * wrows."""
    M, K = e.shape
    N = wt.shape[0]
    _check(e, "e")
    _check(wt, "wt")
    _check(wrows, "wrows")
    c = _out(M, N, e.device, out, e.dtype)
    _lib.call(_sym("nsa_gemm_nt4_xdx", e), _lib.ptr(e), e.stride(0), _lib.ptr(wt), wt.stride(0), _lib.ptr(c), c.stride(0),
              _lib.ptr(wrows), _lib.ptr(coef), M, N, K, nt_grid(e.device), _lib.stream())
    return c


WGRAD_FILL = float(os.environ.get("NSA_WGRAD_FILL", "0.97"))
WGRAD_SPLITS = int(os.environ.get("NSA_WGRAD_SPLITS", "0"))  # > 0: force a split count (A/B runs)


def wgrad_splits(n_out, n_in, tokens, cus=256):
    """Fixed K-split rule of the weight-gradient GEMMs (one 256 x 256 tile per workgroup).

    Fewer output tiles than CUs, and one round of CUs at least 90 % busy: as many splits as
    fit that round (27 tiles -> 9, 36 -> 7, 9 -> 28, 49 -> 5).  Otherwise the fewest
    splits (<= 8) whose work items fill at least ``WGRAD_FILL`` of their last round of CUs,
    else the best-filling count (the tied 124M lm_head: 591 tiles x 3 = 1773 items = 99 %
    of 7 rounds; GPT-2 1.5B's 175-tile c_fc / mlp.c_proj dW: 7 splits = 96 % of 5 rounds,
    where one round of 175 workgroups left 32 % of the CUs idle).  On the 124M / 350M
    shapes these are the split counts the round-3 start-up race picked
    (profiles/r3_bench_*.log)."""
    if WGRAD_SPLITS > 0:
        return max(1, min(WGRAD_SPLITS, max(1, tokens // BK)))
    tiles = -(-n_out // TILE) * -(-n_in // TILE)
    nkb = max(1, tokens // BK)
    s = _wgrad_splits_fill(tiles, nkb, cus)
    if nkb < _WG_SHORT * s:
        # short work items: each one's 256 KB fp32 atomic epilogue is no longer small next
        # to its K loop (shakespeare_char, 16384 tokens: 384 x 384 at 64 splits = 41.3 us,
        # 27.6 at 32; scripts/debug/wgrad_small_ab.py, profiles/r5_wgrad_small.log)
        s = _wgrad_splits_cost(tiles, nkb, cus)
    return s


_WG_SHORT = 32  # K-tiles per work item below which the atomic epilogue enters the split rule
_WG_TK, _WG_TA = 2.1, 0.2  # us: one 256 x 256 x 64 K-tile on a CU; one item's fp32 atomics (256 KB at ~1.3 TB/s)


def _wgrad_splits_fill(tiles, nkb, cus):
    if tiles < cus and tiles * min(cus // tiles, nkb) >= 0.9 * cus:
        return max(1, min(cus // tiles, nkb))
    best, best_fill = 1, -1.0
    for s in range(1, min(8, nkb) + 1):
        items = tiles * s
        fill = items / (cus * -(-items // cus))
        if fill >= WGRAD_FILL:
            return s
        if fill > best_fill + 1e-9:
            best, best_fill = s, fill
    return best


def _wgrad_splits_cost(tiles, nkb, cus):
    """The split count minimising rounds x K-tiles per item x _WG_TK + items x _WG_TA (on the
    124M / 350M shapes this model picks the round-fill rule's counts but for one; measured on
    the short shapes only)."""
    best, best_t = 1, None
    for s in range(1, min(64, nkb) + 1):
        items = tiles * s
        t = -(-items // cus) * (nkb / s) * _WG_TK + items * _WG_TA
        if best_t is None or t < best_t - 1e-9:
            best, best_t = s, t
    return best


def wgrad_acc(dy2, x2, g32, splits=None, deterministic=False, gb32=None):
    """g32 (fp32 [N_out, K_in]) += dy2^T @ x2, reduced over the token dim in-kernel.

    Default: every K split adds its partial tile into g32 with fp32 atomics (arrival
    order, so the last bits vary run to run).  ``deterministic``: each split stores
    its partial to a workspace and one pass adds the splits to g32 in split order
    (bitwise reproducible; with one split the single atomic add per element is
    already order-free).

    ``gb32`` (fp32 [N_out], optional): the bias gradient gb32 += dy2.sum(0) as well -- fused
    into the four-wave kernel's atomic path (column sums of the dY fragments it reads
    anyway), else the separate column-sum pass."""
    T, N_out = dy2.shape
    K_in = x2.shape[1]
    _check(dy2, "dy")
    _check(x2, "x")
    _check(g32, "grad")
    if splits is None:
        splits = wgrad_splits(N_out, K_in, T)
    four = wgrad4_supported(N_out, K_in, T)

    if gb32 is not None:
        if not gb32.is_contiguous() or gb32.dtype != torch.float32 or gb32.numel() != N_out:
            raise ValueError("bias grad must be a contiguous fp32 [N_out] tensor")
        # not in deterministic mode at any split count: the fused kernel spreads each bias
        # column's token sum over the column blocks, each adding its own fp32 atomic
        if four and not deterministic:
            _lib.call(_sym("nsa_gemm_wgrad4b", dy2), EPI_ATOMIC, _lib.ptr(dy2), dy2.stride(0), _lib.ptr(x2), x2.stride(0),
                      _lib.ptr(g32), K_in, _lib.ptr(gb32), N_out, K_in, T, splits, _lib.stream())
            return g32
        wgrad_acc(dy2, x2, g32, splits, deterministic)
        bias_grad_acc(dy2, gb32, deterministic)
        return g32

    def launch(epi, C):
        if four:
            _lib.call(_sym("nsa_gemm_wgrad4", dy2), epi, _lib.ptr(dy2), dy2.stride(0), _lib.ptr(x2), x2.stride(0), _lib.ptr(C),
                      K_in, N_out, K_in, T, splits, _lib.stream())
        else:
            _lib.call(_sym("nsa_gemm", dy2), LAYOUT_TN, epi, _lib.ptr(dy2), dy2.stride(0), _lib.ptr(x2), x2.stride(0),
                      _lib.ptr(C), K_in, None, None, N_out, K_in, T, splits, _lib.stream())

    if deterministic and splits > 1:
        ws = torch.empty(splits, N_out, K_in, device=g32.device, dtype=torch.float32)
        launch(EPI_STORE_F32, ws)
        _lib.call("nsa_splitk_reduce", _lib.ptr(ws), _lib.ptr(g32), g32.numel(), splits, _lib.stream())
        return g32
    launch(EPI_ATOMIC, g32)
    return g32


def bias_grad_acc(dy2, gb32, deterministic=False):
    """gb32 (fp32 [N]) += column sums of dy2 [T, N] (bf16): one partial pass over row slices
    plus the column reduction into the gradient (ordered in deterministic mode)."""
    T, N = dy2.shape
    _check(dy2, "dy")
    nblk = max(1, min(256, T // 64))
    part = torch.empty(nblk, N, device=dy2.device, dtype=torch.float32)
    _lib.call(_sym("nsa_colsum_bf16_partial", dy2), _lib.ptr(dy2), dy2.stride(0), T, N, _lib.ptr(part), nblk, _lib.stream())
    _lib.call("nsa_colsum_accum_ordered" if deterministic else "nsa_colsum_accum", _lib.ptr(part), _lib.ptr(gb32),
              nblk, N, _lib.stream())
    return gb32
