"""Autograd functions for every op of the GPT hot path.

Each op has exactly one GPU implementation — our gfx950 HIP kernels from
``libnsa_kernels.so``, GEMMs included (``ops/gemm_dispatch.py`` picks the kernel
from the shape by a fixed rule; no vendor BLAS on the bf16 path) — and a CPU
implementation in plain fp32 torch that doubles as the numerics reference for
the kernel tests.  The choice is by tensor device and dtype, not a backend switch.

Op inventory (nanoGPT ``model.py`` call sites):

=========  ==========================================  =========================
op         computes                                     nanoGPT site
=========  ==========================================  =========================
K11/K12    ``drop(wte[idx] + wpe[t])``                 ``GPT.forward``
K3         LayerNorm, eps 1e-5, optional bias           ``LayerNorm.forward``
K5-K9      ``x @ W^T + b`` (bias in the GEMM epilogue)   ``nn.Linear``
K4         exact-erf GELU (in the c_fc GEMM epilogue)   ``MLP.forward``
K1/K2      causal flash attention (+dropout)            ``CausalSelfAttention``
K8+K10     tied lm_head + fused cross-entropy           ``GPT.forward`` loss
=========  ==========================================  =========================

Gradient accumulation is fused: if a parameter carries ``main_grad`` (a view
into the flat fp32 gradient buffer owned by ``optim.flat.FlatParamStore``),
weight gradients are accumulated straight into it — for Linear weights inside
the split-K GEMM itself (fp32 atomics into the flat buffer) — and the parameter's
``_nsa_grad_hook`` is called so the bucketed reducer can launch an all-reduce
as soon as a bucket is complete.  Without ``main_grad`` the gradient is
returned to autograd normally (plain ``.grad`` semantics, used by torch DDP
and the gradcheck tests).
"""

from __future__ import annotations

import contextlib
import math
import os
from typing import NamedTuple

import torch
import torch.nn.functional as F

from . import _lib
from . import gemm as _gemm
from . import gemm_dispatch as _gd

BF16 = torch.bfloat16
F16 = torch.float16
F32 = torch.float32
KDT = (BF16, F16)  # the compute dtypes our kernels take (fp16: nanoGPT dtype='float16')


def _sym(name, dtype):
    """NAME for bf16, NAME_h for the fp16 instantiation of the same kernel."""
    return name + "_h" if dtype == F16 else name


# ----------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------

def compute_weight(p: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """The tensor used for compute: the bf16 shadow kept by the optimizer if present."""
    c = getattr(p, "compute", None)
    if c is not None and c.dtype == dtype:
        return c
    p = p.detach()
    return p if p.dtype == dtype else p.to(dtype)


def notify_grad_ready(p: torch.Tensor) -> None:
    hook = getattr(p, "_nsa_grad_hook", None)
    if hook is not None:
        hook(p)


def _accumulate(p: torch.Tensor, g: torch.Tensor):
    """Add ``g`` (fp32) into ``p.main_grad`` if fused accumulation is on; else return it."""
    mg = getattr(p, "main_grad", None)
    if mg is None:
        return g.to(p.dtype).view_as(p)
    mg.add_(g.view_as(mg))
    notify_grad_ready(p)
    return None


def weight_grad(p: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor):
    """dW = dy2^T @ x2 accumulated in fp32 (into ``p.main_grad`` when present).

    On MI355X the accumulate runs in the GEMM itself: our split-K MFMA kernel adds its
    fp32 partial tiles straight into the flat gradient (no bf16 dW, no separate
    accumulate pass)."""
    mg = getattr(p, "main_grad", None)
    if dy2.is_cuda and dy2.dtype in KDT:
        dy2 = dy2.contiguous()
        x2 = x2.contiguous()
        if mg is not None:
            _gd.wgrad_acc(dy2, x2, mg)
            notify_grad_ready(p)
            return None
        g = torch.zeros(p.shape, device=dy2.device, dtype=F32)
        _gd.wgrad_acc(dy2, x2, g)
        return g.to(p.dtype)
    g = dy2.t().float() @ x2.float()
    return _accumulate(p, g)


def weight_bias_grad(w: torch.Tensor, b, dy2: torch.Tensor, x2: torch.Tensor):
    """(dW, db) of one Linear: with both gradients accumulated into flat ``main_grad``
    buffers on the GPU, one weight-grad kernel launch also forms the bias gradient from
    the dY fragments it reads (``gemm_wg4.hip`` BG), instead of a second pass over dY."""
    if b is None:
        return weight_grad(w, dy2, x2), None
    mw, mb = getattr(w, "main_grad", None), getattr(b, "main_grad", None)
    if dy2.is_cuda and dy2.dtype in KDT and mw is not None and mb is not None:
        _gd.wgrad_acc(dy2.contiguous(), x2.contiguous(), mw, gb32=mb)
        notify_grad_ready(w)
        notify_grad_ready(b)
        return None, None
    return weight_grad(w, dy2, x2), bias_grad(b, dy2)


def bias_grad(p, dy2: torch.Tensor):
    """db = dy2.sum(0) accumulated in fp32 (into ``p.main_grad`` when present): our
    column-sum kernel on MI355X."""
    if p is None:
        return None
    mg = getattr(p, "main_grad", None)
    if dy2.is_cuda and dy2.dtype in KDT:
        dy2 = dy2.contiguous()
        if mg is not None:
            _gd.bias_grad_acc(dy2, mg)
            notify_grad_ready(p)
            return None
        g = torch.zeros(p.shape, device=dy2.device, dtype=F32)
        _gd.bias_grad_acc(dy2, g)
        return g.to(p.dtype)
    return _accumulate(p, dy2.float().sum(0))


def new_seed() -> int:
    # drawn from torch's CPU generator so activation checkpointing (which
    # restores RNG state on recompute) replays the same dropout masks
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def set_deterministic(flag: bool) -> None:
    """Bitwise-reproducible training (config key ``deterministic``): weight gradients
    reduce split-K partials in a fixed order and the embedding backward sums each vocab
    row's tokens in token order (no fp32 atomics anywhere on the step).  Every other
    kernel of the step is already order-deterministic."""
    _gd.DETERMINISTIC = bool(flag)


def rng_set(device, value: int = 0) -> None:
    """Set the kernels' device-side dropout step counter (a run starts at 0, so two
    runs with the same seed in one process draw the same masks)."""
    if torch.device(device).type == "cuda":
        _lib.call("nsa_rng_set", int(value), _lib.stream())


def rng_advance(device) -> None:
    """Bump the kernels' device-side dropout step counter (once per micro-step).

    The per-call salts from ``new_seed`` are host values, baked into a captured
    HIP graph; the counter is device state the kernels mix into every salt, and
    this bump is itself a stream operation, so a replayed micro-step (forward,
    backward and any recompute) draws masks no earlier replay used
    (csrc/kernels/common.h ``nsa_seed``).  No-op on CPU."""
    if torch.device(device).type == "cuda":
        _lib.call("nsa_rng_advance", _lib.stream())


# ----------------------------------------------------------------------------
# dropout (hash-based on GPU: the mask is regenerated in backward, never stored)
# ----------------------------------------------------------------------------

def _cpu_keep_mask(shape, p, seed, device=None):
    """Keep-mask of the torch reference path, a pure function of ``seed``: the forward
    and the backward redraw it rather than store it.  A GPU tensor (fp32 compute on the
    GPU) draws it with a device generator seeded the same way, so the mask never crosses
    the host link (a full [B, H, T, T] attention mask per layer would otherwise be drawn
    on the CPU and copied, twice per step)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda":
        g = torch.Generator(device=dev).manual_seed(seed)
        return torch.rand(shape, generator=g, device=dev) >= p
    g = torch.Generator().manual_seed(seed)
    m = torch.rand(shape, generator=g) >= p
    return m if device is None else m.to(device)


def _kern(t) -> bool:
    """Whether an activation runs on our kernels: bf16 or fp16 on the GPU (the fp16 kernels
    are the same sources instantiated with fp16 conversions and v_mfma_*_f16).  fp32 compute
    on the GPU (``--dtype=float32``) takes the plain torch reference path of each op (the
    numerics contract, not the performance path)."""
    return t.is_cuda and t.dtype in KDT


class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        seed = new_seed()
        ctx.p, ctx.seed = p, seed
        if _kern(x):
            y = torch.empty_like(x)
            xc = x.contiguous()
            _lib.call(_sym("nsa_dropout", x.dtype), _lib.ptr(xc), _lib.ptr(y), x.numel(), p, seed, _lib.stream())
            return y
        mask = _cpu_keep_mask(x.shape, p, seed, x.device)
        return x * mask / (1.0 - p)

    @staticmethod
    def backward(ctx, dy):
        if _kern(dy):
            dx = torch.empty_like(dy)
            dyc = dy.contiguous()
            _lib.call(_sym("nsa_dropout", dy.dtype), _lib.ptr(dyc), _lib.ptr(dx), dy.numel(), ctx.p, ctx.seed,
                      _lib.stream())
            return dx, None
        mask = _cpu_keep_mask(dy.shape, ctx.p, ctx.seed, dy.device)
        return dy * mask / (1.0 - ctx.p), None


def dropout(x, p: float, training: bool):
    if not training or p == 0.0:
        return x
    return DropoutFn.apply(x, p)


# ----------------------------------------------------------------------------
# embedding: x = drop(wte[idx] + wpe[arange(T)])
# ----------------------------------------------------------------------------

class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe, p, dtype, cdtype):
        B, T = idx.shape
        V, C = wte.shape
        seed = new_seed() if p > 0 else 0
        ctx.p, ctx.seed, ctx.shape = p, seed, (B, T, V, C)
        ctx.kern = idx.is_cuda and cdtype in KDT
        # the kernels index idx as a dense [B*T] array in both passes: save the
        # contiguous copy (a sliced batch such as d[:, :-1] has row stride T+1)
        idx = idx.contiguous()
        ctx.save_for_backward(idx, wte, wpe)
        if ctx.kern:
            # bf16 weight shadows; the sum (the residual stream) is written in ``dtype``:
            # fp32 (nanoGPT autocast contract) or bf16
            assert C % 8 == 0, "embedding kernel needs n_embd % 8 == 0"
            assert dtype in (F32, BF16) and (cdtype == BF16 or dtype == F32), "fp16 weights take an fp32 stream"
            out = torch.empty(B, T, C, device=idx.device, dtype=dtype)
            # keep the 16-bit weight copies referenced until the launch: without an optimizer's
            # persistent shadow they are temporaries, and the caching allocator would hand
            # the first one's block to the second before the kernel is enqueued
            wte_c, wpe_c = compute_weight(wte, cdtype), compute_weight(wpe, cdtype)
            name = _sym("nsa_embedding_fwd_x32", cdtype) if dtype == F32 else "nsa_embedding_fwd"
            _lib.call(name, _lib.ptr(idx),
                      _lib.ptr(wte_c), _lib.ptr(wpe_c), _lib.ptr(out), B * T, T, C, p, seed, _lib.stream())
            return out
        # fp32 master weights, as nanoGPT's autocast leaves nn.Embedding in fp32
        x = wte.detach().float()[idx] + wpe.detach().float()[:T].unsqueeze(0)
        if p > 0:
            x = x * _cpu_keep_mask(x.shape, p, seed, x.device) / (1.0 - p)
        return x.to(dtype)

    @staticmethod
    def backward(ctx, dx):
        idx, wte, wpe = ctx.saved_tensors
        B, T, V, C = ctx.shape
        if ctx.kern:
            assert idx.is_contiguous()
            dx = dx.contiguous()
            gwte = getattr(wte, "main_grad", None)
            gwpe = getattr(wpe, "main_grad", None)
            ret_wte = gwte is None
            ret_wpe = gwpe is None
            if ret_wte:
                gwte = torch.zeros(V, C, device=dx.device, dtype=F32)
            if ret_wpe:
                gwpe = torch.zeros(wpe.shape[0], C, device=dx.device, dtype=F32)
            assert dx.dtype in (F32, BF16)
            if not _gd.DETERMINISTIC and _seg_lds_fits(V, C):
                # a small vocabulary (a character corpus): the LDS-privatised scatter-add
                # (csrc/kernels/segsum.h); per-row global atomics pile onto a few hot rows
                part = _seg_lds_part(B * T, V, C, dx.device)
                _lib.call("nsa_embedding_bwd_lds", _lib.ptr(idx), _lib.ptr(dx), _lib.ptr(gwte), _lib.ptr(gwpe),
                          _lib.ptr(part), B, T, C, V, 1 if dx.dtype == F32 else 0, ctx.p, ctx.seed, _lib.stream())
            elif _gd.DETERMINISTIC or B * T >= _EMB_SORTED_MIN_TOKENS:
                # atomic-free: token positions stably sorted by id, one writer per vocab row
                # segment starts by binary search over the sorted ids: no host sync
                # (torch.bincount reads its max back to the host, which HIP-graph
                # capture forbids).  Also the faster form from ~64K tokens: B120 T1024
                # C768, wte + wpe grads 313.6 vs 369.5 us with fp32 atomics
                # (scripts/emb_bwd_ab.py, profiles/r5_emb_bwd.md), and deterministic for free.
                ids, order, seg = sort_keys(idx.view(-1), V)
                # partial sums of the segments that cross a 16-position chunk (two slots a chunk)
                part = torch.empty(2 * ((B * T + 15) // 16), C, device=dx.device, dtype=F32)
                _lib.call("nsa_embedding_bwd_det", _lib.ptr(ids), _lib.ptr(order), _lib.ptr(seg), _lib.ptr(part),
                          _lib.ptr(dx), _lib.ptr(gwte), _lib.ptr(gwpe), B, T, C, V, 1 if dx.dtype == F32 else 0, ctx.p,
                          ctx.seed, _lib.stream())
            else:
                _lib.call("nsa_embedding_bwd_x32" if dx.dtype == F32 else "nsa_embedding_bwd", _lib.ptr(idx),
                          _lib.ptr(dx), _lib.ptr(gwte), _lib.ptr(gwpe), B, T, C, ctx.p, ctx.seed, _lib.stream())
            out_wte = gwte.to(wte.dtype) if ret_wte else None
            out_wpe = gwpe.to(wpe.dtype) if ret_wpe else None
            if not ret_wte:
                notify_grad_ready(wte)
            if not ret_wpe:
                notify_grad_ready(wpe)
            return None, out_wte, out_wpe, None, None, None
        d = dx.float()
        if ctx.p > 0:
            d = d * _cpu_keep_mask(d.shape, ctx.p, ctx.seed, d.device) / (1.0 - ctx.p)
        gwte = torch.zeros(V, C, dtype=F32, device=d.device)
        gwte.index_add_(0, idx.reshape(-1), d.reshape(-1, C))
        gwpe = torch.zeros(wpe.shape[0], C, dtype=F32, device=d.device)
        gwpe[:T] = d.sum(0)
        return None, _accumulate(wte, gwte), _accumulate(wpe, gwpe), None, None, None


# our stable key sort (csrc/kernels/keysort.hip) instead of torch.sort + searchsorted for the
# sorted scatter-adds; NSA_KEYSORT=0 falls back to torch's (rocprim) sort
KEYSORT = os.environ.get("NSA_KEYSORT", "1") == "1"


def sort_keys(keys, V):
    """(ids, order, seg) of ``keys`` (int32 / int64, values -1 .. V-1): the stable ascending
    sort, the positions it came from (int64), and seg[v] = #{keys < v} for v = 0 .. V --
    torch.sort(stable=True) + searchsorted(arange(V + 1)), as one HIP radix pass per 8-bit
    digit (no host sync: HIP-graph capturable)."""
    flat = keys.reshape(-1)
    if KEYSORT and flat.is_cuda and V + 1 <= 65536 and flat.dtype in (torch.int32, torch.int64) and flat.numel() > 0:
        n = flat.numel()
        flat = flat.contiguous()
        ids = torch.empty_like(flat)
        order = torch.empty(n, device=flat.device, dtype=torch.int64)
        seg = torch.empty(V + 1, device=flat.device, dtype=torch.int64)
        ws = torch.empty(_lib.call_ret("nsa_keysort_ws_bytes", n), device=flat.device, dtype=torch.uint8)
        _lib.call("nsa_keysort", _lib.ptr(flat), 1 if flat.dtype == torch.int64 else 0, n, V, _lib.ptr(ids),
                  _lib.ptr(order), _lib.ptr(seg), _lib.ptr(ws), _lib.stream())
        return ids, order, seg
    ids, order = torch.sort(flat, stable=True)
    seg = torch.searchsorted(ids, torch.arange(V + 1, device=flat.device, dtype=ids.dtype))
    return ids, order, seg


# below this the fp32-atomic embedding backward (no sort launches) unless deterministic:
# the sort + searchsorted cost ~60 us flat, the atomics ~3 us per 1K tokens against ~2 for
# the sorted kernels (scripts/emb_bwd_ab.py: 16K tokens 55.5 vs 96.2 us, GPT-2 122880
# tokens 369.5 vs 313.6 us, profiles/r5_emb_bwd.md) -> crossover near 64K tokens
_EMB_SORTED_MIN_TOKENS = 65536
_SEG_LDS_BYTES = 128 * 1024  # segsum.h kSegLdsBytes: the padded V x (C + C/8) fp32 table of the LDS scatter-add


def _seg_lds_fits(V, C):
    """The LDS scatter-add's rule: the padded V x (C + C/8) fp32 table fits its LDS budget."""
    return C % 8 == 0 and V * (C + C // 8) * 4 <= _SEG_LDS_BYTES


def _seg_lds_part(n_rows, V, C, device):
    """Scratch of the LDS scatter-add: one V x C fp32 partial table per workgroup."""
    return torch.empty(_lib.call_ret("nsa_seg_lds_parts", n_rows), V * C, device=device, dtype=F32)


def embedding(idx, wte, wpe, p: float, training: bool, dtype=F32, cdtype=None):
    """x = drop(wte[idx] + wpe[t]) in ``dtype`` (the residual stream).  ``cdtype``: the compute
    dtype of the weights (default: bf16 on the GPU -> our kernel; anything else, or the CPU,
    takes the fp32 torch path)."""
    if cdtype is None:
        cdtype = BF16 if idx.is_cuda else F32
    if cdtype not in KDT:
        cdtype = F32  # fp32 compute: the torch path
    return EmbeddingFn.apply(idx, wte, wpe, p if training else 0.0, dtype, cdtype)


# ----------------------------------------------------------------------------
# LayerNorm (eps 1e-5, optional bias)
# ----------------------------------------------------------------------------

LN_EPS = 1e-5
# LayerNorm backward grid: every block resident at once (3 x 256-thread blocks per
# CU at the kernel's ~146 VGPRs, 256 CUs), rows strided over the blocks; measured
# 144 us at 122880 x 768 (5.2 TB/s) vs 148-168 us for 1024-3072 blocks
# (scripts/membound_ab.py)
_LN_BWD_BLOCKS = 768
# fp32 residual stream: ~174 VGPRs -> 2 resident 256-thread blocks per CU
_LN_BWD_BLOCKS_X32 = int(os.environ.get("NSA_LN_BWD_BLOCKS", "512"))
# split-plane residual gradients between our LayerNorm backward passes (NSA_LN_SPLIT=0: plain
# fp32 + a bf16 copy, for A/B); see LayerNormFn and csrc/kernels/layernorm.hip split8
LN_SPLIT = os.environ.get("NSA_LN_SPLIT", "1") != "0"


def split_planes(g: torch.Tensor) -> torch.Tensor:
    """fp32 [.., C] -> the split-plane encoding of csrc/kernels/layernorm.hip (split8), as an
    fp32 tensor of the same shape: hi = bf16(g) rounded to nearest, ties away from zero, in the
    first half of its bytes, the int16 correction bits(g) - (hi << 16) in the second."""
    n = g.numel()
    bits = g.detach().contiguous().view(torch.int32).reshape(-1).to(torch.int64) & 0xFFFFFFFF
    hi = ((bits + 0x8000) >> 16) & 0xFFFF
    hi = torch.where(torch.isnan(g.detach().reshape(-1)), ((bits >> 16) | 0x40) & 0xFFFF, hi)
    lo = (bits - (hi << 16)) & 0xFFFF
    out = torch.empty(2 * n, dtype=torch.int16, device=g.device)
    out[:n] = torch.where(hi >= 0x8000, hi - 0x10000, hi).to(torch.int16)
    out[n:] = torch.where(lo >= 0x8000, lo - 0x10000, lo).to(torch.int16)
    return out.view(torch.float32).view(g.shape)


def unsplit_planes(t: torch.Tensor) -> torch.Tensor:
    """Inverse of ``split_planes``: the fp32 values, bit for bit."""
    n = t.numel()
    raw = t.detach().contiguous().reshape(-1).view(torch.int16)
    hi = raw[:n].to(torch.int64) & 0xFFFF
    lo = raw[n:].to(torch.int64)  # sign-extended correction
    bits = ((hi << 16) + lo) & 0xFFFFFFFF
    bits = torch.where(bits >= 0x80000000, bits - 0x100000000, bits).to(torch.int32)
    return bits.view(torch.float32).view(t.shape)


def split_planes_h(g: torch.Tensor) -> torch.Tensor:
    """fp32 [.., C] -> the fp16-compute split-plane encoding (csrc/kernels/layernorm.hip
    split8h): hi = fp16(g) (round to nearest even) in the first half of the bytes, the int16
    q = (g - hi) * 2^(39 - max(E, 1)) (E = hi's exponent field) in the second; exact for
    |g| >= 2^-14, 2^-39 absolute below, inf at |g| >= 65520."""
    gd = g.detach().contiguous().reshape(-1)
    hi = gd.to(torch.float16)
    e = ((hi.view(torch.int16).to(torch.int32) >> 10) & 31).clamp(min=1)
    r = gd - hi.float()
    q = torch.round(torch.ldexp(r, (39 - e).float()))
    q = torch.where(torch.isfinite(hi), q, torch.zeros_like(q)).to(torch.int16)
    n = gd.numel()
    out = torch.empty(2 * n, dtype=torch.int16, device=g.device)
    out[:n] = hi.view(torch.int16)
    out[n:] = q
    return out.view(torch.float32).view(g.shape)


def unsplit_planes_h(t: torch.Tensor) -> torch.Tensor:
    """Inverse of ``split_planes_h``."""
    n = t.numel()
    raw = t.detach().contiguous().reshape(-1).view(torch.int16)
    hi = raw[:n].view(torch.float16)
    e = ((raw[:n].to(torch.int32) >> 10) & 31).clamp(min=1)
    return (hi.float() + torch.ldexp(raw[n:].float(), (e - 39).float())).view(t.shape)


def _is_split(g) -> bool:
    return g is not None and getattr(g, "_nsa_split", None) is not None


def _unsplit(g):
    """A split-plane gradient decoded (the encoding is named by its ``_nsa_split`` dtype)."""
    return unsplit_planes_h(g) if g._nsa_split == F16 else unsplit_planes(g)


class LayerNormFn(torch.autograd.Function):
    """h = LN(x [+ y]).  With ``y`` the residual add is fused: returns (s = x + y, h).

    The residual stream x / s (and its gradient) keeps x's dtype; y and h are in
    the compute dtype.  On MI355X with an fp32 residual stream (nanoGPT's autocast
    contract: fp32 embedding sum, fp32 + bf16 residual adds) h is bf16 and the
    backward hands y a bf16 copy of the fp32 residual gradient written by the same
    kernel pass.

    Backward of the fused form: ds_total = LN'(dh) + ds (gradient that reached s
    through the residual stream), computed in one kernel pass, and returned as
    the gradient of both x and y — no separate autograd add kernel.

    ``split_grad`` (the GPT trunk, where x comes from another of these nodes and has no other
    consumer): with the fp32 stream and bf16 compute the backward returns x's gradient in the
    split-plane encoding (``split_planes``; the tensor carries ``_nsa_split``), whose first
    half IS the bf16 gradient handed to y — 4 bytes written per element instead of fp32 + a
    bf16 copy (6).  The producing LayerNorm's kernel reads it back exactly; any other
    receiver decodes it with ``unsplit_planes``.  The bf16 half rounds ties away from zero
    (torch's cast: to even), the one difference, at elements whose low 16 bits are 0x8000."""

    @staticmethod
    def forward(ctx, x, y, w, b, out_dtype, passthrough=False, split_grad=False, drop_p=0.0):
        ctx.set_materialize_grads(False)
        # the branch's resid dropout fused into the kernel (add_layer_norm routes only the
        # fp32-stream kernel case here): sum = x + dropout(y), y's gradient masked alike
        ctx.drop = (float(drop_p), new_seed()) if drop_p > 0 else None
        C = x.shape[-1]
        x2 = x.reshape(-1, C)
        N = x2.shape[0]
        ctx.has_bias = b is not None
        ctx.fused = y is not None or passthrough
        ctx.passthrough = passthrough and y is None
        out_dtype = out_dtype or (y.dtype if y is not None else x.dtype)
        ctx.y_dtype = y.dtype if y is not None else None
        ctx.kern = x.is_cuda and out_dtype in KDT
        ctx.split_out = bool(split_grad and LN_SPLIT and ctx.kern and y is not None and x.dtype == F32
                             and out_dtype in (BF16, F16))
        if ctx.kern:
            assert C % 8 == 0 and C <= 8192, "layernorm kernel: C % 8 == 0 and C <= 8192"
            x32 = x.dtype == F32
            assert x.dtype in (F32, BF16) and (x32 or out_dtype == BF16), \
                "layernorm kernel: bf16 stream with bf16 out, or fp32 stream with bf16 / fp16 out"
            x2 = x2.contiguous()
            y2 = y.reshape(-1, C).contiguous() if y is not None else None
            if y2 is not None:
                assert y2.dtype == out_dtype
            s2 = torch.empty_like(x2) if y is not None else None
            h = torch.empty(N, C, device=x.device, dtype=out_dtype)
            mean = torch.empty(N, device=x.device, dtype=F32)
            rstd = torch.empty(N, device=x.device, dtype=F32)
            wc = compute_weight(w, out_dtype)
            bc = compute_weight(b, out_dtype) if b is not None else None
            if ctx.drop is not None:
                assert x32 and y2 is not None
                _lib.call(_sym("nsa_layernorm_fwd_x32d", out_dtype), _lib.ptr(x2), _lib.ptr(y2), _lib.ptr(s2),
                          _lib.ptr(wc), _lib.ptr(bc), _lib.ptr(h), _lib.ptr(mean), _lib.ptr(rstd), N, C, LN_EPS,
                          ctx.drop[0], ctx.drop[1], _lib.stream())
            else:
                _lib.call(_sym("nsa_layernorm_fwd_x32", out_dtype) if x32 else "nsa_layernorm_fwd", _lib.ptr(x2),
                          _lib.ptr(y2),
                          _lib.ptr(s2), _lib.ptr(wc), _lib.ptr(bc), _lib.ptr(h), _lib.ptr(mean), _lib.ptr(rstd), N,
                          C, LN_EPS, _lib.stream())
            inp = s2 if y is not None else x2
        else:
            assert ctx.drop is None, "fused branch dropout is a kernel path (add_layer_norm applies it otherwise)"
            xf = x2.float()
            if y is not None:
                xf = xf + y.reshape(-1, C).float()
            inp = xf.to(x.dtype)
            mean = xf.mean(-1)
            var = xf.var(-1, unbiased=False)
            rstd = torch.rsqrt(var + LN_EPS)
            h = (xf - mean[:, None]) * rstd[:, None] * w.detach().float()
            if b is not None:
                h = h + b.detach().float()
            h = h.to(out_dtype)
        ctx.save_for_backward(inp, w, b if b is not None else mean, mean, rstd)
        hshape = (*x.shape[:-1], C)
        if y is not None:
            return inp.view(x.shape), h.view(hshape)
        if ctx.passthrough:
            return x.view_as(x), h.view(hshape)
        return h.view(hshape)

    @staticmethod
    def backward(ctx, *grads):
        if ctx.fused:
            ds, dh = grads
        else:
            ds, dh = None, grads[0]
        if dh is None and ds is None:  # no output reached the loss (grads are not materialised)
            return None, None, None, None, None, None, None, None
        x2, w, b_or_mean, mean, rstd = ctx.saved_tensors
        ds_split = _is_split(ds)
        if ds_split and (dh is None or not ctx.kern or x2.dtype != F32 or dh.dtype != ds._nsa_split):
            ds, ds_split = _unsplit(ds), False  # a receiver the split kernel does not cover
        b = b_or_mean if ctx.has_bias else None
        C = x2.shape[-1]
        N = x2.shape[0]
        shape = (*(dh if dh is not None else ds).shape[:-1], C)
        if dh is None:  # only the residual output was used
            dyb = ds.to(ctx.y_dtype) if (ctx.fused and not ctx.passthrough) else None
            return ds, _drop_grad(ctx, dyb), None, None, None, None, None, None
        dy2 = dh.reshape(-1, C)
        if ctx.kern:
            x32 = x2.dtype == F32
            dy2 = dy2.contiguous()
            ds2 = ds.reshape(-1, C).contiguous() if ds is not None else None
            if ds2 is not None and ds2.dtype != x2.dtype:
                ds2 = ds2.to(x2.dtype)
            dx = torch.empty_like(x2)
            split_out = ctx.split_out and x32 and dy2.dtype in (BF16, F16)
            # the fused form also hands the branch (y) its gradient in y's dtype (split: the
            # hi plane of dx itself)
            if split_out:
                dyb = dx.view(dy2.dtype).view(-1)[:N * C].view(N, C)
            else:
                dyb = (torch.empty(N, C, device=dh.device, dtype=ctx.y_dtype)
                       if (ctx.fused and x32 and not ctx.passthrough) else None)
            nblk = min(_LN_BWD_BLOCKS_X32 if x32 else _LN_BWD_BLOCKS, max(1, (N + 7) // 8))
            dw_part = torch.empty(nblk, C, device=dh.device, dtype=F32)
            db_part = torch.empty(nblk, C, device=dh.device, dtype=F32) if b is not None else None
            wc = compute_weight(w, dy2.dtype)
            if x32 and (ds_split or split_out):
                _lib.call(_sym("nsa_layernorm_bwd_x32s", dy2.dtype), _lib.ptr(dy2), _lib.ptr(x2), _lib.ptr(wc), _lib.ptr(mean),
                          _lib.ptr(rstd), _lib.ptr(ds2), _lib.ptr(dx), None, _lib.ptr(dw_part),
                          _lib.ptr(db_part), N, C, nblk, (1 if ds_split else 0) | (2 if split_out else 0),
                          _lib.stream())
            elif x32:
                _lib.call(_sym("nsa_layernorm_bwd_x32", dy2.dtype), _lib.ptr(dy2), _lib.ptr(x2), _lib.ptr(wc), _lib.ptr(mean),
                          _lib.ptr(rstd), _lib.ptr(ds2), _lib.ptr(dx), _lib.ptr(dyb), _lib.ptr(dw_part),
                          _lib.ptr(db_part), N, C, nblk, _lib.stream())
            else:
                _lib.call("nsa_layernorm_bwd", _lib.ptr(dy2), _lib.ptr(x2), _lib.ptr(wc), _lib.ptr(mean),
                          _lib.ptr(rstd), _lib.ptr(ds2), _lib.ptr(dx), _lib.ptr(dw_part), _lib.ptr(db_part), N, C,
                          nblk, _lib.stream())
            gw = _colsum_into(w, dw_part)
            gb = _colsum_into(b, db_part) if b is not None else None
            dx = dx.view(shape)
            if split_out:
                dx._nsa_split = dy2.dtype
            if not ctx.fused or ctx.passthrough:
                return dx, None, gw, gb, None, None, None, None
            return dx, _drop_grad(ctx, dyb.view(shape) if dyb is not None else dx), gw, gb, None, None, None, None
        xf = x2.float()
        d = dy2.float()
        xhat = (xf - mean[:, None]) * rstd[:, None]
        wf = w.detach().float()
        dxhat = d * wf
        dx = rstd[:, None] * (dxhat - dxhat.mean(-1, keepdim=True) - xhat * (dxhat * xhat).mean(-1, keepdim=True))
        if ds is not None:
            dx = dx + ds.reshape(-1, C).float()
        gw = _accumulate(w, (d * xhat).sum(0))
        gb = _accumulate(b, d.sum(0)) if b is not None else None
        dxs = dx.to(x2.dtype).view(shape)
        if not ctx.fused or ctx.passthrough:
            return dxs, None, gw, gb, None, None, None, None
        return dxs, dx.to(ctx.y_dtype).view(shape), gw, gb, None, None, None, None


def _drop_grad(ctx, g):
    """The branch gradient through the fused resid dropout: nsa_dropout's mask for the
    forward's seed (a new tensor: with split planes g is a view of the residual gradient)."""
    if ctx.drop is None or g is None:
        return g
    out = torch.empty_like(g)
    gc = g.contiguous()
    _lib.call(_sym("nsa_dropout", g.dtype), _lib.ptr(gc), _lib.ptr(out), g.numel(), ctx.drop[0], ctx.drop[1],
              _lib.stream())
    return out


def _colsum_into(p, partial):
    """Reduce per-block partial column sums into p.main_grad (fused) or a fresh fp32 grad."""
    mg = getattr(p, "main_grad", None)
    rows, C = partial.shape
    fn = "nsa_colsum_accum_ordered" if _gd.DETERMINISTIC else "nsa_colsum_accum"
    if mg is not None:
        _lib.call(fn, _lib.ptr(partial), _lib.ptr(mg), rows, C, _lib.stream())
        notify_grad_ready(p)
        return None
    out = torch.zeros(C, device=partial.device, dtype=F32)
    _lib.call(fn, _lib.ptr(partial), _lib.ptr(out), rows, C, _lib.stream())
    return out.to(p.dtype)


def layer_norm(x, w, b, out_dtype=None):
    """LN(x); ``out_dtype`` (default x's dtype) is the dtype of the normalised output."""
    return LayerNormFn.apply(x, None, w, b, out_dtype)


def layer_norm_pass(x, w, b, out_dtype=None):
    """(x, LN(x)) as one node: the returned x is the residual stream's continuation,
    so its gradient enters the LayerNorm backward kernel as the residual input (one
    pass computes dx = LN'(dh) + ds) instead of being summed with LN's own input
    gradient by a separate add kernel."""
    return LayerNormFn.apply(x, None, w, b, out_dtype, True)


# NSA_LN_DROPOUT=0: the branch's resid dropout as its own pass before the fused add + LN
LN_DROPOUT = os.environ.get("NSA_LN_DROPOUT", "1") != "0"


def add_layer_norm(x, y, w, b, out_dtype=None, split_grad=False, drop_p=0.0):
    """Fused residual add + LayerNorm: returns (x + y, LN(x + y)).

    x + y keeps x's (residual-stream) dtype; LN(x + y) is in ``out_dtype``
    (default y's dtype, the compute dtype).  ``split_grad``: x is the residual output of
    another ``add_layer_norm`` / ``layer_norm_pass`` and nothing else reads it, so x's
    gradient may travel in the split-plane encoding (see LayerNormFn).  ``drop_p``: the
    branch's resid dropout (nanoGPT ``resid_dropout``), x + dropout(y): fused into the
    LayerNorm kernel on the fp32-stream kernel path (the same mask and rounding as
    ``dropout``), a separate ``dropout`` elsewhere."""
    if drop_p > 0:
        od = out_dtype or y.dtype
        if not (LN_DROPOUT and x.is_cuda and x.dtype == F32 and od in KDT and y.dtype == od):
            return LayerNormFn.apply(x, dropout(y, drop_p, True), w, b, out_dtype, False, split_grad)
    return LayerNormFn.apply(x, y, w, b, out_dtype, False, split_grad, drop_p)


# ----------------------------------------------------------------------------
# Linear: out = x @ W^T + b (+ residual)   (our MFMA GEMMs, bias in the epilogue, fp32 dW fused)
# ----------------------------------------------------------------------------

class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, residual):
        K = x.shape[-1]
        Nout = w.shape[0]
        x2 = x.reshape(-1, K)
        wc = compute_weight(w, x.dtype)
        bc = compute_weight(b, x.dtype) if b is not None else None
        if x2.is_cuda and x2.dtype in KDT:
            out = _gd.fwd(x2.contiguous(), wc, bc)
        else:
            out = x2 @ wc.t()
            if bc is not None:
                out = out + bc
        if residual is not None:  # (tests only: the model fuses its residual adds into LayerNorm)
            out = out + residual.reshape(-1, Nout)
        ctx.has_residual = residual is not None
        ctx.save_for_backward(x2, w, b)
        return out.view(*x.shape[:-1], Nout)

    @staticmethod
    def backward(ctx, dout):
        x2, w, b = ctx.saved_tensors
        Nout = w.shape[0]
        d2 = dout.reshape(-1, Nout)
        dx = None
        if ctx.needs_input_grad[0]:
            wc = compute_weight(w, d2.dtype)
            dx = _gd.dgrad(d2.contiguous(), wc) if d2.is_cuda and d2.dtype in KDT else d2 @ wc
            dx = dx.view(*dout.shape[:-1], x2.shape[-1])
        gw, gb = weight_bias_grad(w, b, d2, x2)
        dres = dout if ctx.has_residual else None
        return dx, gw, gb, dres


def linear(x, w, b=None, residual=None):
    return LinearFn.apply(x, w, b, residual)


# ----------------------------------------------------------------------------
# MLP: c_proj(gelu(c_fc(x))) with the GELU in the GEMM epilogues (MI355X path)
# ----------------------------------------------------------------------------

class MLPFn(torch.autograd.Function):
    """c_proj(gelu(c_fc(x) + b_fc)) + b_proj as ONE autograd node.

    Forward: the c_fc GEMM's epilogue adds b_fc and writes g = gelu(u) and gelu'(u) (fp16,
    the backward's only use of u); the c_proj GEMM adds b_proj.  Backward: du = (dy W_proj) *
    gelu'(u) from one GEMM epilogue (a multiply),
    dx = du W_fc, both weight gradients accumulated in fp32 by the split-K GEMM, the bias
    gradients from the same kernel's dY fragments (``weight_bias_grad``)."""

    @staticmethod
    def forward(ctx, x, w_fc, b_fc, w_proj, b_proj, recompute=False):
        C = x.shape[-1]
        x2 = x.reshape(-1, C).contiguous()
        wf = compute_weight(w_fc, x.dtype)
        bf = compute_weight(b_fc, x.dtype) if b_fc is not None else None
        bp = compute_weight(b_proj, x.dtype) if b_proj is not None else None
        gp, g = _gd.fwd_gelu(x2, wf, bf)
        y = _gd.fwd(g, compute_weight(w_proj, x.dtype), bp)
        # recompute (selective recomputation, config key recompute_mlp): keep only the block's
        # input x2; the backward re-runs the c_fc GEMM and its GELU epilogue for gelu(u) /
        # gelu'(u) -- 16 of the ~36 bytes per token and channel a block keeps (utils/memory.py)
        ctx.recompute = bool(recompute)
        if ctx.recompute:
            ctx.save_for_backward(x2, w_fc, b_fc, w_proj, b_proj)
        else:
            ctx.save_for_backward(x2, gp, g, w_fc, b_fc, w_proj, b_proj)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w_proj.shape[0])

    @staticmethod
    def backward(ctx, dy):
        if ctx.recompute:
            x2, w_fc, b_fc, w_proj, b_proj = ctx.saved_tensors
            bf = compute_weight(b_fc, x2.dtype) if b_fc is not None else None
            gp, g = _gd.fwd_gelu(x2, compute_weight(w_fc, x2.dtype), bf)
        else:
            x2, gp, g, w_fc, b_fc, w_proj, b_proj = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        gw_proj, gb_proj = weight_bias_grad(w_proj, b_proj, dy2, g)
        du = _gd.dgrad_dgelu(dy2, compute_weight(w_proj, dy.dtype), gp)
        gw_fc, gb_fc = weight_bias_grad(w_fc, b_fc, du, x2)
        dx = _gd.dgrad(du, compute_weight(w_fc, dy.dtype))
        return dx.view(ctx.xshape), gw_fc, gb_fc, gw_proj, gb_proj, None


def mlp(x, w_fc, b_fc, w_proj, b_proj, recompute=False):
    """c_proj(gelu(c_fc(x))): one fused autograd node on MI355X (bf16 / fp16).  ``recompute``:
    the node keeps only its input and redoes the c_fc GEMM + GELU in the backward."""
    if x.is_cuda and x.dtype in KDT:
        return MLPFn.apply(x, w_fc, b_fc, w_proj, b_proj, recompute)
    return linear(gelu(linear(x, w_fc, b_fc)), w_proj, b_proj)


# ----------------------------------------------------------------------------
# GELU (exact erf, nn.GELU() default)
# ----------------------------------------------------------------------------

_INV_SQRT2 = 1.0 / math.sqrt(2.0)
_INV_SQRT2PI = 1.0 / math.sqrt(2.0 * math.pi)


class GeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        if _kern(x):
            x = x.contiguous()
            y = torch.empty_like(x)
            _lib.call(_sym("nsa_gelu_fwd", x.dtype), _lib.ptr(x), _lib.ptr(y), x.numel(), _lib.stream())
            return y
        return F.gelu(x.float()).to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        if _kern(dy):
            dy = dy.contiguous()
            dx = torch.empty_like(x)
            _lib.call(_sym("nsa_gelu_bwd", dy.dtype), _lib.ptr(dy), _lib.ptr(x), _lib.ptr(dx), x.numel(), _lib.stream())
            return dx
        xf = x.float()
        cdf = 0.5 * (1.0 + torch.erf(xf * _INV_SQRT2))
        pdf = torch.exp(-0.5 * xf * xf) * _INV_SQRT2PI
        return (dy.float() * (cdf + xf * pdf)).to(dy.dtype)


def gelu(x):
    return GeluFn.apply(x)


# ----------------------------------------------------------------------------
# causal self-attention on the packed qkv activation [B, T, 3C]
# ----------------------------------------------------------------------------

def _attn_reference(q, k, v, p, seed):
    """fp32 causal attention with a reproducible dropout mask. q,k,v: [B,H,T,D]."""
    T, D = q.shape[-2], q.shape[-1]
    att = (q @ k.transpose(-2, -1)) * (1.0 / math.sqrt(D))
    mask = torch.ones(T, T, dtype=torch.bool, device=q.device).tril()
    att = att.masked_fill(~mask, float("-inf"))
    att = torch.softmax(att, dim=-1)
    if p > 0:
        att = att * _cpu_keep_mask(att.shape, p, seed, att.device) / (1.0 - p)
    return att @ v


_FLASH_FWD = {"auto": 0, "v1": 1, "v5": 5}
_FLASH_BWD = {"v1": 1, "v2": 2, "v3": 3}


@contextlib.contextmanager
def flash_variant(fwd: str | None = None, bwd: str | None = None, order: int | None = None):
    """Select flash-attention kernels for the duration of a ``with`` block (tests, A/B).

    The library resolves its choice once per process (``NSA_FLASH_FWD`` / ``NSA_FLASH_BWD``
    / ``NSA_ATTN_ORDER``, csrc/kernels/flash_attn.hip FlashConfig); this switches it through
    ``nsa_flash_set_variant`` and restores the previous selection afterwards."""
    prev = _lib.call_ret("nsa_flash_set_variant", _FLASH_FWD[fwd] if fwd else -1, _FLASH_BWD[bwd] if bwd else -1,
                         -1 if order is None else int(order))
    try:
        yield
    finally:
        _lib.call_ret("nsa_flash_set_variant", prev & 0xF, (prev >> 4) & 0xF, (prev >> 8) & 0xF)


class AttentionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, n_head, p):
        B, T, C3 = qkv.shape
        C = C3 // 3
        H = n_head
        D = C // H
        seed = new_seed() if p > 0 else 0
        ctx.meta = (B, T, H, D, p, seed)
        scale = 1.0 / math.sqrt(D)
        ctx.kern = _kern(qkv)
        if ctx.kern:
            assert D in (32, 64, 128), "flash kernel supports head_dim 32/64/128"
            qkv = qkv.contiguous()
            y = torch.empty(B, T, C, device=qkv.device, dtype=qkv.dtype)
            lse = torch.empty(B, H, T, device=qkv.device, dtype=F32)
            _lib.call(_sym("nsa_flash_fwd", qkv.dtype), _lib.ptr(qkv), _lib.ptr(y), _lib.ptr(lse), B, T, H, D,
                      scale, p, seed, _lib.stream())
            ctx.save_for_backward(qkv, y, lse)
            return y
        q, k, v = qkv.float().view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
        y = _attn_reference(q, k, v, p, seed).transpose(1, 2).reshape(B, T, C)
        ctx.save_for_backward(qkv)
        return y.to(qkv.dtype)

    @staticmethod
    def backward(ctx, dy):
        B, T, H, D, p, seed = ctx.meta
        C = H * D
        if ctx.kern:
            qkv, y, lse = ctx.saved_tensors
            dy = dy.contiguous()
            dqkv = torch.empty_like(qkv)
            # 2 x [B, H, T] fp32 workspace for the per-query row constants (delta, lse);
            # dQ is written once, in bf16, by its own kernel (no atomics: a fused dK/dV/dQ
            # kernel with dQ by float atomics measured slower, profiles/r5_attn_fused_experiment.md)
            ws = torch.empty(2, B, H, T, device=dy.device, dtype=F32)
            dy = dy.to(qkv.dtype)
            _lib.call(_sym("nsa_flash_bwd2", qkv.dtype), _lib.ptr(qkv), _lib.ptr(y), _lib.ptr(dy), _lib.ptr(lse),
                      _lib.ptr(ws), _lib.ptr(dqkv), B, T, H, D, 1.0 / math.sqrt(D), p, seed, _lib.stream())
            return dqkv, None, None
        (qkv,) = ctx.saved_tensors
        with torch.enable_grad():
            x = qkv.detach().float().requires_grad_(True)
            q, k, v = x.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
            y = _attn_reference(q, k, v, p, seed).transpose(1, 2).reshape(B, T, C)
            (g,) = torch.autograd.grad(y, x, dy.float())
        return g.to(qkv.dtype), None, None


def attention(qkv, n_head: int, p: float, training: bool):
    return AttentionFn.apply(qkv, n_head, p if training else 0.0)


# ----------------------------------------------------------------------------
# incremental decoding: KV cache append + single-query attention over the cache
# (runtime/decode.py; csrc/kernels/decode.hip).  Inference only (no autograd).
# ----------------------------------------------------------------------------

def kv_append(qkv, kc, vc, pos=None, pos0: int = 0):
    """Write the K / V rows of ``qkv`` [B, S, 3C] into the caches [B, H, Tmax, D] at
    positions p0 .. p0+S-1, p0 = ``pos`` (int64 device tensor, graph-safe) or ``pos0``."""
    B, S, C3 = qkv.shape
    _, H, Tmax, D = kc.shape
    if qkv.is_cuda and qkv.dtype == BF16 and D % 8 == 0:
        qkv = qkv.contiguous()
        _lib.call("nsa_kv_append", _lib.ptr(qkv), _lib.ptr(kc), _lib.ptr(vc), _lib.ptr(pos), int(pos0), B, S, H, D,
                  Tmax, _lib.stream())
        return
    p0 = int(pos.item()) if pos is not None else int(pos0)
    k, v = qkv.view(B, S, 3, H, D)[:, :, 1:].permute(2, 0, 3, 1, 4)
    kc[:, :, p0:p0 + S] = k.to(kc.dtype)
    vc[:, :, p0:p0 + S] = v.to(vc.dtype)


class AttnPartials(NamedTuple):
    """Un-combined flash-decoding partials of one decode row (``decode_attention(...,
    combine=False)``): (m, l, o[64]) per (head, 256-key chunk) in ``ws``.  Only
    ``decode_linear`` consumes them: it combines the chunks in its own prologue."""
    ws: torch.Tensor
    n_split: int
    C: int


def decode_attention(qkv, kc, vc, pos, n_head: int, append: bool = False, combine: bool = True):
    """Causal attention of the newest token (position ``pos``) over the caches:
    qkv [B, 1, 3C] -> [B, 1, C].  ``append``: also store the token's K / V at ``pos``
    (the fused form of ``kv_append``).  GPU (head dim 64): split-K flash-decoding
    kernels; otherwise fp32 torch (CPU reference).  ``combine=False`` with one row on the
    GPU returns the partials (``AttnPartials``) for ``decode_linear`` to combine."""
    B, S, C3 = qkv.shape
    C = C3 // 3
    _, H, Tmax, D = kc.shape
    scale = 1.0 / math.sqrt(D)
    if qkv.is_cuda and qkv.dtype == BF16 and D == 64:
        qkv = qkv.contiguous()
        n_split = -(-Tmax // 256)
        ws = torch.empty(B * H * n_split * (4 + D), device=qkv.device, dtype=F32)  # (m, l, pad, o[D]) per chunk
        partial = not combine and B == 1 and GEMV_MAX_ROWS >= 1 and C <= 8192
        out = None if partial else torch.empty(B, 1, C, device=qkv.device, dtype=qkv.dtype)
        _lib.call("nsa_decode_attn", _lib.ptr(qkv), _lib.ptr(kc), _lib.ptr(vc), _lib.ptr(pos), _lib.ptr(ws),
                  _lib.ptr(out), B, H, D, Tmax, scale, 1 if append else 0, _lib.stream())
        return AttnPartials(ws, n_split, C) if partial else out
    if append:
        kv_append(qkv, kc, vc, pos)
    p = int(pos.item())
    q = qkv.view(B, 3, H, D)[:, 0].float()                      # [B, H, D]
    k = kc[:, :, :p + 1].float()                                 # [B, H, p+1, D]
    v = vc[:, :, :p + 1].float()
    att = torch.softmax(torch.einsum("bhd,bhkd->bhk", q, k) * scale, dim=-1)
    y = torch.einsum("bhk,bhkd->bhd", att, v)
    return y.reshape(B, 1, C).to(qkv.dtype)


GEMV_MAX_ROWS = int(os.environ.get("NSA_GEMV_MAX_ROWS", "1"))
# decode batches of 2..SKINNY_MAX_ROWS rows: the MFMA weight-streaming kernel (nsa_skinny_gemm).
# HIP-graph decode, ms/token (GPT-2 124M / 1.5B): batch 8 0.685 / 4.24 with the library GEMM,
# 0.549 / 3.24 with this kernel; batch 64 0.938 / 5.45 vs 0.946 / 6.62 (every 16-column
# workgroup re-reads the whole 64-row X, 4x its weight bytes), so M > 16 goes to ``linear``
# (round 2 measured against the library GEMM; ``linear`` now runs our small-tile / NT kernels).
SKINNY_MAX_ROWS = int(os.environ.get("NSA_SKINNY_MAX_ROWS", "16"))
# residual add + LayerNorm recomputed in the skinny GEMM's prologue (nsa_skinny_ln_gemm) up to
# this many rows; HIP-graph decode ms/token, 124M / 1.5B: batch 8 0.532 / 3.34 unfused vs
# 0.532 / 3.18 fused; batch 16 0.597 / 3.78 unfused vs 0.667 / 4.10 fused (every workgroup
# normalises all rows: the per-workgroup prologue outgrows the saved launch)
SKINNY_LN_MAX_ROWS = int(os.environ.get("NSA_SKINNY_LN_MAX_ROWS", "8"))


def decode_linear(x, w, b=None, gelu: bool = False, out_f32: bool = False):
    """act(x @ W^T + b) for a decode batch: with <= GEMV_MAX_ROWS rows one weight-streaming
    kernel with the bias / exact GELU in its epilogue on the GPU (bf16, K % 8 == 0);
    otherwise ``linear`` (+ ``gelu``).  Inference only.  Measured (GPT-2 124M / 1.5B
    decode, HIP graph): batch 1 0.69 / 3.02 ms per token vs 0.90 / 4.70 with the (round-2)
    library GEMM + bias copy.  The vector GEMV's VALU grows with the rows (batch 4: 1.52 ms
    per token at 124M in round 2), so the default cap is 1 row (``NSA_GEMV_MAX_ROWS``) and
    batches of 2 .. ``NSA_SKINNY_MAX_ROWS`` (16) rows run on ``nsa_skinny_gemm`` (MFMA
    weight stream, bias / GELU epilogue) when N % 16 == 0 and K % 32 == 0; larger batches go
    to ``linear`` (our small-tile / NT kernels: no library GEMM on this path)."""
    N = w.shape[0]
    if isinstance(x, AttnPartials):  # one row; the attention combine runs in the GEMV prologue
        y = torch.empty(N, device=x.ws.device, dtype=F32 if out_f32 else BF16)
        _lib.call("nsa_gemv_attn", _lib.ptr(x.ws), x.n_split, _lib.ptr(compute_weight(w, BF16)),
                  _lib.ptr(compute_weight(b, BF16) if b is not None else None), _lib.ptr(y), N, x.C,
                  1 if gelu else 0, 1 if out_f32 else 0, _lib.stream())
        return y.view(1, 1, N)
    K = x.shape[-1]
    rows = x.numel() // K
    if x.is_cuda and x.dtype == BF16 and rows <= GEMV_MAX_ROWS and K % 8 == 0:
        x2 = x.reshape(rows, K).contiguous()
        wc = compute_weight(w, BF16)
        bc = compute_weight(b, BF16) if b is not None else None
        y = torch.empty(rows, N, device=x.device, dtype=F32 if out_f32 else BF16)
        _lib.call("nsa_gemv", _lib.ptr(x2), _lib.ptr(wc), _lib.ptr(bc), _lib.ptr(y), rows, N, K, 1 if gelu else 0,
                  1 if out_f32 else 0, _lib.stream())
        return y.view(*x.shape[:-1], N)
    if (x.is_cuda and x.dtype == BF16 and 2 <= rows <= SKINNY_MAX_ROWS and K % 32 == 0 and N % 16 == 0
            and not (gelu and out_f32)):
        x2 = x.reshape(rows, K).contiguous()
        wc = compute_weight(w, BF16)
        bc = compute_weight(b, BF16) if b is not None else None
        y = torch.empty(rows, N, device=x.device, dtype=F32 if out_f32 else BF16)
        _lib.call("nsa_skinny_gemm", _lib.ptr(x2), _lib.ptr(wc), _lib.ptr(bc), _lib.ptr(y), rows, N, K,
                  1 if gelu else 0, 1 if out_f32 else 0, _lib.stream())
        return y.view(*x.shape[:-1], N)
    y = linear(x, w, b)
    if gelu:
        y = GeluFn.apply(y)
    return y.float() if out_f32 else y


def decode_linear_ln(res, branch, ln_w, ln_b, w, b=None, gelu: bool = False, out_f32: bool = False,
                     out_dtype=None, pos_inc=None):
    """One decode row through residual add + LayerNorm + linear:
    s = res + branch, y = act(LN(s) @ W^T + b); returns (s, y) (s is res itself when
    ``branch`` is None).  GPU (fp32 residual, bf16 weights, one row): one kernel that
    recomputes the LayerNorm per workgroup (``nsa_gemv_ln``); otherwise add_layer_norm
    + ``decode_linear`` (``out_dtype``: the LayerNorm output dtype there).  ``pos_inc``: an
    int64 device tensor incremented by one after the row (inside the kernel on the fused
    path: the decode step's position update without its own launch).  Inference only."""
    C = res.shape[-1]
    rows = res.numel() // C
    if (res.is_cuda and res.dtype == F32 and rows == 1 and GEMV_MAX_ROWS >= 1 and C % 8 == 0 and C <= 8192
            and (branch is None or branch.dtype == BF16)):
        N = w.shape[0]
        r2 = res.reshape(C).contiguous()
        br = branch.reshape(C).contiguous() if branch is not None else None
        s_out = torch.empty_like(r2) if branch is not None else None
        lw, lb = compute_weight(ln_w, BF16), compute_weight(ln_b, BF16) if ln_b is not None else None
        wc = compute_weight(w, BF16)
        bc = compute_weight(b, BF16) if b is not None else None
        y = torch.empty(N, device=res.device, dtype=F32 if out_f32 else BF16)
        _lib.call("nsa_gemv_ln", _lib.ptr(r2), _lib.ptr(br), _lib.ptr(s_out), _lib.ptr(lw), _lib.ptr(lb), _lib.ptr(wc),
                  _lib.ptr(bc), _lib.ptr(y), N, C, LN_EPS, 1 if gelu else 0, 1 if out_f32 else 0, _lib.ptr(pos_inc),
                  _lib.stream())
        s_new = s_out.view(res.shape) if branch is not None else res
        return s_new, y.view(*res.shape[:-1], N)
    N = w.shape[0]
    if (res.is_cuda and res.dtype == F32 and 2 <= rows <= min(SKINNY_MAX_ROWS, SKINNY_LN_MAX_ROWS) and C % 32 == 0
            and C <= 1920
            and N % 16 == 0 and not (gelu and out_f32) and (branch is None or branch.dtype == BF16)
            and out_dtype in (None, BF16)):
        # 2..16 rows: residual add + LayerNorm recomputed per workgroup in the skinny GEMM's prologue
        r2 = res.reshape(rows, C).contiguous()
        br = branch.reshape(rows, C).contiguous() if branch is not None else None
        s_out = torch.empty_like(r2) if branch is not None else None
        lw, lb = compute_weight(ln_w, BF16), compute_weight(ln_b, BF16) if ln_b is not None else None
        wc = compute_weight(w, BF16)
        bc = compute_weight(b, BF16) if b is not None else None
        y = torch.empty(rows, N, device=res.device, dtype=F32 if out_f32 else BF16)
        _lib.call("nsa_skinny_ln_gemm", _lib.ptr(r2), _lib.ptr(br), _lib.ptr(s_out), _lib.ptr(lw), _lib.ptr(lb),
                  LN_EPS, _lib.ptr(wc), _lib.ptr(bc), _lib.ptr(y), rows, N, C, 1 if gelu else 0,
                  1 if out_f32 else 0, _lib.stream())
        if pos_inc is not None:
            pos_inc.add_(1)
        s_new = s_out.view(res.shape) if branch is not None else res
        return s_new, y.view(*res.shape[:-1], N)
    if branch is None:
        s_new, h = layer_norm_pass(res, ln_w, ln_b, out_dtype=out_dtype)
    else:
        s_new, h = add_layer_norm(res, branch, ln_w, ln_b, out_dtype=out_dtype)
    y = decode_linear(h, w, b, gelu=gelu, out_f32=out_f32)
    if pos_inc is not None:
        pos_inc.add_(1)
    return s_new, y


def decode_embed_linear_ln(tok, pos, wte, wpe, ln_w, ln_b, w, b=None, dtype=BF16, res_dtype=F32, out_dtype=None):
    """First linear of a decode step with the embedding in front: x = wte[tok] + wpe[pos]
    (rows of the ``dtype`` weight copies summed in fp32, stored as ``res_dtype``: the
    residual stream), y = LN(x) @ W^T + b; returns (x [B, 1, C], y [B, 1, N]).  One GPU
    kernel for a single bf16 row with an fp32 stream (``nsa_gemv_emb_ln``)."""
    B = tok.numel()
    C = wte.shape[1]
    wte_c, wpe_c = compute_weight(wte, dtype), compute_weight(wpe, dtype)
    if (tok.is_cuda and B == 1 and dtype == BF16 and res_dtype == F32 and GEMV_MAX_ROWS >= 1 and C % 8 == 0
            and C <= 8192):
        N = w.shape[0]
        x = torch.empty(1, 1, C, device=tok.device, dtype=F32)
        y = torch.empty(N, device=tok.device, dtype=BF16)
        lw, lb = compute_weight(ln_w, BF16), compute_weight(ln_b, BF16) if ln_b is not None else None
        wc = compute_weight(w, BF16)
        bc = compute_weight(b, BF16) if b is not None else None
        _lib.call("nsa_gemv_emb_ln", _lib.ptr(tok), _lib.ptr(pos), _lib.ptr(wte_c), _lib.ptr(wpe_c), _lib.ptr(x),
                  _lib.ptr(lw), _lib.ptr(lb), _lib.ptr(wc), _lib.ptr(bc), _lib.ptr(y), N, C, LN_EPS, 0, 0,
                  _lib.stream())
        return x, y.view(1, 1, N)
    x = wte_c.index_select(0, tok.view(-1)).float() + wpe_c.index_select(0, pos.view(-1)).float()
    x = x.to(res_dtype).view(B, 1, C)
    return decode_linear_ln(x, None, ln_w, ln_b, w, b, out_dtype=out_dtype)


def sample_topk_(logits, temperature: float, top_k, salt: int, pos, tok, gen, salt_dev=None):
    """Device-side nanoGPT sampling (logits / temperature, top-k, softmax, multinomial)
    of logits [B, V] fp32: the drawn ids go to ``tok`` [B, 1] and ``gen[:, pos]``
    (``pos``: int64 device scalar).  One kernel, graph-capturable; the uniform draw is a
    counter hash of (salt ^ salt_dev, row, position), so a run is reproducible from its
    salts.  ``salt_dev`` (int64 device scalar, optional) is read at run time: rewriting it
    gives a captured sampling graph a fresh stream."""
    B, V = logits.shape
    k = 0 if top_k is None else min(int(top_k), V)
    if logits.is_cuda:
        lg = logits if logits.dtype == F32 and logits.stride(1) == 1 else logits.float().contiguous()
        _lib.call("nsa_sample_topk", _lib.ptr(lg), B, V, lg.stride(0), float(temperature), k, int(salt) & (2 ** 64 - 1),
                  _lib.ptr(salt_dev), _lib.ptr(pos), _lib.ptr(tok), _lib.ptr(gen), gen.stride(0), _lib.stream())
        return
    lg = logits.float() / temperature
    if k > 0:
        v, _ = torch.topk(lg, k)
        lg = lg.masked_fill(lg < v[:, -1:], -float("Inf"))
    nxt = torch.multinomial(torch.softmax(lg, dim=-1), num_samples=1)
    tok.copy_(nxt.view_as(tok))
    gen.index_copy_(1, pos, nxt)


# ----------------------------------------------------------------------------
# tied lm_head + cross-entropy (ignore_index=-1, mean over valid targets)
# ----------------------------------------------------------------------------

def lm_head_rows(V: int) -> int:
    """Rows of the lm_head GEMM operand: V padded to a multiple of 64 (and >= 256, one NT
    tile) so every vocabulary runs on the persistent GEMM kernel.  GPT-2's 50257 -> 50304
    (the same padding nanoGPT's scratch config applies to the vocabulary itself); the
    padding rows are zero and their logits are excluded from the softmax."""
    return V if (V % 64 == 0 and V >= 256) else max(256, -(-V // 64) * 64)


def _lm_weight(w, dtype=BF16):
    """(16-bit [Vpad, C] operand in ``dtype``, fp32 [Vpad, C] gradient view or None).  A
    FlatParamStore keeps padded views of the tied weight (``compute_padded`` /
    ``main_grad_padded``); otherwise the padded operand is a per-call copy and the gradient is
    returned to autograd."""
    V, C = w.shape
    Vp = lm_head_rows(V)
    cp = getattr(w, "compute_padded", None)
    if cp is not None and cp.dtype == dtype:
        return cp, getattr(w, "main_grad_padded", None)
    if Vp == V:
        return compute_weight(w, dtype), getattr(w, "main_grad", None)
    # no flat store (sample / eval scripts): the padded operand is cached on the weight for
    # its current contents (generation, version, storage), so a token-by-token generate()
    # does not allocate and copy the whole [Vpad, C] table per token; never cached while a
    # HIP graph is being captured (the copy is then part of the graph)
    capturing = w.is_cuda and torch.cuda.is_current_stream_capturing()
    key = (_gd._weight_gen, w._version, w.data_ptr(), dtype)
    hit = getattr(w, "_nsa_lm_pad", None)
    if not capturing and hit is not None and hit[0] == key:
        return hit[1], None
    # a fresh buffer on every key change: a consumer still holding the operand of
    # an earlier forward keeps the weights it was given
    wp = torch.zeros(Vp, C, device=w.device, dtype=dtype)
    wp[:V] = compute_weight(w, dtype)
    if not capturing:
        try:
            w._nsa_lm_pad = (key, wp)
        except (AttributeError, RuntimeError):
            pass
    return wp, None


def _lm_grad_out(w, gw, scratch):
    """Finish the lm_head weight gradient: ``gw`` is the padded gradient view itself (already
    accumulated), or a scratch [Vpad, C] buffer whose first V rows go to ``main_grad`` (or to
    autograd when there is none)."""
    V = w.shape[0]
    if scratch:
        mg = getattr(w, "main_grad", None)
        if mg is None:
            return gw[:V].to(w.dtype)
        mg.add_(gw[:V])
    notify_grad_ready(w)
    return None


def _fused_xent_ok(M, C, Vp):
    # deterministic mode too once the onehot dW term is the sorted form: every other piece
    # writes each output once (row-sum slots, ordered combine, per-row fix-up) and the dW GEMM
    # reduces its K splits in order there
    return ((not _gd.DETERMINISTIC or XENT_FIX_SORTED) and M % 4 == 0 and _gemm.nt_supported(M, Vp, C)
            and _gemm.nt_supported(M, C, Vp) and C <= 8192)


# The fused cross-entropy for fp16 compute (default; NSA_XENT_F16=0 selects autocast's form:
# fp16 logits, the fp32 softmax pass, fp16 dlogits): 13.5 ms/step faster at GPT-2 124M
# (413.5 vs 427.0 ms).  Its dW = E^T (x g / S) carries a row's 1/S on the fp16 x operand,
# which for a large S (the target logit far below the row max) lands in fp16's subnormal
# range: ~5e-3 relative error on the vocabulary rows no token targets at init-like logits,
# against 4e-4 for autocast's form.  Everywhere else it is the more accurate of the two
# (fp16 dlogits round every p - onehot to 2^-11 and go subnormal below p = 6e-5): against
# fp32 on the same fp16 inputs at the bench's g, dW 5.4e-5 vs 2.1e-4 and dX 2.1e-4 vs
# 2.9e-4 at init-like logits, dW 1.4e-4 vs 1.2e-3 and dX 2.1e-4 vs 1.2e-3 at sharp ones
# (scripts/debug/xent_f16_vs_autocast.py, profiles/r5_xent16_vs_autocast.log).
XENT_F16 = os.environ.get("NSA_XENT_F16", "1") == "1"


class XentF16Guard:
    """Falls back from the fused fp16 cross-entropy when its exact fix-up gets expensive.

    fp16 E flags every row whose largest logit passes its target's by ~11 nats, and each
    flagged row costs two V x C passes in ``nsa_xent_fixup``: at GPT-2 124M shapes the loss
    forward goes from 9.6 ms to 17.0 / 35.9 / 141.5 ms with 0.1 / 1 / 5 % of the rows flagged
    (profiles/r6_xent_f16_cliff.md).  That share grows as a model trains, so the fused form is
    only kept while the flagged share stays under ``max_frac``.

    The forward adds each call's flagged count and row count into two device counters. Both
    adds are stream-ordered, so they also happen inside a captured HIP graph. ``poll()`` runs
    once per optimizer step. It copies the counters to pinned host memory without blocking
    and reads the copy from the previous poll once that copy's event has completed. When the
    share over at least ``min_rows`` rows exceeds ``max_frac``, the guard trips. Every later
    fp16 call then takes autocast's form (fp16 logits and the fp32 softmax pass). ``poll()``
    returns True on that step, so the trainer can drop a graph captured with the fused form.
    """

    def __init__(self, max_frac: float = 0.002, min_rows: int = 1 << 20):
        self.max_frac = float(max_frac)
        self.min_rows = int(min_rows)
        self.active = True
        self.counts = None  # device int64 [flagged, rows]
        self._host = None
        self._event = None
        self.last = None  # (flagged, rows) as last read

    def note(self, nfix, n_rows: int):
        if self.counts is None or self.counts.device != nfix.device:
            self.counts = torch.zeros(2, dtype=torch.int64, device=nfix.device)
        self.counts[0:1].add_(nfix)
        self.counts[1:2].add_(n_rows)

    def poll(self) -> bool:
        if not self.active or self.counts is None:
            return False
        if self.counts.device.type != "cuda":  # (CPU tests) a synchronous read
            vals = self.counts.tolist()
        else:
            vals = None
            if self._event is not None and self._event.query():
                vals = self._host.tolist()
            if self._host is None:
                self._host = torch.empty(2, dtype=torch.int64, pin_memory=True)
            if vals is not None or self._event is None:
                self._host.copy_(self.counts, non_blocking=True)
                self._event = torch.cuda.Event()
                self._event.record()
        if vals is None:
            return False
        self.last = (int(vals[0]), int(vals[1]))
        flagged, rows = self.last
        if rows >= self.min_rows and flagged > self.max_frac * rows:
            self.active = False
            print(f"[nanosandbox_amd] fused fp16 cross-entropy: {flagged} of {rows} rows needed the exact "
                  f"fix-up (> {self.max_frac:.2%}); switching to autocast's form (fp16 logits, fp32 softmax)")
            return True
        return False


XENT_F16_GUARD = XentF16Guard(float(os.environ.get("NSA_XENT_F16_MAXFIX", "0.002")))
# the lm_head dW onehot term by target-sorted rows (segsum.h) instead of fp32 atomics
XENT_FIX_SORTED = os.environ.get("NSA_XENT_FIX_SORTED", "1") == "1"


def _xent_range(dtype):
    """(shift, lo, hi) of the fused cross-entropy: the row sums S of E = exp(logit - target logit
    - shift) kept, outside [lo, hi] a row is recomputed exactly.  bf16 and fp16 both anchor E at
    the target logit (shift 0): fp16 E then spans autocast's fp16-dlogits precision, and its
    epilogue marks a saturated row (an entry above 65504: a logit ~11 nats above the target)
    with an inf sum."""
    return 0.0, 0.5, 1e30


class LMHeadLossFn(torch.autograd.Function):
    """loss = cross_entropy(x @ wte^T, targets, ignore_index=-1).

    GPU, fused (``csrc/kernels/xent_fused.hip``; bf16 or fp16): the lm_head GEMM's epilogue
    writes E = exp(logit - target logit) and per-tile row sums instead of the logits, so the
    [N, V] logits are never stored and never re-read; the backward GEMMs consume E with
    the softmax normalisation and the onehot term applied in fp32 in their epilogue / a
    row-scatter.  GPU, deterministic mode or shapes outside the NT kernel: logits GEMM +
    the separate cross-entropy pass that overwrites the logits with (softmax - onehot).
    """

    @staticmethod
    def forward(ctx, x, w, targets, need_grad):
        C = x.shape[-1]
        x2 = x.reshape(-1, C)
        t = targets.reshape(-1)
        N = x2.shape[0]
        V = w.shape[0]
        ctx.xshape = x.shape
        ctx.V = V
        if x.is_cuda and x.dtype in KDT:
            x2 = x2.contiguous()
            t = t.contiguous()
            wp, _ = _lm_weight(w, x.dtype)
            Vp = wp.shape[0]
            row_loss = torch.empty(N, device=x.device, dtype=F32)
            # E = exp(logit - target logit) in the compute dtype; fp16 unless XENT_F16 is off (see there)
            ctx.fused = _fused_xent_ok(N, C, Vp) and (x.dtype == BF16 or (XENT_F16 and XENT_F16_GUARD.active))
            if ctx.fused:
                shift, lo, hi = _xent_range(x.dtype)
                crow = torch.empty(N, device=x.device, dtype=F32)
                t32 = torch.empty(N, device=x.device, dtype=torch.int32)
                _lib.call(_sym("nsa_xent_tlogit", x.dtype), _lib.ptr(x2), C, _lib.ptr(wp), C, _lib.ptr(t),
                          _lib.ptr(crow), _lib.ptr(t32), N, C, V, shift, _lib.stream())
                slots = 2 * (-(-Vp // _gemm.TILE))
                part = torch.empty(slots, N, device=x.device, dtype=F32)
                e = _gemm.nt_xent(x2, wp, crow, part, V)
                _gd.record("lm_head_xent", N, Vp, C, "nt4/xent")
                inv_s = torch.empty(N, device=x.device, dtype=F32)
                nfix = torch.zeros(1, device=x.device, dtype=torch.int32)
                fixlist = torch.empty(N, device=x.device, dtype=torch.int32)
                _lib.call("nsa_xent_combine", _lib.ptr(part), slots, _lib.ptr(t32), _lib.ptr(row_loss),
                          _lib.ptr(inv_s), _lib.ptr(nfix), _lib.ptr(fixlist), N, lo, hi, shift, _lib.stream())
                _lib.call(_sym("nsa_xent_fixup", x.dtype), _lib.ptr(x2), C, _lib.ptr(wp), C, _lib.ptr(e), Vp,
                          _lib.ptr(t32),
                          _lib.ptr(nfix), _lib.ptr(fixlist), _lib.ptr(row_loss), _lib.ptr(inv_s), C, V, Vp,
                          _lib.stream())
                if x.dtype == F16:
                    XENT_F16_GUARD.note(nfix, N)
                n_valid = (t32 >= 0).sum().to(F32)
                ctx.save_for_backward(x2, w, e, t32, inv_s, n_valid)
            else:
                logits = _gd.fwd(x2, wp)
                _lib.call(_sym("nsa_xent_fwd", x.dtype), _lib.ptr(logits), _lib.ptr(t), _lib.ptr(row_loss), N, V, Vp,
                          1 if need_grad else 0, _lib.stream())
                n_valid = ((t >= 0) & (t < V)).sum().to(F32)
                ctx.save_for_backward(x2, w, logits, n_valid)
            return row_loss.sum() / n_valid
        ctx.fused = False
        wc = compute_weight(w, x.dtype)
        logits = x2.float() @ wc.float().t()
        logp = torch.log_softmax(logits, dim=-1)
        valid = t != -1
        n_valid = valid.sum().to(F32)
        tt = t.clamp(min=0)
        row_loss = -logp.gather(1, tt[:, None]).squeeze(1) * valid
        loss = row_loss.sum() / n_valid
        dlogits = logp.exp()
        dlogits[torch.arange(N, device=dlogits.device), tt] -= 1.0
        dlogits = dlogits * valid[:, None]
        ctx.save_for_backward(x2, w, dlogits, n_valid)
        return loss

    @staticmethod
    def backward(ctx, gl):
        V = ctx.V
        if ctx.fused:
            x2, w, e, t32, inv_s, n_valid = ctx.saved_tensors
            N, C = x2.shape
            wp, gwp = _lm_weight(w, x2.dtype)
            Vp = wp.shape[0]
            g = (gl.float() / n_valid).reshape(1).contiguous()
            coef = torch.empty(N, 2, device=x2.device, dtype=F32)
            wrows = torch.empty(N, C, device=x2.device, dtype=x2.dtype)
            xs = torch.empty(N, C, device=x2.device, dtype=x2.dtype)
            _lib.call(_sym("nsa_xent_bwd_prep", x2.dtype), _lib.ptr(x2), C, _lib.ptr(wp), C, _lib.ptr(t32),
                      _lib.ptr(inv_s), _lib.ptr(g), _lib.ptr(coef), _lib.ptr(wrows), _lib.ptr(xs), N, C,
                      _lib.stream())
            dx = _gemm.nt_xdx(e, _gd._wt(wp), wrows, coef)
            _gd.record("lm_head_xdx", N, C, Vp, "nt4/xdx")
            ret = gwp is None
            gw = torch.zeros(Vp, C, device=x2.device, dtype=F32) if ret else gwp
            _gd.wgrad_acc(e, xs, gw)
            if not _gd.DETERMINISTIC and _seg_lds_fits(V, C):
                # a small vocabulary: the LDS-privatised scatter-add over the targets
                part = _seg_lds_part(N, V, C, x2.device)
                _lib.call(_sym("nsa_xent_dw_fix_lds", x2.dtype), _lib.ptr(x2), C, _lib.ptr(e), Vp, _lib.ptr(t32),
                          _lib.ptr(inv_s), _lib.ptr(g), _lib.ptr(part), _lib.ptr(gw), C, N, C, V, _lib.stream())
            elif XENT_FIX_SORTED:
                # the onehot term atomic-free: rows sorted by target, one writer per vocab row
                ids, order, seg = sort_keys(t32, Vp)
                part = torch.empty(2 * (-(-N // 16)), C, device=x2.device, dtype=F32)
                _lib.call(_sym("nsa_xent_dw_fix_sorted", x2.dtype), _lib.ptr(x2), C, _lib.ptr(e), Vp, _lib.ptr(t32),
                          _lib.ptr(inv_s), _lib.ptr(g), _lib.ptr(ids), _lib.ptr(order), _lib.ptr(seg),
                          _lib.ptr(part), _lib.ptr(gw), C, N, C, Vp, _lib.stream())
            else:
                _lib.call(_sym("nsa_xent_dw_fix", x2.dtype), _lib.ptr(x2), C, _lib.ptr(e), Vp, _lib.ptr(t32),
                          _lib.ptr(inv_s), _lib.ptr(g), _lib.ptr(gw), C, N, C, _lib.stream())
            return dx.view(ctx.xshape), _lm_grad_out(w, gw, ret), None, None
        x2, w, dlogits, n_valid = ctx.saved_tensors
        g = (gl.float() / n_valid)
        if x2.is_cuda and x2.dtype in KDT:
            # the loss scale g = grad / n_valid stays fp32 (a device scalar read by the
            # kernel): only the scaled products are rounded to bf16 / fp16, not g itself
            wp, gwp = _lm_weight(w, x2.dtype)
            Vp = wp.shape[0]
            g = g.reshape(1).contiguous()
            xs = torch.empty_like(x2)
            scale_rows = _sym("nsa_scale_rows_bf16", x2.dtype)
            _lib.call(scale_rows, _lib.ptr(x2), _lib.ptr(xs), _lib.ptr(g), xs.numel(), _lib.stream())
            dx = _gd.dgrad(dlogits, wp)
            _lib.call(scale_rows, _lib.ptr(dx), _lib.ptr(dx), _lib.ptr(g), dx.numel(), _lib.stream())
            ret = gwp is None
            gw = torch.zeros(Vp, x2.shape[1], device=x2.device, dtype=F32) if ret else gwp
            _gd.wgrad_acc(dlogits, xs, gw)
            return dx.view(ctx.xshape), _lm_grad_out(w, gw, ret), None, None
        wc = compute_weight(w, x2.dtype)
        dx = (dlogits @ wc.float()) * g
        gw = weight_grad(w, dlogits, x2.float() * g)
        return dx.to(x2.dtype).view(ctx.xshape), gw, None, None


def lm_head_loss(x, w, targets):
    # grad mode is off inside Function.forward, so decide here whether the
    # fused kernel must also write d(loss)/d(logits) into the logits buffer
    need_grad = torch.is_grad_enabled() and (x.requires_grad or w.requires_grad)
    return LMHeadLossFn.apply(x, w, targets, need_grad)


def lm_head_logits(x, w):
    """Inference-time logits for the given positions: x @ wte^T (fp32 result)."""
    if x.is_cuda and x.dtype == BF16:
        V, C = w.shape
        wp, _ = _lm_weight(w)
        y = _gd.fwd(x.reshape(-1, C).contiguous(), wp)
        return y[:, :V].float().view(*x.shape[:-1], V)
    wc = compute_weight(w, x.dtype)
    return (x @ wc.t()).float()
