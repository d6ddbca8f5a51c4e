"""Per-shape GEMM backend selection (our gfx950 MFMA kernel vs hipBLASLt).

Every training GEMM shape is timed once, on first use, with both backends and
the faster one is cached (process-wide, optionally persisted to
``$NSA_GEMM_TUNE_FILE`` as JSON).  Measured on MI355X (profiles/, scripts/gemm_shapes.py):
our split-K weight-gradient kernel (fp32 accumulate straight into the flat
gradient) beats hipBLASLt's fp32-output path by 1.2-1.8x on every transformer
linear, the LDS-DMA ring kernel wins some input-gradient shapes (K-contiguous B
operand, e.g. c_attn and the 50304-wide lm_head), and hipBLASLt wins the plain
forwards — so the choice is per shape, not per op.

The MLP's activation can ride in a GEMM epilogue: ``fwd_gelu`` (u and gelu(u)
from one pass) and ``dgrad_dgelu`` (dY·W scaled by gelu'(u)) time the fused
epilogue variants of our kernel against "best GEMM + standalone GELU kernel",
so a fusion is used exactly where it measures faster.

Candidate names: ``hipblaslt`` / ``hipblaslt_t`` (the library, input grads also on the
cached weight transpose), ``nt`` (our persistent NT kernel, ``csrc/kernels/gemm_nt.hip``:
forward and — through the cached K-contiguous weight transpose — input grads),
``ntgelu`` / ``ntdgelu`` (the same kernel with the GELU / GELU' epilogue), ``nt4`` /
``nt4gelu`` / ``nt4dgelu`` (the four-wave persistent kernel, ``csrc/kernels/gemm_nt4.hip``), ``nsa<v>``
(weight grads: split-K kernel variant v of ``csrc/kernels/gemm.hip``).  Weight-gradient
candidates are timed into a scratch buffer so the real accumulator is touched exactly once.
Our kernels win ties: a library candidate is picked only when it is more than
``NSA_NATIVE_MARGIN`` (default 3 %) faster than the best native one.
``NSA_GEMM_BACKEND=nsa|hipblaslt`` pins a backend family (tests, A/B runs).
"""

from __future__ import annotations

import json
import os
import threading

import torch

from . import _lib
from . import gemm as _gemm

F32 = torch.float32
_table: dict = {}
_lock = threading.RLock()  # re-entrant: a "split" candidate tunes its inner GEMM while timed
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
        # per-process temp name: under torchrun every rank saves, and a shared
        # temp file could interleave writes before the atomic replace
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump({json.dumps(list(k)): v for k, v in _table.items()}, f, indent=1)
        os.replace(tmp, path)
    except OSError:
        pass


WGRAD_ALLOW_BF16 = os.environ.get("NSA_WGRAD_ALLOW_BF16", "0") == "1"
# Deterministic mode (config key ``deterministic``, ops.set_deterministic): weight
# gradients reduce their K splits in a fixed order (no fp32 atomics) and the library
# GEMM is left out of the weight-gradient race (its split-K reduction order is not ours
# to pin); the embedding backward switches to its sorted, atomic-free kernel.
DETERMINISTIC = False
NATIVE_MARGIN = float(os.environ.get("NSA_NATIVE_MARGIN", "0.03"))
# weight-grad split counts that fill whole CU rounds as tuner candidates (NSA_WGRAD_FULL_ROUNDS=0: off)
WGRAD_FULL_ROUNDS = os.environ.get("NSA_WGRAD_FULL_ROUNDS", "1") != "0"
WGRAD_VARIANTS = (1, 7, 9, 10)   # weight-grad (fp32 atomic epilogue) candidates: ring, ring64, phase, four-wave
# four-wave weight grads with stored split partials + an ordered reduce pass as candidates
# beside the atomic epilogue (NSA_WGRAD_STORE=1: on; off by default -- the tuner picks them
# for c_attn / c_fc dW by 2-3 %, but the step time does not move, docs/performance.md)
WGRAD_STORE_CANDS = os.environ.get("NSA_WGRAD_STORE", "0") != "0"


def _time_all(candidates: dict, rounds=3, reps=3):
    """Median-of-rounds time per candidate, rounds interleaved across candidates.

    A candidate timed alone in a short burst runs at the boost clock the idle chip
    grants; interleaving puts every candidate in the same power/thermal state, so
    compute-bound and memory-bound candidates compare fairly.
    """
    names = list(candidates)
    for n in names:  # warm: first launch, cache state
        candidates[n]()
    samples = {n: [] for n in names}
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for n in names:
            fn = candidates[n]
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            samples[n].append(e0.elapsed_time(e1) / reps)
    return {n: sorted(v)[len(v) // 2] for n, v in samples.items()}


def _is_library(name: str) -> bool:
    return name.startswith("hipblaslt") or name == "split_lib"


def choose(key, candidates: dict, fixed: str | None = None) -> str:
    """Return the name of the fastest candidate for ``key`` (timed once, then cached).

    Native candidates win within ``NATIVE_MARGIN`` of the fastest library candidate."""
    if FORCE:
        for name in candidates:
            if FORCE == "nsa" and not _is_library(name):
                return name
            if FORCE != "nsa" and name.startswith(FORCE):
                return name
        return next(iter(candidates))
    _load()
    hit = _table.get(key)
    if hit in candidates:
        return hit
    with _lock:
        if DETERMINISTIC:
            # no timing race: a fixed rule, identical in every run: the native
            # candidate (or the caller's ``fixed`` pick), else the first one
            best = fixed if fixed in candidates else next(
                (n for n in candidates if n.startswith("nt4")),
                next((n for n in candidates if n.startswith("nt") or n.startswith("det")), next(iter(candidates))))
        else:
            best = _pick_timed(candidates)
        best = _agree(best)
        _table[key] = best
        _save()
    return best


VERBOSE = os.environ.get("NSA_GEMM_TUNE_VERBOSE", "0") == "1"


def _pick_timed(candidates: dict) -> str:
    times = _time_all(candidates)
    if VERBOSE:
        print("gemm tune:", {n: round(t * 1e3, 1) for n, t in sorted(times.items(), key=lambda kv: kv[1])},
              flush=True)
    best = min(times, key=times.get)
    native = {n: t for n, t in times.items() if not _is_library(n)}
    if _is_library(best) and native:
        nb = min(native, key=native.get)
        if native[nb] <= times[best] * (1.0 + NATIVE_MARGIN):
            best = nb
    return best


def _agree(best: str) -> str:
    """Under DDP every rank must run the same kernels (identical numerics, one tuning pass
    instead of eight racing under shared power/thermal limits): rank 0's pick is broadcast.
    Every rank reaches each tuning decision at the same point of the same program, so the
    broadcasts pair up in order."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return best
    obj = [best]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def table():
    return dict(_table)


# ------------------------------------------------------------------ ops
def _nsa_ok(*ts):
    return all(t.is_contiguous() and t.data_ptr() % 16 == 0 for t in ts)


def _variant(name):
    """'nsa7' -> 7, 'nsa7/s28' -> 7, 'fused8' -> 8."""
    return int(name.split("/")[0].lstrip("abcdefghijklmnopqrstuvwxyz_"))


def _splits(name):
    return int(name.split("/s")[1]) if "/s" in name else None


def _library_ok(M, N, K):
    """Whether a library GEMM may run on the main stream.

    With the weight-gradient side stream on (ops/streams.py), shapes for which
    hipBLASLt's gfx950 pick is a persistent Stream-K kernel (``_SK3``: its
    workgroups wait on each other's partial tiles) must not share the GPU with a
    concurrent stream — measured on the 768 x 768 projection (attn.c_proj fwd and
    input grad at n_embd = 768, M = 122880); those go to our kernel instead."""
    from . import streams

    return not (streams.ENABLED and streams.CONCURRENT_COMPUTE and N <= 1024 and K <= 1024
                and M * N * K >= 2 ** 34)


def _fwd_pick(x2, w):
    """The forward backend for this shape ("hipblaslt" / "nt"; tuned on first use)."""
    M, K = x2.shape
    N = w.shape[0]
    if not (_nsa_ok(x2, w) and _gemm.nt_supported(M, N, K)):
        return "hipblaslt"
    cands = {"hipblaslt": lambda: x2 @ w.t()} if _library_ok(M, N, K) else {}
    cands["nt"] = lambda: _gemm.nt(x2, w)
    if _gemm.nt4_supported(M, N, K):
        cands["nt4"] = lambda: _gemm.nt(x2, w, w4=True)
    return choose(("fwd", M, N, K), cands)


def _native(name, a, b, epi=0, u=None):
    """Run native candidate ``name`` ("nt*": eight-wave kernel, "nt4*": four-wave kernel)."""
    return _gemm.nt(a, b, epi=epi, u=u, w4=name.startswith("nt4"))


def fwd(x2, w):
    """y = x2 @ w^T (bf16)."""
    name = _fwd_pick(x2, w)
    return x2 @ w.t() if name == "hipblaslt" else _native(name, x2, w)


# Weight generation: bumped whenever the bf16 compute weights are rewritten outside
# torch's in-place ops (fused AdamW kernel, FlatParamStore.refresh_compute), so cached
# derived copies of a weight (its transpose, below) are rebuilt once per optimizer step.
_weight_gen = 0


def weights_changed():
    global _weight_gen
    _weight_gen += 1


def _wt(w):
    """w^T as a contiguous tensor, cached on the weight tensor for the current generation.

    hipBLASLt runs dX = dY·W much faster with W stored K-contiguous (the forward's
    "TN" layout) than as the row-major nn.Linear weight ("NN"): 652 vs ~480 us for
    mlp.c_proj at 122880 tokens.  Transposing a weight costs microseconds and is
    amortised over every micro-step of an optimizer step.  Inside HIP-graph capture
    the transpose is recomputed (captured into the graph) instead of cached."""
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
    if w.is_cuda and w.dtype == torch.bfloat16 and R % 64 == 0 and C % 64 == 0 and w.is_contiguous():
        if out is None or out.shape != (C, R) or out.dtype != w.dtype or out.device != w.device:
            out = torch.empty(C, R, device=w.device, dtype=w.dtype)
        _lib.call("nsa_transpose_bf16", _lib.ptr(w), _lib.ptr(out), R, C, _lib.stream())
        return out
    return w.t().contiguous()


def _dgrad_pick(dy2, w):
    """The input-gradient backend for this shape (tuned on first use)."""
    M, N = dy2.shape
    K = w.shape[1]
    if not (_nsa_ok(dy2, w) and _gemm.nt_supported(M, K, N)):
        return "hipblaslt"
    cands = {"hipblaslt": lambda: dy2 @ w, "hipblaslt_t": lambda: dy2 @ _wt(w).t()} if _library_ok(M, K, N) else {}
    cands["nt"] = lambda: _gemm.nt(dy2, _wt(w))
    if _gemm.nt4_supported(M, K, N):
        cands["nt4"] = lambda: _gemm.nt(dy2, _wt(w), w4=True)
    return choose(("dgrad", M, N, K), cands)


def dgrad(dy2, w):
    """dx = dy2 @ w (bf16)."""
    from . import streams

    streams.before_compute(dy2)  # the side stream's weight GEMMs never share the GPU with this one
    name = _dgrad_pick(dy2, w)
    if name == "hipblaslt":
        return dy2 @ w
    if name == "hipblaslt_t":
        return dy2 @ _wt(w).t()
    return _native(name, dy2, _wt(w))


def _gelu_fwd(u):
    from . import _lib

    g = torch.empty_like(u)
    _lib.call("nsa_gelu_fwd", _lib.ptr(u), _lib.ptr(g), u.numel(), _lib.stream())
    return g


def _gelu_bwd(dg, u):
    from . import _lib

    du = torch.empty_like(dg)
    _lib.call("nsa_gelu_bwd", _lib.ptr(dg), _lib.ptr(u), _lib.ptr(du), du.numel(), _lib.stream())
    return du


def fwd_gelu(x2, w):
    """(u, gelu(u)) with u = x2 @ w^T: fused GEMM epilogue or GEMM + GELU kernel, whichever is faster."""
    M, K = x2.shape
    N = w.shape[0]
    if not (_nsa_ok(x2, w) and _gemm.nt_supported(M, N, K)):
        u = x2 @ w.t()
        return u, _gelu_fwd(u)

    def split():
        u = fwd(x2, w)
        return u, _gelu_fwd(u)

    # the split form counts as a library candidate when its GEMM is the library's, so the
    # fused kernel wins within NATIVE_MARGIN of it (as against a plain library GEMM)
    sname = "split_lib" if _is_library(_fwd_pick(x2, w)) else "split"
    cands = {sname: split, "ntgelu": lambda: _gemm.nt(x2, w, epi=_gemm.NT_EPI_GELU)}
    if _gemm.nt4_supported(M, N, K):
        cands["nt4gelu"] = lambda: _gemm.nt(x2, w, epi=_gemm.NT_EPI_GELU, w4=True)
    name = choose(("fwd_gelu", M, N, K), cands)
    return split() if name.startswith("split") else _native(name, x2, w, epi=_gemm.NT_EPI_GELU)


def dgrad_dgelu(dy2, w, u, between=None):
    """(dy2 @ w) * gelu'(u): fused GEMM epilogue or GEMM + GELU-backward kernel.

    ``between`` (optional callable) runs after the GEMM is issued and before the
    GELU backward of the split form (after the fused kernel otherwise): the side
    stream's weight-GEMM fork point (ops/streams.py)."""
    M, N = dy2.shape
    K = w.shape[1]
    if not (_nsa_ok(dy2, w, u) and _gemm.nt_supported(M, K, N)):
        dg = dy2 @ w
        if between is not None:
            between()
        return _gelu_bwd(dg, u)

    def split(hook=None):
        dg = dgrad(dy2, w)
        if hook is not None:
            hook()
        return _gelu_bwd(dg, u)

    sname = "split_lib" if _is_library(_dgrad_pick(dy2, w)) else "split"
    cands = {sname: split, "ntdgelu": lambda: _gemm.nt(dy2, _wt(w), epi=_gemm.NT_EPI_DGELU, u=u)}
    if _gemm.nt4_supported(M, K, N):
        cands["nt4dgelu"] = lambda: _gemm.nt(dy2, _wt(w), epi=_gemm.NT_EPI_DGELU, u=u, w4=True)
    name = choose(("dgrad_dgelu", M, N, K), cands)
    if name.startswith("split"):
        return split(between)
    du = _native(name, dy2, _wt(w), epi=_gemm.NT_EPI_DGELU, u=u)
    if between is not None:
        between()
    return du


def _hip_wgrad(dy2, x2, g32):
    torch.addmm(g32, dy2.t(), x2, out_dtype=F32, out=g32)


def _hip_wgrad_bf16(dy2, x2, g32):
    """bf16 library GEMM, then fp32 accumulate: the rounding nanoGPT's autocast
    weight grads get (bf16 matmul output added into the fp32 .grad)."""
    g32.add_(dy2.t() @ x2)


def wgrad_acc(dy2, x2, g32):
    """g32 += dy2^T @ x2 in fp32."""
    T, N = dy2.shape
    K = x2.shape[1]
    ok = _nsa_ok(dy2, x2, g32) and T % 64 == 0 and N % 8 == 0 and K % 8 == 0
    if not ok:
        if DETERMINISTIC:
            g32.add_(dy2.t().float() @ x2.float())  # plain fp32 GEMM, then one add
        else:
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

    if DETERMINISTIC:
        # same kernels and split counts, partials reduced in split order
        sdef = _gemm.wgrad_splits(N, K, T)
        tiles = -(-N // _gemm.TILE) * -(-K // _gemm.TILE)
        splits = {sdef, _gemm.wgrad_splits_balanced(N, K, T)}
        splits.update(r * 256 // tiles for r in (1, 2, 3))
        dc = {f"det{v}/s{sb}": cand(lambda a, b, c, v=v, sb=sb: _gemm.wgrad_acc(a, b, c, splits=sb, variant=v,
                                                                                deterministic=True))
              for v in WGRAD_VARIANTS for sb in sorted(x for x in splits if 1 <= x <= max(1, T // _gemm.BK))}
        name = choose(("wgrad_det", T, N, K), dc, fixed=f"det{WGRAD_VARIANTS[-1]}/s{sdef}")
        _gemm.wgrad_acc(dy2, x2, g32, splits=_splits(name), variant=_variant(name), deterministic=True)
        return
    # every default candidate keeps dW in fp32 until it is added into the fp32
    # accumulator; the bf16-rounding library path changes gradient precision, so a
    # speed race never picks it unless asked for (NSA_WGRAD_ALLOW_BF16=1)
    cands = {"hipblaslt": cand(_hip_wgrad)}
    if WGRAD_ALLOW_BF16:
        cands["hipblaslt_bf16"] = cand(_hip_wgrad_bf16)
    cands.update({f"nsa{v}": cand(lambda a, b, c, v=v: _gemm.wgrad_acc(a, b, c, variant=v)) for v in WGRAD_VARIANTS})
    # the same kernels with a split count that fills whole rounds of CUs
    # ... and the split counts that fill 1 / 2 / 3 whole rounds as nearly as possible
    sdef = _gemm.wgrad_splits(N, K, T)
    tiles = -(-N // _gemm.TILE) * -(-K // _gemm.TILE)
    extra = {_gemm.wgrad_splits_balanced(N, K, T)}
    extra.update(r * 256 // tiles for r in (1, 2, 3))
    if WGRAD_FULL_ROUNDS:
        # split counts up to 8 whose work items fill >= 95 % of their last CU round (the tied
        # lm_head dW has 591 output tiles: 3 splits = 1773 items = 99 % of 7 rounds)
        extra.update(sp for sp in range(1, 9)
                     if tiles * sp / (256 * -(-(tiles * sp) // 256)) >= 0.95)
    for sb in sorted(x for x in extra if 1 <= x <= max(1, T // _gemm.BK) and x != sdef):
        cands.update({f"nsa{v}/s{sb}": cand(lambda a, b, c, v=v, sb=sb: _gemm.wgrad_acc(a, b, c, splits=sb, variant=v))
                      for v in WGRAD_VARIANTS})
    # the four-wave kernel with its splits' partials stored (plain stores) and added in one
    # ordered pass instead of fp32 atomics: every work item of a many-split shape (the
    # 768 x 768 dW: 9 tiles x 28 splits) ends in the same instant, where the atomics queue
    if WGRAD_STORE_CANDS and WGRAD_VARIANTS[-1] == _gemm.WGRAD4:
        v = _gemm.WGRAD4
        for sb in sorted(x for x in extra | {sdef} if 2 <= x <= max(1, T // _gemm.BK)):
            cands[f"det{v}/s{sb}"] = cand(lambda a, b, c, v=v, sb=sb: _gemm.wgrad_acc(a, b, c, splits=sb, variant=v,
                                                                                     deterministic=True))
    name = choose(("wgrad", T, N, K), cands)
    if name == "hipblaslt":
        _hip_wgrad(dy2, x2, g32)
    elif name == "hipblaslt_bf16":
        _hip_wgrad_bf16(dy2, x2, g32)
    else:
        _gemm.wgrad_acc(dy2, x2, g32, splits=_splits(name), variant=_variant(name),
                        deterministic=name.startswith("det"))
