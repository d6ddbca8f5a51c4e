"""Loader for the in-tree gfx950 kernel library ``nanosandbox_amd/lib/libnsa_kernels.so``.

The kernels are plain HIP C++ (``csrc/kernels/*.hip``) compiled by ``hipcc
--offload-arch=gfx950`` into one shared object with a C ABI (every entry point is an
``NSA_API`` function, ``csrc/kernels/common.h``; its ctypes signature is listed in
``_SIGNATURES`` below).  We bind it with ctypes rather than a torch C++
extension: the library does not depend on torch headers or ABI, builds in
seconds, and every launch takes raw device pointers plus the current HIP
stream, so it composes with torch's stream/graph semantics.

There is deliberately no silent fallback: on a GPU device every op calls into
this library and raises if it is missing (run ``python -m nanosandbox_amd.build``).
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch

_LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib")
# NSA_KERNEL_LIB points at an alternative build (e.g. an A/B probe variant from
# ``nanosandbox_amd.build.build_variant``); default is the in-tree library.
LIB_PATH = os.environ.get("NSA_KERNEL_LIB") or os.path.join(_LIB_DIR, "libnsa_kernels.so")

_lock = threading.Lock()
_lib = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_uint64 = ctypes.c_uint64
c_float = ctypes.c_float

# name -> argtypes (restype is always int = hipError_t)
_SIGNATURES = {
    "nsa_embedding_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_uint64, c_void_p],
    "nsa_embedding_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_uint64, c_void_p],
    "nsa_embedding_fwd_x32": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_uint64,
                              c_void_p],
    "nsa_embedding_bwd_x32": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_uint64,
                              c_void_p],
    "nsa_layernorm_fwd_x32": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_int, c_int, c_float, c_void_p],
    "nsa_layernorm_bwd_x32": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_int, c_int, c_int, c_void_p],
    "nsa_layernorm_bwd_x32s": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
    "nsa_layernorm_fwd_x32d": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_int, c_int, c_float, c_float, c_uint64, c_void_p],
    "nsa_layernorm_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_int, c_int, c_float, c_void_p],
    "nsa_layernorm_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_int, c_int, c_int, c_void_p],
    "nsa_colsum_accum": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "nsa_colsum_accum_ordered": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "nsa_gelu_fwd": [c_void_p, c_void_p, c_int64, c_void_p],
    "nsa_gelu_bwd": [c_void_p, c_void_p, c_void_p, c_int64, c_void_p],
    "nsa_dropout": [c_void_p, c_void_p, c_int64, c_float, c_uint64, c_void_p],
    "nsa_xent_fwd": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
    "nsa_scale_rows_bf16": [c_void_p, c_void_p, c_void_p, c_int64, c_void_p],
    "nsa_adamw_step": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                       c_float, c_float, c_float, c_float, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p],
    "nsa_sumsq_partial": [c_void_p, c_int64, c_void_p, c_int, c_float, c_void_p, c_void_p],
    "nsa_clip_coef": [c_void_p, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p, c_float, c_float, c_float,
                      c_void_p],
    "nsa_cast_f32_bf16": [c_void_p, c_void_p, c_int64, c_void_p],
    "nsa_flash_fwd": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_float, c_uint64, c_void_p],
    "nsa_flash_set_variant": [c_int, c_int, c_int],
    "nsa_ew_set_nt": [c_int],
    "nsa_ln_set_nt": [c_int],
    "nsa_kv_append": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nsa_decode_attn": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                        c_float, c_int, c_void_p],
    "nsa_sample_topk": [c_void_p, c_int, c_int, c_int, c_float, c_int, c_uint64, c_void_p, c_void_p, c_void_p,
                        c_void_p, c_int, c_void_p],
    "nsa_gemv": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nsa_skinny_gemm": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nsa_skinny_ln_gemm": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p,
                           c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nsa_gemv_emb_ln": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_void_p, c_int, c_int, c_float, c_int, c_int, c_void_p],
    "nsa_gemv_attn": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
    "nsa_gemv_ln": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                    c_float, c_int, c_int, c_void_p, c_void_p],
    "nsa_flash_bwd2": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_int, c_int, c_int, c_int, c_float, c_float, c_uint64, c_void_p],
    "nsa_rng_advance": [c_void_p],
    "nsa_rng_set": [c_uint64, c_void_p],
    "nsa_splitk_reduce": [c_void_p, c_void_p, c_int64, c_int, c_void_p],
    "nsa_embedding_bwd_det": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                              c_int, c_int, c_int, c_float, c_uint64, c_void_p],
    "nsa_transpose_bf16": [c_void_p, c_void_p, c_int, c_int, c_void_p],
    "nsa_gemm": [c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                 c_int, c_int, c_int, c_int, c_void_p],
    "nsa_gemm_wgrad4": [c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                        c_void_p],
    "nsa_gemm_wgrad4b": [c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int,
                         c_void_p],
    "nsa_gemm_nt4": [c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                     c_int, c_int, c_int, c_int, c_void_p],
    "nsa_gemm_small": [c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                       c_int, c_int, c_int, c_void_p],
    "nsa_gemm_nt4_xent": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                          c_int, c_int, c_void_p],
    "nsa_gemm_nt4_xdx": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                         c_int, c_void_p],
    "nsa_xent_tlogit": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float,
                        c_void_p],
    "nsa_xent_combine": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_float, c_float,
                         c_float, c_void_p],
    "nsa_xent_fixup": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_void_p, c_int, c_int, c_int, c_void_p],
    "nsa_xent_bwd_prep": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_int, c_int, c_void_p],
    "nsa_xent_dw_fix": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                        c_void_p],
    "nsa_xent_dw_fix_sorted": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
    "nsa_embedding_bwd_lds": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                              c_float, c_uint64, c_void_p],
    "nsa_seg_lds_parts": [c_int],
    "nsa_xent_dw_fix_lds": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_int, c_int, c_int, c_int, c_void_p],
    "nsa_colsum_bf16_partial": [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p],
    "nsa_keysort": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "nsa_keysort_ws_bytes": [c_int],
    "nsa_probe_spin": [c_int, c_uint64, c_void_p, c_void_p],
    "nsa_probe_mark": [c_void_p, c_void_p],
}
# entry points whose return value is not a hipError_t
_RESTYPES = {"nsa_keysort_ws_bytes": c_int64}


class KernelLibraryMissing(RuntimeError):
    pass


def lib():
    """Return the loaded kernel library (raises loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise KernelLibraryMissing(
                f"HIP kernel library not found at {LIB_PATH}; build it with "
                "`python -m nanosandbox_amd.build` (hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in _SIGNATURES.items():
            # NAME_h: the fp16 instantiation of an entry point, same C signature
            for sym in (name, name + "_h"):
                fn = getattr(L, sym, None)
                if fn is None:
                    continue  # optional entry points (checked at call time)
                fn.argtypes = argtypes
                fn.restype = _RESTYPES.get(name, c_int)
        _lib = L
        return _lib


def available() -> bool:
    return os.path.exists(LIB_PATH)


def ptr(t):
    """Device pointer of a tensor (or NULL for None)."""
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def call_ret(name, *args):
    """Call an entry point that returns a value (not a hipError_t)."""
    fn = getattr(lib(), name, None)
    if fn is None:
        raise KernelLibraryMissing(f"{name} missing from {LIB_PATH}; rebuild the kernel library")
    return fn(*args)


def call(name, *args):
    fn = getattr(lib(), name, None)
    if fn is None:
        raise KernelLibraryMissing(f"{name} missing from {LIB_PATH}; rebuild the kernel library")
    err = fn(*args)
    if err != 0:
        raise RuntimeError(f"{name} failed with hipError {err}")
