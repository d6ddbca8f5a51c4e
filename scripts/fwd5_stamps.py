"""Phase timing of the ping-pong forward (v5) from a diagnostic build with s_memtime stamps.

    python -c "from nanosandbox_amd.build import build_variant; build_variant('fwd5stamp', ['NSA_FWD5_STAMPS=1'])"
    NSA_KERNEL_LIB=build/variants/fwd5stamp/libnsa_kernels.so python scripts/fwd5_stamps.py

Prints per-wave averages over the grid (cycles): the whole loop, M-phase work, the wait
after M (DMA wait + barrier), V-phase work, the wait after V, and tiles computed; split by
wave half (0-3 run M first, 4-7 half a step behind).
"""
import ctypes
import json
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import _lib  # noqa: E402
from nanosandbox_amd.ops.functional import flash_variant  # noqa: E402


def main():
    B, T, H, D = 120, 1024, 12, 64
    C = H * D
    qkv = torch.randn(B, T, 3 * C, device="cuda").to(torch.bfloat16)
    y = torch.empty(B, T, C, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, T, device="cuda")
    n_wg = (T // 256) * B * H
    with flash_variant(fwd=os.environ.get("FWD", "v5")):
        for _ in range(3):
            _lib.call("nsa_flash_fwd", _lib.ptr(qkv), _lib.ptr(y), _lib.ptr(lse), B, T, H, D, 1.0 / math.sqrt(D), 0.0,
                      0, _lib.stream())
        torch.cuda.synchronize()
    buf = np.zeros(n_wg * 8 * 6, dtype=np.uint64)
    fn = _lib.lib().nsa_fwd5_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert fn(buf.ctypes.data, buf.size) == 0
    a = buf.reshape(n_wg, 8, 6).astype(np.float64)
    names = ["loop", "M_work", "wait_after_M", "V_work", "wait_after_V", "tiles"]
    for half, sl in (("waves0-3", slice(0, 4)), ("waves4-7", slice(4, 8))):
        m = a[:, sl, :].reshape(-1, 6).mean(0)
        out = {k: round(float(v), 1) for k, v in zip(names, m)}
        out["per_tile"] = {k: round(float(m[i] / max(1.0, m[5])), 1) for i, k in enumerate(names[:5])}
        print(json.dumps({half: out}), flush=True)


if __name__ == "__main__":
    main()
