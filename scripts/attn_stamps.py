"""Where the forward v3 tile loop spends its cycles, from a diagnostic build with s_memtime
stamps (no output is computed from them).

    python -c "from nanosandbox_amd.build import build_variant; build_variant('fwd3stamp', ['NSA_FWD3_STAMPS=1'])"
    NSA_KERNEL_LIB=build/variants/fwd3stamp/libnsa_kernels.so python scripts/attn_stamps.py

Per-wave totals averaged over the grid (cycles) and per computed tile: S MFMA issue (with
the K fragment reads), the wait for S plus the softmax VALU, the P·V issue (with the V
fragment reads), the DMA wait plus barrier at the end of every tile.
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
    with flash_variant(fwd="v3"):
        for _ in range(3):
            _lib.call("nsa_flash_fwd", _lib.ptr(qkv), _lib.ptr(y), _lib.ptr(lse), B, T, H, D, 1.0 / math.sqrt(D), 0.0,
                      0, _lib.stream())
        torch.cuda.synchronize()
    buf = np.zeros(n_wg * 4 * 6, dtype=np.uint64)
    fn = _lib.lib().nsa_fwd3_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert fn(buf.ctypes.data, buf.size) == 0
    a = buf.reshape(n_wg, 4, 6).astype(np.float64)
    names = ["loop", "S_issue", "S_wait_softmax", "PV_issue", "dma_wait_barrier", "tiles"]
    m = a.reshape(-1, 6).mean(0)
    out = {k: round(float(v), 1) for k, v in zip(names, m)}
    loops = a[:, :, 0].sum(1) / 4
    out["per_tile"] = {k: round(float(m[i] / max(1.0, m[5])), 1) for i, k in enumerate(names[1:5], 1)}
    out["wg_loop_cycles_mean"] = round(float(loops.mean()), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
