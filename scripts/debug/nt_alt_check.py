"""Bitwise check of an alternative kernel-library build's NT GEMM against the default one on
odd shapes (tail tiles in both dimensions, one K-tile, a single tile, more tiles than CUs).

    python scripts/debug/nt_alt_check.py build/variants/<name>/libnsa_kernels.so
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd.ops import _lib, gemm  # noqa: E402


def main():
    alt = ctypes.CDLL(sys.argv[1]).nsa_gemm_nt4
    alt.argtypes = _lib._SIGNATURES["nsa_gemm_nt4"]
    alt.restype = ctypes.c_int
    torch.manual_seed(0)
    bad = 0
    for (m, n, k) in ((256, 256, 64), (256, 256, 256), (1000, 520, 320), (777, 1288, 640), (4096, 50304, 256),
                      (300, 2304, 64), (122880, 768, 768), (61440, 2304, 768), (2048, 3072, 1600)):
        x = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(n, k, device="cuda") * 2 - 1).to(torch.bfloat16)
        ref = gemm.nt(x, w)
        for grid in (gemm.num_cus(x.device), 7, 1):
            c = torch.full((m, n), float("nan"), device="cuda", dtype=torch.bfloat16)
            err = alt(int(os.environ.get("ALT_EPI", "0")), _lib.ptr(x), x.stride(0), _lib.ptr(w), w.stride(0), _lib.ptr(c), c.stride(0), None, None,
                      None, m, n, k, grid, _lib.stream())
            assert err == 0, err
            torch.cuda.synchronize()
            eq = torch.equal(c, ref)
            bad += not eq
            print(json.dumps({"m": m, "n": n, "k": k, "grid": grid, "equal": eq,
                              "nan": int(torch.isnan(c).sum().item())}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
