"""Which E elements a fused-cross-entropy GEMM leaves unwritten (NaN-prefilled output)."""
import sys, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nanosandbox_amd.ops import gemm  # noqa: E402

for (M, N, K, nv) in ((512, 256, 768, 65), (2048, 50304, 768, 50257), (1024, 1024, 128, 1024)):
    for grid in (None, 1, 2):
        x = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * 0.1).to(torch.bfloat16)
        crow = torch.zeros(M, device="cuda")
        part = torch.empty(2 * ((N + 255) // 256), M, device="cuda")
        e = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        if grid is None:
            gemm.nt_xent(x, w, crow, part, nv, out=e)
        else:
            from nanosandbox_amd.ops import _lib
            _lib.call("nsa_gemm_nt4_xent", _lib.ptr(x), K, _lib.ptr(w), K, _lib.ptr(e), N, _lib.ptr(crow),
                      _lib.ptr(part), M, N, nv, K, grid, _lib.stream())
        torch.cuda.synchronize()
        bad = torch.isnan(e)
        rows = bad.any(1).nonzero().flatten().tolist()
        cols = bad.any(0).nonzero().flatten().tolist()
        print(M, N, K, "grid", grid, "nan", int(bad.sum()), "rows", rows[:12], len(rows), "cols", cols[:6], cols[-3:] if cols else [], len(cols), flush=True)
