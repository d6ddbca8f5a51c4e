"""GPU probe: nsa_layernorm_bwd_x32s split-plane input decode (dy = 0 makes dx = dres exactly)."""
import torch

from nanosandbox_amd.ops import _lib
from nanosandbox_amd.ops.functional import split_planes

DEV, BF = "cuda", torch.bfloat16
torch.manual_seed(11)
for (N, C) in [(8, 64), (300, 768), (1100, 768)]:
    s = torch.randn(N, C, device=DEV)
    w = torch.ones(C, device=DEV).to(BF)
    mean = s.mean(-1)
    rstd = torch.rsqrt(s.var(-1, unbiased=False) + 1e-5)
    dres = torch.randn(N, C, device=DEV) * 0.1
    for dyz in (True, False):
        dh = torch.zeros(N, C, device=DEV).to(BF) if dyz else torch.randn(N, C, device=DEV).to(BF)
        nblk = 16
        dx0 = torch.full((N, C), float("nan"), device=DEV)
        dwp = torch.empty(nblk, C, device=DEV)
        rc0 = _lib.call_ret("nsa_layernorm_bwd_x32", _lib.ptr(dh), _lib.ptr(s), _lib.ptr(w), _lib.ptr(mean),
                            _lib.ptr(rstd), _lib.ptr(dres), _lib.ptr(dx0), None, _lib.ptr(dwp), None, N, C, nblk,
                            _lib.stream())
        din = split_planes(dres)
        dx1 = torch.full((N, C), float("nan"), device=DEV)
        rc1 = _lib.call_ret("nsa_layernorm_bwd_x32s", _lib.ptr(dh), _lib.ptr(s), _lib.ptr(w), _lib.ptr(mean),
                            _lib.ptr(rstd), _lib.ptr(din), _lib.ptr(dx1), None, _lib.ptr(dwp), None, N, C, nblk, 1,
                            _lib.stream())
        torch.cuda.synchronize()
        bad = (dx1.view(torch.int32) != dx0.view(torch.int32))
        print(f"N={N} C={C} dy0={dyz} rc={rc0},{rc1} mismatches={int(bad.sum())} "
              f"dx0==dres(dy0)={bool(torch.equal(dx0, dres)) if dyz else '-'}")
        if bad.any():
            idx = bad.nonzero()[:6].tolist()
            for r, c in idx:
                print("   ", r, c, f"dx1={dx1[r, c].item():.6g} dx0={dx0[r, c].item():.6g} dres={dres[r, c].item():.6g}",
                      hex(dx1[r, c].view(torch.int32).item() & 0xffffffff), hex(dx0[r, c].view(torch.int32).item() & 0xffffffff))
