"""Our persistent NT GEMM (csrc/kernels/gemm_nt4.hip) on the GPT-2 training shapes, with torch's
matmul (hipBLASLt) timed beside it as an oracle / yardstick only — it is never dispatched to.

Correctness: each shape is checked against an fp32 product of the same bf16 operands.
Timing: interleaved rounds in one process on uniform [-1, 1) operands
(cdna_hip_programming.md §5.4 rules 24/25).

    python scripts/gemm_nt_ab.py [--m 122880] [--rounds 5] [--probe] [--epi] [--gms 1,4] [--vars 1,2] [--ovls 1,2]

``--probe`` needs a library built with -DNSA_PROBES (the structure probes: no DMA, no vmcnt
wait, no barrier, no epilogue, no stores).  ``--alt-lib PATH`` loads a second build of the
kernel library (e.g. ``nanosandbox_amd.build.build_variant``) beside the default one and times
its nt4 kernel as "nt4_alt" in the same interleaved rounds.
"""

import ctypes

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import gemm  # noqa: E402
from nanosandbox_amd.ops import _lib  # noqa: E402


def uni(*shape, scale=1.0):
    return (torch.rand(*shape, device="cuda").mul_(2).sub_(1) * scale).to(torch.bfloat16)


def rel(got, ref):
    return ((got.float() - ref).norm() / ref.norm()).item()


SHAPES = {"c_attn": (2304, 768), "attn.c_proj": (768, 768), "c_fc": (3072, 768), "mlp.c_proj": (768, 3072),
          "lm_head": (50304, 768), "c_attn.dx": (768, 2304), "c_fc.dx": (768, 3072),
          "mlp.c_proj.dx": (3072, 768), "lm_head.dx": (768, 50304)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=122880)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--probe", action="store_true")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--epi", action="store_true", help="also time the GELU / GELU' epilogues")
    ap.add_argument("--gms", default="", help="extra tile-group sizes to time, e.g. 1,4,8")
    ap.add_argument("--vars", default="0", help="epilogue store policies to time (0 auto, 1 nontemporal, 2 plain)")
    ap.add_argument("--small", action="store_true", help="also time the bounds-checked small-tile kernel")
    ap.add_argument("--xent", action="store_true", help="lm_head: also time the fused cross-entropy (XENT) GEMM")
    ap.add_argument("--xdx", action="store_true", help="lm_head.dx: also time the fused cross-entropy dX (XDX) GEMM")
    ap.add_argument("--ovls", default="", help="overlapped-epilogue policies to time beside auto, e.g. 1,2")
    ap.add_argument("--alt-lib", default="")
    ap.add_argument("--alt-ovl", type=int, default=0, help="overlapped-epilogue policy bits for the --alt-lib calls")
    a = ap.parse_args()
    alt = alt_xent = alt_xdx = None
    if a.alt_lib:
        alt = ctypes.CDLL(a.alt_lib).nsa_gemm_nt4
        alt.argtypes = _lib._SIGNATURES["nsa_gemm_nt4"]
        alt.restype = ctypes.c_int
        alt_xent = ctypes.CDLL(a.alt_lib).nsa_gemm_nt4_xent
        alt_xent.argtypes = _lib._SIGNATURES["nsa_gemm_nt4_xent"]
        alt_xent.restype = ctypes.c_int
        alt_xdx = ctypes.CDLL(a.alt_lib).nsa_gemm_nt4_xdx
        alt_xdx.argtypes = _lib._SIGNATURES["nsa_gemm_nt4_xdx"]
        alt_xdx.restype = ctypes.c_int

    def nt_alt(x, w, epi=0, u=None):
        M_, K_ = x.shape
        N_ = w.shape[0]
        c = torch.empty(M_, N_, device=x.device, dtype=torch.float16 if epi == gemm.NT_EPI_GELU else torch.bfloat16)
        c2 = torch.empty(M_, N_, device=x.device, dtype=torch.bfloat16) if epi == gemm.NT_EPI_GELU else None
        if epi == gemm.NT_EPI_GELU:
            u = gemm.gelu_table(x.device)
        err = alt(epi | (gemm.NT_VAR << 12) | (a.alt_ovl << 14), _lib.ptr(x), x.stride(0), _lib.ptr(w), w.stride(0), _lib.ptr(c),
                  c.stride(0), _lib.ptr(c2), _lib.ptr(u), None, M_, N_, K_, gemm.num_cus(x.device), _lib.stream())
        assert err == 0, err
        return (c, c2) if epi == gemm.NT_EPI_GELU else c
    M = a.m
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print(json.dumps({"device": torch.cuda.get_device_name(), "cus": gemm.num_cus()}), flush=True)
    for (m_, n_, k_) in ((1000, 520, 320), (256, 256, 256), (777, 1288, 640), (4096, 50304, 256)):
        x, w = uni(m_, k_), uni(n_, k_)
        ref = x.float() @ w.float().t()
        print(json.dumps({"check_odd": [m_, n_, k_], "rel_err": rel(gemm.nt(x, w), ref),
                          "rel_err_small": rel(gemm.small(x, w), ref)}), flush=True)
    for name in a.shapes.split(","):
        N, K = SHAPES[name] if name in SHAPES else map(int, name.split("x"))  # or "NxK"
        fl = 2.0 * M * N * K
        x = uni(M, K)
        w = uni(N, K, scale=0.05)
        got = gemm.nt(x, w)
        rows = slice(0, 4096) if N > 8192 else slice(None)
        ref = x[rows].float() @ w.float().t()
        tail = ((got[-256:].float() - x[-256:].float() @ w.float().t()).abs().max()).item()
        print(json.dumps({"check": name, "rel_err": rel(got[rows], ref), "tail_maxabs": tail}), flush=True)
        cands = {"torch_matmul": lambda: x @ w.t(), "nt4": lambda: gemm.nt(x, w)}
        if alt is not None:
            assert torch.equal(nt_alt(x, w), got)
            cands["nt4_alt"] = lambda: nt_alt(x, w)
        for gm_ in [int(t) for t in a.gms.split(",") if t]:
            cands[f"nt4_gm{gm_}"] = lambda gm_=gm_: gemm.nt(x, w, gm=gm_)
        if a.small:
            cands["small"] = lambda: gemm.small(x, w)
        if a.xent and name == "lm_head":
            nvalid = 50257
            crow = (x[:, :64].float().sum(1) * 0.05).contiguous()  # a per-row shift of the logits' scale
            part = torch.empty(2 * ((N + 255) // 256), M, device=x.device)
            e_ref = gemm.nt_xent(x, w, crow, part, nvalid)
            part_ref = part.clone()
            cands["nt4_xent"] = lambda: gemm.nt_xent(x, w, crow, part, nvalid, out=e_ref)
            if alt_xent is not None:
                part2 = torch.empty_like(part)
                e2 = torch.empty_like(e_ref)

                def xent_alt():
                    err = alt_xent(_lib.ptr(x), x.stride(0), _lib.ptr(w), w.stride(0), _lib.ptr(e2), e2.stride(0),
                                   _lib.ptr(crow), _lib.ptr(part2), M, N, nvalid, K, gemm.num_cus(x.device),
                                   _lib.stream())
                    assert err == 0, err
                xent_alt()
                torch.cuda.synchronize()
                print(json.dumps({"check": "lm_head/xent_vs_alt", "E_equal": torch.equal(e2, e_ref),
                                  "part_maxrel": ((part2 - part_ref).abs() / part_ref.abs().clamp_min(1e-30)).max().item()}),
                      flush=True)
                cands["nt4_alt_xent"] = xent_alt
        if a.xdx and name == "lm_head.dx":
            wrows = uni(M, N)
            coef = torch.rand(M, 2, device=x.device)
            c_ref = gemm.nt_xdx(x, w, wrows, coef)
            cands["nt4_xdx"] = lambda: gemm.nt_xdx(x, w, wrows, coef, out=c_ref)
            if a.alt_lib:
                c2 = torch.empty_like(c_ref)

                def xdx_alt():
                    err = alt_xdx(_lib.ptr(x), x.stride(0), _lib.ptr(w), w.stride(0), _lib.ptr(c2), c2.stride(0),
                                  _lib.ptr(wrows), _lib.ptr(coef), M, N, K, gemm.num_cus(x.device), _lib.stream())
                    assert err == 0, err
                xdx_alt()
                torch.cuda.synchronize()
                print(json.dumps({"check": "lm_head.dx/xdx_vs_alt", "equal": torch.equal(c2, c_ref)}), flush=True)
                cands["nt4_alt_xdx"] = xdx_alt
        for ov in [int(t) for t in a.ovls.split(",") if t]:
            cands[f"nt4_ovl{ov}"] = lambda ov=ov: gemm.nt(x, w, ovl=ov)
            assert torch.equal(gemm.nt(x, w, ovl=ov), got), ov
        for v in [int(t) for t in a.vars.split(",") if t and t != "0"]:
            cands[f"nt4_v{v}"] = lambda v=v: gemm.nt(x, w, var=v)
            print(json.dumps({"check": f"{name}/v{v}", "rel_err": rel(gemm.nt(x, w, var=v)[rows], ref)}), flush=True)
        del ref
        if a.probe:
            for pr, nm in ((1, "nodma"), (2, "novmwait"), (3, "nobarrier"), (4, "noepi"), (5, "nostore")):
                cands[f"nt4_{nm}"] = lambda pr=pr: gemm.nt(x, w, probe=pr)
        if a.epi and name == "c_fc":
            gp, g = gemm.nt(x, w, epi=gemm.NT_EPI_GELU)
            u = gemm.nt(x, w)
            eg = ((g.float() - torch.nn.functional.gelu(u.float())).abs().max()).item()
            print(json.dumps({"check": name + "/gelu", "maxabs_g_vs_gelu(u)": eg}), flush=True)

            def split():
                uu = x @ w.t()
                gg = torch.empty_like(uu)
                _lib.call("nsa_gelu_fwd", _lib.ptr(uu), _lib.ptr(gg), uu.numel(), _lib.stream())
            cands["torch_matmul+gelu"] = split
            cands["nt4_gelu"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_GELU)
            if a.probe:  # the GELU epilogue without its stores / without any epilogue
                cands["nt4_gelu_nostore"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_GELU, probe=5)
                cands["nt4_gelu_noepi"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_GELU, probe=4)
            if alt is not None:
                cands["nt4_alt_gelu"] = lambda: nt_alt(x, w, epi=gemm.NT_EPI_GELU)
                gp2, g2 = nt_alt(x, w, epi=gemm.NT_EPI_GELU)
                print(json.dumps({"check": name + "/gelu_vs_alt", "g_ulp_diff_frac": (g2 != g).float().mean().item(),
                                  "gp_maxabs": (gp2.float() - gp.float()).abs().max().item()}), flush=True)
        if a.epi and name == "mlp.c_proj.dx":
            u = uni(M, N, scale=3.0)
            uf = u.float()
            gp = (0.5 * (1 + torch.erf(uf / 2 ** 0.5)) + uf * torch.exp(-0.5 * uf * uf) * 0.3989422804014327).half()
            got = gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=gp)  # U = gelu'(u) in fp16 (the GELU epilogue's output)
            ref = (x.float() @ w.float().t()).to(torch.bfloat16).float() * gp.float()
            print(json.dumps({"check": name + "/dgelu", "rel_err": rel(got, ref)}), flush=True)
            del ref, uf

            def split2():
                dg = x @ w.t()
                du = torch.empty_like(dg)
                _lib.call("nsa_gelu_bwd", _lib.ptr(dg), _lib.ptr(u), _lib.ptr(du), du.numel(), _lib.stream())
            cands["torch_matmul+dgelu"] = split2
            cands["nt4_dgelu"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=gp)
            if a.probe:
                cands["nt4_dgelu_nostore"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=gp, probe=5)
            if alt is not None:
                cands["nt4_alt_dgelu"] = lambda: nt_alt(x, w, epi=gemm.NT_EPI_DGELU, u=gp)
        for fn in cands.values():
            fn()
        torch.cuda.synchronize()
        samples = {k: [] for k in cands}
        names = list(cands)
        for r in range(a.rounds):
            # the starting candidate rotates every round: the same kernel timed in different
            # slots of one round has measured up to ~4 % apart (profiles/r6_nt4_ovl.md)
            for k in names[r % len(names):] + names[:r % len(names)]:
                fn = cands[k]
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                e1.synchronize()
                samples[k].append(e0.elapsed_time(e1) / a.reps)
        out = {}
        for k, s in samples.items():
            med = sorted(s)[len(s) // 2]
            out[k] = {"us": round(med * 1e3, 1), "TF": round(fl / (med * 1e-3) / 1e12, 1)}
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "res": out}), flush=True)


if __name__ == "__main__":
    main()
