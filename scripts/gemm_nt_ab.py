"""Persistent NT GEMM (csrc/kernels/gemm_nt.hip) vs hipBLASLt on the GPT-2 training shapes.

Correctness: each shape is checked against an fp32 product of the same bf16 operands.
Timing: interleaved rounds in one process on uniform [-1, 1) operands
(cdna_hip_programming.md §5.4 rules 24/25).

    python scripts/gemm_nt_ab.py [--m 122880] [--rounds 5] [--probe] [--tuned]

--tuned replays the TunableOp hipBLASLt/rocBLAS solution table the trainer and bench.py
use (ops/blas_tuning.py), i.e. the library GEMM the tuner actually races against.
"""

import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import gemm  # noqa: E402
from nanosandbox_amd.ops import _lib  # noqa: E402


def uni(*shape, scale=1.0):
    return (torch.rand(*shape, device="cuda").mul_(2).sub_(1) * scale).to(torch.bfloat16)


def gelu_ref(x):
    return torch.nn.functional.gelu(x.float())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=122880)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--probe", action="store_true", help="also time the no-DMA structure probe")
    ap.add_argument("--shapes", default="c_attn,attn.c_proj,c_fc,mlp.c_proj,lm_head,c_attn.dx,c_fc.dx,"
                                        "mlp.c_proj.dx,lm_head.dx")
    ap.add_argument("--epi", action="store_true", help="also time the GELU / GELU' epilogues")
    ap.add_argument("--tuned", action="store_true", help="hipBLASLt with the tuned solution table")
    ap.add_argument("--alt", default="", help="NAME=PATH,... stand-alone NT builds (scripts/build_nt_variants.sh)")
    ap.add_argument("--oldlib", default="", help="PATH of a build of the round-2 gemm.hip: times its 4-wave "
                    "kernel (variant 11) in the NT layout as 'w4'")
    ap.add_argument("--gms", default="", help="extra tile-group sizes to time, e.g. 1,4,8")
    ap.add_argument("--vars", default="0", help="epilogue store policies to time (0 auto, 1 nontemporal, 2 plain)")
    a = ap.parse_args()
    M = a.m
    alts = {}
    for spec in [t for t in a.alt.split(",") if t]:
        nm, path = spec.split("=", 1)
        L = ctypes.CDLL(os.path.abspath(path))
        fn = getattr(L, "nsa_gemm_nt4", None) or L.nsa_gemm_nt
        fn.argtypes = _lib._SIGNATURES["nsa_gemm_nt"]
        fn.restype = ctypes.c_int
        alts[nm] = fn

    old = None
    if a.oldlib:
        old = ctypes.CDLL(os.path.abspath(a.oldlib))
        old.nsa_gemm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        old.nsa_gemm.restype = ctypes.c_int

    def old_nt(x, w, variant=11):
        Mx, Kx = x.shape
        Nx = w.shape[0]
        out = torch.empty(Mx, Nx, device=x.device, dtype=torch.bfloat16)
        err = old.nsa_gemm(0, variant << 8, x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(),
                           out.stride(0), None, None, Mx, Nx, Kx, 1, _lib.stream())
        assert err == 0, err
        return out

    def alt_nt(L, x, w, epi=0, u=None):
        Mx, Kx = x.shape
        Nx = w.shape[0]
        out = torch.empty(Mx, Nx, device=x.device, dtype=torch.bfloat16)
        act = torch.empty_like(out) if epi == gemm.NT_EPI_GELU else None
        err = L(epi, x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0),
                            None if act is None else act.data_ptr(), None if u is None else u.data_ptr(), Mx, Nx, Kx,
                            gemm.num_cus(), _lib.stream())
        assert err == 0, err
        return (out, act) if act is not None else out
    if a.tuned:
        from nanosandbox_amd.ops import blas_tuning
        print(json.dumps({"tuned_table": blas_tuning.enable()}), flush=True)
    # name -> (N, K): C[M, N] = A[M, K] B[N, K]^T
    shapes = {"c_attn": (2304, 768), "attn.c_proj": (768, 768), "c_fc": (3072, 768), "mlp.c_proj": (768, 3072),
              "lm_head": (50304, 768), "c_attn.dx": (768, 2304), "c_fc.dx": (768, 3072),
              "mlp.c_proj.dx": (3072, 768), "lm_head.dx": (768, 50304)}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print(json.dumps({"device": torch.cuda.get_device_name(), "cus": gemm.num_cus()}), flush=True)
    for (m_, n_, k_) in ((1000, 520, 320), (256, 256, 256), (777, 1288, 640), (4096, 50304, 256)):
        x = uni(m_, k_)
        w = uni(n_, k_)
        ref = x.float() @ w.float().t()
        got = gemm.nt(x, w).float()
        got4 = gemm.nt(x, w, w4=True).float()
        print(json.dumps({"check_odd": [m_, n_, k_], "rel_err": ((got - ref).norm() / ref.norm()).item(),
                          "rel_err_w4": ((got4 - ref).norm() / ref.norm()).item(),
                          "maxabs_w4": (got4 - ref).abs().max().item()}), flush=True)
    for name in a.shapes.split(","):
        N, K = shapes[name]
        fl = 2.0 * M * N * K
        x = uni(M, K)
        w = uni(N, K, scale=0.05)
        # correctness on a row slice (full fp32 reference of 122880 x 50304 is too big)
        got = gemm.nt(x, w)
        rows = slice(0, 4096) if N > 8192 else slice(None)
        ref = x[rows].float() @ w.float().t()
        ref_n = ref.norm()
        err = ((got[rows].float() - ref).norm() / ref_n).item()
        tail = ((got[-256:].float() - x[-256:].float() @ w.float().t()).abs().max()).item()
        print(json.dumps({"check": name, "rel_err": err, "tail_maxabs": tail}), flush=True)
        del ref
        got4 = gemm.nt(x, w, w4=True)
        err4 = ((got4[rows].float() - x[rows].float() @ w.float().t()).norm() / ref_n).item()
        tail4 = ((got4[-256:].float() - x[-256:].float() @ w.float().t()).abs().max()).item()
        print(json.dumps({"check": name + "/w4", "rel_err": err4, "tail_maxabs": tail4}), flush=True)
        del got4
        cands = {"hipblaslt": lambda: x @ w.t(), "nt": lambda: gemm.nt(x, w), "nt4": lambda: gemm.nt(x, w, w4=True)}
        if old is not None:
            cands["w4"] = lambda: old_nt(x, w)
            e = ((old_nt(x, w)[rows].float() - x[rows].float() @ w.float().t()).norm() / ref_n).item()
            print(json.dumps({"check": f"{name}/w4", "rel_err": e}), flush=True)
        for nm, L in alts.items():
            cands[f"nt_{nm}"] = lambda L=L: alt_nt(L, x, w)
            e = ((alt_nt(L, x, w)[rows].float() - x[rows].float() @ w.float().t()).norm() / ref_n).item()
            print(json.dumps({"check": f"{name}/{nm}", "rel_err": e}), flush=True)
        for gm_ in [int(t) for t in a.gms.split(",") if t]:
            cands[f"nt_gm{gm_}"] = lambda gm_=gm_: gemm.nt(x, w, gm=gm_)
            cands[f"nt4_gm{gm_}"] = lambda gm_=gm_: gemm.nt(x, w, gm=gm_, w4=True)
        for v in [int(t) for t in a.vars.split(",") if t and t != "0"]:
            cands[f"nt_v{v}"] = lambda v=v: gemm.nt(x, w, var=v)
            if v:
                got = gemm.nt(x, w, var=v)
                e = ((got[rows].float() - x[rows].float() @ w.float().t()).norm() / ref_n).item()
                print(json.dumps({"check": f"{name}/v{v}", "rel_err": e}), flush=True)
        if a.probe:
            for pr, nm in ((1, "nodma"), (4, "nostore")):
                cands[f"nt_{nm}"] = lambda pr=pr: gemm.nt(x, w, probe=pr)
            for pr, nm in ((1, "nodma"), (2, "novmwait"), (3, "nobarrier"), (4, "noepi"), (5, "nostore")):
                cands[f"nt4_{nm}"] = lambda pr=pr: gemm.nt(x, w, probe=pr, w4=True)
        if a.epi and name in ("c_fc", "mlp.c_proj.dx"):
            if name == "c_fc":
                u, g = gemm.nt(x, w, epi=gemm.NT_EPI_GELU)
                ref_u = (x.float() @ w.float().t())
                eu = ((u.float() - ref_u).norm() / ref_u.norm()).item()
                eg = ((g.float() - gelu_ref(u)).abs().max()).item()
                print(json.dumps({"check": name + "/gelu", "rel_err_u": eu, "maxabs_g_vs_gelu(u)": eg}), flush=True)
                del ref_u

                def split():
                    uu = x @ w.t()
                    gg = torch.empty_like(uu)
                    _lib.call("nsa_gelu_fwd", _lib.ptr(uu), _lib.ptr(gg), uu.numel(), _lib.stream())
                cands["hipblaslt+gelu"] = split
                cands["nt_gelu"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_GELU)
                cands["nt4_gelu"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_GELU, w4=True)
                u4, g4 = gemm.nt(x, w, epi=gemm.NT_EPI_GELU, w4=True)
                print(json.dumps({"check": name + "/gelu_w4", "maxabs_u": (u4.float() - u.float()).abs().max().item(),
                                  "maxabs_g": (g4.float() - g.float()).abs().max().item()}), flush=True)
                cands["nt_gelu_nopost"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_GELU, probe=2)
                for nm, L in alts.items():
                    cands[f"nt_gelu_{nm}"] = lambda L=L: alt_nt(L, x, w, epi=gemm.NT_EPI_GELU)
            else:
                u = uni(M, N, scale=3.0)
                got = gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=u)
                ref = (x.float() @ w.float().t()).to(torch.bfloat16).float()
                uf = u.float()
                cdf = 0.5 * (1 + torch.erf(uf / 2 ** 0.5))
                pdf = torch.exp(-0.5 * uf * uf) / (2 * 3.141592653589793) ** 0.5
                ref = ref * (cdf + uf * pdf)
                e = ((got.float() - ref).norm() / ref.norm()).item()
                print(json.dumps({"check": name + "/dgelu", "rel_err": e}), flush=True)
                del ref, uf, cdf, pdf

                def split2():
                    dg = x @ w.t()
                    du = torch.empty_like(dg)
                    _lib.call("nsa_gelu_bwd", _lib.ptr(dg), _lib.ptr(u), _lib.ptr(du), du.numel(), _lib.stream())
                cands["hipblaslt+dgelu"] = split2
                cands["nt_dgelu"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=u)
                cands["nt4_dgelu"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=u, w4=True)
                e4 = ((gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=u, w4=True).float() - got.float()).abs().max()).item()
                print(json.dumps({"check": name + "/dgelu_w4_vs_nt_maxabs", "v": e4}), flush=True)
                cands["nt_dgelu_nopost"] = lambda: gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=u, probe=2)
                for nm, L in alts.items():
                    cands[f"nt_dgelu_{nm}"] = lambda L=L: alt_nt(L, x, w, epi=gemm.NT_EPI_DGELU, u=u)
        for fn in cands.values():
            fn()
        torch.cuda.synchronize()
        samples = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, fn in cands.items():
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                e1.synchronize()
                samples[k].append(e0.elapsed_time(e1) / a.reps)
        out = {}
        for k, s in samples.items():
            s = sorted(s)
            med = s[len(s) // 2]
            out[k] = {"us": round(med * 1e3, 1), "TF": round(fl / (med * 1e-3) / 1e12, 1)}
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "res": out}), flush=True)


if __name__ == "__main__":
    main()
