"""A/B timing of weight-gradient GEMM strategies on the GPT-2 training shapes.

dW[N_out, K_in] (fp32) += dY[T, N_out]^T · X[T, K_in] over T tokens, as:
  * nsa<v>/s<S>   our split-K kernel (fp32 atomics), the tuner's candidates
  * det<v>/s<S>   the same kernel storing per-split partials + one ordered reduction (--det)
  * blt           one hipBLASLt addmm with fp32 output
  * bmm<S>        hipBLASLt strided-batched split-K: S partial [N_out, K_in] fp32 products
                  (bmm out_dtype=fp32), then one fixed-order reduction pass (nsa_splitk_reduce)
plus, for calibration, hipBLASLt on a square TN shape with >= 256 output tiles.
Candidates are interleaved per round (same clocks); TFLOP/s from the median round.

    python scripts/wgrad_ab.py [--m 122880] [--rounds 5]
"""

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import _lib, gemm  # noqa: E402

F32 = torch.float32


def uni(*shape):
    return (torch.rand(*shape, device="cuda").mul_(2).sub_(1)).to(torch.bfloat16)


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=122880)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--shapes", default="c_attn,attn.c_proj,c_fc,mlp.c_proj,lm_head,sq4096")
    ap.add_argument("--bmm-splits", default="2,4,7,8,14")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--variants", default="1,7")
    ap.add_argument("--det", action="store_true", help="also the deterministic form (partials + ordered reduce)")
    ap.add_argument("--only", default="", help="comma list of candidate names to keep (e.g. nsa7/s7,nsa11/s7)")
    a = ap.parse_args()
    T = a.m
    shapes = {"c_attn": (2304, 768), "attn.c_proj": (768, 768), "c_fc": (3072, 768), "mlp.c_proj": (768, 3072),
              "lm_head": (50304, 768), "sq4096": (4096, 4096)}
    for name in a.shapes.split(","):
        N, K = shapes[name]
        dy, x = uni(T, N), uni(T, K)
        g = torch.zeros(N, K, device="cuda", dtype=F32)
        flops = 2.0 * T * N * K
        cands = {"blt": lambda: torch.addmm(g, dy.t(), x, out_dtype=F32, out=g)}
        if name != "sq4096":
            sdef = gemm.wgrad_splits(N, K, T)
            tiles = -(-N // gemm.TILE) * -(-K // gemm.TILE)
            ss = {sdef, gemm.wgrad_splits_balanced(N, K, T)} | {r * 256 // tiles for r in (1, 2, 3)}
            for s in sorted(x for x in ss if 1 <= x <= T // gemm.BK):
                for v in [int(t) for t in a.variants.split(",")]:
                    sv = s
                    cands[f"nsa{v}/s{sv}"] = (lambda sv=sv, v=v: gemm.wgrad_acc(dy, x, g, splits=sv, variant=v))
                    if a.det and sv > 1:
                        cands[f"det{v}/s{sv}"] = (lambda sv=sv, v=v: gemm.wgrad_acc(dy, x, g, splits=sv, variant=v,
                                                                                    deterministic=True))
        for S in [int(v) for v in a.bmm_splits.split(",") if v]:
            if T % S or (T // S) % 8:
                continue
            ws = torch.empty(S, N, K, device="cuda", dtype=F32)
            dyb = dy.view(S, T // S, N).transpose(1, 2)
            xb = x.view(S, T // S, K)

            def run(ws=ws, dyb=dyb, xb=xb, S=S):
                torch.bmm(dyb, xb, out_dtype=F32, out=ws)
                _lib.call("nsa_splitk_reduce", _lib.ptr(ws), _lib.ptr(g), g.numel(), S, _lib.stream())
            cands[f"bmm{S}"] = run
        if a.only:
            keep = set(a.only.split(","))
            cands = {n: f for n, f in cands.items() if n in keep}
        if a.check:
            ref = dy.float().t() @ x.float()
            for n, fn in cands.items():
                g.zero_()
                fn()
                torch.cuda.synchronize()
                err = ((g - ref).norm() / ref.norm()).item()
                print(f"  check {name} {n}: rel err {err:.2e}", flush=True)
        for fn in cands.values():
            fn()
        torch.cuda.synchronize()
        res = {n: [] for n in cands}
        for _ in range(a.rounds):
            for n, fn in cands.items():
                res[n].append(timeit(fn, a.reps))
        print(f"== {name}: T={T} N_out={N} K_in={K}", flush=True)
        for n, ts in sorted(res.items(), key=lambda kv: sorted(kv[1])[len(kv[1]) // 2]):
            med = sorted(ts)[len(ts) // 2]
            print(f"  {n:12s} {med:9.1f} us  {flops / med / 1e6:7.1f} TF/s", flush=True)
        del dy, x, g
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
