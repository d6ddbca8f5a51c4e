"""Pick hipBLASLt/rocBLAS solutions for the library GEMMs of GPT-2 training (PyTorch TunableOp).

For every forward / input-grad shape of a micro-step at each token count M:
  1. time torch's default heuristic pick (TunableOp off),
  2. let TunableOp search the hipBLASLt + rocBLAS solutions for that shape,
  3. time the tuned pick the same way (interleaved with the default, same process),
and keep only the entries whose tuned pick is faster by --min-gain.  The kept
entries (plus TunableOp's validator lines: torch/HIP/hipBLASLt/rocBLAS versions
and gfx arch) are written to --out, which ``nanosandbox_amd.ops.blas_tuning``
loads with tuning disabled.

    python scripts/tune_blas.py --m 122880,61440 --out nanosandbox_amd/ops/tuned/gfx950_gpt2.csv
"""

import argparse
import os
import sys

import torch
import torch.cuda.tunable as tn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, rounds=5, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(rounds):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    return sorted(out)[len(out) // 2]


def uni(*shape, scale=1.0):
    return (torch.rand(*shape, device="cuda").mul_(2).sub_(1) * scale).to(torch.bfloat16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="122880,61440")
    ap.add_argument("--c", type=int, default=768)
    ap.add_argument("--v", type=int, default=50304)
    ap.add_argument("--ops", default="fwd,dx,dw")
    ap.add_argument("--min-gain", type=float, default=0.02)
    ap.add_argument("--iters", type=int, default=20, help="TunableOp max tuning iterations per solution")
    ap.add_argument("--out", default="nanosandbox_amd/ops/tuned/gfx950_gpt2.csv")
    ap.add_argument("--shapes", default="c_attn,attn.c_proj,c_fc,mlp.c_proj,lm_head")
    a = ap.parse_args()
    C, V = a.c, a.v
    shapes = {"c_attn": (3 * C, C), "attn.c_proj": (C, C), "c_fc": (4 * C, C), "mlp.c_proj": (C, 4 * C),
              "lm_head": (V, C)}
    tn.enable(False)
    tn.set_max_tuning_iterations(a.iters)
    tn.set_filename("/tmp/nsa_tunableop_scratch.csv")  # TunableOp writes its own results file at exit
    keep = {}
    for M in [int(m) for m in a.m.split(",")]:
        for name, (N, K) in shapes.items():
            if name not in a.shapes.split(","):
                continue
            x, w, dy = uni(M, K), uni(N, K, scale=0.05), uni(M, N)
            wt = w.t().contiguous()
            fns = {}
            if "fwd" in a.ops.split(","):
                fns["fwd"] = lambda: x @ w.t()
            if "dx" in a.ops.split(","):
                fns["dx"] = lambda: dy @ w
            if "dxt" in a.ops.split(","):
                # input grad through the cached K-contiguous weight transpose (ops/gemm_tune._wt)
                fns["dxt"] = lambda: dy @ wt.t()
            if "dw" in a.ops.split(","):
                # weight grad with a bf16 result (nanoGPT + autocast semantics), dY^T X
                fns["dw"] = lambda: dy.t() @ x
            for op, fn in fns.items():
                tn.enable(False)
                fn()
                before = set(tuple(r) for r in tn.get_results())
                t_default = timed(fn)
                tn.enable(True)
                tn.tuning_enable(True)
                fn()  # TunableOp searches the solutions for this shape here
                tn.tuning_enable(False)
                new = [tuple(r) for r in tn.get_results() if tuple(r) not in before]
                t_tuned = timed(fn)
                # interleave once more so both see the same clock state
                tn.enable(False)
                t_default = min(t_default, timed(fn))
                tn.enable(True)
                t_tuned = min(t_tuned, timed(fn))
                gain = t_default / t_tuned - 1.0
                fl = 2.0 * M * N * K
                print(f"M={M} {name}/{op}: default {fl / t_default / 1e9:.0f} TF/s, tuned {fl / t_tuned / 1e9:.0f} TF/s "
                      f"({gain * 100:+.1f} %) {new}", flush=True)
                if gain >= a.min_gain:
                    for r in new:
                        keep[tuple(r[:2])] = r
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        for k, v in tn.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for r in keep.values():
            f.write(",".join(str(x) for x in r) + "\n")
    print(f"wrote {len(keep)} tuned entries to {a.out}")


if __name__ == "__main__":
    main()
