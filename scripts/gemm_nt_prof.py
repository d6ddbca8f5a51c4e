"""Run one NT-GEMM configuration repeatedly (a rocprofv3 --pmc target).

    python scripts/gemm_nt_prof.py --n 768 --k 50304 --probe 0 --iters 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nanosandbox_amd.ops import gemm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=122880)
ap.add_argument("--n", type=int, default=768)
ap.add_argument("--k", type=int, default=50304)
ap.add_argument("--probe", type=int, default=0)
ap.add_argument("--var", type=int, default=0)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--lib", action="store_true", help="torch matmul (hipBLASLt) as a yardstick")
a = ap.parse_args()
x = (torch.rand(a.m, a.k, device="cuda") * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(a.n, a.k, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
for _ in range(a.iters):
    if a.lib:
        y = x @ w.t()
    else:
        y = gemm.nt(x, w, probe=a.probe, var=a.var)
torch.cuda.synchronize()
print("done", y.shape)
