"""Run the native RCCL micro-benchmark (``csrc/comm/rccl_bench.cpp``) and parse it.

    python -m nanosandbox_amd.parallel.rccl_bench --ranks 8 --max-mb 512
    torchrun --nproc-per-node 8 -m nanosandbox_amd.parallel.rccl_bench --multi-proc

The last line of the tool's output recommends a DDP bucket size: the smallest
all-reduce message whose bus bandwidth reaches ``target`` of the best measured
one (the per-link-bound ring over point-to-point xGMI).  Feed it
to training as ``--ddp_bucket_mb=<N>``.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

from .. import build as _build


def binary() -> str:
    path = _build.RCCL_BENCH
    if not os.path.exists(path):
        _build.build_tools(verbose=False)
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} missing; run `python -m nanosandbox_amd.build`")
    return path


def run(ranks=0, min_mb=1.0, max_mb=512.0, iters=20, warmup=5, dtype="f32", ops=("all_reduce",), target=0.9,
        id_file=None, timeout=600):
    """Execute the benchmark; returns (rows, recommendation dict or None)."""
    cmd = [binary(), "--min-mb", str(min_mb), "--max-mb", str(max_mb), "--iters", str(iters), "--warmup",
           str(warmup), "--dtype", dtype, "--ops", ",".join(ops), "--target", str(target)]
    if id_file:
        cmd += ["--id-file", id_file]
    elif ranks:
        cmd += ["--ranks", str(ranks)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    if out.returncode != 0:
        raise RuntimeError(f"rccl_bench failed ({out.returncode}): {out.stderr.strip()}")
    return parse(out.stdout)


def parse(text: str):
    rows, rec = [], None
    for line in text.splitlines():
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "recommend_bucket_mb" in d:
            rec = d
        else:
            rows.append(d)
    return rows, rec


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--ranks", type=int, default=0, help="single-process mode: GPUs to use (0 = all)")
    ap.add_argument("--multi-proc", action="store_true",
                    help="one process per GPU (RANK/WORLD_SIZE/LOCAL_RANK from torchrun)")
    ap.add_argument("--id-file", default="/dev/shm/nsa_rccl_bench.id")
    ap.add_argument("--min-mb", type=float, default=1.0)
    ap.add_argument("--max-mb", type=float, default=512.0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    ap.add_argument("--ops", default="all_reduce")
    ap.add_argument("--target", type=float, default=0.9)
    a = ap.parse_args(argv)
    rows, rec = run(ranks=a.ranks, min_mb=a.min_mb, max_mb=a.max_mb, iters=a.iters, warmup=a.warmup, dtype=a.dtype,
                    ops=a.ops.split(","), target=a.target, id_file=a.id_file if a.multi_proc else None)
    if int(os.environ.get("RANK", "0")) == 0:
        for r in rows:
            print(json.dumps(r))
        if rec:
            print(json.dumps(rec))
    return 0


if __name__ == "__main__":
    sys.exit(main())
