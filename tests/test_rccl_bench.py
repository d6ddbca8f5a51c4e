"""RCCL bucket-sizing micro-benchmark (csrc/comm/rccl_bench.cpp): build, CLI, parsing, 1-GPU run."""
import subprocess

import pytest

from nanosandbox_amd import build
from nanosandbox_amd.parallel import rccl_bench


def test_rccl_bench_builds_and_prints_help():
    path = build.build_tools(verbose=False)
    assert path is not None
    out = subprocess.run([path, "--help"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0
    assert "--id-file" in out.stdout


def test_parse_recommendation():
    text = "\n".join([
        "RCCL INFO noise",
        '{"op": "all_reduce", "ranks": 8, "dtype": "f32", "mib": 1.0, "time_us": 50.0, "algbw_GBps": 20.0, '
        '"busbw_GBps": 35.0}',
        '{"recommend_bucket_mb": 64.0, "best_busbw_GBps": 300.0, "target_fraction": 0.9, "ranks": 8}',
    ])
    rows, rec = rccl_bench.parse(text)
    assert len(rows) == 1 and rows[0]["busbw_GBps"] == 35.0
    assert rec["recommend_bucket_mb"] == 64.0


@pytest.mark.gpu
def test_rccl_bench_single_gpu_runs():
    rows, rec = rccl_bench.run(ranks=1, min_mb=1, max_mb=8, iters=3, warmup=1,
                               ops=("all_reduce", "all_gather", "broadcast"))
    ops = {r["op"] for r in rows}
    assert ops == {"all_reduce", "all_gather", "broadcast"}
    assert all(r["time_us"] > 0 for r in rows)
    assert rec is not None and rec["ranks"] == 1
