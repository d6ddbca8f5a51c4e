"""bench.py batch plan: the 491,520-token optimizer step is fixed for every N (strong scaling)."""
import importlib.util
import os

import pytest

_spec = importlib.util.spec_from_file_location(
    "nsa_bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
bench = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(bench)


@pytest.mark.parametrize("world,expect_micro", [(1, 120), (2, 120), (4, 120), (8, 60), (3, 80)])
def test_auto_plan_keeps_global_batch(world, expect_micro):
    micro, total_micro = bench.batch_plan(world)
    assert micro == expect_micro
    assert total_micro % world == 0
    assert micro * total_micro == 480  # sequences per optimizer step
    assert micro * total_micro * 1024 == 491_520


def test_nanogpt_schedule_reproducible():
    # --micro-batch 12 reproduces train_gpt2's 12 x 40 (5 x 8 on 8 ranks)
    assert bench.batch_plan(1, 12) == (12, 40)
    assert bench.batch_plan(8, 12) == (12, 40)


def test_bad_plans_rejected():
    with pytest.raises(AssertionError):
        bench.batch_plan(7)
    with pytest.raises(AssertionError):
        bench.batch_plan(1, 7)


@pytest.mark.slow
def test_multirank_record_carries_rccl_block(tmp_path):
    """bench.py's N > 1 path (torchrun, 2 ranks, gloo on the CPU, the tiny plumbing model):
    the one stdout JSON record carries the per-rank transport and the all-reduce sweep, so a
    driver SCALE run needs no log scraping."""
    import json
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=root)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                        "--gpus", "2", "--device", "cpu", "--model", "tiny", "--micro-batch", "24",
                        "--block-size", "32", "--steps", "1", "--warmup", "1", "--rccl-sweep", "1,2"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    rc = rec["rccl"]
    assert rc["backend"] == "gloo"
    assert set(rc["transport_by_rank"]) == {"0", "1"}
    assert [r["MiB"] for r in rc["sweep"]] == [1, 2] and all(r["busbw_GBps"] > 0 for r in rc["sweep"])
    assert rc["allreduce_64MiB_ms"] > 0
    # the bucket layout and the exposed all-reduce per timed step
    assert rc["buckets"] and rc["buckets"][-1]["late"]
    assert rc["exposed_allreduce_ms"] is not None and rc["exposed_allreduce_ms"] >= 0
    assert len(rc["exposed_allreduce_ms_per_step"]) == 1
    assert all(n >= 1 for n in rc["buckets_launched_in_backward"])
    assert "gemm_kernels" in rec  # per GEMM shape the kernel that ran it (empty on the CPU)
    assert "box" in rec and rec["box"] is None  # clocks + calibration GEMM: GPU runs only


def test_read_clocks_parses_dpm_tables(tmp_path, monkeypatch):
    """the bench record's clock fields come from the amdgpu DPM tables;
    the '*' level is the one in use, the top level is the card's maximum."""
    from nanosandbox_amd.utils import boxcal

    dev = tmp_path / "card1" / "device"
    dev.mkdir(parents=True)
    (dev / "pp_dpm_sclk").write_text("0: 500Mhz\n1: 1800Mhz *\n2: 2400Mhz\n")
    (dev / "pp_dpm_mclk").write_text("0: 900Mhz\n1: 1900Mhz *\n")
    monkeypatch.setattr(boxcal.glob, "glob", lambda pat: [str(dev)])
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    c = boxcal.read_clocks(0)
    assert c["sclk"] == {"cur_mhz": 1800, "max_mhz": 2400} and c["mclk"] == {"cur_mhz": 1900, "max_mhz": 1900}
    assert c["source"] == "sysfs:card1"
    monkeypatch.setattr(boxcal.glob, "glob", lambda pat: [])
    monkeypatch.setattr(boxcal.shutil, "which", lambda name: None)
    assert boxcal.read_clocks(0) == {"sclk": None, "mclk": None, "source": None}


def test_bench_record_has_box_block():
    """The record carries a 'box' block (clocks before / after the timed loop + calibration
    GEMM TF/s) next to the timing; bench.py's CLI exposes the calibration length."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "bench.py")).read()
    assert '"box": box' in src and "--calib-seconds" in src
    assert "clocks_before" in src and "clocks_after" in src and "calibration_gemm" in src


def test_per_rank_emulation_model_and_record():
    """--per-rank-of N: one rank's micro-batch plan of an N-GPU job, the
    flat reducer's buckets with each all-reduce modelled as a ring at an assumed bus bandwidth,
    and a record that says it is a projection (never the headline metric)."""
    import torch

    import bench
    from nanosandbox_amd.models import GPT, GPTConfig
    from nanosandbox_amd.optim import FlatParamStore
    from nanosandbox_amd.parallel.emulate import EmulatedAllReduce

    assert bench.batch_plan(8, 60) == (60, 8)  # 60 x 1 per rank: the N = 8 share of 480 sequences
    cfg = GPTConfig(n_layer=12, n_head=12, n_embd=768, block_size=1024, vocab_size=50304, bias=False)
    store = FlatParamStore(GPT(cfg), "cpu")
    emu = EmulatedAllReduce(store, 8, bucket_cap_mb=64, busbw_GBps=300.0, nwg=32)
    m = emu.model()
    assert m["world"] == 8 and m["busbw_GBps"] == 300.0 and m["nwg"] == 32
    assert len(m["allreduce_us_by_bucket"]) == len(emu.buckets) == 7
    b = emu.buckets[0]
    want = 2 * 7 / 8 * (b.end - b.start) * 4 / 300e3
    assert abs(m["allreduce_us_by_bucket"][0] - round(want, 1)) < 0.11
    assert emu.grad_scale == 1.0
    torch.distributed.destroy_process_group()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "bench.py")).read()
    assert "--per-rank-of" in src and '"projection": True' in src and "PROJECTED tokens/sec" in src
