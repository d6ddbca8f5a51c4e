"""Data-parallel correctness without GPUs: gloo, world_size 2.

* our flat bucketed reducer and torch DDP must give identical parameters on
  every rank, equal to single-process training on the same global batch with
  the same number of micro-steps (gradient accumulation / world-size semantics);
* ranks start from *different* random inits: the initial broadcast must fix that;
* bf16-compressed reduction stays close;
* buckets launch in order and overlap the backward (launched before finish()).
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from nanosandbox_amd.models import GPT, GPTConfig
from nanosandbox_amd.optim import FlatParamStore
from nanosandbox_amd.parallel import FlatBucketReducer

CFG = dict(n_layer=2, n_head=2, n_embd=32, block_size=16, vocab_size=64, bias=True)
STEPS = 3
GLOBAL_MICRO = 4  # micro-steps per optimizer step across all ranks
MB = 3  # micro-batch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches():
    g = torch.Generator().manual_seed(123)
    return [[torch.randint(0, 64, (MB, 17), generator=g) for _ in range(GLOBAL_MICRO)] for _ in range(STEPS)]


def _build(seed, fused_grad=True):
    torch.manual_seed(seed)
    m = GPT(GPTConfig(**CFG))
    store = FlatParamStore(m, "cpu", fused_grad=fused_grad)
    opt = m.configure_optimizers(0.1, 1e-2, (0.9, 0.95), "cpu", store=store)
    return m, store, opt


def _train(model, store, opt, micro_batches, gas, before_backward=None, after_backward=None):
    for step_batches in micro_batches:
        for i, d in enumerate(step_batches):
            sync = i == gas - 1
            if before_backward:
                before_backward(sync)
            _, loss = model(d[:, :-1], d[:, 1:])
            (loss / gas).backward()
        if after_backward:
            after_backward()
        opt.clip_grad_norm_(1.0)
        opt.step()
        opt.zero_grad()
    return store.master.clone()


def _worker(rank, world, port, mode, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    gas = GLOBAL_MICRO // world
    mine = [[b[rank * gas + i] for i in range(gas)] for b in _batches()]
    info = {}
    if mode in ("flat", "flat_bf16"):
        model, store, opt = _build(seed=100 + rank)  # different init per rank: broadcast must fix it
        red = FlatBucketReducer(store, bucket_cap_mb=0.02 if mode == "flat" else 1,
                                reduce_dtype=torch.bfloat16 if mode == "flat_bf16" else torch.float32)
        red.broadcast_parameters()
        opt.grad_scale = red.grad_scale
        launched_early = []

        def after():
            launched_early.append(sum(b.work is not None for b in red.buckets))
            red.finish()

        final = _train(model, store, opt, mine, gas, before_backward=red.prepare, after_backward=after)
        info["n_buckets"] = len(red.buckets)
        info["launched_before_finish"] = launched_early
    else:  # torch DDP
        from torch.nn.parallel import DistributedDataParallel as DDP
        model, store, opt = _build(seed=100 + rank, fused_grad=False)
        ddp = DDP(model)
        store.zero_grad()

        def before(sync):
            ddp.require_backward_grad_sync = sync

        final = _train(ddp, store, opt, mine, gas, before_backward=before)
    torch.save({"final": final, "info": info}, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def _run(mode, world, tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, mode, str(tmp_path)), nprocs=world, join=True)
    return [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(world)]


def _reference():
    model, store, opt = _build(seed=100)  # rank 0's init
    return _train(model, store, opt, _batches(), GLOBAL_MICRO)


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["flat", "torch"])
def test_ddp_matches_single_process(mode, tmp_path):
    res = _run(mode, 2, tmp_path)
    ref = _reference()
    assert torch.equal(res[0]["final"], res[1]["final"]), "ranks diverged"
    # Adam normalises per element, so fp32 summation-order noise on near-zero
    # gradients shows up at ~1e-5 absolute in a handful of elements
    assert torch.allclose(res[0]["final"], ref, atol=2e-5, rtol=1e-5)
    assert (res[0]["final"] - ref).abs().mean() < 1e-7
    if mode == "flat":
        info = res[0]["info"]
        assert info["n_buckets"] > 1
        # first step discovers contribution counts (no overlap); later steps launch during backward
        assert info["launched_before_finish"][0] == 0
        assert all(n == info["n_buckets"] for n in info["launched_before_finish"][1:])


@pytest.mark.slow
def test_ddp_bf16_compressed_reduction(tmp_path):
    res = _run("flat_bf16", 2, tmp_path)
    ref = _reference()
    assert torch.equal(res[0]["final"], res[1]["final"])
    d = (res[0]["final"] - ref).abs()
    # bf16 gradient rounding can flip Adam's per-element step on tiny gradients;
    # each step moves a weight by at most ~lr (1e-2), so bound by steps * lr
    assert d.max() <= STEPS * 1e-2 + 1e-6
    assert d.mean() < 1e-3


def test_bucket_layout_contiguous_reverse_order():
    model, store, _ = _build(0)
    b = store.buckets(4 * 1024)
    assert b[0][0] == 0 and b[-1][1] == store.numel
    for (s0, e0, _), (s1, e1, _) in zip(b, b[1:]):
        assert e0 == s1
    names = [s.name for s in store.slots]
    assert names[0].startswith("transformer.ln_f") and names[-1] == "transformer.wte.weight"


def test_bucket_cap_rule_gpt2_124m():
    """a bucket is closed before the parameter that would push it past
    the cap, so no bucket exceeds ``ddp_bucket_mb`` unless it is one oversized parameter or
    the late embedding tail (wte + wpe, final only after the embedding backward), and the
    tail shares no bucket with block weights."""
    from nanosandbox_amd.models import GPT, GPTConfig

    cfg = GPTConfig(n_layer=12, n_head=12, n_embd=768, block_size=1024, vocab_size=50304, bias=False)
    store = FlatParamStore(GPT(cfg), "cpu")
    cap = 64 << 20
    b = store.buckets(cap)
    for s, e, members in b:
        late = [getattr(m.param, "_nsa_late_grad", False) for m in members]
        assert all(late) or not any(late), "late embeddings share a bucket with block weights"
        if (e - s) * 4 > cap:
            assert len(members) == 1 or all(late)
    assert {m.name for m in b[-1][2]} == {"transformer.wte.weight", "transformer.wpe.weight"}
    sizes = [(e - s) * 4 / 2 ** 20 for s, e, _ in b]
    assert len(b) == 7 and all(v <= 64 for v in sizes[:-1]), sizes


def test_reducer_records_layout_and_exposure(tmp_path):
    """The reducer's record for the bench JSON: bucket layout, buckets launched while the
    backward ran, and the exposed wait in finish() per synchronised step (gloo, 2 ranks)."""
    port = _free_port()
    mp.spawn(_exposure_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    rec = torch.load(os.path.join(tmp_path, "exposure0.pt"), weights_only=True)
    assert len(rec["layout"]) == rec["n_buckets"] > 1
    assert rec["layout"][-1]["late"] and not any(x["late"] for x in rec["layout"][:-1])
    assert all(x["MiB"] > 0 and x["first"] and x["last"] for x in rec["layout"])
    assert len(rec["exposed"]) == STEPS and all(v >= 0 for v in rec["exposed"])
    # the first step discovers contribution counts; later ones launch during the backward
    assert rec["early"][0] == 0 and all(n >= 1 for n in rec["early"][1:])
    assert rec["early"][1:] == [rec["n_buckets"]] * (STEPS - 1)


def _exposure_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    gas = GLOBAL_MICRO // world
    mine = [[b[rank * gas + i] for i in range(gas)] for b in _batches()]
    model, store, opt = _build(seed=100)
    red = FlatBucketReducer(store, bucket_cap_mb=0.02)
    opt.grad_scale = red.grad_scale
    _train(model, store, opt, mine, gas, before_backward=red.prepare, after_backward=red.finish)
    early = list(red.launched_in_backward)
    rec = {"layout": red.layout(), "n_buckets": len(red.buckets), "early": early, "exposed": red.exposed_ms()}
    if rank == 0:
        torch.save(rec, os.path.join(out_dir, "exposure0.pt"))
    dist.destroy_process_group()


def test_rccl_env_presets(monkeypatch):
    """RCCL presets fill only unset variables: xGMI (single node) sets the torch NCCL
    knobs; the socket preset adds the reference's TCP-only transport (README.md:101)."""
    from nanosandbox_amd.parallel import dist

    for k in list(dist.XGMI_ENV) + list(dist.SOCKET_ENV):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "ens5")
    applied = dist.rccl_env_defaults("socket")
    assert applied["NCCL_IB_DISABLE"] == "1" and "NCCL_SOCKET_IFNAME" not in applied
    import os
    assert os.environ["NCCL_SOCKET_IFNAME"] == "ens5"  # an operator's setting wins
    for k in dist.XGMI_ENV:
        assert os.environ[k] == dist.XGMI_ENV[k]
    assert dist.rccl_env_defaults("xgmi") == {}  # idempotent


def _sweep_worker(rank, world, port, out_dir):
    import json
    import os

    import torch.distributed as dist

    from nanosandbox_amd.parallel import allreduce_sweep
    from nanosandbox_amd.parallel.dist import init_distributed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    info = init_distributed("gloo", "cpu")
    rows = allreduce_sweep(info, (1, 2), iters=1, verbose=False)
    with open(os.path.join(out_dir, f"sweep{rank}.json"), "w") as f:
        json.dump(rows, f)
    dist.destroy_process_group()


def test_allreduce_sweep_rows(tmp_path):
    """bench.py's pre-timing bucket-size sweep (world > 1): one row per size, positive bus
    bandwidth, on every rank."""
    import json

    port = _free_port()
    mp.spawn(_sweep_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        rows = json.load(open(tmp_path / f"sweep{r}.json"))
        assert [x["MiB"] for x in rows] == [1, 2]
        assert all(x["busbw_GBps"] > 0 and x["ms"] > 0 for x in rows)


def _bounded_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    model, store, opt = _build(seed=100)
    red = FlatBucketReducer(store, bucket_cap_mb=0.02, history=8)
    d = torch.randint(0, 64, (MB, 17), generator=torch.Generator().manual_seed(7))
    sizes = []
    for _ in range(40):  # a training loop that never calls exposed_ms()
        red.prepare(True)
        _, loss = model(d[:, :-1], d[:, 1:])
        loss.backward()
        red.finish()
        opt.zero_grad()
        sizes.append((len(red._exposed), len(red.launched_in_backward)))
    rec = {"sizes": sizes, "exposed": red.exposed_ms(), "after": (len(red._exposed), len(red.launched_in_backward))}
    if rank == 0:
        torch.save(rec, os.path.join(out_dir, "bounded0.pt"))
    dist.destroy_process_group()


def test_reducer_history_is_bounded(tmp_path):
    """finish() records an event pair per synchronised step; a run that never
    drains them through exposed_ms() (train.py) must not grow without bound."""
    port = _free_port()
    mp.spawn(_bounded_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    rec = torch.load(os.path.join(tmp_path, "bounded0.pt"), weights_only=True)
    assert max(a for a, _ in rec["sizes"]) == 8 and max(b for _, b in rec["sizes"]) == 8
    assert len(rec["exposed"]) == 8 and rec["after"] == (0, 0)
