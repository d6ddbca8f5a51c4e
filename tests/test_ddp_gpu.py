"""Data-parallel training through the GPU kernel path, two ranks on one MI355X.

RCCL refuses two ranks on one device, so the rehearsal runs the collectives
over gloo (which stages CUDA tensors through the host) while every kernel —
GEMMs, flash attention, LayerNorm, fused AdamW, the flat bucketed reducer's
hooks — runs on cuda:0 exactly as in an 8-GPU job (``NSA_REHEARSAL_ONE_GPU``,
parallel/dist.py).  Checks: the initial broadcast fixes different per-rank
inits, ranks stay bit-identical, and the result matches single-process GPU
training on the same global batch (gradient accumulation / world-size
semantics).
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(n_layer=2, n_head=2, n_embd=128, block_size=64, vocab_size=512, bias=False, dropout=0.0)
STEPS = 3
GLOBAL_MICRO = 4
MB = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# production-kernel rehearsal: every GEMM dimension >= 256 so the forward / input-grad
# GEMMs take the persistent NT kernel and the weight grads the four-wave split-K kernel
# (CFG's widths run on the small-tile / ring64 kernels)
CFG_PROD = dict(n_layer=2, n_head=4, n_embd=256, block_size=256, vocab_size=1024, bias=False, dropout=0.0)


def _batches(cfg=CFG):
    g = torch.Generator().manual_seed(7)
    T, V = cfg["block_size"], cfg["vocab_size"]
    return [[torch.randint(0, V, (MB, T + 1), generator=g) for _ in range(GLOBAL_MICRO)] for _ in range(STEPS)]


def _build(seed, cfg=CFG):
    from nanosandbox_amd.models import GPT, GPTConfig
    from nanosandbox_amd.optim import FlatParamStore

    torch.manual_seed(seed)
    m = GPT(GPTConfig(**cfg)).to("cuda:0").set_compute_dtype(torch.bfloat16)
    store = FlatParamStore(m, "cuda:0", compute_dtype=torch.bfloat16)
    opt = m.configure_optimizers(0.1, 3e-3, (0.9, 0.95), "cuda", store=store)
    return m, store, opt


def _train(model, store, opt, micro_batches, gas, before=None, after=None):
    for step_batches in micro_batches:
        for i, d in enumerate(step_batches):
            if before:
                before(i == gas - 1)
            d = d.to("cuda:0")
            _, loss = model(d[:, :-1], d[:, 1:])
            (loss / gas).backward()
        if after:
            after()
        opt.clip_grad_norm_(1.0)
        opt.step()
        opt.zero_grad()
    torch.cuda.synchronize()
    return store.master.detach().cpu().clone()


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NSA_REHEARSAL_ONE_GPU="1")
    from nanosandbox_amd.parallel import FlatBucketReducer
    from nanosandbox_amd.parallel.dist import init_distributed

    info = init_distributed("nccl", "cuda")
    assert info.device == "cuda:0" and info.world_size == world
    gas = GLOBAL_MICRO // world
    mine = [[b[rank * gas + i] for i in range(gas)] for b in _batches()]
    model, store, opt = _build(seed=200 + rank)  # different init per rank: the broadcast must fix it
    red = FlatBucketReducer(store, bucket_cap_mb=1)
    red.broadcast_parameters()
    opt.grad_scale = red.grad_scale
    final = _train(model, store, opt, mine, gas, before=red.prepare, after=red.finish)
    torch.save({"final": final, "n_buckets": len(red.buckets)}, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_ddp_gpu_two_ranks_match_single_process(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    res = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    assert res[0]["n_buckets"] > 1
    assert torch.equal(res[0]["final"], res[1]["final"]), "ranks diverged"
    model, store, opt = _build(seed=200)  # rank 0's init, all micro-batches in one process
    ref = _train(model, store, opt, _batches(), GLOBAL_MICRO)
    d = (res[0]["final"] - ref).abs()
    # the remaining differences: summation order (gloo's rank sum vs sequential
    # accumulation, split-K / embedding / LayerNorm-partial atomics); Adam turns that noise
    # into <= lr-sized steps on near-zero gradients
    assert d.max() <= STEPS * 3e-3 + 1e-6
    assert d.mean() < 2e-5


def _worker_prod(rank, world, port, out_dir, mode):
    """As _worker, with the production-size GEMMs (NT and four-wave weight-grad kernels, by
    the fixed shape rule every rank evaluates identically) in default or deterministic mode.
    Collectives still run over gloo (one GPU)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NSA_REHEARSAL_ONE_GPU="1")
    from nanosandbox_amd import ops
    from nanosandbox_amd.ops import gemm_dispatch
    from nanosandbox_amd.parallel import FlatBucketReducer
    from nanosandbox_amd.parallel.dist import init_distributed

    ops.set_deterministic(mode == "deterministic")
    info = init_distributed("nccl", "cuda")
    assert info.world_size == world
    gas = GLOBAL_MICRO // world
    mine = [[b[rank * gas + i] for i in range(gas)] for b in _batches(CFG_PROD)]
    model, store, opt = _build(seed=300 + rank, cfg=CFG_PROD)
    red = FlatBucketReducer(store, bucket_cap_mb=1)
    red.broadcast_parameters()
    opt.grad_scale = red.grad_scale
    final = _train(model, store, opt, mine, gas, before=red.prepare, after=red.finish)
    used = {repr(k): v for k, v in gemm_dispatch.kernels_used().items()}
    torch.save({"final": final, "n_buckets": len(red.buckets), "used": used},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["default", "deterministic"])
def test_ddp_gpu_production_kernels(tmp_path, mode):
    """The flat reducer's bucket hooks, our split-K weight-gradient kernels accumulating
    into the flat gradient and the NT forward / input-gradient GEMMs, together under DDP.
    Every rank runs the same kernels (a fixed shape rule: no tuning decision to agree on)
    and ranks agree bitwise; a single-process run of the global batch differs only in the
    gradient summation order."""
    from nanosandbox_amd import ops

    port = _free_port()
    mp.spawn(_worker_prod, args=(2, port, str(tmp_path), mode), nprocs=2, join=True)
    res = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(2)]
    assert res[0]["n_buckets"] > 1
    assert res[0]["used"] == res[1]["used"]
    used = res[0]["used"]
    assert any(v.startswith("wgrad4") for v in used.values()), used
    assert any(v == "nt4" for v in used.values()), used
    assert not any(v == "torch" for v in used.values()), used
    assert torch.equal(res[0]["final"], res[1]["final"]), "ranks diverged"
    ops.set_deterministic(mode == "deterministic")
    try:
        model, store, opt = _build(seed=300, cfg=CFG_PROD)
        ref = _train(model, store, opt, _batches(CFG_PROD), GLOBAL_MICRO)
    finally:
        ops.set_deterministic(False)
    d = (res[0]["final"] - ref).abs()
    assert d.max() <= STEPS * 3e-3 + 1e-6
    assert d.mean() < 2e-5


def _worker_trainer(rank, world, port, out_dir, cfg, compile_):
    """Trainer-level DDP rehearsal (flat reducer over gloo, one GPU): compile=True captures
    the accumulation micro-steps as a HIP graph and runs the synchronising one eagerly."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NSA_REHEARSAL_ONE_GPU="1")
    from nanosandbox_amd.train import Trainer

    torch.manual_seed(0)
    c = dict(cfg, compile=compile_, out_dir=os.path.join(out_dir, f"c{int(compile_)}_r{rank}"))
    tr = Trainer(c)
    X, Y = tr.batches.get_batch("train")
    losses = []
    for _ in range(4):
        for g in tr.optimizer.param_groups:
            g["lr"] = 1e-3
        loss, _, X, Y = tr.train_step(X, Y)
        losses.append(loss.item() * tr.gas)
    torch.cuda.synchronize()
    torch.save({"losses": losses, "final": tr.store.master.detach().cpu().clone(), "use_graph": tr.use_graph,
                "replays": tr.graph.replays if tr.graph is not None else 0, "gas": tr.gas},
               os.path.join(out_dir, f"t{int(compile_)}_rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_ddp_gpu_compile_graph_with_reducer(tmp_path):
    """compile=True at world_size 2: the gas - 1 accumulation micro-steps
    replay a HIP graph captured with the bucket hooks disarmed, the last one runs eagerly
    with the reducer armed; ranks stay bitwise identical and training tracks eager DDP."""
    from nanosandbox_amd.config import TRAIN_DEFAULTS
    from nanosandbox_amd.data.prepare import synthetic_corpus, write_char_dataset

    write_char_dataset(str(tmp_path / "data" / "chars"), synthetic_corpus(200_000))
    cfg = dict(TRAIN_DEFAULTS)
    cfg.update(dataset="chars", data_dir=str(tmp_path / "data"), n_layer=2, n_head=4, n_embd=256, block_size=256,
               batch_size=4, gradient_accumulation_steps=6, max_iters=10, eval_interval=1000, eval_iters=1,
               log_interval=1000, device="cuda", backend="nccl", dropout=0.0, bias=False, seed=1234,
               ddp_impl="flat", ddp_bucket_mb=1, tensorboard_dir="", always_save_checkpoint=False)
    res = {}
    for compile_ in (True, False):
        port = _free_port()
        mp.spawn(_worker_trainer, args=(2, port, str(tmp_path), cfg, compile_), nprocs=2, join=True)
        res[compile_] = [torch.load(os.path.join(tmp_path, f"t{int(compile_)}_rank{r}.pt"), weights_only=True)
                         for r in range(2)]
    g, e = res[True], res[False]
    assert g[0]["use_graph"] and not e[0]["use_graph"]
    assert g[0]["gas"] == 3 and g[0]["replays"] == 4 * (g[0]["gas"] - 1)
    for r in (g, e):
        assert torch.equal(r[0]["final"], r[1]["final"]), "ranks diverged"
    for a, b in zip(g[0]["losses"], e[0]["losses"]):
        assert abs(a - b) < 2e-2 * abs(b), (g[0]["losses"], e[0]["losses"])
    d = (g[0]["final"] - e[0]["final"]).abs()
    assert d.max() < 4 * 3e-3 and d.mean() < 2e-5


def _worker_fit(rank, world, port, out_dir, cfg):
    """Trainer.fit() under DDP (flat reducer over gloo, one GPU): rank 0 evaluates alone at
    iteration 0 and at the eval interval while the other rank trains on; nothing may pair
    up wrongly or hang (no collective outside the reducer's ordered buckets)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), NSA_REHEARSAL_ONE_GPU="1")
    from nanosandbox_amd.train import Trainer

    torch.manual_seed(0)
    tr = Trainer(dict(cfg, out_dir=os.path.join(out_dir, f"fit_r{rank}")))
    tr.fit()
    torch.cuda.synchronize()
    torch.save({"final": tr.store.master.detach().cpu().clone(), "iter": tr.iter_num},
               os.path.join(out_dir, f"fit_rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_ddp_gpu_fit_with_rank0_eval(tmp_path):
    from nanosandbox_amd.config import TRAIN_DEFAULTS
    from nanosandbox_amd.data.prepare import synthetic_corpus, write_char_dataset

    write_char_dataset(str(tmp_path / "data" / "chars"), synthetic_corpus(200_000))
    cfg = dict(TRAIN_DEFAULTS)
    cfg.update(dataset="chars", data_dir=str(tmp_path / "data"), n_layer=2, n_head=4, n_embd=256, block_size=256,
               batch_size=4, gradient_accumulation_steps=4, max_iters=6, eval_interval=3, eval_iters=2,
               log_interval=1, device="cuda", backend="nccl", dropout=0.0, bias=True, seed=1234, compile=False,
               ddp_impl="flat", ddp_bucket_mb=1, tensorboard_dir="", always_save_checkpoint=False)
    port = _free_port()
    mp.spawn(_worker_fit, args=(2, port, str(tmp_path), cfg), nprocs=2, join=True)
    res = [torch.load(os.path.join(tmp_path, f"fit_rank{r}.pt"), weights_only=True) for r in range(2)]
    assert res[0]["iter"] == res[1]["iter"] == 7
    assert torch.equal(res[0]["final"], res[1]["final"]), "ranks diverged"
