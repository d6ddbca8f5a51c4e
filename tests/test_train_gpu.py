"""End-to-end trainer on the GPU: loss decreases, checkpoint is written and resumes."""

import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(tmp_path, **kw):
    from nanosandbox_amd.config import TRAIN_DEFAULTS
    from nanosandbox_amd.data.prepare import synthetic_corpus, write_char_dataset

    if not (tmp_path / "data" / "chars" / "train.bin").exists():
        write_char_dataset(str(tmp_path / "data" / "chars"), synthetic_corpus(300_000))
    c = dict(TRAIN_DEFAULTS)
    c.update(dataset="chars", data_dir=str(tmp_path / "data"), out_dir=str(tmp_path), n_layer=2, n_head=4, n_embd=256, block_size=256,
             batch_size=8, gradient_accumulation_steps=2, max_iters=30, eval_interval=15, eval_iters=2,
             log_interval=5, learning_rate=3e-3, warmup_iters=2, lr_decay_iters=30, min_lr=3e-4,
             compile=False, device="cuda", always_save_checkpoint=True, tensorboard_dir=str(tmp_path / "runs"))
    c.update(kw)
    return c


def test_train_and_resume(kernels, tmp_path):
    from nanosandbox_amd.train import Trainer
    from nanosandbox_amd.utils.tfevents import read_events

    tr = Trainer(_cfg(tmp_path))
    tr.fit()
    ck = os.path.join(tmp_path, "ckpt.pt")
    assert os.path.exists(ck)
    sd = torch.load(ck, weights_only=True)
    assert sd["iter_num"] == 30 and "lm_head.weight" in sd["model"]
    assert len(sd["optimizer"]["state"]) == len(list(tr.raw_model.parameters()))
    import json
    recs = [json.loads(l) for l in open(os.path.join(tmp_path, "metrics.jsonl"))]
    train = [r for r in recs if r["kind"] == "train"]
    assert train[-1]["loss"] < 0.8 * train[0]["loss"]  # learnable char data
    ev = [f for f in os.listdir(tmp_path / "runs" / "gpt2")]
    assert ev and read_events(str(tmp_path / "runs" / "gpt2" / ev[0]))

    tr2 = Trainer(_cfg(tmp_path, init_from="resume", max_iters=32))
    assert tr2.iter_num == 30
    # the checkpoint is written at the eval of iter 30, before that iteration's step
    for k, v in tr2.raw_model.state_dict().items():
        assert torch.equal(v.cpu(), sd["model"][k]), k
    st = tr2.optimizer.state_dict()["state"]
    for i, s in sd["optimizer"]["state"].items():
        assert torch.equal(st[i]["exp_avg"].cpu(), s["exp_avg"])
    tr2.fit()


def test_compile_hip_graph_matches_eager(kernels, tmp_path):
    """compile=True captures the fwd+bwd micro-step as a HIP graph; training must track eager."""
    from nanosandbox_amd.train import Trainer

    def run(compile_):
        torch.manual_seed(0)
        tr = Trainer(_cfg(tmp_path, compile=compile_, dropout=0.0, bias=False, max_iters=8, eval_interval=1000,
                          out_dir=str(tmp_path / f"o{int(compile_)}"), seed=1234))
        X, Y = tr.batches.get_batch("train")
        losses = []
        for it in range(6):
            for g in tr.optimizer.param_groups:
                g["lr"] = 1e-3
            loss, _, X, Y = tr.train_step(X, Y)
            losses.append(loss.item() * tr.gas)
        return tr, losses

    tg, lg = run(True)
    te, le = run(False)
    assert tg.use_graph and tg.graph is not None and tg.graph.replays == 6 * tg.gas
    assert not te.use_graph
    for a, b in zip(lg, le):
        assert abs(a - b) < 2e-2 * abs(b), (lg, le)
    assert lg[-1] < lg[0]


def test_compile_hip_graph_with_dropout(kernels, tmp_path):
    """compile=True with dropout (the char config's p = 0.2): the captured micro-step
    bumps the device-side dropout counter, so replays on the same batch draw different
    masks, and graph training tracks eager training."""
    from nanosandbox_amd.train import Trainer

    def run(compile_, steps=12):
        torch.manual_seed(0)
        tr = Trainer(_cfg(tmp_path, compile=compile_, dropout=0.2, bias=False, max_iters=steps,
                          eval_interval=1000, out_dir=str(tmp_path / f"d{int(compile_)}"), seed=1234))
        X, Y = tr.batches.get_batch("train")
        losses = []
        for _ in range(steps):
            for g in tr.optimizer.param_groups:
                g["lr"] = 2e-3
            loss, _, X, Y = tr.train_step(X, Y)
            losses.append(loss.item() * tr.gas)
        return tr, losses

    tg, lg = run(True)
    assert tg.use_graph and tg.graph is not None
    # two replays on one batch: fresh masks -> different losses
    X, Y = tg.batches.get_batch("train")
    l1 = tg.graph.run(X, Y).item()
    l2 = tg.graph.run(X, Y).item()
    assert l1 != l2
    te, le = run(False)
    assert lg[-1] < 0.9 * lg[0] and le[-1] < 0.9 * le[0]
    assert abs(sum(lg[-4:]) - sum(le[-4:])) < 0.1 * abs(sum(le[-4:])), (lg, le)


def test_sample_from_checkpoint_gpu(kernels, tmp_path):
    """sample.py on the GPU (bf16 compute, last-position logits, top-k multinomial) from a
    checkpoint the GPU trainer wrote; the char codec comes from the dataset's meta.pkl."""
    from nanosandbox_amd.sample import main as sample_main
    from nanosandbox_amd.train import Trainer

    Trainer(_cfg(tmp_path, max_iters=4, eval_interval=4)).fit()
    outs = sample_main([f"--out_dir={tmp_path}", "--num_samples=2", "--max_new_tokens=40", "--start=ab",
                        "--device=cuda"])
    assert len(outs) == 2
    for text in outs:
        assert text.startswith("ab") and len(text) == 42


def test_deterministic_training_is_bitwise_reproducible(kernels, tmp_path):
    """deterministic=True: two identical runs give bitwise-identical parameters and
    optimizer state (fixed-order split-K weight gradients, sorted embedding backward,
    ordered LayerNorm dW/db reduction); the default atomic kernels are only expected
    to agree to rounding."""
    from nanosandbox_amd import ops
    from nanosandbox_amd.train import Trainer

    def run(det):
        torch.manual_seed(0)
        tr = Trainer(_cfg(tmp_path, compile=False, dropout=0.1, bias=True, max_iters=5, eval_interval=1000,
                          out_dir=str(tmp_path / f"det{int(det)}"), seed=77, deterministic=det))
        X, Y = tr.batches.get_batch("train")
        for _ in range(4):
            _, _, X, Y = tr.train_step(X, Y)
        torch.cuda.synchronize()
        return {k: v.detach().float().cpu().clone() for k, v in tr.raw_model.state_dict().items()}

    try:
        a = run(True)
        b = run(True)
        for k in a:
            assert torch.equal(a[k], b[k]), k
        c = run(False)
        for k in a:
            # AdamW turns rounding-level gradient differences of near-zero-gradient
            # entries into up-to-lr-sized steps (the key bias's gradient is exactly zero
            # in exact arithmetic: its updates are noise-driven in either mode), so only
            # the weight matrices are compared, as whole tensors
            if a[k].dim() < 2:
                continue
            err = ((a[k] - c[k]).norm() / (c[k].norm() + 1e-12)).item()
            assert err < 5e-2, (k, err)
    finally:
        ops.set_deterministic(False)


@pytest.mark.parametrize("dtype", ["float16", "float32"])
def test_train_dtype_contract(kernels, tmp_path, dtype):
    """nanoGPT's --dtype on the GPU: float16 runs the fp16 HIP kernels with the dynamic loss
    scale on the device (compile=True captures its micro-step as a HIP graph, the
    scale read from device memory), float32 the torch reference ops (eager micro-steps);
    both learn like bf16."""
    import json

    from nanosandbox_amd.train import Trainer

    tr = Trainer(_cfg(tmp_path, dtype=dtype, max_iters=20, eval_interval=1000, compile=True,
                      tensorboard_dir=""))
    assert tr.raw_model.compute_dtype == {"float16": torch.float16, "float32": torch.float32}[dtype]
    assert tr.use_graph == (dtype == "float16")
    assert (tr.scaler is not None) == (dtype == "float16")
    tr.fit()
    recs = [json.loads(l) for l in open(os.path.join(tmp_path, "metrics.jsonl"))]
    train = [r for r in recs if r["kind"] == "train"]
    assert all(r["loss"] == r["loss"] for r in train)  # finite
    assert train[-1]["loss"] < 0.85 * train[0]["loss"]
    if dtype == "float16":
        assert tr.scaler.scale > 0


def test_fp16_loss_scale_skips_overflowing_steps(kernels, tmp_path):
    """An absurd initial loss scale overflows fp16 gradients: the step is skipped (weights
    unchanged) and the scale backs off until steps go through (GradScaler semantics)."""
    from nanosandbox_amd.train import Trainer

    tr = Trainer(_cfg(tmp_path, dtype="float16", max_iters=5, eval_interval=1000, compile=False,
                      tensorboard_dir=""))
    tr.scaler.scale = 2.0 ** 60
    w0 = tr.store.master.clone()
    X, Y = tr.batches.get_batch("train")
    for g in tr.optimizer.param_groups:
        g["lr"] = 1e-3
    tr.train_step(X, Y)
    assert tr.scaler.skipped == 1 and tr.scaler.scale == 2.0 ** 59
    assert torch.equal(tr.store.master, w0)
    for _ in range(60):  # every overflow halves the scale: 2^59 -> ~2^20 in ~40 skipped steps
        X, Y = tr.batches.get_batch("train")
        tr.train_step(X, Y)
        if not torch.equal(tr.store.master, w0):
            break
    assert not torch.equal(tr.store.master, w0)  # a step went through once the scale fit
    assert tr.scaler.scale < 2.0 ** 59 and tr.scaler.skipped >= 1


def test_recompute_mlp_matches_resident_bitwise(kernels, tmp_path):
    """recompute_mlp=True (selective recomputation): the MLP keeps only its
    input and re-runs c_fc + GELU in the backward.  The recomputed gelu(u) / gelu'(u) come from
    the same kernel on the same operands, so with deterministic reductions the trained
    parameters are bitwise those of the resident run; the planner reports the mode."""
    from nanosandbox_amd import ops
    from nanosandbox_amd.train import Trainer

    def run(rm):
        torch.manual_seed(0)
        tr = Trainer(_cfg(tmp_path, compile=False, dropout=0.1, bias=True, max_iters=5, eval_interval=1000,
                          out_dir=str(tmp_path / f"rm{int(rm)}"), seed=77, deterministic=True, recompute_mlp=rm))
        assert tr.raw_model.recompute_mlp == rm
        X, Y = tr.batches.get_batch("train")
        for _ in range(3):
            _, _, X, Y = tr.train_step(X, Y)
        torch.cuda.synchronize()
        return {k: v.detach().float().cpu().clone() for k, v in tr.raw_model.state_dict().items()}

    try:
        a, b = run(False), run(True)
        for k in a:
            assert torch.equal(a[k], b[k]), k
    finally:
        ops.set_deterministic(False)
