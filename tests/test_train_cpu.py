"""CPU end-to-end (BASELINE config 1: char model, world_size 1): the reference's
smoke flags (notebooks/colab_nanoGPT_companion.ipynb:70-79), stdout contract,
metrics files, checkpoint layout/resume, auto-resume after an injected fault,
and sampling from the checkpoint."""

import json
import os

import pytest
import torch

from nanosandbox_amd.config import TRAIN_DEFAULTS, apply_overrides
from nanosandbox_amd.data.prepare import synthetic_corpus, write_char_dataset

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def cfg(tmp_path):
    write_char_dataset(str(tmp_path / "data" / "shakespeare_char"), synthetic_corpus(100_000))
    c = apply_overrides(dict(TRAIN_DEFAULTS), [os.path.join(ROOT, "config", "smoke_cpu.py"),
                                               f"--data_dir={tmp_path / 'data'}", f"--out_dir={tmp_path / 'out'}",
                                               "--max_iters=12", "--eval_interval=6", "--eval_iters=3",
                                               "--always_save_checkpoint=True",
                                               f"--tensorboard_dir={tmp_path / 'runs'}"], verbose=False)
    return c


def test_cpu_smoke_train_resume_sample(cfg, tmp_path, capsys):
    from nanosandbox_amd.sample import main as sample_main
    from nanosandbox_amd.train import Trainer
    from nanosandbox_amd.utils.tfevents import read_events

    tr = Trainer(cfg)
    tr.fit()
    out = capsys.readouterr().out
    assert "tokens per iteration will be: 2,048" in out
    assert "step 0: train loss" in out and "step 6: train loss" in out
    assert "iter 12: loss" in out and "mfu" in out
    assert "saving checkpoint to" in out
    ck = torch.load(tmp_path / "out" / "ckpt.pt", weights_only=True)
    assert set(ck) == {"model", "optimizer", "model_args", "iter_num", "best_val_loss", "config"}
    assert ck["iter_num"] == 12 and ck["model_args"]["n_layer"] == 2
    assert ck["optimizer"]["param_groups"][0]["weight_decay"] == 0.1
    assert ck["optimizer"]["param_groups"][1]["weight_decay"] == 0.0
    assert ck["config"]["dataset"] == "shakespeare_char"
    recs = [json.loads(l) for l in open(tmp_path / "out" / "metrics.jsonl")]
    assert {r["kind"] for r in recs} == {"train", "eval"}
    ev = os.listdir(tmp_path / "runs" / "gpt2")
    assert any(t == "eval/val_loss" for _, t, _ in read_events(str(tmp_path / "runs" / "gpt2" / ev[0])))

    # a torch AdamW can load our optimizer state (checkpoint compatibility both ways)
    from nanosandbox_amd.models import GPT, GPTConfig
    m = GPT(GPTConfig(**ck["model_args"]))
    opt = m.configure_optimizers(0.1, 1e-3, (0.9, 0.95), "cpu")
    opt.load_state_dict(ck["optimizer"])

    # resume continues from iter 12
    c2 = dict(cfg, init_from="resume", max_iters=14)
    tr2 = Trainer(c2)
    assert tr2.iter_num == 12
    # the checkpoint is written at the eval of iter 12, before that iteration's step
    st = tr2.optimizer.state_dict()["state"]
    for i, s in ck["optimizer"]["state"].items():
        assert torch.equal(st[i]["exp_avg"], s["exp_avg"])
    for k, v in tr2.raw_model.state_dict().items():
        assert torch.equal(v, ck["model"][k]), k
    tr2.fit()

    outs = sample_main([f"--out_dir={tmp_path / 'out'}", "--device=cpu", "--num_samples=1",
                        "--max_new_tokens=20", f"--data_dir={tmp_path / 'data'}", "--start=KING:"])
    assert outs[0].startswith("KING:") and len(outs[0]) == len("KING:") + 20


def test_fault_job_key_default_rdzv_id(monkeypatch):
    """torchrun's default --rdzv-id makes TORCHELASTIC_RUN_ID 'none' for every
    job, so it cannot key the marker; two default-launched jobs (different elastic agents)
    get different keys, while one job's restarted workers (same agent) keep theirs."""
    import os

    from nanosandbox_amd import train

    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    monkeypatch.setattr(os, "getppid", lambda: 4242)
    k1 = train._fault_job_key()
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")  # the same job after a restart
    assert train._fault_job_key() == k1
    monkeypatch.setattr(os, "getppid", lambda: 4343)  # a second job: another agent
    assert train._fault_job_key() != k1
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job-x")
    assert train._fault_job_key() == "runjob-x"
    monkeypatch.delenv("TORCHELASTIC_RUN_ID")
    monkeypatch.delenv("TORCHELASTIC_RESTART_COUNT")
    assert train._fault_job_key() == f"pid{os.getpid()}"


def test_fault_injection_and_auto_resume(cfg, tmp_path, monkeypatch):
    from nanosandbox_amd.train import Trainer

    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job-a")
    c = dict(cfg, fault_inject_iter=8, fault_inject_rank=0, auto_resume=True)
    with pytest.raises(RuntimeError, match="injected fault"):
        Trainer(c).fit()
    assert (tmp_path / "out" / "ckpt.pt").exists()  # saved at iter 6
    assert (tmp_path / "out" / ".fault_injected_rank0.runjob-a").exists()
    # the same job configuration restarted (what torchrun --max-restarts / a k8s restart
    # does): the fault fired once per job, so the restart resumes at 6 and runs through
    tr = Trainer(c)
    assert tr.iter_num == 6
    tr.fit()
    assert tr.iter_num == 13
    # a later job reusing the out_dir gets its own fault (the marker is keyed to the job)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job-b")
    c2 = dict(c, fault_inject_iter=14, max_iters=20)
    with pytest.raises(RuntimeError, match="injected fault at iter 14"):
        Trainer(c2).fit()


def test_eval_only(cfg, capsys):
    from nanosandbox_amd.train import Trainer

    Trainer(dict(cfg, eval_only=True)).fit()
    out = capsys.readouterr().out
    assert "step 0:" in out and "iter 0:" not in out


def test_nanogpt_checkpoint_with_compile_prefix_loads(cfg, tmp_path):
    """A checkpoint written by a torch.compile'd nanoGPT model carries '_orig_mod.' keys."""
    from nanosandbox_amd.models import GPT, GPTConfig
    from nanosandbox_amd.train import Trainer

    args = dict(n_layer=2, n_head=2, n_embd=64, block_size=128, bias=False, vocab_size=None, dropout=0.0)
    tr = Trainer(cfg)
    args["vocab_size"] = tr.model_args["vocab_size"]
    m = GPT(GPTConfig(**args))
    sd = {"_orig_mod." + k: v for k, v in m.state_dict().items()}
    opt = m.configure_optimizers(0.1, 1e-3, (0.9, 0.95), "cpu")
    os.makedirs(tmp_path / "out", exist_ok=True)
    torch.save({"model": sd, "optimizer": opt.state_dict(), "model_args": args, "iter_num": 3,
                "best_val_loss": torch.tensor(2.5), "config": {}}, tmp_path / "out" / "ckpt.pt")
    tr2 = Trainer(dict(cfg, init_from="resume"))
    assert tr2.iter_num == 3 and tr2.best_val_loss == 2.5
    for (k, a), b in zip(tr2.raw_model.state_dict().items(), m.state_dict().values()):
        assert torch.equal(a, b), k


def test_graph_capture_policy(monkeypatch):
    """compile=True at world_size > 1 captures the accumulation micro-steps with the flat
    reducer (the synchronising one runs eagerly); torch DDP and gas = 1 stay eager."""
    import torch

    from nanosandbox_amd.runtime.hipgraph import graph_capture_supported

    assert not graph_capture_supported("cpu", 0.0, 1)[0]
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    assert graph_capture_supported("cuda:0", 0.0, 1)[0]
    assert graph_capture_supported("cuda:0", 0.2, 8, "flat", 4)[0]
    ok, why = graph_capture_supported("cuda:0", 0.0, 8, "flat", 1)
    assert not ok and "one micro-step" in why
    ok, why = graph_capture_supported("cuda:0", 0.0, 2, "torch", 4)
    assert not ok and "torch DDP" in why


def test_dtype_key_contract():
    """nanoGPT's dtype key: bfloat16 / float16 / float32 accepted (anything else refused
    loudly); the CPU computes in fp32 whatever the key (nanoGPT's nullcontext)."""
    import torch

    from nanosandbox_amd.train import _compute_dtype

    assert _compute_dtype("cuda", "bfloat16") == torch.bfloat16
    assert _compute_dtype("cuda", "float16") == torch.float16
    assert _compute_dtype("cuda", "float32") == torch.float32
    for d in ("bfloat16", "float16", "float32"):
        assert _compute_dtype("cpu", d) == torch.float32
    with pytest.raises(ValueError, match="dtype must be one of"):
        _compute_dtype("cuda", "fp8")


def test_dynamic_loss_scale_policy():
    """GradScaler's policy: back off x0.5 and count a skip on overflow, grow x2 after
    growth_interval clean steps."""
    from nanosandbox_amd.optim.loss_scale import DynamicLossScale

    s = DynamicLossScale(init_scale=1024.0, growth_interval=3)
    assert not s.finite(float("inf")) and not s.finite(float("nan")) and s.finite(3.0)
    s.update(True)
    assert s.scale == 512.0 and s.skipped == 1
    for _ in range(2):
        s.update(False)
    assert s.scale == 512.0
    s.update(False)
    assert s.scale == 1024.0
    sd = s.state_dict()
    s2 = DynamicLossScale()
    s2.load_state_dict(sd)
    assert s2.scale == 1024.0


def test_cpu_trainer_accepts_float16_key(cfg):
    """--dtype=float16 on the CPU trains in fp32 without a scaler (nanoGPT: GradScaler is
    disabled off CUDA)."""
    from nanosandbox_amd.train import Trainer

    tr = Trainer(dict(cfg, dtype="float16", max_iters=2))
    assert tr.scaler is None
    tr.fit()
