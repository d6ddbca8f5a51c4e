"""Deployment layer: k8s manifests (static checks), scripts, entrypoint rank logic,
and a local emulation of the multi-Pod topology."""

import glob
import os
import re
import socket
import subprocess
import sys

import pytest
import yaml

from nanosandbox_amd.parallel import node_rank_from_hostname

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENTRY = os.path.join(ROOT, "container", "entrypoint.sh")


from test_manifests import _docs, _container  # noqa: E402


def test_train_args_are_valid_config_overrides():
    from nanosandbox_amd.config import TRAIN_DEFAULTS, apply_overrides
    d = _docs()
    for k in [("Job", "train-singlepod"), ("StatefulSet", "train-multipod")]:
        _, c = _container(d[k])
        args = c["args"]
        assert args[0] == "train.py"
        cfg = [os.path.join(ROOT, a) if not a.startswith("--") else a for a in args[1:]]
        apply_overrides(dict(TRAIN_DEFAULTS), cfg, verbose=False)  # raises on unknown keys / bad types


def _dry(env, *args):
    e = dict(os.environ, NSA_DRY_RUN="1", **env)
    r = subprocess.run(["bash", ENTRY, *args], env=e, capture_output=True, text=True, check=True)
    return r.stdout


def test_entrypoint_rank_from_ordinal():
    out = _dry({"HOSTNAME": "train-multipod-3", "NNODES": "8", "MASTER_ADDR": "train-multipod-0.train-mp-headless",
                "RDZV_BACKEND": "static"}, "train.py", "config/train_gpt2.py")
    assert "--node-rank=3" in out and "--master-addr=train-multipod-0.train-mp-headless" in out
    assert "train.py config/train_gpt2.py" in out
    out = _dry({"POD_NAME": "train-multipod-5", "NNODES": "8", "MASTER_ADDR": "m", "RDZV_BACKEND": "c10d"}, "x.py")
    assert "--rdzv-backend=c10d" in out and "--rdzv-endpoint=m:29500" in out and "--node-rank=5" in out
    out = _dry({"HOSTNAME": "anything", "NNODES": "1", "NPROC_PER_NODE": "8"}, "x.py")
    assert "--standalone" in out and "--nproc-per-node=8" in out
    assert node_rank_from_hostname("train-multipod-12") == 12


def test_entrypoint_rejects_unranked_multinode():
    e = dict(os.environ, NSA_DRY_RUN="1", HOSTNAME="nohyphen", NNODES="2", MASTER_ADDR="x")
    e.pop("POD_NAME", None)
    r = subprocess.run(["bash", ENTRY, "x.py"], env=e, capture_output=True, text=True)
    assert r.returncode == 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
@pytest.mark.parametrize("rdzv", ["static", "c10d", "c10d-xgmi-pods"])
def test_multipod_emulation(tmp_path, rdzv):
    """Two 'pods' (torchrun agents started through the real entrypoint with
    HOSTNAME=train-multipod-{0,1}) rendezvous on 127.0.0.1 and train on gloo.  The xgmi-pods
    case goes through Topology B over xGMI's path (k8s/statefulset/42-train-multipod-xgmi.yaml):
    preset xgmi-pods and the GPU chosen by ordinal, which must reach every rank."""
    from nanosandbox_amd.data.prepare import synthetic_corpus, write_char_dataset
    write_char_dataset(str(tmp_path / "datasets" / "shakespeare_char"), synthetic_corpus(60_000))
    port = _port()
    procs = []
    xgmi = rdzv.endswith("xgmi-pods")
    for k in range(2):
        env = dict(os.environ, HOSTNAME=f"train-multipod-{k}", NNODES="2", NPROC_PER_NODE="1",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RDZV_BACKEND=rdzv.split("-")[0], RDZV_ID="emu",
                   PYTHON=sys.executable, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
        env.pop("POD_NAME", None)
        env.pop("NSA_LOCAL_DEVICE", None)
        if xgmi:
            env.update(NSA_RCCL_PRESET="xgmi-pods", NSA_DEVICE_SELECT="ordinal", NSA_GPUS_PER_NODE="8",
                       NCCL_HOSTID="emu-node")
        procs.append(subprocess.Popen(
            ["bash", ENTRY, os.path.join(ROOT, "train.py"), os.path.join(ROOT, "config", "smoke_cpu.py"),
             f"--data_dir={tmp_path / 'datasets'}", f"--out_dir={tmp_path / 'out'}", "--max_iters=6",
             "--eval_interval=5", "--eval_iters=2", "--gradient_accumulation_steps=2", "--log_interval=2",
             "--always_save_checkpoint=True"],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, cwd=str(tmp_path)))
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
        outs.append(o)
    assert all(p.returncode == 0 for p in procs), outs[0][-3000:] + "\n----\n" + outs[1][-3000:]
    log = "".join(outs)
    assert "tokens per iteration will be: 4,096" in log  # 2 ranks x 1 micro-step x 16 x 128
    assert "iter 6:" in log and "saving checkpoint" in log
    assert (tmp_path / "out" / "ckpt.pt").exists()
    if xgmi:
        for k in range(2):
            assert f"NSA_LOCAL_DEVICE={k} (of 8)" in outs[k]  # entrypoint
            assert f"rank {k}: device by ordinal NSA_LOCAL_DEVICE={k}" in log  # trainer


def test_local_device_index(monkeypatch):
    from nanosandbox_amd.parallel.dist import local_device_index
    monkeypatch.delenv("NSA_LOCAL_DEVICE", raising=False)
    assert local_device_index(3) == 3
    monkeypatch.setenv("NSA_LOCAL_DEVICE", "6")
    assert local_device_index(0) == 6


@pytest.mark.slow
def test_elastic_restart_resumes_through_entrypoint(tmp_path):
    """Elastic recovery end to end (README.md:116-120): 2 ranks launched
    through the real entrypoint with MAX_RESTARTS=1; rank 1 fails at iter 5 (fault
    injection); torchrun restarts the group, every rank auto-resumes from ckpt.pt at the
    saved iter_num, the job finishes, and both replicas end bit-identical."""
    from nanosandbox_amd.data.prepare import synthetic_corpus, write_char_dataset
    write_char_dataset(str(tmp_path / "datasets" / "shakespeare_char"), synthetic_corpus(60_000))
    env = dict(os.environ, HOSTNAME="train-singlepod", NNODES="1", NPROC_PER_NODE="2", MAX_RESTARTS="1",
               PYTHON=sys.executable, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", NSA_PARAM_DIGEST="1",
               MASTER_ADDR="127.0.0.1")
    env.pop("POD_NAME", None)
    env.pop("TORCHELASTIC_RESTART_COUNT", None)
    p = subprocess.run(
        ["bash", ENTRY, "--local-addr=127.0.0.1", os.path.join(ROOT, "train.py"),
         os.path.join(ROOT, "config", "smoke_cpu.py"), f"--data_dir={tmp_path / 'datasets'}",
         f"--out_dir={tmp_path / 'out'}", "--max_iters=8", "--eval_interval=4", "--eval_iters=2",
         "--gradient_accumulation_steps=2", "--log_interval=1", "--always_save_checkpoint=True",
         "--auto_resume=True", "--fault_inject_iter=5", "--fault_inject_rank=1"],
        env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, cwd=str(tmp_path), timeout=400)
    log = p.stdout
    assert p.returncode == 0, log[-4000:]
    assert "injected fault at iter 5 on rank 1" in log
    assert "auto_resume: found" in log and "Resuming training from" in log
    assert list((tmp_path / "out").glob(".fault_injected_rank1.*"))
    digests = {}
    for line in log.splitlines():
        if "param digest rank" in line:
            # two ranks share the pipe: another rank's output can follow on the same line
            # ("... 9iter 7: loss ..."), so take only the leading digits of the count
            parts = line.split("param digest rank ")[1].split()
            digests[int(parts[0].rstrip(":"))] = (parts[1], int(re.match(r"\d+", parts[3]).group()))
    assert set(digests) == {0, 1}, log[-3000:]
    assert digests[0] == digests[1]  # identical replicas after the restart
    assert digests[0][1] == 9  # iterations 0..max_iters ran, the last one after the resume
