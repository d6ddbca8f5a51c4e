"""Deployment layer: k8s manifests (static checks), scripts, entrypoint rank logic,
and a local emulation of the multi-Pod topology."""

import glob
import os
import socket
import subprocess
import sys

import pytest
import yaml

from nanosandbox_amd.parallel import node_rank_from_hostname

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENTRY = os.path.join(ROOT, "container", "entrypoint.sh")


def _docs():
    out = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "k8s", "**", "*.yaml"), recursive=True)):
        for d in yaml.safe_load_all(open(f)):
            if d:
                out[(d["kind"], d["metadata"]["name"])] = d
    return out


def test_manifests_parse_and_names():
    d = _docs()
    assert ("Namespace", "disttrain") in d
    assert ("ConfigMap", "proxy-config") in d
    assert ("PersistentVolume", "disttrain-pv") in d and ("PersistentVolumeClaim", "disttrain-pvc") in d
    assert d[("PersistentVolume", "disttrain-pv")]["spec"]["hostPath"]["path"] == "/var/lib/disttrain"
    for k in [("Job", "download-tiny-shakespeare"), ("Job", "train-singlepod"), ("StatefulSet", "train-multipod"),
              ("Service", "train-mp-headless"), ("Job", "prepare-owt-subset")]:
        assert k in d, k
        if k[0] != "PersistentVolume":
            assert d[k]["metadata"].get("namespace", "disttrain") == "disttrain"


def test_no_proxy_keeps_cluster_traffic_direct():
    cm = _docs()[("ConfigMap", "proxy-config")]["data"]
    for h in [".svc", ".cluster.local", "127.0.0.1", "localhost"]:
        assert h in cm["NO_PROXY"]


def _container(obj):
    spec = obj["spec"]["template"]["spec"]
    return spec, spec["containers"][0]


def _env(c):
    return {e["name"]: e.get("value") for e in c.get("env", [])}


def test_singlepod_job_uses_all_gpus_standalone():
    spec, c = _container(_docs()[("Job", "train-singlepod")])
    env = _env(c)
    assert c["resources"]["limits"]["amd.com/gpu"] == int(env["NPROC_PER_NODE"]) == 8
    assert env["NNODES"] == "1"
    assert any(m["mountPath"] == "/data" for m in c["volumeMounts"])
    assert any(m["mountPath"] == "/dev/shm" for m in c["volumeMounts"])
    assert "nvidia.com/gpu" not in str(spec)


def test_statefulset_rendezvous_consistency():
    d = _docs()
    sts = d[("StatefulSet", "train-multipod")]
    svc = d[("Service", "train-mp-headless")]
    spec, c = _container(sts)
    env = _env(c)
    assert sts["spec"]["serviceName"] == svc["metadata"]["name"]
    assert svc["spec"]["clusterIP"] == "None"
    assert svc["spec"]["selector"] == sts["spec"]["selector"]["matchLabels"]
    assert int(env["NNODES"]) == sts["spec"]["replicas"] == 8
    assert env["NPROC_PER_NODE"] == "1" and c["resources"]["limits"]["amd.com/gpu"] == 1
    assert env["MASTER_ADDR"] == f"{sts['metadata']['name']}-0.{svc['metadata']['name']}"
    assert env["MASTER_PORT"] == str(svc["spec"]["ports"][0]["port"])
    assert env["RDZV_BACKEND"] == "c10d"
    assert any(e["name"] == "POD_NAME" for e in c["env"])
    assert any(a.startswith("config/train_gpt2_350m.py") for a in c["args"])


def test_train_args_are_valid_config_overrides():
    from nanosandbox_amd.config import TRAIN_DEFAULTS, apply_overrides
    d = _docs()
    for k in [("Job", "train-singlepod"), ("StatefulSet", "train-multipod")]:
        _, c = _container(d[k])
        args = c["args"]
        assert args[0] == "train.py"
        cfg = [os.path.join(ROOT, a) if not a.startswith("--") else a for a in args[1:]]
        apply_overrides(dict(TRAIN_DEFAULTS), cfg, verbose=False)  # raises on unknown keys / bad types


@pytest.mark.parametrize("f", sorted(glob.glob(os.path.join(ROOT, "scripts", "*.sh"))) + [ENTRY])
def test_shell_syntax(f):
    subprocess.run(["bash", "-n", f], check=True)


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
@pytest.mark.parametrize("rdzv", ["static", "c10d"])
def test_multipod_emulation(tmp_path, rdzv):
    """Two 'pods' (torchrun agents started through the real entrypoint with
    HOSTNAME=train-multipod-{0,1}) rendezvous on 127.0.0.1 and train on gloo."""
    from nanosandbox_amd.data.prepare import synthetic_corpus, write_char_dataset
    write_char_dataset(str(tmp_path / "datasets" / "shakespeare_char"), synthetic_corpus(60_000))
    port = _port()
    procs = []
    for k in range(2):
        env = dict(os.environ, HOSTNAME=f"train-multipod-{k}", NNODES="2", NPROC_PER_NODE="1",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RDZV_BACKEND=rdzv, RDZV_ID="emu",
                   PYTHON=sys.executable, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
        env.pop("POD_NAME", None)
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
