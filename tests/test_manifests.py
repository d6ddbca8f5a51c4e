"""Static checks of the deployment layer.

Torch-free on purpose: the CI ``lint`` job (.github/workflows/lint.yml) runs this file with
only PyYAML and pytest installed.
"""

import glob
import os
import subprocess

import pytest
import yaml

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


@pytest.mark.parametrize("f", sorted(glob.glob(os.path.join(ROOT, "scripts", "*.sh"))) + [ENTRY])
def test_shell_syntax(f):
    subprocess.run(["bash", "-n", f], check=True)


def _volumes(obj):
    spec = obj["spec"]["template"]["spec"]
    return {v["name"]: v for v in spec.get("volumes", [])}


def test_host_ipc_pods_share_the_host_dev_shm():
    """hostIPC is only useful to RCCL's SHM transport when /dev/shm is the host's: a
    per-pod memory emptyDir mounted there hides it (round-2 verdict, D11)."""
    for (kind, name), obj in _docs().items():
        if kind not in ("StatefulSet", "Job", "Deployment"):
            continue
        spec, c = _container(obj)
        mounts = {m["mountPath"]: m["name"] for m in c.get("volumeMounts", [])}
        if spec.get("hostIPC"):
            assert "/dev/shm" in mounts, name
            vol = _volumes(obj)[mounts["/dev/shm"]]
            assert vol.get("hostPath", {}).get("path") == "/dev/shm", (name, vol)
            assert "emptyDir" not in vol, name


def test_multipod_transport_preset_is_consistent():
    """The StatefulSet (1 GPU per pod) cannot get P2P over xGMI; it must ask for SHM and
    give every pod of a node one RCCL host id (docs/rccl.md)."""
    d = _docs()
    spec, c = _container(d[("StatefulSet", "train-multipod")])
    env = {e["name"]: e for e in c["env"]}
    assert env["NSA_RCCL_PRESET"]["value"] == "shm"
    assert env["NCCL_HOSTID"]["valueFrom"]["fieldRef"]["fieldPath"] == "spec.nodeName"
    assert spec.get("hostIPC") is True
    spec1, c1 = _container(d[("Job", "train-singlepod")])
    env1 = {e["name"]: e.get("value") for e in c1["env"]}
    assert env1["NSA_RCCL_PRESET"] == "xgmi"  # all 8 GPUs in one pod: P2P over xGMI


def test_multipod_xgmi_variant_exposes_peer_gpus():
    """Topology B over xGMI (VERDICT r5 missing item 1): one GPU per pod for the scheduler,
    every render node + /dev/kfd mounted so RCCL can open the peers, the pod's GPU chosen by
    its ordinal, all pods on one node, shared IPC / PID namespaces and the host /dev/shm."""
    d = _docs()
    sts = d[("StatefulSet", "train-multipod-xgmi")]
    svc = d[("Service", "train-mpx-headless")]
    spec, c = _container(sts)
    env = _env(c)
    assert sts["spec"]["serviceName"] == svc["metadata"]["name"] and svc["spec"]["clusterIP"] == "None"
    assert svc["spec"]["selector"] == sts["spec"]["selector"]["matchLabels"]
    assert int(env["NNODES"]) == sts["spec"]["replicas"] == int(env["NSA_GPUS_PER_NODE"]) == 8
    assert env["NPROC_PER_NODE"] == "1" and c["resources"]["limits"]["amd.com/gpu"] == 1
    assert env["MASTER_ADDR"] == f"{sts['metadata']['name']}-0.{svc['metadata']['name']}"
    assert env["NSA_RCCL_PRESET"] == "xgmi-pods" and env["NSA_DEVICE_SELECT"] == "ordinal"
    hostid = next(e for e in c["env"] if e["name"] == "NCCL_HOSTID")
    assert hostid["valueFrom"]["fieldRef"]["fieldPath"] == "spec.nodeName"
    mounts = {m["mountPath"]: m["name"] for m in c["volumeMounts"]}
    vols = _volumes(sts)
    assert vols[mounts["/dev/kfd"]]["hostPath"]["path"] == "/dev/kfd"
    assert vols[mounts["/dev/dri"]]["hostPath"]["path"] == "/dev/dri"
    assert vols[mounts["/dev/shm"]]["hostPath"]["path"] == "/dev/shm"
    assert spec["hostIPC"] is True and spec["hostPID"] is True
    assert c["securityContext"]["privileged"] is True
    aff = spec["affinity"]["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"][0]
    assert aff["topologyKey"] == "kubernetes.io/hostname"
    assert aff["labelSelector"]["matchLabels"] == sts["spec"]["selector"]["matchLabels"]


def test_entrypoint_selects_device_by_ordinal():
    e = dict(os.environ, NSA_DRY_RUN="1", POD_NAME="train-multipod-xgmi-5", NNODES="8", NPROC_PER_NODE="1",
             MASTER_ADDR="m", RDZV_BACKEND="c10d", NSA_RCCL_PRESET="xgmi-pods", NSA_DEVICE_SELECT="ordinal",
             NSA_GPUS_PER_NODE="8", NCCL_HOSTID="node-a")
    r = subprocess.run(["bash", ENTRY, "x.py"], env=e, capture_output=True, text=True, check=True)
    assert "NSA_LOCAL_DEVICE=5" in r.stderr and "--node-rank=5" in r.stdout
    e["NPROC_PER_NODE"] = "2"  # ordinal selection is for one process per pod only
    r = subprocess.run(["bash", ENTRY, "x.py"], env=e, capture_output=True, text=True)
    assert r.returncode == 2
