"""Process-group setup for one-process-per-GPU data parallelism.

Contract (nanoGPT ``train.py`` DDP block; topologies from
reference ``README.md:7-8,102``):

* ``ddp = RANK in env``; then ``init_process_group(backend)``, read
  ``RANK/LOCAL_RANK/WORLD_SIZE``, pin ``cuda:{LOCAL_RANK}``; rank 0 is the
  master process; the seed offset is the rank; gradient accumulation steps
  are divided by the world size.

On ROCm the ``nccl`` backend *is* RCCL; single-node ranks talk over xGMI
peer-to-peer.  ``rccl_env_defaults`` documents/sets the presets we use (the
reference's ``NCCL_IB_DISABLE=1``/``NCCL_SOCKET_IFNAME=eth0`` TCP preset is
kept only for the multi-Pod fallback where pods cannot share IPC).
"""

from __future__ import annotations

import os
import re
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    ddp: bool
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    device: str = "cpu"

    @property
    def master_process(self) -> bool:
        return self.rank == 0

    @property
    def seed_offset(self) -> int:
        return self.rank


# Single-node xGMI preset: RCCL picks P2P over xGMI by itself; these only make
# the choice explicit and keep the communicator's kernels on a high-priority
# stream so bucket all-reduces overlap the backward GEMMs.
XGMI_ENV = {
    "TORCH_NCCL_HIGH_PRIORITY": "1",
    "TORCH_NCCL_ASYNC_ERROR_HANDLING": "1",
}
# Multi-Pod fallback when pods do not share IPC/devices (reference README.md:101).
SOCKET_ENV = {
    "NCCL_IB_DISABLE": "1",
    "NCCL_SOCKET_IFNAME": "eth0",
}


# Pods of one node sharing the host /dev/shm but not their GPUs: RCCL's SHM transport
# (host memory).  NCCL_HOSTID (the node name, set by the StatefulSet) makes the pods
# one "host" to RCCL; NCCL_SHM_DISABLE=0 keeps SHM eligible.
SHM_ENV = {
    "NCCL_SHM_DISABLE": "0",
}
# Topology B over xGMI (k8s/statefulset/42-train-multipod-xgmi.yaml): one GPU per pod for the
# scheduler, but every pod mounts all GPUs of its node and pins the one its ordinal names
# (NSA_LOCAL_DEVICE); with one NCCL_HOSTID and shared IPC / PID namespaces RCCL connects the
# pods peer to peer over xGMI.  SHM stays eligible (RCCL's fallback if P2P setup fails).
XGMI_PODS_ENV = dict(SHM_ENV)
# transport kind each preset expects (report_transport warns on a mismatch)
PRESET_TRANSPORT = {"xgmi": "P2P", "xgmi-pods": "P2P", "shm": "SHM", "socket": "NET"}


def rccl_env_defaults(preset: str = "xgmi") -> dict:
    env = dict(XGMI_ENV)
    if preset == "socket":
        env.update(SOCKET_ENV)
    elif preset == "shm":
        env.update(SHM_ENV)
    elif preset == "xgmi-pods":
        env.update(XGMI_PODS_ENV)
    applied = {}
    for k, v in env.items():
        if k not in os.environ:
            os.environ[k] = v
            applied[k] = v
    return applied


def node_rank_from_hostname(hostname: str) -> int:
    """StatefulSet ordinal -> NODE_RANK (``train-multipod-2`` -> 2); the
    ``container/entrypoint.sh`` logic, reference README.md:21,102."""
    m = re.search(r"-(\d+)$", hostname)
    if not m:
        raise ValueError(f"hostname {hostname!r} has no StatefulSet ordinal suffix")
    return int(m.group(1))


# ---------------------------------------------------------------------------------
# Transport check: which RCCL transport carries each peer connection (P2P over xGMI,
# SHM through host memory, NET sockets), read from RCCL's own INIT log, plus one timed
# all-reduce.  The reference's multi-Pod path falls back to TCP silently
# (README.md:101); here a fallback is reported, and flagged when the xgmi preset is on.
# ---------------------------------------------------------------------------------
_TRANSPORT_RE = re.compile(r"->\s*\d+\[\d+\]\s+via\s+(\S+)")
_rccl_log_dir = None


def enable_transport_log() -> str | None:
    """Route RCCL's INIT-subsystem log to a per-process file (before the communicator
    exists).  A user who set NCCL_DEBUG or NCCL_DEBUG_FILE keeps their own log untouched (the
    transport then reads 'unknown'); NSA_RCCL_TRANSPORT_LOG=0 opts out.  The file's directory
    is removed once ``report_transport`` has read it."""
    global _rccl_log_dir
    if (os.environ.get("NSA_RCCL_TRANSPORT_LOG", "1") == "0" or "NCCL_DEBUG_FILE" in os.environ
            or "NCCL_DEBUG" in os.environ):
        return None
    import tempfile
    _rccl_log_dir = tempfile.mkdtemp(prefix="nsa_rccl_")
    os.environ.setdefault("NCCL_DEBUG", "INFO")
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT")
    os.environ["NCCL_DEBUG_FILE"] = os.path.join(_rccl_log_dir, "rccl.%h.%p.log")
    return _rccl_log_dir


def parse_transports(lines) -> dict:
    """Count the transports of RCCL's channel-connection lines
    (``Channel 00/0 : 0[0] -> 1[1] via P2P/IPC``): {'P2P/IPC': 14, ...}."""
    out: dict = {}
    for line in lines:
        m = _TRANSPORT_RE.search(line)
        if m:
            out[m.group(1)] = out.get(m.group(1), 0) + 1
    return out


def transport_kind(counts: dict) -> str:
    """Collapse transport names to P2P / SHM / NET / mixed; 'unknown' when no channel line
    was parsed (log not captured)."""
    kinds = {k.split("/")[0] for k in counts}
    if not kinds:
        return "unknown"
    return kinds.pop() if len(kinds) == 1 else "mixed:" + "+".join(sorted(kinds))


def _own_log_lines() -> list:
    if _rccl_log_dir is None:
        return []
    import glob
    lines = []
    for f in glob.glob(os.path.join(_rccl_log_dir, f"rccl.*.{os.getpid()}.log")):
        with open(f, errors="replace") as fh:
            lines += fh.readlines()
    return lines


def report_transport(info: "DistInfo", nbytes: int = 64 << 20, iters: int = 5, verbose: bool = True) -> dict:
    """Time an ``nbytes`` fp32 all-reduce (bus bandwidth = 2(n-1)/n * bytes / time) and
    collect every rank's transport counts on rank 0.  Rank 0 prints one JSON line and a
    WARNING when the xgmi preset is on but a connection is not P2P."""
    import json
    import time
    if not info.ddp or not dist.is_initialized():
        return {}
    be = dist.get_backend()
    dev = torch.device(info.device) if be == "nccl" else torch.device("cpu")
    x = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
    dist.all_reduce(x)  # communicator init (the INIT log is complete after this)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(x)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / iters
    n = info.world_size
    busbw = 2 * (n - 1) / n * nbytes / dt / 1e9
    counts = parse_transports(_own_log_lines()) if be == "nccl" else {"gloo": 1}
    _drop_transport_log()
    gathered = [None] * n
    dist.all_gather_object(gathered, {"rank": info.rank, "transports": counts})
    rep = {"backend": be, "preset": os.environ.get("NSA_RCCL_PRESET", "xgmi"), "world": n,
           "allreduce_MiB": nbytes >> 20, "allreduce_ms": round(dt * 1e3, 3), "busbw_GBps": round(busbw, 1),
           "transport": {g["rank"]: transport_kind(g["transports"]) for g in gathered},
           "connections": {g["rank"]: g["transports"] for g in gathered}}
    if info.rank == 0 and verbose:
        print("rccl: " + json.dumps(rep), flush=True)
        want = PRESET_TRANSPORT.get(rep["preset"])
        bad = {r: k for r, k in rep["transport"].items() if k not in (want, "unknown")}
        if be == "nccl" and want and bad:
            print(f"WARNING: NSA_RCCL_PRESET={rep['preset']} expects {want} but RCCL picked {bad}; "
                  "see docs/rccl.md 'Which transport each topology gets'", flush=True)
    return rep


def _drop_transport_log():
    global _rccl_log_dir
    if _rccl_log_dir is not None:
        import shutil
        shutil.rmtree(_rccl_log_dir, ignore_errors=True)
        _rccl_log_dir = None


def allreduce_sweep(info: "DistInfo", sizes_mib=(4, 16, 64, 256), iters: int = 3, verbose: bool = True) -> list:
    """All-reduce bus bandwidth by message size (the gradient bucket size trade-off of
    docs/rccl.md: per-call latency vs per-link bandwidth over xGMI).  Rank 0 prints one
    ``rccl sweep:`` JSON line; every rank returns the rows."""
    import json
    import time
    if not info.ddp or not dist.is_initialized():
        return []
    be = dist.get_backend()
    dev = torch.device(info.device) if be == "nccl" else torch.device("cpu")
    n = info.world_size
    rows = []
    for mib in sizes_mib:
        x = torch.ones((int(mib) << 20) // 4, dtype=torch.float32, device=dev)
        dist.all_reduce(x)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / iters
        rows.append({"MiB": mib, "ms": round(dt * 1e3, 3),
                     "busbw_GBps": round(2 * (n - 1) / n * x.numel() * 4 / dt / 1e9, 1)})
        del x
    if info.rank == 0 and verbose:
        print("rccl sweep: " + json.dumps({"backend": be, "world": n, "rows": rows}), flush=True)
    return rows


def _attempt_store(rank: int, world: int):
    """The rendezvous store for an elastic restart, namespaced by the attempt.

    After ``torchrun --max-restarts`` restarts the worker group, the new workers can
    read the dead attempt's gloo/RCCL address keys from the reused store and fail to
    connect (observed with --standalone: "connectFullMesh ... Connection refused").
    Prefixing every key with the restart count isolates the attempts.  Returns None on
    the first attempt (plain env:// init)."""
    restart = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0)
    if restart <= 0 or "MASTER_ADDR" not in os.environ or "MASTER_PORT" not in os.environ:
        return None
    from datetime import timedelta
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
    store = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                          is_master=(not agent and rank == 0), timeout=timedelta(minutes=10),
                          multi_tenant=not agent)
    return dist.PrefixStore(f"nsa/attempt_{restart}", store)


def local_device_index(local_rank: int) -> int:
    """GPU index this process pins: ``NSA_LOCAL_DEVICE`` when the launcher chose one (Topology
    B over xGMI selects the pod's GPU by its StatefulSet ordinal, container/entrypoint.sh),
    else LOCAL_RANK (nanoGPT's ``cuda:{LOCAL_RANK}``)."""
    v = os.environ.get("NSA_LOCAL_DEVICE", "")
    return int(v) if v.strip() else local_rank


def init_distributed(backend: str, device: str) -> DistInfo:
    ddp = int(os.environ.get("RANK", -1)) != -1
    if not ddp:
        return DistInfo(ddp=False, device=device)
    if backend == "nccl" and not device.startswith("cuda"):
        backend = "gloo"
    if backend == "nccl":
        rccl_env_defaults(os.environ.get("NSA_RCCL_PRESET", "xgmi"))
        if os.environ.get("NSA_REHEARSAL_ONE_GPU") != "1":
            enable_transport_log()
    rank = int(os.environ["RANK"])
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ["WORLD_SIZE"])
    store = _attempt_store(rank, world)
    kw = {} if store is None else {"store": store, "rank": rank, "world_size": world}
    if device.startswith("cuda") and os.environ.get("NSA_REHEARSAL_ONE_GPU") == "1":
        # multi-rank rehearsal on a 1-GPU box: every rank shares cuda:0 and the
        # collectives go through gloo (RCCL refuses two ranks on one device)
        device = "cuda:0"
        torch.cuda.set_device(device)
        dist.init_process_group(backend="gloo", **kw)
    elif device.startswith("cuda"):
        device = f"cuda:{local_device_index(local_rank)}"
        torch.cuda.set_device(device)
        dist.init_process_group(backend=backend, device_id=torch.device(device), **kw)
    else:
        dist.init_process_group(backend=backend, **kw)
    return DistInfo(ddp=True, rank=rank, local_rank=local_rank, world_size=world, device=device)


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
