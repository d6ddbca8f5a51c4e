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


def rccl_env_defaults(preset: str = "xgmi") -> dict:
    env = dict(XGMI_ENV)
    if preset == "socket":
        env.update(SOCKET_ENV)
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


def init_distributed(backend: str, device: str) -> DistInfo:
    ddp = int(os.environ.get("RANK", -1)) != -1
    if not ddp:
        return DistInfo(ddp=False, device=device)
    if backend == "nccl" and not device.startswith("cuda"):
        backend = "gloo"
    if backend == "nccl":
        rccl_env_defaults(os.environ.get("NSA_RCCL_PRESET", "xgmi"))
    rank = int(os.environ["RANK"])
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    world = int(os.environ["WORLD_SIZE"])
    if device.startswith("cuda") and os.environ.get("NSA_REHEARSAL_ONE_GPU") == "1":
        # multi-rank rehearsal on a 1-GPU box: every rank shares cuda:0 and the
        # collectives go through gloo (RCCL refuses two ranks on one device)
        device = "cuda:0"
        torch.cuda.set_device(device)
        dist.init_process_group(backend="gloo")
    elif device.startswith("cuda"):
        device = f"cuda:{local_rank}"
        torch.cuda.set_device(device)
        dist.init_process_group(backend=backend, device_id=torch.device(device))
    else:
        dist.init_process_group(backend=backend)
    return DistInfo(ddp=True, rank=rank, local_rank=local_rank, world_size=world, device=device)


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
