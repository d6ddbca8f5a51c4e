"""One rank of an N-GPU data-parallel job, on ONE GPU.

The driver's 8-GPU scaling run is the headline, and no 8-GPU node has been available to
measure it before.  ``EmulatedAllReduce`` runs the flat reducer's real bucket logic (its hooks,
bucket order and ``finish()``) but replaces each RCCL all-reduce with a kernel of the
collective's footprint on a high-priority side stream (``nsa_probe_spin``: ``nwg`` 256-thread
workgroups, 8 KiB of LDS, spinning for the all-reduce's modelled duration), launched exactly
where ProcessGroupNCCL would launch it: behind the compute stream at the bucket-ready hook.
So the per-rank step time it measures includes what the collective's kernels do to the
backward's persistent GEMMs (and what they do to it), and the exposed tail all-reduce.

The all-reduce duration is a MODEL, not a measurement: a ring over N ranks moves
2 (N - 1) / N x bucket bytes per rank at ``busbw`` (bus bandwidth, GB/s); RCCL's real number
on an MI355X node has not been measured here (no multi-GPU box), so every projection built
on it is labelled as one (bench.py ``--per-rank-of``).
"""

from __future__ import annotations

import torch
import torch.distributed as dist

from .reducer import FlatBucketReducer


class _SideWork:
    """What reducer.finish() waits on: the compute stream waits for the side stream."""

    def __init__(self, side):
        self.ev = torch.cuda.Event()
        self.ev.record(side)

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


def ensure_single_process_group():
    """The reducer reads the world size from a process group: a gloo group of one."""
    if not dist.is_initialized():
        # an in-process store: no rendezvous address, nothing written to the environment
        dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1)


class EmulatedAllReduce(FlatBucketReducer):
    """The flat reducer with each bucket's all-reduce replaced by a collective-shaped kernel."""

    def __init__(self, store, world: int, bucket_cap_mb: int = 64, busbw_GBps: float = 300.0, nwg: int = 32,
                 wire_bytes_per_elem: int = 4):
        ensure_single_process_group()
        super().__init__(store, bucket_cap_mb=bucket_cap_mb)
        self.emu_world = int(world)
        self.busbw = float(busbw_GBps)
        self.nwg = int(nwg)
        self.wire = int(wire_bytes_per_elem)
        self.side = None  # high-priority side stream (TORCH_NCCL_HIGH_PRIORITY=1), made at the first launch
        self.stamps = torch.zeros(len(self.buckets), 2 * self.nwg, dtype=torch.int64, device=store.grad.device)

    def modelled_us(self, b) -> float:
        n = self.emu_world
        nbytes = (b.end - b.start) * self.wire
        return 2.0 * (n - 1) / n * nbytes / (self.busbw * 1e3)  # bytes / (GB/s) -> us

    def model(self) -> dict:
        return {"world": self.emu_world, "busbw_GBps": self.busbw, "nwg": self.nwg, "wire_bytes": self.wire,
                "allreduce_us_by_bucket": [round(self.modelled_us(b), 1) for b in self.buckets]}

    def _launch(self, b):
        from ..ops import _lib

        ticks = max(1, int(self.modelled_us(b) * 100))  # 100 MHz real-time counter
        if self.side is None:
            self.side = torch.cuda.Stream(device=self.store.grad.device, priority=-1)
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            _lib.call("nsa_probe_spin", self.nwg, ticks, _lib.ptr(self.stamps[b.index]), _lib.stream())
        b.work = _SideWork(self.side)
        b.comm_buf = self.store.grad[b.start:b.end]  # nothing to copy back

    @property
    def grad_scale(self) -> float:
        return 1.0  # the one process's gradient is the job's mean (every rank would be identical)
