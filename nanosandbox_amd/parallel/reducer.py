"""Bucketed gradient all-reduce over the flat gradient buffer (our DDP).

Why not a line-by-line DDP: the reference relies on torch DDP's reducer, which
copies gradients into its own 25 MiB buckets and back.
Here the gradient already lives in one flat fp32 buffer laid out in
backward-completion order (``FlatParamStore``), so a bucket is just a slice:

* backward kernels accumulate into ``param.main_grad`` and call the param's
  ``_nsa_grad_hook``; on the synchronising micro-step the hook counts
  contributions per bucket and, once a bucket is complete, issues an async
  ``all_reduce(SUM)`` on that slice — overlapping RCCL with the rest of the
  backward pass.  Buckets are launched strictly in index order on every rank
  (a ready bucket waits for its predecessors), so collective order is
  identical across ranks by construction.
* the expected number of contributions per parameter (2 for the tied
  wte/lm_head weight) is discovered on the first synchronised backward, which
  runs without overlap; later steps use the recorded counts (static graph).
* 1/world_size is folded into the fused AdamW kernel's gradient multiplier,
  so there is no separate divide pass.
* bucket size is chosen for xGMI: an MI355X has 7 point-to-point links of
  ~153 GB/s; a ring all-reduce is per-link bound, so buckets should be large
  enough that each RCCL call streams for tens of microseconds on every
  channel.  The 64 MiB default gives GPT-2 124M five 63 MiB buckets, one 9 MiB
  bucket and the 150 MiB wte + wpe tail (``FlatParamStore.buckets``), against
  torch DDP's 19 buckets of 25 MiB.
* the tail bucket (the embeddings, final only after the embedding backward) is the
  one all-reduce that cannot overlap the backward.  ``finish()`` measures what is
  exposed: HIP events on the compute stream before and after its waits give the
  time the compute stream stood still for communication (``exposed_ms``, reported
  by bench.py as ``rccl.exposed_allreduce_ms``).
* optional bf16 compression (``grad_reduce_dtype='bfloat16'``) halves the
  bytes on the wire; the fp32 buffer is restored from the reduced bf16 copy.

The initial parameter broadcast (DDP ctor, C3) is a single broadcast of the
flat fp32 master buffer.
"""

from __future__ import annotations

import collections
import time

import torch
import torch.distributed as dist

from ..optim.flat import FlatParamStore


class _Bucket:
    __slots__ = ("index", "start", "end", "params", "names", "expected", "count", "work", "comm_buf", "early")

    def __init__(self, index, start, end, params, names):
        self.index = index
        self.start = start
        self.end = end
        self.params = params
        self.names = names
        self.expected = 0
        self.count = 0
        self.work = None
        self.comm_buf = None
        self.early = False  # launched by a gradient hook, i.e. before the backward returned


class FlatBucketReducer:
    # per-step records kept for ``exposed_ms``: a long training run that never drains them
    # holds at most this many event pairs (they grew by two HIP events per step)
    HISTORY = 256

    def __init__(self, store: FlatParamStore, process_group=None, bucket_cap_mb: int = 64,
                 reduce_dtype: torch.dtype = torch.float32, history: int = HISTORY):
        assert store.fused_grad, "FlatBucketReducer needs fused main_grad accumulation"
        self.store = store
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.reduce_dtype = reduce_dtype
        cap = max(1, int(bucket_cap_mb * 1024 * 1024))
        self.buckets = [_Bucket(i, s, e, [m.param for m in members], [m.name for m in members])
                        for i, (s, e, members) in enumerate(store.buckets(cap))]
        self._bucket_of = {}
        for b in self.buckets:
            for p in b.params:
                self._bucket_of[id(p)] = b
        self._contrib = {id(s.param): 0 for s in store.slots}
        self.discovered = False
        self.armed = False
        self._next_launch = 0
        self._in_finish = False
        # per synchronised step: buckets launched during the backward, and the exposed
        # communication (HIP event pairs on the compute stream, read lazily; host wall
        # time on the CPU), bounded to the last ``history`` steps
        self._history = max(1, int(history))
        self.launched_in_backward: collections.deque = collections.deque(maxlen=self._history)
        self._exposed: collections.deque = collections.deque(maxlen=self._history)
        for s in store.slots:
            s.param._nsa_grad_hook = self._on_grad

    def layout(self) -> list[dict]:
        """Bucket layout for the bench record: size, parameter count, the first and last
        parameter (backward-completion order), and whether it is the late embedding tail."""
        return [{"index": b.index, "MiB": round((b.end - b.start) * 4 / 2 ** 20, 2), "n_params": len(b.params),
                 "first": b.names[0], "last": b.names[-1],
                 "late": any(getattr(p, "_nsa_late_grad", False) for p in b.params)} for b in self.buckets]

    def exposed_ms(self, clear: bool = True) -> list[float]:
        """Milliseconds per synchronised step between the end of the backward on the compute
        stream and the point where every bucket's all-reduce had landed (synchronises)."""
        out = []
        for e in self._exposed:
            if isinstance(e, tuple):
                e[1].synchronize()
                out.append(float(e[0].elapsed_time(e[1])))
            else:
                out.append(float(e))
        if clear:
            self._exposed.clear()
            self.launched_in_backward.clear()
        return out

    # --------------------------------------------------------------- setup
    @torch.no_grad()
    def broadcast_parameters(self, src: int = 0):
        """One broadcast of the flat master buffer from ``src`` (replaces DDP's per-tensor sync)."""
        dist.broadcast(self.store.master, src=src, group=self.pg)
        self.store.refresh_compute()

    # ------------------------------------------------------------ per step
    def prepare(self, sync: bool):
        """Call before each micro-step backward; ``sync`` on the last micro-step."""
        self.armed = sync
        for b in self.buckets:
            b.count = 0
            b.work = None
            b.early = False
        self._next_launch = 0
        if sync and not self.discovered:
            for k in self._contrib:
                self._contrib[k] = 0

    def _on_grad(self, p):
        if not self.armed:
            return
        if not self.discovered:
            self._contrib[id(p)] += 1
            return
        b = self._bucket_of[id(p)]
        b.count += 1
        if b.count == b.expected:
            self._launch_ready()

    def _launch_ready(self):
        while self._next_launch < len(self.buckets):
            b = self.buckets[self._next_launch]
            if b.count < b.expected:
                return
            self._launch(b)
            b.early = not self._in_finish
            self._next_launch += 1

    def _launch(self, b: _Bucket):
        flat = self.store.grad[b.start:b.end]
        if self.reduce_dtype == torch.float32:
            b.comm_buf = flat
        else:
            b.comm_buf = flat.to(self.reduce_dtype)
        b.work = dist.all_reduce(b.comm_buf, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    @torch.no_grad()
    def finish(self):
        """Wait for every bucket of the synchronising micro-step (launching stragglers)."""
        if not self.armed:
            return
        cuda = self.store.grad.is_cuda
        if cuda:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        else:
            t0 = time.perf_counter()
        self.launched_in_backward.append(sum(b.work is not None for b in self.buckets))
        if not self.discovered:
            for b in self.buckets:
                b.expected = sum(self._contrib[id(p)] for p in b.params)
            self.discovered = True
        for b in self.buckets:
            b.count = max(b.count, b.expected)
        self._in_finish = True
        self._launch_ready()
        self._in_finish = False
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                if b.comm_buf is not None and b.comm_buf.data_ptr() != self.store.grad[b.start:].data_ptr():
                    self.store.grad[b.start:b.end].copy_(b.comm_buf)
                b.work = None
                b.comm_buf = None
        if cuda:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self._exposed.append((ev0, ev1))
        else:
            self._exposed.append((time.perf_counter() - t0) * 1000.0)
        self.armed = False

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world
