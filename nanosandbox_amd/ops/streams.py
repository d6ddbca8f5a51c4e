"""Side HIP stream for weight-gradient GEMMs.

In a transformer backward the input-gradient chain is strictly serial
(dgrad -> GELU' -> dgrad -> LayerNorm' -> flash-attention backward -> ...),
but each weight gradient dW = dY^T X only needs tensors that already exist
when its layer's dgrad is issued.  Launching the dW GEMMs on a second stream
lets the GPU run them beside the serial chain: a compute-bound split-K GEMM
next to the memory-bound GELU / LayerNorm backward kernels and the
latency-bound flash-attention backward (one 8-wave workgroup per CU), which
fills CUs that would otherwise idle (MI355X has 4 hardware queues per process;
two streams map to two of them).

Protocol (all calls are no-ops on CPU tensors and during HIP-graph capture):

* ``fork(*tensors)`` — side stream waits for the main stream's current
  position (so the operands are complete and any earlier ``zero_grad`` of the
  flat gradient is ordered before the accumulate), and the operands are kept
  referenced until an event recorded after the side GEMM has passed (checked
  without blocking at the next ``fork``; all released at ``join``).  That one
  mechanism covers both hazards: the caching allocator cannot hand their
  memory to the main stream early, and autograd cannot accumulate another
  gradient in place into them (it only does so for buffers nobody else
  references; the residual stream's dY is both a weight-GEMM operand and an
  accumulation target).  ``record_stream`` is deliberately not used: its
  deferred frees pile up when the host runs steps ahead of the GPU and pushed
  the caching allocator into its synchronising free-and-retry path (7x slower
  steps measured on MI355X).
  Returns a context manager that makes the side stream current.
* ``join()`` — the main stream waits for every side launch so far.  The
  first ``fork`` of a backward pass queues it as an autograd final callback,
  so when ``loss.backward()`` returns every weight gradient is ordered before
  the caller's stream (plain ``.main_grad`` reads are safe).  It is also
  called before anything reads or rewrites the flat gradient outside a GEMM:
  the embedding backward (tied wte/lm_head gradient), grad-norm / AdamW,
  ``zero_grad``.  Bucket all-reduces are issued from the side stream itself
  (parallel/reducer.py), so they never stall the main stream.

Scheduling: a weight GEMM is forked right after the input-gradient GEMM of the
same layer, so it starts when that GEMM is done and runs beside the
memory-bound kernel that follows on the main stream (GELU backward, LayerNorm
backward); ``before_compute`` makes the main stream wait for the side stream
before its next compute-bound launch (input-gradient GEMM, flash-attention
backward).  Two compute kernels never share the GPU that way: measured on
MI355X, a side weight GEMM left running beside the next input-gradient GEMM
held the CUs it had (one 139 KB-LDS workgroup per CU, for the kernel's whole
500 us) and stretched that GEMM from ~0.46 to ~8 ms, a zero-sum reshuffle;
hipBLASLt's gfx950 picks for some shapes are also persistent Stream-K kernels
(``_SK3``) whose workgroups wait on each other and stalled whole steps when a
concurrent stream held CUs.  ``NSA_WGRAD_CONCURRENT=1`` drops the
``before_compute`` waits (and keeps such library shapes off hipBLASLt) for A/B runs.

Opt-in (``NSA_WGRAD_STREAM=1``); the default keeps every weight gradient on
the main stream.
"""

from __future__ import annotations

import contextlib
import os

import torch

ENABLED = os.environ.get("NSA_WGRAD_STREAM", "0") == "1"
CONCURRENT_COMPUTE = os.environ.get("NSA_WGRAD_CONCURRENT", "0") == "1"

_side: dict = {}
_pending: set = set()
_callback_queued = False
_held: list = []  # (side-stream event, operands) not yet known to be consumed


def _end_of_backward():
    global _callback_queued
    _callback_queued = False
    join()


def side_stream(device) -> torch.cuda.Stream:
    idx = torch.device(device).index
    if idx is None:
        idx = torch.cuda.current_device()
    s = _side.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _side[idx] = s
    return s


def active(t: torch.Tensor) -> bool:
    return ENABLED and t.is_cuda and not torch.cuda.is_current_stream_capturing()


def fork(*tensors: torch.Tensor):
    """Context manager running the enclosed launches on the side stream (see module doc)."""
    t0 = tensors[0]
    if not active(t0):
        return contextlib.nullcontext()
    s = side_stream(t0.device)
    s.wait_stream(torch.cuda.current_stream(t0.device))
    while _held and _held[0][0].query():  # operands the side stream has finished with
        _held.pop(0)
    _pending.add(s.device.index if s.device.index is not None else torch.cuda.current_device())
    global _callback_queued
    if not _callback_queued:
        try:  # only possible inside a backward pass; outside one the caller joins explicitly
            torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
            _callback_queued = True
        except RuntimeError:
            pass
    return _on_side(s, tensors)


@contextlib.contextmanager
def _on_side(s, tensors):
    with torch.cuda.stream(s):
        yield
    _held.append((s.record_event(), tensors))


def before_compute(t: torch.Tensor) -> None:
    """Main stream waits for the side stream before a compute-bound launch (see module doc)."""
    if _pending and not CONCURRENT_COMPUTE and t.is_cuda:
        join(t.device)


def join(device=None) -> None:
    """Make the current stream wait for all side-stream work launched so far."""
    if not _pending:
        return
    if torch.cuda.is_current_stream_capturing():
        return
    idxs = list(_pending) if device is None else [torch.device(device).index or torch.cuda.current_device()]
    for idx in idxs:
        s = _side.get(idx)
        if s is not None:
            torch.cuda.current_stream(idx).wait_stream(s)
        _pending.discard(idx)
    _held.clear()  # everything the main stream does from here on is ordered after the side work
