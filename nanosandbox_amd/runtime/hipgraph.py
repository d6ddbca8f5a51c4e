"""HIP-graph capture of one training micro-step (``compile=True``).

nanoGPT's ``compile=True`` runs ``torch.compile`` (Inductor/Triton).  This stack
has no tracing compiler: the hot ops are already fused HIP kernels.  What a
compiler would still buy is the removal of per-kernel host overhead, and on
MI355X that is exactly what a HIP graph does.  The forward, the loss scaling and
the backward of one micro-step (~1,000 kernel launches at GPT-2 124M) are
captured once into a ``torch.cuda.CUDAGraph`` (hipGraph on ROCm) and replayed
for every micro-step, with the batch copied into static input buffers.

Why it is sound here:
* every parameter gradient accumulates into the flat fp32 buffer
  (``param.main_grad``) from inside our autograd ops; torch's AccumulateGrad is
  never involved, so replaying the captured backward gas times accumulates
  exactly like gas eager backwards;
* weights are read through the static bf16 shadow buffer that the optimizer
  refreshes in place, and the learning rate lives in the (eager) optimizer step;
* the GEMM autotuner is warmed up before capture, so no timing runs are captured.

* dropout (the char config's p = 0.2): the per-call dropout salts are host values
  and get baked into the graph, but every dropout kernel mixes them with a
  device-side step counter that the captured micro-step bumps first
  (``ops.rng_advance``), so each replay draws fresh masks, identical between its
  forward and backward.

More than one rank (flat bucket reducer only): the gradient-bucket hooks are Python
callbacks that launch RCCL all-reduces as buckets complete, so the synchronising micro-step
cannot be a replay.  The captured graph (reducer disarmed, no communication) runs the
gas - 1 accumulation micro-steps; the last micro-step runs eagerly with the reducer armed,
its bucket all-reduces overlapping its backward as without graphs.  At gas = 1 (one
micro-step per rank, e.g. 8 ranks on the 480-sequence batch) nothing is captured.

When it is not used (eager fallback, decided by ``graph_capture_supported``): CPU
devices, and torch's own DDP wrapper (its reducer hooks autograd itself).
"""

from __future__ import annotations

import torch


def graph_capture_supported(device: str, dropout: float, world_size: int, ddp_impl: str = "flat",
                            gas: int = 2) -> tuple[bool, str]:
    if not str(device).startswith("cuda") or not torch.cuda.is_available():
        return False, "graph capture needs a GPU device"
    if world_size > 1 and ddp_impl != "flat":
        return False, "torch DDP: its reducer hooks autograd (use ddp_impl='flat')"
    if world_size > 1 and gas < 2:
        return False, "one micro-step per rank: the synchronising micro-step always runs eagerly"
    return True, ""


class MicroStepGraph:
    """Captured ``loss = model(X, Y)[1] / gas; loss.backward()``, replayed per micro-step."""

    def __init__(self, model, X: torch.Tensor, Y: torch.Tensor, gas: int, warmup: int = 2, zero_grad=None,
                 dropout: bool = False, loss_scale: torch.Tensor | None = None):
        """``loss_scale``: the fp16 dynamic loss scale as a 1-element device tensor; the
        backward is taken of loss * scale, with the scale read at replay time (it changes
        between steps on the device)."""
        from ..ops import rng_advance

        self.model = model
        self.gas = gas
        self.X = X.detach().clone()
        self.Y = Y.detach().clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):  # tuner timing runs, allocator warm-up, lazy init
                if dropout:
                    rng_advance(self.X.device)
                _, loss = model(self.X, self.Y)
                ((loss / gas) * loss_scale if loss_scale is not None else loss / gas).backward()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if zero_grad is not None:
            zero_grad()  # the warm-up backwards accumulated into the gradient buffer
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            if dropout:
                rng_advance(self.X.device)  # replayed: fresh dropout masks per micro-step
            _, loss = model(self.X, self.Y)
            self.loss = loss / gas
            (self.loss * loss_scale if loss_scale is not None else self.loss).backward()
        self.replays = 0

    def run(self, X: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
        """Copy the batch into the static inputs and replay; returns the (static) scaled loss."""
        self.X.copy_(X, non_blocking=True)
        self.Y.copy_(Y, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        return self.loss
