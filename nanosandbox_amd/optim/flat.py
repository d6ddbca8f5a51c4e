"""Flat parameter / gradient / compute-shadow storage.

MI355X-first layout (288 GB HBM per GPU makes the memory cost irrelevant; the
win is in the number and size of passes):

* ``master`` — one contiguous fp32 buffer holding every parameter; the
  ``nn.Parameter`` objects become views into it.
* ``grad``   — one contiguous fp32 buffer; each parameter's ``main_grad`` is a
  view.  Linear/LayerNorm/Embedding backward kernels accumulate into it
  directly, and the DDP reducer all-reduces contiguous slices of it (buckets)
  with zero copies.
* ``compute`` — one contiguous bf16 (or fp16, dtype='float16') buffer, the forward/backward weights
  (``param.compute``), rewritten by the fused AdamW kernel in the same pass
  that updates ``master`` — so no per-micro-step autocast weight casts.
* ``wd_mask`` — one byte per 64-element chunk: 1 where weight decay applies
  (nanoGPT rule: tensors with ``dim >= 2``).  Each parameter is padded to a
  multiple of 64 elements so a chunk never straddles two parameters.
* row padding — a parameter tagged ``_nsa_pad_rows = R`` (the tied wte / lm_head weight
  of a vocabulary that is not a multiple of 64, e.g. GPT-2's 50257) gets R rows of room;
  ``param.compute_padded`` / ``param.main_grad_padded`` view them as [R, C] for the lm_head
  GEMMs.  The extra rows start at zero and stay zero (zero gradient, zero AdamW update).

Parameters are laid out in *reverse registration order*, which is the order
their gradients become final during backward (ln_f, last block ... first
block, wpe, wte — the tied wte/lm_head gradient is complete only after the
embedding backward).  Buckets are therefore contiguous and fire in order.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch

CHUNK = 64  # elements per weight-decay flag; also the per-parameter padding granule


@dataclass
class ParamSlot:
    name: str
    param: torch.nn.Parameter
    offset: int
    numel: int
    padded: int
    decay: bool


class FlatParamStore:
    def __init__(self, model: torch.nn.Module, device, compute_dtype=None, fused_grad=True):
        self.device = torch.device(device)
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]  # dedups tied weights
        self.slots: list[ParamSlot] = []
        off = 0
        for name, p in reversed(named):
            n = p.numel()
            rows = getattr(p, "_nsa_pad_rows", None)
            room = rows * p.shape[1] if rows and p.dim() == 2 and rows > p.shape[0] else n
            padded = (room + CHUNK - 1) // CHUNK * CHUNK
            self.slots.append(ParamSlot(name, p, off, n, padded, p.dim() >= 2))
            off += padded
        self.numel = off
        self.master = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=self.device)
        flags = torch.zeros(off // CHUNK, dtype=torch.uint8)
        with torch.no_grad():
            for s in self.slots:
                view = self.master[s.offset:s.offset + s.numel]
                view.copy_(s.param.detach().reshape(-1).to(self.device, torch.float32))
                s.param.data = view.view(s.param.shape)
                if s.decay:
                    flags[s.offset // CHUNK:(s.offset + s.padded) // CHUNK] = 1
        self.wd_mask = flags.to(self.device)
        self.fused_grad = fused_grad
        for s in self.slots:
            g = self.grad[s.offset:s.offset + s.numel].view(s.param.shape)
            if fused_grad:
                s.param.main_grad = g
                pr = self._pad_shape(s)
                if pr is not None:
                    s.param.main_grad_padded = self.grad[s.offset:s.offset + pr[0] * pr[1]].view(pr)
            else:
                s.param.grad = g
        self.compute_dtype = compute_dtype
        self.compute = None
        if compute_dtype is not None and compute_dtype != torch.float32:
            self.compute = torch.empty(off, dtype=compute_dtype, device=self.device)
            for s in self.slots:
                s.param.compute = self.compute[s.offset:s.offset + s.numel].view(s.param.shape)
                pr = self._pad_shape(s)
                if pr is not None:
                    s.param.compute_padded = self.compute[s.offset:s.offset + pr[0] * pr[1]].view(pr)
            self.refresh_compute()

    @staticmethod
    def _pad_shape(s: ParamSlot):
        rows = getattr(s.param, "_nsa_pad_rows", None)
        if rows and s.param.dim() == 2 and rows > s.param.shape[0]:
            return (rows, s.param.shape[1])
        return None

    # ----------------------------------------------------------------- views
    def slot_of(self, p) -> ParamSlot:
        for s in self.slots:
            if s.param is p:
                return s
        raise KeyError("parameter not in store")

    def param_view(self, buf: torch.Tensor, s: ParamSlot) -> torch.Tensor:
        return buf[s.offset:s.offset + s.numel].view(s.param.shape)

    # ------------------------------------------------------------ operations
    @torch.no_grad()
    def refresh_compute(self):
        """Re-derive the bf16 compute shadow from the fp32 master (after load/broadcast)."""
        from ..ops import gemm_dispatch
        gemm_dispatch.weights_changed()
        if self.compute is None:
            return
        if self.device.type == "cuda":
            from ..ops import _lib
            name = "nsa_cast_f32_bf16_h" if self.compute.dtype == torch.float16 else "nsa_cast_f32_bf16"
            _lib.call(name, _lib.ptr(self.master), _lib.ptr(self.compute), self.numel, _lib.stream())
        else:
            self.compute.copy_(self.master)

    @torch.no_grad()
    def zero_grad(self):
        self.grad.zero_()
        if not self.fused_grad:
            # torch DDP / plain autograd path: keep .grad pointing at the flat buffer
            for s in self.slots:
                if s.param.grad is None or s.param.grad.data_ptr() != self.param_view(self.grad, s).data_ptr():
                    s.param.grad = self.param_view(self.grad, s)

    def buckets(self, cap_bytes: int):
        """Contiguous [start, end) element ranges of ``grad``, cut at parameter boundaries
        so that no bucket exceeds ``cap_bytes`` (fp32) unless it holds a single parameter
        larger than the cap, or is the late tail below.  A bucket is closed *before* the
        parameter that would push it past the cap: with the 64 MiB default GPT-2 124M gets five
        63 MiB buckets and a 9 MiB one (the round-4 rule closed a bucket only after it passed
        the cap: about 85 MiB each).
        Parameters tagged ``_nsa_late_grad`` (wte, wpe: complete only after the embedding
        backward, the last kernel of the step) never share a bucket with earlier ones; they
        form one tail bucket (GPT-2 124M: 150 MiB, the one all-reduce that cannot overlap
        the backward)."""
        out = []
        start = 0
        size = 0
        members = []
        late = False
        for s in self.slots:
            nbytes = s.padded * 4
            is_late = bool(getattr(s.param, "_nsa_late_grad", False))
            # the late parameters all become final in the same kernel: one collective for them
            if members and (is_late != late or (size + nbytes > cap_bytes and not is_late)):
                out.append((start, s.offset, members))
                start = s.offset
                size = 0
                members = []
            members.append(s)
            size += nbytes
            late = is_late
        if members:
            out.append((start, self.numel, members))
        return out
