"""Fused flat AdamW (+ global grad-norm clipping) over a ``FlatParamStore``.

One optimizer step is three kernels regardless of the parameter count:

1. ``nsa_sumsq_partial`` — per-block partial sum of squares of the flat fp32
   gradient (deterministic two-level reduction, no atomics),
2. ``nsa_clip_coef``     — one block folds the partials into the global norm
   and writes the combined gradient multiplier
   ``grad_scale * min(1, max_norm / (norm + 1e-6))`` to device memory,
3. ``nsa_adamw_step``    — one streaming pass that reads (p, g, m, v), applies
   decoupled weight decay (per-64-element-chunk mask), updates m/v/p and also
   writes the bf16 compute shadow.  ~30 B/param, HBM-bound.

Nothing is read back to the host (lr/betas/bias corrections are host scalars
computed from the step counter), so the step is graph-capturable.  With an fp16 dynamic
loss scale attached (``attach_loss_scale``) the three kernels also run GradScaler's
unscale / inf check / skip / scale update on the device (``optim/loss_scale.py``).

Math and state layout match ``torch.optim.AdamW`` (``decoupled_weight_decay``):
``state_dict()`` / ``load_state_dict()`` speak torch's format — per-parameter
``step``/``exp_avg``/``exp_avg_sq`` indexed in param-group order and two param
groups (decay / no decay) — so nanoGPT checkpoints resume across both
(SURVEY.md §2.9.6, §7.4 item 3).  Clipping follows
``torch.nn.utils.clip_grad_norm_`` (coef = max_norm / (norm + 1e-6), clamped to 1).
"""

from __future__ import annotations

import math

import torch

from .flat import FlatParamStore

_NORM_BLOCKS = 1024


class FusedAdamW:
    def __init__(self, store: FlatParamStore, param_groups, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0):
        self.store = store
        dev = store.device
        self.param_groups = []
        for g in param_groups:
            d = dict(weight_decay=g.get("weight_decay", weight_decay), lr=g.get("lr", lr),
                     betas=tuple(g.get("betas", betas)), eps=g.get("eps", eps), amsgrad=False, maximize=False,
                     foreach=None, capturable=False, differentiable=False, fused=True,
                     decoupled_weight_decay=True)
            d["params"] = list(g["params"])
            self.param_groups.append(d)
        for g in self.param_groups:
            for p in g["params"]:
                s = store.slot_of(p)
                want_decay = g["weight_decay"] != 0.0
                if want_decay != s.decay and g["weight_decay"] != 0.0:
                    raise ValueError("fused AdamW: decay groups must follow the dim>=2 rule of the flat store")
        self.exp_avg = torch.zeros(store.numel, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(store.numel, dtype=torch.float32, device=dev)
        self.step_count = 0
        self.grad_scale = 1.0  # set by the reducer (1/world_size when it sums)
        self._coef = torch.ones(1, dtype=torch.float32, device=dev)
        self._norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self._partial = torch.zeros(2 * _NORM_BLOCKS, dtype=torch.float32, device=dev)
        self._clip_pending = False
        self.loss_scale = None  # DynamicLossScale (fp16), see attach_loss_scale

    def attach_loss_scale(self, ls) -> None:
        """Run the fp16 dynamic loss scale's policy inside the optimizer kernels: the
        gradient multiplier divides by the device scale, a step whose gradients hold an
        inf / NaN is skipped on the device, and AdamW's bias correction counts good steps."""
        self.loss_scale = ls

    # -------------------------------------------------------------- helpers
    @property
    def _is_gpu(self):
        return self.store.device.type == "cuda"

    def _hyper(self):
        g0 = self.param_groups[0]
        lrs = {g["lr"] for g in self.param_groups}
        if len(lrs) != 1:
            raise ValueError("fused AdamW applies one learning rate to all groups")
        wd = max(g["weight_decay"] for g in self.param_groups)
        return g0["lr"], g0["betas"], g0["eps"], wd

    # ------------------------------------------------------------ grad norm
    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global L2 norm of the (scaled) gradient; arms clipping for the next step.

        Returns the pre-clip total norm as a 1-element device tensor (no sync)."""
        g = self.store.grad
        ls = self.loss_scale
        if self._is_gpu:
            from ..ops import _lib
            lsp = _lib.ptr(ls.state) if ls is not None else None
            _lib.call("nsa_sumsq_partial", _lib.ptr(g), g.numel(), _lib.ptr(self._partial), _NORM_BLOCKS,
                      float(self.grad_scale), lsp, _lib.stream())
            _lib.call("nsa_clip_coef", _lib.ptr(self._partial), _NORM_BLOCKS, float(self.grad_scale),
                      float(max_norm), _lib.ptr(self._norm), _lib.ptr(self._coef), lsp,
                      ls.growth_factor if ls else 0.0, ls.backoff_factor if ls else 0.0,
                      float(ls.growth_interval) if ls else 0.0, _lib.stream())
        elif ls is not None:  # host reference of the kernels' loss-scale path
            from .loss_scale import LS_SCALE
            gs = float(self.grad_scale) / float(ls.state[LS_SCALE])
            found = not bool(torch.isfinite(g).all())
            norm = float("inf") if found else float((g.double() * gs).pow(2).sum().sqrt())
            self._norm.fill_(norm)
            c = min(1.0, max_norm / (norm + 1e-6)) if (max_norm > 0 and not found) else 1.0
            self._coef.fill_(0.0 if found else gs * c)
            ls.update(found)
        else:
            norm = g.double().pow(2).sum().sqrt().float() * self.grad_scale
            self._norm.copy_(norm.view(1))
            c = min(1.0, max_norm / (float(norm) + 1e-6)) if max_norm > 0 else 1.0
            self._coef.fill_(self.grad_scale * c)
        self._clip_pending = True
        return self._norm

    @property
    def last_norm(self) -> torch.Tensor:
        """Device norm of the last gradient check: the user's ``clip_grad_norm_`` or, with a
        loss scale and no clipping, the inf check ``step()`` runs itself (inf on a step the
        loss scale skipped).  No sync."""
        return self._norm

    # ----------------------------------------------------------------- step
    @torch.no_grad()
    def step(self):
        ls = self.loss_scale
        if not self._clip_pending:
            if ls is not None:  # the inf check / unscale / scale update still has to run
                self.clip_grad_norm_(0.0)
            else:
                self._coef.fill_(self.grad_scale)
        self._clip_pending = False
        if ls is not None and not self._is_gpu and ls.found_inf:
            return  # host reference: GradScaler skips the step
        self.step_count += 1
        lr, (beta1, beta2), eps, wd = self._hyper()
        t = self.step_count
        bc1 = 1.0 - beta1 ** t
        bc2_sqrt = math.sqrt(1.0 - beta2 ** t)
        st = self.store
        if self._is_gpu:
            from ..ops import _lib, gemm_dispatch
            gemm_dispatch.weights_changed()  # the kernel rewrites the bf16 compute weights
            # the fp16 instantiation writes an fp16 compute shadow (dtype float16)
            name = "nsa_adamw_step_h" if st.compute is not None and st.compute.dtype == torch.float16 else "nsa_adamw_step"
            _lib.call(name, _lib.ptr(st.master), _lib.ptr(st.grad), _lib.ptr(self.exp_avg),
                      _lib.ptr(self.exp_avg_sq), _lib.ptr(st.compute), _lib.ptr(st.wd_mask), st.numel,
                      float(lr), float(beta1), float(beta2), float(eps), float(wd), float(bc1), float(bc2_sqrt),
                      _lib.ptr(self._coef), _lib.ptr(ls.state) if ls is not None else None, _lib.stream())
            return
        if ls is not None:  # bias correction counts the good steps only
            t = ls.good_steps
            bc1 = 1.0 - beta1 ** t
            bc2_sqrt = math.sqrt(1.0 - beta2 ** t)
        # CPU reference (same math as the kernel, torch.optim.AdamW semantics)
        p, m, v = st.master, self.exp_avg, self.exp_avg_sq
        g = st.grad * self._coef
        mask = st.wd_mask.repeat_interleave(p.numel() // st.wd_mask.numel()).bool()
        p.mul_(torch.where(mask, 1.0 - lr * wd, 1.0))
        m.mul_(beta1).add_(g, alpha=1.0 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
        denom = (v.sqrt() / bc2_sqrt).add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)
        if st.compute is not None:
            st.compute.copy_(p)
            from ..ops import gemm_dispatch
            gemm_dispatch.weights_changed()

    def zero_grad(self, set_to_none: bool = True):
        # the flat buffer is persistent (gradient views, bucket views) -> zero instead of None
        self.store.zero_grad()

    # ----------------------------------------------------------- state dict
    def _ordered_params(self):
        return [p for g in self.param_groups for p in g["params"]]

    def state_dict(self):
        st = self.store
        state = {}
        step = self.loss_scale.good_steps if self.loss_scale is not None else self.step_count
        for i, p in enumerate(self._ordered_params()):
            s = st.slot_of(p)
            state[i] = {
                "step": torch.tensor(float(step), dtype=torch.float32),
                "exp_avg": st.param_view(self.exp_avg, s).detach().clone(),
                "exp_avg_sq": st.param_view(self.exp_avg_sq, s).detach().clone(),
            }
        groups = []
        idx = 0
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(idx, idx + len(g["params"])))
            idx += len(g["params"])
            groups.append(d)
        return {"state": state, "param_groups": groups}

    @torch.no_grad()
    def load_state_dict(self, sd):
        params = self._ordered_params()
        groups = sd["param_groups"]
        if len(groups) != len(self.param_groups):
            raise ValueError("loaded state dict has a different number of parameter groups")
        for g_saved, g in zip(groups, self.param_groups):
            if len(g_saved["params"]) != len(g["params"]):
                raise ValueError("loaded state dict contains a parameter group that doesn't match the size")
            for k in ("lr", "betas", "eps", "weight_decay"):
                if k in g_saved:
                    g[k] = tuple(g_saved[k]) if k == "betas" else g_saved[k]
        st = self.store
        steps = []
        for i, p in enumerate(params):
            s_saved = sd["state"].get(i, sd["state"].get(str(i)))
            if s_saved is None:
                continue
            s = st.slot_of(p)
            st.param_view(self.exp_avg, s).copy_(s_saved["exp_avg"].to(self.exp_avg.device).view(p.shape))
            st.param_view(self.exp_avg_sq, s).copy_(s_saved["exp_avg_sq"].to(self.exp_avg.device).view(p.shape))
            steps.append(int(float(s_saved["step"])))
        if steps:
            self.step_count = max(steps)
            if self.loss_scale is not None:
                from .loss_scale import LS_STEP
                self.loss_scale.state[LS_STEP] = float(self.step_count)
