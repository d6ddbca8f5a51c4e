"""Dynamic loss scaling for ``--dtype=float16`` (nanoGPT ``train.py``:
``scaler = torch.cuda.amp.GradScaler(enabled=(dtype == 'float16'))``).

The same policy as torch's GradScaler: start at 2^16; after ``growth_interval`` consecutive
steps with finite gradients multiply the scale by ``growth_factor``; on a step whose
gradients hold an inf / NaN skip the optimizer step and multiply it by ``backoff_factor``.

The state lives in one small fp32 tensor (slots ``LS_*``, mirrored in
``csrc/kernels/optim.hip``).  On the GPU the whole policy runs inside the fused optimizer's
three kernels (``FusedAdamW.attach_loss_scale``): the trainer multiplies the loss by the
device scale, the grad-norm pass squares the *unscaled* gradient (finite scaled gradients
cannot overflow the sum) and counts non-finite elements separately (torch's
per-element check), the clip kernel updates the scale, and the AdamW kernel skips a step
whose gradients overflowed.  Nothing is read back to the host, so an fp16 step has no
sync (GradScaler's ``step`` has one).  ``update()`` is the same policy on the host, used
off the GPU and as the reference the kernel is tested against.
"""

from __future__ import annotations

import math

import torch

LS_SCALE, LS_TRACKER, LS_FOUND, LS_SKIPPED, LS_STEP = range(5)
LS_SLOTS = 8


class DynamicLossScale:
    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000, device="cpu"):
        self.growth_factor = float(growth_factor)
        self.backoff_factor = float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self.state = torch.zeros(LS_SLOTS, dtype=torch.float32, device=device)
        self.state[LS_SCALE] = float(init_scale)

    # ------------------------------------------------------------ device view
    @property
    def scale_t(self) -> torch.Tensor:
        """The current scale as a 1-element device tensor (multiply the loss by it: no sync)."""
        return self.state[LS_SCALE:LS_SCALE + 1]

    @property
    def scale(self) -> float:
        return float(self.state[LS_SCALE].item())

    @scale.setter
    def scale(self, v: float) -> None:
        self.state[LS_SCALE] = float(v)

    @property
    def skipped(self) -> int:
        return int(self.state[LS_SKIPPED].item())

    @property
    def good_steps(self) -> int:
        """Optimizer steps taken (skipped ones excluded): AdamW's bias-correction step."""
        return int(self.state[LS_STEP].item())

    @property
    def found_inf(self) -> bool:
        return bool(self.state[LS_FOUND].item())

    # ------------------------------------------------------------ host policy
    @staticmethod
    def finite(norm) -> bool:
        return math.isfinite(float(norm))

    def update(self, found_inf: bool) -> None:
        s = self.state
        s[LS_FOUND] = 1.0 if found_inf else 0.0
        if found_inf:
            s[LS_SCALE] *= self.backoff_factor
            s[LS_TRACKER] = 0.0
            s[LS_SKIPPED] += 1.0
            return
        s[LS_STEP] += 1.0
        s[LS_TRACKER] += 1.0
        if s[LS_TRACKER].item() >= self.growth_interval:
            s[LS_SCALE] *= self.growth_factor
            s[LS_TRACKER] = 0.0

    def state_dict(self) -> dict:
        return {"scale": self.scale, "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": int(self.state[LS_TRACKER].item())}

    def load_state_dict(self, sd: dict) -> None:
        self.state[LS_SCALE] = float(sd["scale"])
        self.state[LS_TRACKER] = float(sd.get("_growth_tracker", 0))
