"""Dynamic loss scaling for ``--dtype=float16`` (nanoGPT ``train.py``:
``scaler = torch.cuda.amp.GradScaler(enabled=(dtype == 'float16'))``).

The same policy as torch's GradScaler: start at 2^16; after ``growth_interval`` consecutive
steps with finite gradients multiply the scale by ``growth_factor``; on a step whose
gradients hold an inf / NaN skip the optimizer step and multiply it by ``backoff_factor``.
The trainer scales the loss before backward and folds 1 / scale into the fused AdamW
kernel's gradient multiplier (and the clip norm), so unscaling costs no extra pass; the
inf check reads the global gradient norm the clip already computes (a host sync, as
GradScaler's ``step`` has).
"""

from __future__ import annotations

import math


class DynamicLossScale:
    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000):
        self.scale = float(init_scale)
        self.growth_factor = float(growth_factor)
        self.backoff_factor = float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self._good_steps = 0
        self.skipped = 0

    @staticmethod
    def finite(norm) -> bool:
        return math.isfinite(float(norm))

    def update(self, found_inf: bool) -> None:
        if found_inf:
            self.scale *= self.backoff_factor
            self._good_steps = 0
            self.skipped += 1
            return
        self._good_steps += 1
        if self._good_steps >= self.growth_interval:
            self.scale *= self.growth_factor
            self._good_steps = 0

    def state_dict(self) -> dict:
        return {"scale": self.scale, "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": self._good_steps}

    def load_state_dict(self, sd: dict) -> None:
        self.scale = float(sd["scale"])
        self._good_steps = int(sd.get("_growth_tracker", 0))
