"""Training observability: nanoGPT stdout lines + JSONL + TensorBoard scalars.

The stdout format is the contract read through ``kubectl logs`` (reference
README.md:59,69-71)::

    step {it}: train loss {:.4f}, val loss {:.4f}
    iter {it}: loss {:.4f}, time {dt_ms:.2f}ms, mfu {mfu:.2f}%

On top of that every logged iteration is appended to ``<out_dir>/metrics.jsonl``
(iter, loss, lr, dt_ms, tokens/s, mfu, grad_norm) and, if requested, to a
tfevents file under ``tensorboard_dir``.
"""

from __future__ import annotations

import json
import os
import time

from .tfevents import EventWriter


class MetricsLogger:
    def __init__(self, out_dir: str, jsonl: bool = True, tensorboard_dir: str = "", run_name: str = "run",
                 enabled: bool = True):
        self.enabled = enabled
        self._jsonl = None
        self._tb = None
        if not enabled:
            return
        if jsonl:
            os.makedirs(out_dir, exist_ok=True)
            self._jsonl = open(os.path.join(out_dir, "metrics.jsonl"), "a")
        if tensorboard_dir:
            self._tb = EventWriter(os.path.join(tensorboard_dir, run_name))

    def log(self, kind: str, step: int, **values):
        if not self.enabled:
            return
        if self._jsonl is not None:
            rec = {"kind": kind, "iter": step, "time": time.time()}
            rec.update({k: (float(v) if isinstance(v, (int, float)) else v) for k, v in values.items()})
            self._jsonl.write(json.dumps(rec) + "\n")
            self._jsonl.flush()
        if self._tb is not None:
            for k, v in values.items():
                if isinstance(v, (int, float)):
                    self._tb.add_scalar(f"{kind}/{k}", float(v), step)
            self._tb.flush()

    def close(self):
        if self._jsonl is not None:
            self._jsonl.close()
        if self._tb is not None:
            self._tb.close()
