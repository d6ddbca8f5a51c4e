"""Learning-rate schedule (nanoGPT ``train.py::get_lr``).

Linear warmup for ``warmup_iters`` steps, ``it > lr_decay_iters`` -> ``min_lr``,
otherwise cosine decay down to ``min_lr``.
"""

from __future__ import annotations

import math


def get_lr(it: int, learning_rate: float, warmup_iters: int, lr_decay_iters: int, min_lr: float) -> float:
    # 1) linear warmup for warmup_iters steps
    if it < warmup_iters:
        return learning_rate * (it + 1) / (warmup_iters + 1)
    # 2) if it > lr_decay_iters, return min learning rate
    if it > lr_decay_iters:
        return min_lr
    # 3) in between, use cosine decay down to min learning rate
    decay_ratio = (it - warmup_iters) / (lr_decay_iters - warmup_iters)
    assert 0 <= decay_ratio <= 1
    coeff = 0.5 * (1.0 + math.cos(math.pi * decay_ratio))  # coeff ranges 0..1
    return min_lr + coeff * (learning_rate - min_lr)
