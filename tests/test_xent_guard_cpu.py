"""The fused fp16 cross-entropy's fall-back guard (ops/functional.py XentF16Guard), on CPU
counters: it trips only past its flagged-row share and row minimum, once, and turns the
fused form off (profiles/r6_xent_f16_cliff.md)."""

import torch

from nanosandbox_amd.ops.functional import XentF16Guard


def test_guard_stays_below_threshold():
    g = XentF16Guard(max_frac=0.01, min_rows=1000)
    for _ in range(10):
        g.note(torch.tensor([5], dtype=torch.int32), 1000)  # 0.5 %
        assert g.poll() is False
    assert g.active and g.last == (50, 10000)


def test_guard_waits_for_min_rows_then_trips_once():
    g = XentF16Guard(max_frac=0.002, min_rows=10000)
    g.note(torch.tensor([100], dtype=torch.int32), 4000)  # 2.5 %, but too few rows seen
    assert g.poll() is False and g.active
    g.note(torch.tensor([100], dtype=torch.int32), 8000)
    assert g.poll() is True  # 200 of 12000 rows
    assert not g.active
    g.note(torch.tensor([100], dtype=torch.int32), 8000)
    assert g.poll() is False  # already off: no second trip


def test_guard_counts_accumulate_on_the_counter_device():
    g = XentF16Guard()
    nfix = torch.tensor([3], dtype=torch.int32)
    g.note(nfix, 7)
    g.note(nfix, 7)
    assert g.counts.dtype == torch.int64 and g.counts.tolist() == [6, 14]
