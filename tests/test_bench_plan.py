"""bench.py batch plan: the 491,520-token optimizer step is fixed for every N (strong scaling)."""
import importlib.util
import os

import pytest

_spec = importlib.util.spec_from_file_location(
    "nsa_bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
bench = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(bench)


@pytest.mark.parametrize("world,expect_micro", [(1, 120), (2, 120), (4, 120), (8, 60), (3, 80)])
def test_auto_plan_keeps_global_batch(world, expect_micro):
    micro, total_micro = bench.batch_plan(world)
    assert micro == expect_micro
    assert total_micro % world == 0
    assert micro * total_micro == 480  # sequences per optimizer step
    assert micro * total_micro * 1024 == 491_520


def test_nanogpt_schedule_reproducible():
    # --micro-batch 12 reproduces train_gpt2's 12 x 40 (5 x 8 on 8 ranks)
    assert bench.batch_plan(1, 12) == (12, 40)
    assert bench.batch_plan(8, 12) == (12, 40)


def test_bad_plans_rejected():
    with pytest.raises(AssertionError):
        bench.batch_plan(7)
    with pytest.raises(AssertionError):
        bench.batch_plan(1, 7)
