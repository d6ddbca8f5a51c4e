"""CPU checks of the GPU dispatch helpers: split-K sizing, weight-transpose cache
generations, and the side-stream protocol's CPU no-op behaviour."""

import torch

from nanosandbox_amd.ops import gemm, gemm_tune, streams


def _blocks(n_out, n_in, s):
    return (-(-n_out // gemm.TILE)) * (-(-n_in // gemm.TILE)) * s


def test_wgrad_splits_fill_rounds():
    cus = 256
    for n_out, n_in in [(768, 768), (2304, 768), (3072, 768), (768, 3072), (50304, 768)]:
        s_def = gemm.wgrad_splits(n_out, n_in, 122880, cus)
        assert _blocks(n_out, n_in, s_def) <= 2 * cus or s_def == 1
        s_bal = gemm.wgrad_splits_balanced(n_out, n_in, 122880, cus)
        blocks = _blocks(n_out, n_in, s_bal)
        rounds = -(-blocks // cus)
        assert rounds <= gemm.WGRAD_MAX_ROUNDS
        # at least as well filled as the default rule's last round
        eff_bal = blocks / (rounds * cus)
        b_def = _blocks(n_out, n_in, s_def)
        eff_def = b_def / (-(-b_def // cus) * cus)
        assert eff_bal >= eff_def - 1e-9


def test_lm_head_wgrad_gets_two_splits():
    # 197 x 3 = 591 output tiles: 2.3 rounds unsplit (77 % busy), 4.6 rounds with 2 splits (92 %)
    assert gemm.wgrad_splits_balanced(50304, 768, 122880) == 2


def test_weight_transpose_cache_generations():
    w = torch.randn(6, 4)
    t0 = gemm_tune._wt(w)
    assert torch.equal(t0, w.t())
    assert gemm_tune._wt(w) is t0
    w.add_(1.0)  # version bump
    t1 = gemm_tune._wt(w)
    assert t1 is not t0 and torch.equal(t1, w.t())
    w.data.mul_(3.0)  # no version bump: stale until announced
    assert gemm_tune._wt(w) is t1
    gemm_tune.weights_changed()
    assert torch.equal(gemm_tune._wt(w), w.t())


def test_streams_are_noops_on_cpu():
    x = torch.randn(3)
    assert not streams.active(x)
    with streams.fork(x, x):
        y = x * 2
    streams.join()
    assert torch.equal(y, x * 2)
