"""CPU checks of the fixed GEMM dispatch rule (ops/gemm_dispatch.py): every training GEMM of
every shipped GPT configuration maps to one of our kernels (never the torch/vendor
fallback), the split-K counts are the ones the round-3 start-up race picked, the vocabulary
padding, and the weight-transpose cache generations."""

import glob
import os
import runpy

import pytest
import torch

from nanosandbox_amd.ops import gemm, gemm_dispatch, lm_head_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gemm_shapes(n_embd, vocab, tokens):
    """(op, M, N, K) of every GEMM of one training micro-step (GPT-2 block + tied lm_head)."""
    C, V = n_embd, lm_head_rows(vocab)
    out = []
    for n_out, n_in in [(3 * C, C), (C, C), (4 * C, C), (C, 4 * C)]:
        out += [("fwd", tokens, n_out, n_in), ("dgrad", tokens, n_in, n_out), ("wgrad", n_out, n_in, tokens)]
    out += [("fwd", tokens, V, C), ("dgrad", tokens, C, V), ("wgrad", V, C, tokens)]
    return out


def _configs():
    for path in sorted(glob.glob(os.path.join(ROOT, "config", "*.py"))):
        g = runpy.run_path(path)
        yield os.path.basename(path), g


@pytest.mark.parametrize("name", [os.path.basename(p) for p in sorted(glob.glob(os.path.join(ROOT, "config", "*.py")))])
def test_every_config_runs_on_native_gemms(name):
    """No GEMM of any shipped config reaches the torch fallback (hipBLASLt off the
    training hot path), bias / pretrained-vocab configs included."""
    from nanosandbox_amd.config import TRAIN_DEFAULTS

    cfg = dict(TRAIN_DEFAULTS)
    cfg.update({k: v for k, v in runpy.run_path(os.path.join(ROOT, "config", name)).items()
                if k in TRAIN_DEFAULTS})
    dims = {"gpt2": 768, "gpt2-medium": 1024, "gpt2-large": 1280, "gpt2-xl": 1600}
    n_embd = dims.get(cfg["init_from"], cfg["n_embd"])
    vocab = 50257 if cfg["init_from"].startswith("gpt2") else (65 if "char" in cfg["dataset"] else 50304)
    tokens = cfg["batch_size"] * cfg["block_size"]
    for op, M, N, K in _gemm_shapes(n_embd, vocab, tokens):
        k = gemm_dispatch.kernel_for(op, M, N, K)
        assert k != "torch", (name, op, M, N, K)


def test_gpt2_shapes_take_the_persistent_kernels():
    for op, M, N, K in _gemm_shapes(768, 50304, 122880):
        assert gemm_dispatch.kernel_for(op, M, N, K) == ("wgrad4" if op == "wgrad" else "nt4"), (op, M, N, K)
    # a tiny model (smoke config) takes the bounds-checked kernels
    assert gemm_dispatch.kernel_for("fwd", 256, 192, 64) == "small"
    assert gemm_dispatch.kernel_for("wgrad", 192, 64, 256) == "ring64"
    assert gemm_dispatch.kernel_for("fwd", 256, 192, 60) == "torch"  # K % 8 != 0: out of contract


def test_small_vocab_lds_scatter_rule():
    """The LDS-privatised scatter-add (segsum.h seg_lds_kernel) takes a table whose padded
    V x (C + C/8) fp32 copy fits its 128 KB LDS budget: the char config's 65 x 384 (and the
    reference's companion-notebook char model, 65 x 128), never a GPT-2 vocabulary."""
    from nanosandbox_amd.ops import functional as Fn

    fits = Fn._seg_lds_fits
    assert fits(65, 384) and fits(65, 128)
    assert not fits(50304, 768) and not fits(50257, 1600) and not fits(1000, 384)


def test_wgrad_split_rule_matches_round3_race():
    """The fixed split rule reproduces the start-up race's picks (profiles/r3_bench_glds.log,
    r3_bench_gpt2_medium.log) and fills its last round of CUs."""
    picks = {(2304, 768): 9, (768, 768): 28, (3072, 768): 7, (768, 3072): 7, (50304, 768): 3,
             (1024, 1024): 16, (1024, 4096): 4, (3072, 1024): 5, (4096, 1024): 4, (50304, 1024): 6}
    for (n_out, n_in), s in picks.items():
        assert gemm.wgrad_splits(n_out, n_in, 122880) == s, (n_out, n_in)
    # short work items (shakespeare_char: 16384 tokens): the atomic epilogue caps the count
    # (measured best 12-16 / 24-32 / 12-16, profiles/r5_wgrad_small.log)
    assert gemm.wgrad_splits(1152, 384, 16384) == 16
    assert gemm.wgrad_splits(384, 384, 16384) == 26
    assert gemm.wgrad_splits(1536, 384, 16384) == 15
    # GPT-2 1.5B (61440 tokens) keeps the round-fill picks
    assert gemm.wgrad_splits(1600, 6400, 61440) == 7 and gemm.wgrad_splits(50304, 1600, 61440) == 2
    # never more splits than 64-token K-tiles
    assert gemm.wgrad_splits(768, 768, 256) <= 4
    # GPT-2 1.5B (micro-batch 60 x 1024): 133 / 175 output tiles must not run as one
    # partial round (52 % / 68 % of the CUs): 7 splits fill 91 % / 96 % of their rounds
    for (n_out, n_in), s in {(4800, 1600): 7, (6400, 1600): 7, (1600, 6400): 7, (1600, 1600): 5,
                             (50304, 1600): 2}.items():
        assert gemm.wgrad_splits(n_out, n_in, 61440) == s, (n_out, n_in)


def test_lm_head_rows_padding():
    assert lm_head_rows(50304) == 50304
    assert lm_head_rows(50257) == 50304
    assert lm_head_rows(65) == 256
    assert lm_head_rows(512) == 512


def test_flat_store_pads_the_tied_vocab_rows():
    from nanosandbox_amd.models import GPT, GPTConfig
    from nanosandbox_amd.optim import FlatParamStore

    m = GPT(GPTConfig(n_layer=1, n_head=2, n_embd=64, block_size=32, vocab_size=65, bias=True))
    st = FlatParamStore(m, "cpu")
    w = m.lm_head.weight
    assert w.main_grad_padded.shape == (256, 64)
    assert w.main_grad_padded.data_ptr() == w.main_grad.data_ptr()
    assert torch.equal(st.master[st.slot_of(w).offset + 65 * 64: st.slot_of(w).offset + 256 * 64],
                       torch.zeros(191 * 64))


def test_weight_transpose_cache_generations():
    w = torch.randn(6, 4)
    t0 = gemm_dispatch._wt(w)
    assert torch.equal(t0, w.t())
    assert gemm_dispatch._wt(w) is t0
    w.add_(1.0)  # version bump
    t1 = gemm_dispatch._wt(w)
    assert t1 is not t0 and torch.equal(t1, w.t())
    w.data.mul_(3.0)  # no version bump: stale until announced
    assert gemm_dispatch._wt(w) is t1
    gemm_dispatch.weights_changed()
    assert torch.equal(gemm_dispatch._wt(w), w.t())


def test_cpu_fallbacks_match_torch():
    """Off the GPU the dispatch functions are plain fp32 torch (the kernels' reference)."""
    torch.manual_seed(0)
    x, w, b = torch.randn(5, 8), torch.randn(3, 8), torch.randn(3)
    assert torch.allclose(gemm_dispatch.fwd(x, w, b), x @ w.t() + b)
    gp, g = gemm_dispatch.fwd_gelu(x, w)
    u = x @ w.t()
    assert torch.allclose(g, torch.nn.functional.gelu(u))
    assert gp.dtype == torch.float16  # gelu'(u), the backward's only use of u
    uu = u.clone().requires_grad_(True)
    torch.nn.functional.gelu(uu).backward(torch.ones_like(uu))
    assert torch.allclose(gp.float(), uu.grad, rtol=2 ** -10, atol=1e-6)
    w2, dy2 = torch.randn(4, 3), torch.randn(5, 4)  # the next layer (c_proj: 3 -> 4) and its output grad
    assert torch.allclose(gemm_dispatch.dgrad_dgelu(dy2, w2, gp), (dy2 @ w2) * gp.float())
    gacc = torch.zeros(3, 8)
    gemm_dispatch.wgrad_acc(torch.randn(5, 3), x, gacc)
    gb = torch.zeros(3)
    dy = torch.randn(5, 3)
    gemm_dispatch.bias_grad_acc(dy, gb)
    assert torch.allclose(gb, dy.sum(0))
