"""Training-curve parity on the GPU: the production bf16 stack against an independent
fp32 PyTorch GPT-2 (HuggingFace GPT2LMHeadModel) from identical weights and batches
(nanosandbox_amd/utils/parity.py; the GPT-2 124M-shape run is scripts/loss_parity.py,
its log in profiles/)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_loss_curve_tracks_fp32_reference(kernels):
    pytest.importorskip("transformers")
    import importlib.util
    import os

    from nanosandbox_amd.models import GPTConfig
    from nanosandbox_amd.utils.parity import run_parity

    spec = importlib.util.spec_from_file_location(
        "loss_parity", os.path.join(os.path.dirname(__file__), "..", "scripts", "loss_parity.py"))
    lp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lp)
    cfg = GPTConfig(block_size=256, vocab_size=512, n_layer=4, n_head=4, n_embd=256, dropout=0.0, bias=False)
    batches = lp.char_batches(80, 8, 256)
    recs = run_parity(cfg, batches, lr=1e-3, min_lr=1e-4, warmup=5)
    assert abs(recs[0]["loss"] - recs[0]["loss_ref"]) < 0.01 * recs[0]["loss_ref"]  # same weights, same batch
    rel = [abs(r["loss"] - r["loss_ref"]) / r["loss_ref"] for r in recs]
    assert max(rel) < 0.05, rel
    assert sum(rel) / len(rel) < 0.02, rel
    assert recs[-1]["loss_ref"] < 0.7 * recs[0]["loss_ref"]  # it learned
    assert recs[-1]["loss"] < 0.7 * recs[0]["loss"]
