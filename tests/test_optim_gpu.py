"""Fused AdamW + the fp16 dynamic loss scale on the device (optim.hip), against the host
reference of the same policy (``FusedAdamW`` CPU path, ``DynamicLossScale.update``)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _store(device, seed=0):
    from nanosandbox_amd.models import GPT, GPTConfig
    from nanosandbox_amd.optim import FlatParamStore

    torch.manual_seed(seed)
    m = GPT(GPTConfig(n_layer=1, n_head=2, n_embd=64, block_size=32, vocab_size=128, bias=True))
    store = FlatParamStore(m, device, compute_dtype=torch.bfloat16 if device == "cuda" else None)
    opt = m.configure_optimizers(0.1, 1e-3, (0.9, 0.95), device, store=store)
    return store, opt


def _run(device, grads, clip, init_scale):
    from nanosandbox_amd.optim.loss_scale import DynamicLossScale

    store, opt = _store(device)
    ls = DynamicLossScale(init_scale=init_scale, growth_interval=2, device=device)
    opt.attach_loss_scale(ls)
    norms = []
    for g in grads:
        store.grad.copy_(g.to(device))
        if clip:
            norms.append(float(opt.clip_grad_norm_(clip).item()))
        opt.step()
        opt.zero_grad()
    return store.master.cpu(), ls.state.cpu(), norms


def test_loss_scale_kernels_match_host_policy(kernels):
    """Random scaled gradients, one step with an inf, one with a NaN: the device kernels
    (unscale, non-finite count, skip, backoff / growth, good-step bias correction) match the
    host reference step for step."""
    torch.manual_seed(3)
    store, _ = _store("cpu")
    n = store.numel
    scale = 2.0 ** 12
    grads = [torch.randn(n) * 1e-2 * scale for _ in range(5)]
    grads[1][7] = float("inf")
    grads[3][n // 2] = float("nan")
    for clip in (1.0, 0.0):
        m_gpu, st_gpu, nrm_gpu = _run("cuda", grads, clip, scale)
        m_cpu, st_cpu, nrm_cpu = _run("cpu", grads, clip, scale)
        assert torch.equal(st_gpu[:5], st_cpu[:5]), (st_gpu, st_cpu)  # scale, tracker, found, skipped, step
        assert st_gpu[3].item() == 2 and st_gpu[4].item() == 3
        assert torch.allclose(m_gpu, m_cpu, rtol=1e-5, atol=1e-6)
        if clip:
            assert nrm_gpu[1] == float("inf") and nrm_gpu[3] == float("inf")
            for a, b in zip(nrm_gpu, nrm_cpu):
                assert a == b or abs(a - b) <= 1e-4 * abs(b)


def test_large_finite_scaled_gradients_are_not_skipped(kernels):
    """the sum of squares of the SCALED gradient overflows fp32 for large finite
    values (1e19 squared); the norm is taken over the unscaled gradient, so the step runs."""
    from nanosandbox_amd.optim.loss_scale import DynamicLossScale

    store, opt = _store("cuda")
    ls = DynamicLossScale(init_scale=2.0 ** 16, device="cuda")
    opt.attach_loss_scale(ls)
    w0 = store.master.clone()
    store.grad.fill_(1e19)
    norm = opt.clip_grad_norm_(1.0)
    opt.step()
    assert torch.isfinite(norm).item() and norm.item() > 0
    assert not ls.found_inf and ls.skipped == 0 and ls.good_steps == 1
    assert not torch.equal(store.master, w0) and torch.isfinite(store.master).all()
    # one non-finite element: skipped, weights unchanged, scale halved
    w1 = store.master.clone()
    store.grad.fill_(1.0)
    store.grad[5] = float("-inf")
    opt.clip_grad_norm_(1.0)
    opt.step()
    assert ls.found_inf and ls.skipped == 1 and ls.scale == 2.0 ** 15 and ls.good_steps == 1
    assert torch.equal(store.master, w1)
