"""Finite-difference gradient checks of every autograd op.

The kernel tests (test_kernels_gpu.py) compare each backward against torch's fp32
autograd of the same op.  These check something different: that an op's backward is
the derivative of ITS OWN forward.

* CPU: ``torch.autograd.gradcheck`` on the hand-written backward formulas of the CPU
  paths (fp64 inputs; the paths compute in fp32, so eps/atol are fp32-sized).
* GPU: a directional finite difference through the HIP kernels in bf16.  Both the
  forward and the backward run on the kernels.  The probe direction is the analytic
  gradient itself, the largest-signal direction.  The perturbed inputs are rounded to
  the input dtype, so the prediction uses the perturbation that was actually applied,
  ``g . (x+ - x-)``, rather than ``2h|g|``.  bf16 rounding of the outputs bounds the
  agreement to a few percent.
"""

import pytest
import torch

from nanosandbox_amd.ops import functional as Fn

F64 = torch.float64


@pytest.fixture
def fixed_seed(monkeypatch):
    """Dropout draws a fresh salt per forward; gradcheck re-runs the forward many times,
    so pin the salt (the mask is a function of it)."""
    monkeypatch.setattr(Fn, "new_seed", lambda: 12345)


def _gc(fn, *inputs):
    assert torch.autograd.gradcheck(fn, inputs, eps=1e-3, atol=2e-3, rtol=2e-3, nondet_tol=0.0)


def _leaf(*shape, scale=1.0, shift=0.0):
    return (torch.randn(*shape, dtype=F64) * scale + shift).requires_grad_(True)


# ------------------------------------------------------------------------- CPU
def test_gradcheck_gelu_cpu():
    torch.manual_seed(0)
    _gc(Fn.gelu, _leaf(4, 6, scale=2.0))


@pytest.mark.parametrize("bias", [False, True])
def test_gradcheck_layer_norm_cpu(bias):
    torch.manual_seed(0)
    x, w = _leaf(5, 16, scale=2.0, shift=0.5), _leaf(16, scale=0.5, shift=1.0)
    b = _leaf(16, scale=0.1) if bias else None
    _gc(lambda x, w, *b: Fn.layer_norm(x, w, b[0] if b else None), x, w, *([b] if bias else []))


def test_gradcheck_add_layer_norm_cpu():
    torch.manual_seed(0)
    x, y, w, b = _leaf(3, 4, 16), _leaf(3, 4, 16), _leaf(16, shift=1.0), _leaf(16, scale=0.1)
    _gc(lambda x, y, w, b: Fn.add_layer_norm(x, y, w, b), x, y, w, b)


def test_gradcheck_layer_norm_pass_cpu():
    torch.manual_seed(0)
    x, w = _leaf(6, 8), _leaf(8, shift=1.0)
    _gc(lambda x, w: Fn.layer_norm_pass(x, w, None), x, w)


@pytest.mark.parametrize("bias,residual", [(False, False), (True, False), (True, True)])
def test_gradcheck_linear_cpu(bias, residual):
    torch.manual_seed(0)
    x, w = _leaf(2, 3, 8), _leaf(5, 8, scale=0.3)
    extra = [_leaf(5, scale=0.1) if bias else None, _leaf(2, 3, 5) if residual else None]
    args = [t for t in extra if t is not None]

    def f(x, w, *rest):
        it = iter(rest)
        b = next(it) if bias else None
        r = next(it) if residual else None
        return Fn.linear(x, w, b, r)

    _gc(f, x, w, *args)


def test_gradcheck_mlp_cpu():
    torch.manual_seed(0)
    x, wf, wp = _leaf(2, 3, 8), _leaf(32, 8, scale=0.3), _leaf(8, 32, scale=0.3)
    _gc(lambda x, wf, wp: Fn.mlp(x, wf, None, wp, None), x, wf, wp)


@pytest.mark.parametrize("p", [0.0, 0.25])
def test_gradcheck_embedding_cpu(fixed_seed, p):
    torch.manual_seed(0)
    idx = torch.tensor([[1, 3, 3, 0], [2, 2, 5, 1]])
    wte, wpe = _leaf(6, 8), _leaf(5, 8)
    _gc(lambda wte, wpe: Fn.embedding(idx, wte, wpe, p, True, dtype=F64), wte, wpe)


def test_gradcheck_dropout_cpu(fixed_seed):
    torch.manual_seed(0)
    _gc(lambda x: Fn.dropout(x, 0.3, True), _leaf(64))


@pytest.mark.parametrize("p", [0.0, 0.2])
def test_gradcheck_attention_cpu(fixed_seed, p):
    torch.manual_seed(0)
    B, T, H, D = 1, 5, 2, 4
    _gc(lambda qkv: Fn.attention(qkv, H, p, True), _leaf(B, T, 3 * H * D))


def test_gradcheck_lm_head_loss_cpu():
    torch.manual_seed(0)
    x, w = _leaf(2, 3, 8), _leaf(11, 8, scale=0.5)
    t = torch.tensor([[1, -1, 10], [0, 4, 4]])
    _gc(lambda x, w: Fn.lm_head_loss(x, w, t), x, w)


# ------------------------------------------------------------------------- GPU
DEV = "cuda"
BF = torch.bfloat16


def _fd_check(f, leaves, rel=0.1, rtol=3e-2):
    """Directional finite difference of scalar ``f(*leaves)`` along each leaf's gradient.

    ``rel``: perturbation norm relative to the leaf's norm (one value, or one per leaf).  A
    leaf the output depends on linearly (a bias) takes a large one: there the difference is
    exact up to the outputs' bf16 rounding, which a small perturbation would drown in."""
    loss = f(*leaves)
    grads = torch.autograd.grad(loss, leaves)
    rels = rel if isinstance(rel, (list, tuple)) else [rel] * len(leaves)
    for i, (x, g, rel) in enumerate(zip(leaves, grads, rels)):
        g64 = g.double()
        v = g64 / g64.norm()
        h = rel * x.detach().double().norm()
        xp = (x.detach().double() + h * v).to(x.dtype)
        xm = (x.detach().double() - h * v).to(x.dtype)
        with torch.no_grad():
            args_p = [xp if j == i else t.detach() for j, t in enumerate(leaves)]
            args_m = [xm if j == i else t.detach() for j, t in enumerate(leaves)]
            measured = f(*args_p).double() - f(*args_m).double()
        predicted = (g64 * (xp.double() - xm.double())).sum()
        err = (measured - predicted).abs().item() / predicted.abs().item()
        assert err < rtol, f"leaf {i}: finite difference {measured.item():.6g} vs g.dx {predicted.item():.6g}"


def _proj(*outs):
    """Scalar probe of (possibly several) outputs: sum of out * R with fixed random R."""
    gen = torch.Generator(device=DEV).manual_seed(99)
    total = 0.0
    for o in outs:
        r = torch.randn(o.shape, device=DEV, generator=gen, dtype=torch.float32)
        total = total + (o.float() * r).double().sum()
    return total


@pytest.mark.gpu
def test_fd_gelu_gpu(kernels):
    torch.manual_seed(0)
    x = (torch.randn(64, 256, device=DEV) * 2).to(BF).requires_grad_(True)
    _fd_check(lambda x: _proj(Fn.gelu(x)), [x], rel=0.02)


@pytest.mark.gpu
@pytest.mark.parametrize("x32", [False, True])
def test_fd_layer_norm_gpu(kernels, x32):
    torch.manual_seed(0)
    x = (torch.randn(256, 768, device=DEV) * 2 + 0.5).to(torch.float32 if x32 else BF).requires_grad_(True)
    w = (torch.randn(768, device=DEV) * 0.5 + 1).to(BF).requires_grad_(True)
    b = (torch.randn(768, device=DEV) * 0.1).to(BF).requires_grad_(True)
    _fd_check(lambda x, w, b: _proj(Fn.layer_norm(x, w, b, out_dtype=BF)), [x, w, b], rel=[0.02, 0.05, 0.5])


@pytest.mark.gpu
def test_fd_add_layer_norm_gpu(kernels):
    """The fp32 residual stream: s = x + y (fp32), h = LN(s) (bf16); both outputs probed."""
    torch.manual_seed(0)
    x = torch.randn(256, 768, device=DEV).requires_grad_(True)
    y = torch.randn(256, 768, device=DEV).to(BF).requires_grad_(True)
    w = (torch.randn(768, device=DEV) * 0.5 + 1).to(BF).requires_grad_(True)
    _fd_check(lambda x, y, w: _proj(*Fn.add_layer_norm(x, y, w, None)), [x, y, w], rel=0.02)


@pytest.mark.gpu
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fd_flash_attention_gpu(kernels, fixed_seed, D, p):
    torch.manual_seed(0)
    B, T, H = 2, 192, 2
    qkv = torch.randn(B, T, 3 * H * D, device=DEV).to(BF).requires_grad_(True)
    _fd_check(lambda qkv: _proj(Fn.attention(qkv, H, p, True)), [qkv], rel=0.02)


@pytest.mark.gpu
def test_fd_mlp_gpu(kernels):
    torch.manual_seed(0)
    M, C = 512, 256
    x = torch.randn(M, C, device=DEV).to(BF).requires_grad_(True)
    wf = (torch.randn(4 * C, C, device=DEV) * 0.05).to(BF).requires_grad_(True)
    wp = (torch.randn(C, 4 * C, device=DEV) * 0.05).to(BF).requires_grad_(True)
    _fd_check(lambda x, wf, wp: _proj(Fn.mlp(x, wf, None, wp, None)), [x, wf, wp], rel=0.02)


@pytest.mark.gpu
def test_fd_linear_gpu(kernels):
    torch.manual_seed(0)
    x = torch.randn(384, 256, device=DEV).to(BF).requires_grad_(True)
    w = (torch.randn(768, 256, device=DEV) * 0.05).to(BF).requires_grad_(True)
    _fd_check(lambda x, w: _proj(Fn.linear(x, w)), [x, w], rel=0.02)


@pytest.mark.gpu
def test_fd_lm_head_loss_gpu(kernels):
    torch.manual_seed(0)
    N, V, C = 256, 1024, 128
    x = torch.randn(N, C, device=DEV).to(BF).requires_grad_(True)
    w = (torch.randn(V, C, device=DEV) * 0.1).to(BF).requires_grad_(True)
    t = torch.randint(0, V, (N,), device=DEV)
    t[::7] = -1
    _fd_check(lambda x, w: Fn.lm_head_loss(x, w, t).double(), [x, w], rel=0.02)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fd_embedding_gpu(kernels, fixed_seed, p):
    torch.manual_seed(0)
    B, T, V, C = 4, 64, 300, 256
    idx = torch.randint(0, V, (B, T), device=DEV)
    wte = (torch.randn(V, C, device=DEV) * 0.5).to(BF).requires_grad_(True)
    wpe = (torch.randn(T, C, device=DEV) * 0.5).to(BF).requires_grad_(True)
    _fd_check(lambda wte, wpe: _proj(Fn.embedding(idx, wte, wpe, p, True, dtype=torch.float32)), [wte, wpe],
              rel=0.02)
