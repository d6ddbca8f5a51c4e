"""Our MFMA GEMMs vs fp32 torch matmul: the persistent NT kernel (forward, input grad,
GELU / GELU' epilogues, ragged shapes) and the split-K weight-gradient kernel."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (1024, 2304, 768), (264, 520, 192), (2048, 50304, 768),
                                   (256, 256, 3072), (1000, 1288, 640), (4096, 768, 4608)])
def test_nt_forward_and_gelu_epilogue(kernels, M, N, K):
    """Persistent NT kernels vs fp32 torch (gemm.fwd / fwd_gelu run the four-wave kernel):
    plain, GELU epilogue, ragged M/N (tail tiles shifted back inside the matrix), several
    tiles per workgroup; the eight-wave kernel (gemm_nt.hip) with either store policy gives
    bitwise the same output (same accumulation order)."""
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    y = gemm.fwd(x, w)
    assert rel(y, x.float() @ w.float().t()) < 1e-2
    u, g = gemm.fwd_gelu(x, w)
    assert torch.equal(u, y)
    assert rel(g, F.gelu(u.float())) < 1e-2
    for st in (1, 2):  # nontemporal / plain epilogue stores: identical results
        assert torch.equal(gemm.nt(x, w, var=st), y)


@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (1024, 3072, 768), (264, 512, 256), (2048, 50304, 768),
                                   (8192, 768, 3072), (8200, 768, 3072)])
def test_nt_input_grad_and_dgelu_epilogue(kernels, M, N, K):
    """dX = dY·W through the K-contiguous W^T, plain and with the GELU' epilogue; the
    8192-row shapes give every workgroup several output tiles (deferred epilogue stores,
    and with 8200 rows a shifted tail tile among them)."""
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(0)
    dy = torch.randn(M, N, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    dx = gemm.dgrad(dy, w)
    ref = dy.float() @ w.float()
    assert rel(dx, ref) < 1e-2
    u = torch.randn(M, K, device=DEV).to(BF)
    dxg = gemm.dgrad(dy, w, u=u)
    uf = u.float()
    gp = 0.5 * (1 + torch.erf(uf / 2 ** 0.5)) + uf * torch.exp(-0.5 * uf * uf) / (2 * torch.pi) ** 0.5
    assert rel(dxg, dx.float() * gp) < 1e-2


@pytest.mark.parametrize("T,N,K,splits", [(1024, 768, 768, None), (4096, 2304, 768, None), (512, 520, 200, 2),
                                          (2048, 768, 3072, 4), (1024, 50304, 768, 1),
                                          (1024, 768, 768, 3), (4096, 2304, 768, 28),  # uneven K splits
                                          (1024, 768, 768, 16)])  # one K-tile per split
@pytest.mark.parametrize("variant", [1, 7, 9, 10])
def test_wgrad_acc(kernels, T, N, K, splits, variant):
    from nanosandbox_amd.ops import gemm
    if K % 8:
        K = K - K % 8
    torch.manual_seed(0)
    dy = torch.randn(T, N, device=DEV).to(BF)
    x = torch.randn(T, K, device=DEV).to(BF)
    g = torch.randn(N, K, device=DEV)
    ref = g + dy.float().t() @ x.float()
    gemm.wgrad_acc(dy, x, g, splits=splits, variant=variant)
    assert rel(g, ref) < 5e-3
    # deterministic form: partials reduced in split order, bitwise repeatable
    g1 = torch.randn(N, K, device=DEV)
    g2 = g1.clone()
    gemm.wgrad_acc(dy, x, g1, splits=splits, variant=variant, deterministic=True)
    gemm.wgrad_acc(dy, x, g2, splits=splits, variant=variant, deterministic=True)
    assert torch.equal(g1, g2)


@pytest.mark.parametrize("variant", [1, 7, 9, 10])
def test_asymmetric_identity(kernels, variant):
    """A = I with an asymmetric B catches row/col swaps in the C write (guide §3)."""
    from nanosandbox_amd.ops import gemm
    n = 256
    eye = torch.eye(n, device=DEV).to(BF)
    b = torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n).remainder(251).to(BF)
    assert torch.equal(gemm.fwd(eye, b).float(), b.float().t())  # I @ b^T
    assert torch.equal(gemm.dgrad(eye, b).float(), b.float())     # I @ b
    g = torch.zeros(n, n, device=DEV)
    gemm.wgrad_acc(eye, b, g, variant=variant)                    # I^T @ b
    assert torch.equal(g, b.float())


def test_tuner_prefers_native_within_margin(kernels, monkeypatch):
    """gemm_tune.choose: a library candidate wins only when it is more than NATIVE_MARGIN
    faster than the best native one; deterministic mode picks without timing."""
    from nanosandbox_amd.ops import gemm_tune
    monkeypatch.setattr(gemm_tune, "_time_all", lambda c, **k: {"hipblaslt": 1.0, "nt": 1.01})
    monkeypatch.setattr(gemm_tune, "_table", {})
    monkeypatch.setattr(gemm_tune, "FORCE", "")
    cands = {"hipblaslt": lambda: None, "nt": lambda: None}
    assert gemm_tune.choose(("t", 1), cands) == "nt"
    monkeypatch.setattr(gemm_tune, "_time_all", lambda c, **k: {"hipblaslt": 1.0, "nt": 1.10})
    assert gemm_tune.choose(("t", 2), cands) == "hipblaslt"
    monkeypatch.setattr(gemm_tune, "DETERMINISTIC", True)
    monkeypatch.setattr(gemm_tune, "_time_all", lambda c, **k: (_ for _ in ()).throw(AssertionError("timed")))
    assert gemm_tune.choose(("t", 3), cands) == "nt"


def test_transposed_weight_dgrad_cache(kernels):
    """dX = dY·W through the cached K-contiguous W^T (gemm_tune._wt): equal to the plain
    product, rebuilt after an in-place update (version bump) and after a raw rewrite
    announced by weights_changed() (what the fused AdamW kernel does)."""
    from nanosandbox_amd.ops import gemm_tune

    torch.manual_seed(0)
    dy = torch.randn(512, 384, device="cuda").to(torch.bfloat16)
    w = torch.randn(384, 256, device="cuda").to(torch.bfloat16)

    def via_t():
        return dy @ gemm_tune._wt(w).t()

    assert torch.equal(via_t(), dy @ w)
    t0 = gemm_tune._wt(w)
    assert gemm_tune._wt(w) is t0  # cached
    w.mul_(2.0)  # torch in-place op: version bump invalidates
    assert torch.equal(via_t(), dy @ w)
    w.data.copy_(torch.randn_like(w))  # raw rewrite: no version bump ...
    stale = via_t()
    assert not torch.equal(stale, dy @ w)  # ... so the cache is stale until announced
    gemm_tune.weights_changed()
    assert torch.equal(via_t(), dy @ w)


@pytest.mark.parametrize("R,C", [(768, 3072), (50304, 768), (64, 128), (2304, 768)])
def test_transpose_bf16(kernels, R, C):
    """The weight-transpose kernel behind the cached K-contiguous dgrad weights."""
    from nanosandbox_amd.ops import gemm_tune

    w = torch.randn(R, C, device="cuda").to(torch.bfloat16)
    t = gemm_tune._transpose(w)
    assert t.shape == (C, R) and t.is_contiguous()
    assert torch.equal(t, w.t())
    t2 = gemm_tune._transpose(w * 2, out=t)  # rebuilt in place
    assert t2.data_ptr() == t.data_ptr() and torch.equal(t2, (w * 2).t())


@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (1024, 2304, 768), (264, 520, 192), (2048, 50304, 768),
                                   (256, 256, 64), (1000, 1288, 640), (8200, 768, 3072), (4096, 768, 4608)])
def test_nt4_matches_fp32_and_nt(kernels, M, N, K):
    """Four-wave persistent NT kernel (gemm_nt4.hip) vs fp32 torch, and bitwise against the
    eight-wave kernel (same accumulation order per output: one K-tile at a time, k-steps in
    order) for the plain, GELU and GELU' epilogues; ragged M / N exercise the shifted tail
    tiles and the drained (uncounted) epilogue, 8200 x 768 several tiles per workgroup."""
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    y4 = gemm.nt(x, w, w4=True)
    assert rel(y4, x.float() @ w.float().t()) < 1e-2
    u4, g4 = gemm.nt(x, w, epi=gemm.NT_EPI_GELU, w4=True)
    assert torch.equal(u4, y4)
    assert rel(g4, F.gelu(u4.float())) < 1e-2
    for st in (1, 2):
        assert torch.equal(gemm.nt(x, w, var=st, w4=True), y4)
    u = torch.randn(M, N, device=DEV).to(BF)
    d4 = gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=u, w4=True)
    uf = u.float()
    gp = 0.5 * (1 + torch.erf(uf / 2 ** 0.5)) + uf * torch.exp(-0.5 * uf * uf) / (2 * torch.pi) ** 0.5
    assert rel(d4, y4.float() * gp) < 1e-2


def test_nt4_asymmetric_identity(kernels):
    """A = I with an asymmetric B through the four-wave kernel: a row/column swap or a wrong
    column permutation of the staged B image shows up exactly (guide §3)."""
    from nanosandbox_amd.ops import gemm
    n = 512
    eye = torch.eye(n, device=DEV).to(BF)
    b = torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n).remainder(251).to(BF)
    assert torch.equal(gemm.nt(eye, b, w4=True).float(), b.float().t())
    assert torch.equal(gemm.nt(b, eye, w4=True).float(), b.float())
