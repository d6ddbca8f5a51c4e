"""Our MFMA GEMMs vs fp32 torch matmul, checked element by element.

Every output is written into a NaN-prefilled buffer (a tile that skips rows or columns
leaves NaN behind) and compared per element against the fp32 product of the same
bf16-exact operands with the bound |C - C_ref| <= 2^-8 |C_ref| + 2^-16 (|A| |B|^T)
(one bf16 rounding of the output plus fp32 accumulation-order noise), so a tail tile that
drops or misplaces even one row fails.  Exact permutation / identity products at ragged
shapes pin the tile and epilogue indexing bit for bit (guide §3: asymmetric operands)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16
NAN = float("nan")


def nanbuf(*shape, dtype=BF):
    return torch.full(shape, NAN, device=DEV, dtype=dtype)


def check(c, ref, absab, rel=2 ** -8, name=""):
    """Per-element bound; no NaN / inf anywhere."""
    c = c.float()
    assert torch.isfinite(c).all(), f"{name}: {(~torch.isfinite(c)).sum().item()} non-finite outputs"
    err = (c - ref).abs()
    bound = rel * ref.abs() + 2 ** -16 * absab + 1e-30
    bad = err > bound
    assert not bad.any(), (f"{name}: {bad.sum().item()} elements out of bound, worst at "
                           f"{tuple(torch.nonzero(bad)[0].tolist())}: got {c[bad][0].item()} want {ref[bad][0].item()}")


def gelu_grad(uf):
    return 0.5 * (1 + torch.erf(uf / 2 ** 0.5)) + uf * torch.exp(-0.5 * uf * uf) / (2 * torch.pi) ** 0.5


def check_gelu_pair(gp, g, u, name):
    """The GELU epilogue's outputs for the bf16 pre-activation u: gelu'(u) in fp16 (one fp16
    rounding, 2^-11, plus the erf approximation) and gelu(u) in bf16."""
    assert gp.dtype == torch.float16 and g.dtype == BF
    uf = u.float()
    check(gp, gelu_grad(uf), torch.ones_like(uf), rel=2 ** -10, name=name + " gelu'")
    check(g, F.gelu(uf), uf.abs() + 1, rel=2 ** -7, name=name + " gelu")


NT_SHAPES = [(512, 768, 768), (1024, 2304, 768), (264, 520, 192), (2048, 50304, 768), (256, 256, 64),
             (1000, 1288, 640), (8200, 768, 3072), (257, 264, 64), (4096, 768, 4608)]


@pytest.mark.parametrize("M,N,K", NT_SHAPES)
def test_nt4_elementwise(kernels, M, N, K):
    """Four-wave persistent kernel: plain, bias, GELU (u and gelu(u)), GELU' epilogues;
    ragged M / N exercise the shifted tail tiles, 8200 x 768 several tiles per workgroup."""
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(0)
    x = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = torch.randn(N, device=DEV).to(BF)
    ref = x.float() @ w.float().t()
    absab = x.float().abs() @ w.float().abs().t()
    y = gemm.nt(x, w, out=nanbuf(M, N))
    check(y, ref, absab, name="plain")
    yb = gemm.nt(x, w, bias=b, out=nanbuf(M, N))
    check(yb, ref + b.float(), absab + b.float().abs(), name="bias")
    gp, g = gemm.nt(x, w, epi=gemm.NT_EPI_GELU, bias=b, out=nanbuf(M, N, dtype=torch.float16),
                    out2=nanbuf(M, N))
    check_gelu_pair(gp, g, yb, "nt4")  # u = yb, the bias epilogue's bf16 output
    # the lookup-table path is torch's exact-erf GELU rounded to bf16, bit for bit (rows of a
    # wave holding a u outside the table take the arithmetic path: rare at these values)
    exact = (g == F.gelu(yb.float()).to(BF)).float().mean().item()
    assert exact > 0.999, f"gelu(u) bit-exact on only {exact:.5f} of the elements"
    for st in (1, 2):  # nontemporal / plain epilogue stores: identical results
        assert torch.equal(gemm.nt(x, w, var=st, out=nanbuf(M, N)), y)
    # the overlapped epilogue forced on / off (each tile's stores inside the next tile's first
    # K-tile; tail tiles store every row), also with many tiles per workgroup: identical results
    for ov, grid in ((1, None), (2, None), (1, 7), (1, 1)):
        assert torch.equal(gemm.nt(x, w, ovl=ov, grid=grid, out=nanbuf(M, N)), y), (ov, grid)
    uu = gelu_grad(torch.randn(M, N, device=DEV) * 2).half()
    d = gemm.nt(x, w, epi=gemm.NT_EPI_DGELU, u=uu, out=nanbuf(M, N))
    assert torch.equal(d, (y.float() * uu.float()).to(BF))  # bf16(bf16(acc) * gelu'(u)), bitwise


@pytest.mark.parametrize("M,N,K", [(1000, 1288, 640), (8200, 768, 3072), (257, 264, 64), (2048, 50304, 768)])
def test_nt4_exact_permutation(kernels, M, N, K):
    """A = one-hot rows (row i selects column i % K): C[i, j] = B[j, i % K] exactly, so any
    misplaced row / column of a ragged tail tile shows up bit for bit."""
    from nanosandbox_amd.ops import gemm
    a = torch.zeros(M, K, device=DEV, dtype=BF)
    idx = torch.arange(M, device=DEV) % K
    a[torch.arange(M, device=DEV), idx] = 1
    b = torch.arange(N * K, device=DEV, dtype=torch.float32).view(N, K).remainder(251).sub(125).to(BF)
    c = gemm.nt(a, b, out=nanbuf(M, N))
    assert torch.equal(c.float(), b.float()[:, idx].t())
    assert torch.equal(gemm.nt(a, b, ovl=1, out=nanbuf(M, N)), c)  # the overlapped epilogue


@pytest.mark.parametrize("M,N,K", [(64, 192, 64), (100, 72, 40), (2048, 64, 256), (17, 300, 128), (300, 17, 88)])
def test_small_kernel(kernels, M, N, K):
    """The bounds-checked kernel for shapes below one NT tile: every epilogue, any M / N."""
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(1)
    x = torch.randn(M, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.1).to(BF)
    b = torch.randn(N, device=DEV).to(BF)
    ref = x.float() @ w.float().t()
    absab = x.float().abs() @ w.float().abs().t()
    check(gemm.small(x, w, out=nanbuf(M, N)), ref, absab, name="small")
    yb = gemm.small(x, w, bias=b, out=nanbuf(M, N))
    check(yb, ref + b.float(), absab + b.float().abs(), name="small bias")
    gp, g = gemm.small(x, w, epi=gemm.NT_EPI_GELU, bias=b, out=nanbuf(M, N, dtype=torch.float16), out2=nanbuf(M, N))
    check_gelu_pair(gp, g, yb, "small")
    uu = gelu_grad(torch.randn(M, N, device=DEV) * 2).half()
    d = gemm.small(x, w, epi=gemm.NT_EPI_DGELU, u=uu, out=nanbuf(M, N))
    y = gemm.small(x, w, out=nanbuf(M, N))
    assert torch.equal(d, (y.float() * uu.float()).to(BF))


@pytest.mark.parametrize("T,N,K,splits", [(1024, 768, 768, None), (4096, 2304, 768, None), (512, 520, 200, 2),
                                          (2048, 768, 3072, 4), (1024, 50304, 768, 1), (1088, 1032, 264, 3),
                                          (1024, 768, 768, 3), (4096, 2304, 768, 28),  # uneven K splits
                                          (1024, 768, 768, 16), (512, 192, 64, 2)])  # one K-tile per split; ring64
def test_wgrad_acc(kernels, T, N, K, splits):
    from nanosandbox_amd.ops import gemm
    K = K - K % 8
    torch.manual_seed(0)
    dy = torch.randn(T, N, device=DEV).to(BF)
    x = torch.randn(T, K, device=DEV).to(BF)
    g = torch.randn(N, K, device=DEV)
    ref = g + dy.float().t() @ x.float()
    absab = g.abs() + dy.float().abs().t() @ x.float().abs()
    gemm.wgrad_acc(dy, x, g, splits=splits)
    check(g, ref, absab, rel=2 ** -20, name="wgrad")
    # deterministic form: partials reduced in split order, bitwise repeatable
    g1 = torch.randn(N, K, device=DEV)
    g2 = g1.clone()
    gemm.wgrad_acc(dy, x, g1, splits=splits, deterministic=True)
    gemm.wgrad_acc(dy, x, g2, splits=splits, deterministic=True)
    assert torch.equal(g1, g2)


@pytest.mark.parametrize("T,N,K", [(1088, 1032, 264), (1024, 768, 768), (512, 192, 64)])
def test_wgrad_exact_permutation(kernels, T, N, K):
    """dY[t, n] = 1 iff n == t % N: dW[n] = sum of the x rows t = n, n + N, ... (at most two
    bf16 values: exact in fp32) -- a misplaced output row / column of a ragged tail tile
    fails bit for bit."""
    from nanosandbox_amd.ops import gemm
    dy = torch.zeros(T, N, device=DEV, dtype=BF)
    t = torch.arange(T, device=DEV)
    dy[t, t % N] = 1
    x = torch.arange(T * K, device=DEV, dtype=torch.float32).view(T, K).remainder(97).sub(48).to(BF)
    ref = torch.zeros(N, K, device=DEV)
    ref.index_add_(0, t % N, x.float())
    for det in (False, True):
        g = torch.zeros(N, K, device=DEV)
        gemm.wgrad_acc(dy, x, g, deterministic=det)
        assert torch.equal(g, ref)


def test_asymmetric_identity(kernels):
    """A = I with an asymmetric B catches row/col swaps in the C write (guide §3)."""
    from nanosandbox_amd.ops import gemm, gemm_dispatch
    n = 512
    eye = torch.eye(n, device=DEV).to(BF)
    b = torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n).remainder(251).to(BF)
    assert torch.equal(gemm.nt(eye, b).float(), b.float().t())  # I @ b^T
    assert torch.equal(gemm.nt(b, eye).float(), b.float())
    assert torch.equal(gemm_dispatch.dgrad(eye, b).float(), b.float())  # I @ b
    g = torch.zeros(n, n, device=DEV)
    gemm.wgrad_acc(eye, b, g)  # I^T @ b
    assert torch.equal(g, b.float())


def test_bias_grad(kernels):
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(0)
    for T, N in [(122880 // 16, 768), (300, 72), (64, 2304)]:
        dy = torch.randn(T, N, device=DEV).to(BF)
        gb = torch.randn(N, device=DEV)
        ref = gb + dy.float().sum(0)
        gemm.bias_grad_acc(dy, gb)
        assert torch.allclose(gb, ref, rtol=1e-5, atol=1e-4 * T ** 0.5)
        g1 = torch.zeros(N, device=DEV)
        g2 = torch.zeros(N, device=DEV)
        gemm.bias_grad_acc(dy, g1, deterministic=True)
        gemm.bias_grad_acc(dy, g2, deterministic=True)
        assert torch.equal(g1, g2)


@pytest.mark.parametrize("T,N_out,K_in,splits", [(4096, 768, 768, 4), (2048, 1032, 520, 3), (1024, 3072, 768, 1),
                                                 (2048, 264, 256, 5)])
def test_wgrad_fused_bias_grad(kernels, T, N_out, K_in, splits):
    """The weight-grad kernel's fused bias gradient (column sums of dY from its own A
    fragments, the first column-block tiles only, one atomic per column and split) against
    fp32 sums: ragged N_out (1032: the last row tile shifted back), several splits, and a
    bias view at an odd offset of a flat buffer (no alignment assumed)."""
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(0)
    dy = torch.randn(T, N_out, device=DEV).to(BF)
    x = torch.randn(T, K_in, device=DEV).to(BF)
    g = torch.zeros(N_out, K_in, device=DEV)
    flat = torch.full((N_out + 3,), float("nan"), device=DEV)
    gb = flat[1:1 + N_out]
    gb.zero_()
    gb += 0.5
    gemm.wgrad_acc(dy, x, g, splits=splits, gb32=gb)
    ref_b = dy.float().sum(0) + 0.5
    assert torch.isnan(flat[0]) and torch.isnan(flat[-2:]).all()  # nothing written outside the view
    assert (gb - ref_b).abs().max().item() <= 1e-3 * T ** 0.5, (gb - ref_b).abs().max().item()
    ref_w = dy.float().t() @ x.float()
    assert ((g - ref_w).norm() / ref_w.norm()).item() < 1e-5


@pytest.mark.parametrize("T,N_out,K_in", [(2048, 1024, 4096), (1024, 3072, 768)])
def test_wgrad_bias_deterministic_one_split(kernels, T, N_out, K_in):
    """with one K split the fused bias-grad kernel still adds each bias column
    from several column blocks (fp32 atomics in arrival order), so deterministic mode must
    not use it: weight AND bias gradients bitwise equal across two runs at splits = 1."""
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(1)
    dy = torch.randn(T, N_out, device=DEV).to(BF)
    x = torch.randn(T, K_in, device=DEV).to(BF)
    outs = []
    for _ in range(2):
        g = torch.full((N_out, K_in), 0.25, device=DEV)
        gb = torch.full((N_out,), 0.25, device=DEV)
        gemm.wgrad_acc(dy, x, g, splits=1, deterministic=True, gb32=gb)
        outs.append((g, gb))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref_b = dy.float().sum(0) + 0.25
    assert (outs[0][1] - ref_b).abs().max().item() <= 1e-3 * T ** 0.5


def test_dispatch_records_native_kernels(kernels):
    """The fixed rule's picks as the bench JSON reports them (no library kernel)."""
    from nanosandbox_amd.ops import gemm_dispatch
    x = torch.randn(512, 768, device=DEV).to(BF)
    w = torch.randn(2304, 768, device=DEV).to(BF)
    gemm_dispatch.fwd(x, w)
    gemm_dispatch.fwd(x[:100].contiguous(), w)
    used = gemm_dispatch.kernels_used()
    assert used[("fwd", 512, 2304, 768)] == "nt4"
    assert used[("fwd", 100, 2304, 768)] == "small"


def test_transposed_weight_dgrad_cache(kernels):
    """dX = dY·W through the cached K-contiguous W^T: equal to the plain product, rebuilt after
    an in-place update (version bump) and after a raw rewrite announced by weights_changed()
    (what the fused AdamW kernel does)."""
    from nanosandbox_amd.ops import gemm_dispatch

    torch.manual_seed(0)
    dy = torch.randn(512, 384, device="cuda").to(torch.bfloat16)
    w = torch.randn(384, 256, device="cuda").to(torch.bfloat16)

    def via_t():
        return (dy.float() @ gemm_dispatch._wt(w).t().float())

    assert torch.equal(via_t(), dy.float() @ w.float())
    t0 = gemm_dispatch._wt(w)
    assert gemm_dispatch._wt(w) is t0  # cached
    w.mul_(2.0)  # torch in-place op: version bump invalidates
    assert torch.equal(via_t(), dy.float() @ w.float())
    w.data.copy_(torch.randn_like(w))  # raw rewrite: no version bump ...
    assert not torch.equal(via_t(), dy.float() @ w.float())  # ... so the cache is stale until announced
    gemm_dispatch.weights_changed()
    assert torch.equal(via_t(), dy.float() @ w.float())


@pytest.mark.parametrize("R,C", [(768, 3072), (50304, 768), (64, 128), (2304, 768)])
def test_transpose_bf16(kernels, R, C):
    """The weight-transpose kernel behind the cached K-contiguous dgrad weights."""
    from nanosandbox_amd.ops import gemm_dispatch

    w = torch.randn(R, C, device="cuda").to(torch.bfloat16)
    t = gemm_dispatch._transpose(w)
    assert t.shape == (C, R) and t.is_contiguous()
    assert torch.equal(t, w.t())
    t2 = gemm_dispatch._transpose(w * 2, out=t)  # rebuilt in place
    assert t2.data_ptr() == t.data_ptr() and torch.equal(t2, (w * 2).t())


@pytest.mark.parametrize("M,V,Vp,C", [(2048, 50304, 50304, 768), (1032, 50257, 50304, 768), (512, 65, 256, 384)])
def test_nt4_xent_epilogue(kernels, M, V, Vp, C):
    """Fused cross-entropy forward GEMM: E = exp(x w^T - c) (bf16, padding columns 0) and the
    half-tile row sums, against fp32."""
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(2)
    x = torch.randn(M, C, device=DEV).to(BF)
    w = torch.zeros(Vp, C, device=DEV, dtype=BF)
    w[:V] = (torch.randn(V, C, device=DEV) * 0.05).to(BF)
    crow = torch.randn(M, device=DEV)
    slots = 2 * (-(-Vp // 256))
    part = torch.full((slots, M), NAN, device=DEV)
    e = gemm.nt_xent(x, w, crow, part, V, out=nanbuf(M, Vp))
    ref = torch.exp(x.float() @ w.float().t() - crow[:, None])
    ref[:, V:] = 0
    check(e, ref, ref.abs() * 2 ** -12, rel=2 ** -7, name="E")
    S = part.sum(0)
    assert torch.isfinite(part).all()
    assert torch.allclose(S, ref.sum(1), rtol=1e-4)


@pytest.mark.parametrize("M,K,N", [(2048, 50304, 768), (1032, 50304, 1024)])
def test_nt4_xdx_epilogue(kernels, M, K, N):
    """Fused cross-entropy input-gradient GEMM: cs * (E W) - cw * Wrows, fp32 subtraction."""
    from nanosandbox_amd.ops import gemm
    torch.manual_seed(3)
    e = torch.rand(M, K, device=DEV).to(BF)
    wt = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    wrows = torch.randn(M, N, device=DEV).to(BF)
    coef = torch.rand(M, 2, device=DEV)
    coef[::7] = 0  # ignored rows
    d = gemm.nt_xdx(e, wt, wrows, coef, out=nanbuf(M, N))
    prod = e.float() @ wt.float().t()
    ref = coef[:, :1] * prod - coef[:, 1:] * wrows.float()
    absab = coef[:, :1] * (e.float().abs() @ wt.float().abs().t()) + coef[:, 1:] * wrows.float().abs()
    check(d, ref, absab, name="xdx")
