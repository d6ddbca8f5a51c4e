"""KV-cache decoding on MI355X: the decode kernels against an fp32 torch reference, and the
graph-replayed decode step against the full fused forward."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def _ref_decode(q, kc, vc, p):
    """q [B, H, D], caches [B, H, T, D] -> [B, H, D] (fp32), keys 0..p."""
    k, v = kc[:, :, :p + 1].float(), vc[:, :, :p + 1].float()
    att = torch.softmax(torch.einsum("bhd,bhkd->bhk", q.float(), k) / math.sqrt(q.shape[-1]), dim=-1)
    return torch.einsum("bhk,bhkd->bhd", att, v)


@pytest.mark.parametrize("pos", [0, 37, 255, 256, 700, 1023])
def test_decode_attention_kernel(kernels, pos):
    from nanosandbox_amd import ops

    torch.manual_seed(pos)
    B, H, D, T = 3, 12, 64, 1024
    C = H * D
    kc = torch.randn(B, H, T, D, device=DEV).to(BF)
    vc = torch.randn(B, H, T, D, device=DEV).to(BF)
    qkv = torch.randn(B, 1, 3 * C, device=DEV).to(BF)
    p = torch.tensor([pos], device=DEV, dtype=torch.int64)
    ops.kv_append(qkv, kc, vc, p)  # the new token's K/V land at position pos
    k_new, v_new = qkv.view(B, 3, H, D)[:, 1], qkv.view(B, 3, H, D)[:, 2]
    assert torch.equal(kc[:, :, pos], k_new) and torch.equal(vc[:, :, pos], v_new)
    y = ops.decode_attention(qkv, kc, vc, p, H).float().view(B, H, D)
    ref = _ref_decode(qkv.view(B, 3, H, D)[:, 0], kc, vc, pos)
    err = ((y - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


def test_kv_append_prefill_rows(kernels):
    from nanosandbox_amd import ops

    B, S, H, D, T = 2, 77, 4, 64, 128
    qkv = torch.randn(B, S, 3 * H * D, device=DEV).to(BF)
    kc = torch.zeros(B, H, T, D, device=DEV, dtype=BF)
    vc = torch.zeros_like(kc)
    ops.kv_append(qkv, kc, vc, None, 0)
    k, v = qkv.view(B, S, 3, H, D)[:, :, 1:].permute(2, 0, 3, 1, 4)
    assert torch.equal(kc[:, :, :S], k) and torch.equal(vc[:, :, :S], v)
    assert kc[:, :, S:].abs().sum() == 0


@pytest.mark.parametrize("B,T", [(4, 40), (4, 64), (1, 40), (4, 33), (2, 72)])
def test_embedding_with_fp32_weights(kernels, B, T):
    """Without an optimizer's bf16 shadow the kernel's weight copies are temporaries; both
    must stay alive until the launch (the second copy used to land in the first's freed
    block, so wte rows were read from wpe's data for some shapes)."""
    from nanosandbox_amd import ops

    torch.manual_seed(T)
    wte = torch.randn(512, 256, device=DEV) * 0.02
    wpe = torch.randn(256, 256, device=DEV) * 0.02
    idx = torch.randint(0, 512, (B, T), device=DEV)
    x = ops.embedding(idx, wte, wpe, 0.0, False, dtype=torch.float32)
    ref = wte.to(BF).float()[idx] + wpe.to(BF).float()[:T]
    assert torch.equal(x, ref)


def _model():
    from nanosandbox_amd.models import GPT, GPTConfig

    torch.manual_seed(0)
    m = GPT(GPTConfig(block_size=256, vocab_size=512, n_layer=3, n_head=4, n_embd=256, dropout=0.0, bias=False))
    return m.eval().to(DEV).set_compute_dtype(BF)


@pytest.mark.parametrize("B", [4, 1])
def test_graph_decode_matches_full_forward(kernels, B):
    """B = 4: GEMV / library linears + add+LayerNorm kernels; B = 1: the fused single-row
    path (embedding, LayerNorm and attention combine in the GEMV prologues, the position
    advanced by the head kernel)."""
    from nanosandbox_amd.runtime.decode import Decoder

    m = _model()
    T0, T = 40, 72
    idx = torch.randint(0, 512, (B, T), device=DEV)
    with torch.no_grad():
        full = m.forward_logits(idx)  # [B, T, V] through the training-path fused forward
    dg = Decoder(m, B, use_graph=True)
    de = Decoder(m, B, use_graph=False)
    with torch.no_grad():
        lg, le = dg.prefill(idx[:, :T0]), de.prefill(idx[:, :T0])
        for t in range(T0, T):
            ref = full[:, t - 1] if t == T0 else None
            if ref is not None:
                assert ((lg - ref).norm() / ref.norm()).item() < 2e-2
            lg = dg.step(idx[:, t]).clone()
            le = de.step(idx[:, t])
            assert torch.equal(lg, le), t  # the replayed graph runs exactly the eager kernels
            err = ((lg - full[:, t]).norm() / full[:, t].norm()).item()
            assert err < 3e-2, (t, err)
    assert dg.replays == T - T0 and dg.position == T


def test_cached_generation_on_gpu(kernels):
    m = _model()
    idx = torch.randint(0, 512, (2, 8), device=DEV)
    torch.manual_seed(3)
    out = m.generate_cached(idx, 50, temperature=0.8, top_k=20)
    assert out.shape == (2, 58) and torch.equal(out[:, :8], idx)
    assert int(out.max()) < 512 and int(out.min()) >= 0


def test_reused_decoder_draws_independent_samples(kernels):
    """sample.py's loop reuses one Decoder (and its captured sampling graph) for every
    sample: each generate call must still draw its own tokens (a salt baked into
    the graph made every sample identical)."""
    from nanosandbox_amd.runtime.decode import Decoder

    m = _model()
    idx = torch.randint(0, 512, (1, 8), device=DEV)
    dec = Decoder(m, 1, max_len=m.config.block_size, use_graph=True)
    try:
        outs = [m.generate_cached(idx, 40, temperature=1.0, top_k=None, decoder=dec) for _ in range(3)]
    finally:
        dec.release()
    assert dec.replays > 0
    assert not torch.equal(outs[0], outs[1]) and not torch.equal(outs[1], outs[2])
    torch.manual_seed(11)
    a = m.generate_cached(idx, 20, temperature=1.0)
    torch.manual_seed(11)
    b = m.generate_cached(idx, 20, temperature=1.0)
    assert torch.equal(a, b)  # still reproducible from torch.manual_seed


@pytest.mark.parametrize("B", [3, 1])
def test_graph_sampling_loop_matches_eager_greedy(kernels, B):
    """run(): step + sampling + device-side token feedback replayed as one graph gives the
    eager decoder's greedy tokens."""
    m = _model()
    idx = torch.randint(0, 512, (B, 16), device=DEV)
    a = m.generate_cached(idx, 40, top_k=1, use_graph=True)
    b = m.generate_cached(idx, 40, top_k=1, use_graph=False)
    assert torch.equal(a, b)
    assert not any(hasattr(p, "compute") for p in m.parameters())  # shadows released


@pytest.mark.parametrize("top_k,temperature", [(None, 1.0), (5, 0.7), (1, 1.0), (50, 1.3)])
def test_device_sampling_distribution(kernels, top_k, temperature):
    """ops.sample_topk_ draws from softmax(top-k(logits) / temperature): empirical
    frequencies over 32k draws match (total variation < 0.03; the sampling noise of 32k
    draws over 64 ids is <= 0.018); top_k = 1 is argmax."""
    from nanosandbox_amd import ops

    torch.manual_seed(0)
    V, R = 64, 4096
    base = torch.randn(V, device=DEV) * 2.0
    logits = base.expand(R, V).contiguous()
    ref = base / temperature
    if top_k is not None:
        thr = torch.topk(ref, top_k).values[-1]
        ref = ref.masked_fill(ref < thr, -float("inf"))
    p = torch.softmax(ref, 0)
    counts = torch.zeros(V, device=DEV)
    tok = torch.zeros(R, 1, dtype=torch.int64, device=DEV)
    gen = torch.zeros(R, 8, dtype=torch.int64, device=DEV)
    for step in range(8):
        pos = torch.tensor([step], dtype=torch.int64, device=DEV)
        ops.sample_topk_(logits, temperature, top_k, 1234, pos, tok, gen)
        assert torch.equal(gen[:, step], tok[:, 0])
        counts += torch.bincount(tok[:, 0], minlength=V).float()
    freq = counts / counts.sum()
    if top_k is not None:
        assert counts[p == 0].sum() == 0  # nothing outside the top-k
    tv = 0.5 * (freq - p).abs().sum().item()
    assert tv < 0.03, tv


@pytest.mark.parametrize("rows", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("N,K,bias,gelu,f32", [(768, 768, True, False, False), (3072, 768, True, True, False),
                                              (768, 3072, False, False, False), (50304, 768, False, False, True),
                                              (4800, 1600, True, False, False), (100, 64, True, True, False)])
def test_decode_linear_kernel(kernels, monkeypatch, rows, N, K, bias, gelu, f32):
    from nanosandbox_amd import ops
    from nanosandbox_amd.ops import functional
    import torch.nn.functional as F

    monkeypatch.setattr(functional, "GEMV_MAX_ROWS", 8)  # exercise the kernel at every row count

    torch.manual_seed(rows * 7 + N)
    x = torch.randn(rows, 1, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = (torch.randn(N, device=DEV) * 0.1).to(BF) if bias else None
    y = ops.decode_linear(x, w, b, gelu=gelu, out_f32=f32)
    ref = x.float().view(rows, K) @ w.float().t()
    if b is not None:
        ref = ref + b.float()
    if gelu:
        ref = F.gelu(ref)
    assert y.shape == (rows, 1, N) and y.dtype == (torch.float32 if f32 else BF)
    err = ((y.float().view(rows, N) - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("rows", [2, 3, 8, 15, 16, 17, 31, 33, 64])
@pytest.mark.parametrize("N,K,bias,gelu,f32", [(768, 768, True, False, False), (3072, 768, True, True, False),
                                              (768, 3072, False, False, False), (50304, 768, False, False, True),
                                              (4800, 1600, True, False, False), (6400, 1600, True, True, False),
                                              (16, 32, True, False, False), (48, 448, False, True, False)])
def test_decode_skinny_gemm(kernels, monkeypatch, rows, N, K, bias, gelu, f32):
    """Decode batches of 2..64 rows: the MFMA weight-streaming kernel (nsa_skinny_gemm,
    16 output columns per workgroup, K-units split over 4 waves, tail loop for K not a
    multiple of 512) against the fp32 reference."""
    from nanosandbox_amd import ops
    from nanosandbox_amd.ops import functional
    import torch.nn.functional as F

    monkeypatch.setattr(functional, "GEMV_MAX_ROWS", 1)
    monkeypatch.setattr(functional, "SKINNY_MAX_ROWS", 64)
    calls = []
    real_call = functional._lib.call
    monkeypatch.setattr(functional._lib, "call", lambda name, *a: (calls.append(name), real_call(name, *a))[1])
    torch.manual_seed(rows * 13 + N + K)
    x = torch.randn(rows, 1, K, device=DEV).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = (torch.randn(N, device=DEV) * 0.1).to(BF) if bias else None
    y = ops.decode_linear(x, w, b, gelu=gelu, out_f32=f32)
    assert "nsa_skinny_gemm" in calls
    ref = x.float().view(rows, K) @ w.float().t()
    if b is not None:
        ref = ref + b.float()
    if gelu:
        ref = F.gelu(ref)
    assert y.shape == (rows, 1, N) and y.dtype == (torch.float32 if f32 else BF)
    err = ((y.float().view(rows, N) - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("rows", [2, 5, 16])
@pytest.mark.parametrize("branch", [False, True])
@pytest.mark.parametrize("N,K,bias,gelu,f32", [(2304, 768, True, False, False), (3072, 768, True, True, False),
                                              (50304, 768, False, False, True), (6400, 1600, True, True, False),
                                              (4800, 1600, True, False, False), (48, 1920, False, False, False)])
def test_decode_skinny_ln_kernel(kernels, monkeypatch, rows, branch, N, K, bias, gelu, f32):
    """Residual add + LayerNorm in the skinny GEMM's prologue (2..16 decode rows) against
    fp32 torch on the same bf16-rounded LayerNorm output; s = res + branch in fp32."""
    from nanosandbox_amd import ops
    from nanosandbox_amd.ops import functional
    import torch.nn.functional as F

    monkeypatch.setattr(functional, "SKINNY_LN_MAX_ROWS", 16)  # exercise the kernel at every row count
    calls = []
    real_call = functional._lib.call
    monkeypatch.setattr(functional._lib, "call", lambda name, *a: (calls.append(name), real_call(name, *a))[1])
    torch.manual_seed(N + K + rows)
    res = torch.randn(rows, 1, K, device=DEV) * 3 + 0.5
    br = torch.randn(rows, 1, K, device=DEV).to(BF) if branch else None
    lw = (1 + 0.1 * torch.randn(K, device=DEV)).to(BF)
    lb = (0.1 * torch.randn(K, device=DEV)).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = (torch.randn(N, device=DEV) * 0.1).to(BF) if bias else None
    s, y = ops.decode_linear_ln(res, br, lw, lb, w, b, gelu=gelu, out_f32=f32)
    assert "nsa_skinny_ln_gemm" in calls
    s_ref = res + br.float() if branch else res
    assert torch.allclose(s, s_ref) and (branch or s is res)
    h = F.layer_norm(s_ref.view(rows, K), (K,), lw.float(), lb.float(), 1e-5).to(BF).float()
    ref = h @ w.float().t()
    if b is not None:
        ref = ref + b.float()
    if gelu:
        ref = F.gelu(ref)
    assert y.shape == (rows, 1, N) and y.dtype == (torch.float32 if f32 else BF)
    err = ((y.float().view(rows, N) - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("branch", [False, True])
@pytest.mark.parametrize("N,K,bias,gelu,f32", [(2304, 768, True, False, False), (3072, 768, True, True, False),
                                              (50304, 768, False, False, True), (6400, 1600, True, True, False),
                                              (100, 64, False, False, False)])
def test_decode_linear_ln_kernel(kernels, branch, N, K, bias, gelu, f32):
    """Fused residual add + LayerNorm + GEMV (one decode row) against fp32 torch on the
    same bf16-rounded LayerNorm output."""
    from nanosandbox_amd import ops
    import torch.nn.functional as F

    torch.manual_seed(N + K)
    res = torch.randn(1, 1, K, device=DEV) * 3 + 0.5
    br = torch.randn(1, 1, K, device=DEV).to(BF) if branch else None
    lw = (1 + 0.1 * torch.randn(K, device=DEV)).to(BF)
    lb = (0.1 * torch.randn(K, device=DEV)).to(BF)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
    b = (torch.randn(N, device=DEV) * 0.1).to(BF) if bias else None
    s, y = ops.decode_linear_ln(res, br, lw, lb, w, b, gelu=gelu, out_f32=f32)
    s_ref = res + br.float() if branch else res
    assert torch.allclose(s, s_ref) and (branch or s is res)
    h = F.layer_norm(s_ref.view(1, K), (K,), lw.float(), lb.float(), 1e-5).to(BF).float()
    ref = h @ w.float().t()
    if b is not None:
        ref = ref + b.float()
    if gelu:
        ref = F.gelu(ref)
    assert y.shape == (1, 1, N) and y.dtype == (torch.float32 if f32 else BF)
    err = ((y.float().view(1, N) - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("V,top_k", [(63, 5), (50304, 200), (50304, 1), (4096, 2000), (50304, 1024)])
def test_device_sampling_topk_support(kernels, V, top_k):
    """Top-k restriction on wide rows and on every kernel path (candidate compaction for
    k <= 1024, the register bisection for larger k, the scalar-load path for V % 4 != 0):
    every draw is one of the k largest logits; k = 1 is the argmax."""
    from nanosandbox_amd import ops

    torch.manual_seed(V + top_k)
    R = 64
    logits = torch.randn(R, V, device=DEV) * 3.0
    thr = torch.topk(logits, top_k, dim=1).values[:, -1:]
    tok = torch.zeros(R, 1, dtype=torch.int64, device=DEV)
    gen = torch.zeros(R, 4, dtype=torch.int64, device=DEV)
    seen = set()
    for step in range(4):
        pos = torch.tensor([step], dtype=torch.int64, device=DEV)
        ops.sample_topk_(logits, 0.9, top_k, 77, pos, tok, gen)
        picked = logits.gather(1, tok)
        assert bool((picked >= thr).all()), step
        if top_k == 1:
            assert torch.equal(tok[:, 0], logits.argmax(1))
        seen.update(tok[:, 0].tolist())
    if top_k >= 200:
        assert len(seen) > 64  # draws spread over the kept set


def test_device_sampling_all_ties(kernels):
    """Equal logits: > 4096 candidates tie with the k-th largest, so the kernel takes the
    full bisection path and (ties kept) samples uniformly over the whole row."""
    from nanosandbox_amd import ops

    V, R = 50304, 256
    logits = torch.zeros(R, V, device=DEV)
    tok = torch.zeros(R, 1, dtype=torch.int64, device=DEV)
    gen = torch.zeros(R, 1, dtype=torch.int64, device=DEV)
    ops.sample_topk_(logits, 1.0, 200, 5, torch.zeros(1, dtype=torch.int64, device=DEV), tok, gen)
    assert int(tok.min()) >= 0 and int(tok.max()) < V
    assert len(set(tok[:, 0].tolist())) > 200


def test_decode_embed_linear_ln_kernel(kernels):
    from nanosandbox_amd import ops
    import torch.nn.functional as F

    torch.manual_seed(1)
    V, T, C, N = 512, 128, 768, 2304
    wte = (torch.randn(V, C, device=DEV) * 0.5).to(BF)
    wpe = (torch.randn(T, C, device=DEV) * 0.5).to(BF)
    lw = (1 + 0.1 * torch.randn(C, device=DEV)).to(BF)
    lb = (0.1 * torch.randn(C, device=DEV)).to(BF)
    w = (torch.randn(N, C, device=DEV) * 0.05).to(BF)
    b = (torch.randn(N, device=DEV) * 0.1).to(BF)
    tok = torch.tensor([[311]], device=DEV)
    pos = torch.tensor([77], device=DEV)
    x, y = ops.decode_embed_linear_ln(tok, pos, wte, wpe, lw, lb, w, b)
    x_ref = wte[311].float() + wpe[77].float()
    assert x.dtype == torch.float32 and torch.equal(x.view(C), x_ref)
    h = F.layer_norm(x_ref.view(1, C), (C,), lw.float(), lb.float(), 1e-5).to(BF).float()
    ref = h @ w.float().t() + b.float()
    err = ((y.float().view(1, N) - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("pos", [0, 300, 1023])
def test_attention_partials_into_linear(kernels, pos):
    """decode_attention(combine=False) -> decode_linear (combine in the GEMV prologue)
    equals the combine kernel's output through the plain GEMV."""
    from nanosandbox_amd import ops

    torch.manual_seed(pos)
    H, D, T = 12, 64, 1024
    C = H * D
    kc = torch.randn(1, H, T, D, device=DEV).to(BF)
    vc = torch.randn(1, H, T, D, device=DEV).to(BF)
    qkv = torch.randn(1, 1, 3 * C, device=DEV).to(BF)
    p = torch.tensor([pos], device=DEV, dtype=torch.int64)
    w = (torch.randn(C, C, device=DEV) * 0.05).to(BF)
    b = (torch.randn(C, device=DEV) * 0.1).to(BF)
    y_ref = ops.decode_linear(ops.decode_attention(qkv, kc.clone(), vc.clone(), p, H, append=True), w, b)
    part = ops.decode_attention(qkv, kc, vc, p, H, append=True, combine=False)
    assert isinstance(part, ops.AttnPartials)
    y = ops.decode_linear(part, w, b)
    assert y.shape == y_ref.shape
    err = ((y.float() - y_ref.float()).norm() / y_ref.float().norm()).item()
    assert err < 5e-3, err
