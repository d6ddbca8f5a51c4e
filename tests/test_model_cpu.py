"""GPT model contract on CPU: parameter counts, state-dict keys, init, forward/backward
parity with an independent plain-PyTorch nanoGPT-style reference, generate, surgery."""

import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from nanosandbox_amd.models import GPT, GPTConfig
from nanosandbox_amd.optim import FlatParamStore


# ----------------------------------------------------------- reference model
class RefBlock(nn.Module):
    """Straight PyTorch version of nanoGPT's Block (SDPA math path), used as an oracle."""

    def __init__(self, cfg):
        super().__init__()
        C = cfg.n_embd
        self.ln_1 = nn.LayerNorm(C, bias=cfg.bias)
        self.c_attn = nn.Linear(C, 3 * C, bias=cfg.bias)
        self.c_proj = nn.Linear(C, C, bias=cfg.bias)
        self.ln_2 = nn.LayerNorm(C, bias=cfg.bias)
        self.c_fc = nn.Linear(C, 4 * C, bias=cfg.bias)
        self.mlp_proj = nn.Linear(4 * C, C, bias=cfg.bias)
        self.n_head = cfg.n_head

    def forward(self, x):
        B, T, C = x.shape
        q, k, v = self.c_attn(self.ln_1(x)).split(C, dim=2)
        q, k, v = (t.view(B, T, self.n_head, C // self.n_head).transpose(1, 2) for t in (q, k, v))
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        x = x + self.c_proj(y.transpose(1, 2).contiguous().view(B, T, C))
        return x + self.mlp_proj(F.gelu(self.c_fc(self.ln_2(x))))


class RefGPT(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.wte = nn.Embedding(cfg.vocab_size, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.block_size, cfg.n_embd)
        self.h = nn.ModuleList([RefBlock(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = nn.LayerNorm(cfg.n_embd, bias=cfg.bias)

    def forward(self, idx, targets):
        x = self.wte(idx) + self.wpe(torch.arange(idx.shape[1]))
        for b in self.h:
            x = b(x)
        logits = self.ln_f(x) @ self.wte.weight.t()
        return F.cross_entropy(logits.view(-1, logits.size(-1)), targets.view(-1), ignore_index=-1)


def load_ref(ref, sd, cfg):
    m = {"wte.weight": "transformer.wte.weight", "wpe.weight": "transformer.wpe.weight",
         "ln_f.weight": "transformer.ln_f.weight"}
    if cfg.bias:
        m["ln_f.bias"] = "transformer.ln_f.bias"
    for i in range(cfg.n_layer):
        for a, b in [("ln_1", "ln_1"), ("c_attn", "attn.c_attn"), ("c_proj", "attn.c_proj"), ("ln_2", "ln_2"),
                     ("c_fc", "mlp.c_fc"), ("mlp_proj", "mlp.c_proj")]:
            m[f"h.{i}.{a}.weight"] = f"transformer.h.{i}.{b}.weight"
            if cfg.bias:
                m[f"h.{i}.{a}.bias"] = f"transformer.h.{i}.{b}.bias"
    ref.load_state_dict({k: sd[v] for k, v in m.items()})
    return m


# --------------------------------------------------------------------- tests
def test_gpt2_124m_param_count():
    with torch.device("meta"):
        m = GPT(GPTConfig(n_layer=12, n_head=12, n_embd=768, block_size=1024, vocab_size=50304, bias=False))
    total = sum(p.numel() for p in m.parameters())
    assert total == 124_373_760  # 124.37M with tied wte/lm_head
    assert m.get_num_params() == 123_587_328  # 123.59M non-embedding (wpe subtracted)


def test_state_dict_keys_nanogpt_layout():
    cfg = GPTConfig(n_layer=2, n_head=2, n_embd=32, block_size=16, vocab_size=50, bias=True)
    sd = GPT(cfg).state_dict()
    expect = {"transformer.wte.weight", "transformer.wpe.weight", "transformer.ln_f.weight",
              "transformer.ln_f.bias", "lm_head.weight"}
    for i in range(2):
        for n in ["ln_1", "attn.c_attn", "attn.c_proj", "ln_2", "mlp.c_fc", "mlp.c_proj"]:
            expect |= {f"transformer.h.{i}.{n}.weight", f"transformer.h.{i}.{n}.bias"}
    assert set(sd) == expect
    m = GPT(cfg)
    assert m.transformer.wte.weight is m.lm_head.weight  # weight tying


def test_init_statistics():
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=4, n_head=4, n_embd=256, block_size=64, vocab_size=2000, bias=True)
    m = GPT(cfg)
    assert m.transformer.h[0].attn.c_attn.weight.std().item() == pytest.approx(0.02, rel=0.05)
    assert m.transformer.h[0].mlp.c_proj.weight.std().item() == pytest.approx(0.02 / math.sqrt(8), rel=0.05)
    assert m.transformer.h[0].attn.c_attn.bias.abs().max().item() == 0.0


@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("flat", [False, True])
def test_forward_backward_parity_with_reference(bias, flat):
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=2, n_head=4, n_embd=64, block_size=32, vocab_size=97, bias=bias)
    m = GPT(cfg)
    ref = RefGPT(cfg)
    names = load_ref(ref, m.state_dict(), cfg)
    store = FlatParamStore(m, "cpu") if flat else None
    idx = torch.randint(0, 97, (3, 32))
    tgt = torch.randint(0, 97, (3, 32))
    tgt[0, :4] = -1
    _, loss = m(idx, tgt)
    loss.backward()
    lref = ref(idx, tgt)
    lref.backward()
    assert loss.item() == pytest.approx(lref.item(), rel=1e-5)
    ours = dict(m.named_parameters())
    for rk, ok in names.items():
        p = ours[ok] if ok in ours else m.lm_head.weight
        g = p.main_grad if flat else p.grad
        gr = dict(ref.named_parameters())[rk].grad
        assert torch.allclose(g, gr, atol=1e-5, rtol=1e-4), rk


def test_eval_logits_last_position_and_generate():
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=1, n_head=2, n_embd=32, block_size=16, vocab_size=40)
    m = GPT(cfg).eval()
    idx = torch.randint(0, 40, (2, 10))
    logits, loss = m(idx)
    assert loss is None and logits.shape == (2, 1, 40)
    full = m.forward_logits(idx)
    assert torch.allclose(full[:, -1], logits[:, 0], atol=1e-5)
    out = m.generate(idx, 12, temperature=0.8, top_k=5)
    assert out.shape == (2, 22) and torch.equal(out[:, :10], idx)


def test_crop_block_size():
    cfg = GPTConfig(n_layer=1, n_head=2, n_embd=32, block_size=64, vocab_size=40)
    m = GPT(cfg)
    w = m.transformer.wpe.weight[:16].clone()
    m.crop_block_size(16)
    assert m.config.block_size == 16 and torch.equal(m.transformer.wpe.weight, w)
    with pytest.raises(AssertionError):
        m(torch.zeros(1, 17, dtype=torch.long))


def test_grad_ckpt_matches():
    torch.manual_seed(0)
    cfg = GPTConfig(n_layer=2, n_head=2, n_embd=32, block_size=16, vocab_size=40, dropout=0.1)
    m = GPT(cfg)
    idx = torch.randint(0, 40, (2, 16))
    torch.manual_seed(5)
    _, l1 = m(idx, idx)
    l1.backward()
    g1 = [p.grad.clone() for p in m.parameters()]
    m.zero_grad()
    m.grad_ckpt = True
    torch.manual_seed(5)
    _, l2 = m(idx, idx)
    l2.backward()
    assert l1.item() == pytest.approx(l2.item(), rel=1e-6)
    for a, b in zip(g1, [p.grad for p in m.parameters()]):
        assert torch.allclose(a, b, atol=1e-6)


def test_mfu_uses_mi355x_peak():
    cfg = GPTConfig(n_layer=12, n_head=12, n_embd=768, block_size=1024, vocab_size=50304, bias=False)
    with torch.device("meta"):
        m = GPT(cfg)
    fpt = m.flops_per_token()
    # 6N + 12 L H Q T for 124M at T=1024 ~ 0.855 GFLOP/token
    assert fpt == pytest.approx(0.855e9, rel=0.01)
    mfu = m.estimate_mfu(12 * 40, 1.0)
    assert mfu == pytest.approx(fpt * 1024 * 480 / 2.5e15)


def test_from_pretrained_local_snapshot(tmp_path, monkeypatch):
    """GPT.from_pretrained reads a local HuggingFace-layout safetensors snapshot (no
    network): Conv1D [in, out] weights are transposed into Linear layout, the rest copied,
    lm_head stays tied to wte.  The snapshot here is synthetic (random tensors of the
    gpt2 shapes under the HF key names)."""
    from safetensors.torch import save_file

    torch.manual_seed(0)
    C, L, V, T = 768, 12, 50257, 1024
    sd = {"wte.weight": torch.randn(V, C), "wpe.weight": torch.randn(T, C),
          "ln_f.weight": torch.randn(C), "ln_f.bias": torch.randn(C)}
    for i in range(L):
        p = f"h.{i}."
        sd.update({p + "ln_1.weight": torch.randn(C), p + "ln_1.bias": torch.randn(C),
                   p + "ln_2.weight": torch.randn(C), p + "ln_2.bias": torch.randn(C),
                   p + "attn.c_attn.weight": torch.randn(C, 3 * C), p + "attn.c_attn.bias": torch.randn(3 * C),
                   p + "attn.c_proj.weight": torch.randn(C, C), p + "attn.c_proj.bias": torch.randn(C),
                   p + "attn.bias": torch.ones(1, 1, T, T).tril()[:, :, :8, :8].contiguous(),
                   p + "mlp.c_fc.weight": torch.randn(C, 4 * C), p + "mlp.c_fc.bias": torch.randn(4 * C),
                   p + "mlp.c_proj.weight": torch.randn(4 * C, C), p + "mlp.c_proj.bias": torch.randn(C)})
    snap = tmp_path / "gpt2"
    snap.mkdir()
    save_file(sd, str(snap / "model.safetensors"))
    monkeypatch.setenv("NSA_HF_GPT2_DIR", str(tmp_path))
    m = GPT.from_pretrained("gpt2", {"dropout": 0.1})
    assert m.config.vocab_size == V and m.config.bias and m.config.dropout == 0.1
    blk = m.transformer.h[3]
    assert torch.equal(blk.attn.c_attn.weight, sd["h.3.attn.c_attn.weight"].t())
    assert torch.equal(blk.mlp.c_proj.weight, sd["h.3.mlp.c_proj.weight"].t())
    assert torch.equal(blk.ln_2.bias, sd["h.3.ln_2.bias"])
    assert torch.equal(m.transformer.wpe.weight, sd["wpe.weight"])
    assert m.lm_head.weight is m.transformer.wte.weight
    assert torch.equal(m.lm_head.weight, sd["wte.weight"])


def test_from_pretrained_without_snapshot_says_why(tmp_path, monkeypatch):
    monkeypatch.setenv("NSA_HF_GPT2_DIR", str(tmp_path))
    monkeypatch.setenv("HF_HOME", str(tmp_path))
    with pytest.raises(FileNotFoundError, match="NSA_HF_GPT2_DIR"):
        GPT.from_pretrained("gpt2-medium")


def test_from_pretrained_matches_hf_gpt2_forward(tmp_path, monkeypatch):
    """U-M8 parity against HuggingFace itself (offline): a random-init
    ``transformers.GPT2LMHeadModel`` at gpt2 sizes, saved with ``save_pretrained``
    (safetensors), loaded through ``GPT.from_pretrained('gpt2')`` — the Conv1D
    transposes, tied lm_head and key mapping must reproduce HF's logits.
    ``activation_function='gelu'`` because nanoGPT's MLP is the exact-erf GELU."""
    transformers = pytest.importorskip("transformers")
    torch.manual_seed(0)
    hf_cfg = transformers.GPT2Config(n_layer=12, n_head=12, n_embd=768, n_positions=1024, vocab_size=50257,
                                     activation_function="gelu", resid_pdrop=0.0, embd_pdrop=0.0, attn_pdrop=0.0)
    hf = transformers.GPT2LMHeadModel(hf_cfg).eval()
    snap = tmp_path / "gpt2"
    hf.save_pretrained(str(snap), safe_serialization=True)
    monkeypatch.setenv("NSA_HF_GPT2_DIR", str(tmp_path))
    m = GPT.from_pretrained("gpt2").eval()
    assert m.lm_head.weight is m.transformer.wte.weight
    idx = torch.randint(0, 50257, (2, 64))
    with torch.no_grad():
        out = hf(idx, labels=idx)
        ref = out.logits.float()
        last, _ = m(idx)  # inference path: last-position logits
        _, loss = m(idx[:, :-1], idx[:, 1:])  # training path: fused lm_head + cross-entropy
    rel = ((last[:, -1].float() - ref[:, -1]).norm() / ref[:, -1].norm()).item()
    assert rel < 1e-4, rel
    assert abs(loss.item() - out.loss.item()) < 1e-4 * abs(out.loss.item()), (loss.item(), out.loss.item())


def test_split_planes_roundtrip_bitwise():
    """The split-plane residual-gradient encoding (LayerNorm backward, csrc/kernels/layernorm.hip
    split8): hi + lo give g back bit for bit at binade edges, denormals, signed zeros,
    infinities and arbitrary bit patterns (a NaN stays a NaN); the hi plane is bf16(g) rounded
    to nearest, equal to torch's cast except at exact ties, which round away from zero."""
    from nanosandbox_amd.ops.functional import split_planes, unsplit_planes
    torch.manual_seed(0)
    g = torch.randn(64, 48) * torch.logspace(-40, 38, 48)[None]
    special = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), 1e-45, -1e-45, 3.4e38, -3.4e38,
                            1.00390625, -1.00390625, 1.01171875, 1.0 + 2 ** -8 + 2 ** -20, 255.99998])
    g[0, :special.numel()] = special
    bits = torch.randint(-2 ** 31, 2 ** 31 - 1, (16, 48), dtype=torch.int64).to(torch.int32)
    g[-16:] = bits.view(torch.float32)  # arbitrary bit patterns, NaNs included
    enc = split_planes(g)
    assert enc.dtype == torch.float32 and enc.shape == g.shape
    n = g.numel()
    fin = ~torch.isnan(g)
    tie = (g.view(torch.int32) & 0xFFFF) == 0x8000
    hi = enc.reshape(-1).view(torch.bfloat16)[:n].view(g.shape)
    rne = g.to(torch.bfloat16)
    sel = fin & ~tie
    assert torch.equal(hi.view(torch.int16)[sel], rne.view(torch.int16)[sel])
    assert tie[0, 8] and tie[0, 9] and tie[0, 10]
    assert hi[0, 8].item() == 1.0078125 and hi[0, 9].item() == -1.0078125  # away from zero
    assert hi[0, 10].item() == 1.015625  # (1.01171875 is a tie between 1.0078125 and 1.015625)
    assert torch.isnan(hi[~fin]).all()
    back = unsplit_planes(enc)
    assert torch.equal(back.view(torch.int32)[fin], g.view(torch.int32)[fin])
    assert torch.isnan(back[~fin]).all()


def test_split_planes_fp16_roundtrip():
    """The fp16-compute split encoding (csrc/kernels/layernorm.hip split8h): the hi plane is
    torch's fp16 cast; hi + lo give g back bit for bit for 2^-14 <= |g| < 65520 (binade
    edges, values that round up into the next binade, ties), within 2^-39 below that
    (subnormal and zero hi), an fp16 inf at and above 65520, infinities kept, NaN stays NaN."""
    from nanosandbox_amd.ops.functional import split_planes_h, unsplit_planes_h
    torch.manual_seed(0)
    g = torch.randn(64, 48) * torch.logspace(-12, 4.8, 48)[None]  # up to ~6e4
    special = torch.tensor([2.0 ** -14, -(2.0 ** -14), 2.0 ** -14 * (1 + 2 ** -20), 1.0 + 2 ** -11,
                            1.0 + 3 * 2 ** -11, 2.0 - 2 ** -23, 65504.0, 65519.99, -65519.99, 1.0 + 2 ** -12,
                            3e-5, -1e-8, 0.0, -0.0, 1e-30])
    g[0, :special.numel()] = special
    enc = split_planes_h(g)
    n = g.numel()
    hi = enc.reshape(-1).view(torch.float16)[:n].view(g.shape)
    assert torch.equal(hi.view(torch.int16), g.to(torch.float16).view(torch.int16))
    back = unsplit_planes_h(enc)
    normal = (g.abs() >= 2 ** -14) & (g.abs() < 65520)
    assert torch.equal(back.view(torch.int32)[normal], g.view(torch.int32)[normal])
    tiny = g.abs() < 2 ** -14
    assert ((back - g).abs()[tiny] <= 2.0 ** -39).all()
    assert torch.isinf(back[g.abs() >= 65520]).all()
    edge = torch.tensor([65520.0, -70000.0, float("inf"), float("-inf"), float("nan")])
    be = unsplit_planes_h(split_planes_h(edge))
    assert be[0].item() == float("inf") and be[1].item() == float("-inf")
    assert be[2].item() == float("inf") and be[3].item() == float("-inf") and torch.isnan(be[4])
