"""KV-cache decoding (runtime/decode.py): incremental logits and generations match the
full-recompute model on CPU (the fp32 torch reference of the decode kernels)."""

import pytest
import torch

from nanosandbox_amd.models import GPT, GPTConfig
from nanosandbox_amd.runtime.decode import Decoder


def _model(bias=True, n_layer=2, n_head=4, n_embd=64, block_size=48, vocab_size=97):
    torch.manual_seed(0)
    return GPT(GPTConfig(block_size=block_size, vocab_size=vocab_size, n_layer=n_layer, n_head=n_head,
                         n_embd=n_embd, dropout=0.0, bias=bias)).eval()


@pytest.mark.parametrize("bias", [True, False])
def test_incremental_logits_match_full_forward(bias):
    m = _model(bias=bias)
    idx = torch.randint(0, 97, (3, 20))
    full = m.forward_logits(idx)  # [B, T, V]
    dec = Decoder(m, 3, use_graph=False)
    with torch.no_grad():
        lg = dec.prefill(idx[:, :8])
        assert torch.allclose(lg, full[:, 7], atol=1e-4, rtol=1e-4)
        for t in range(8, 20):
            lg = dec.step(idx[:, t])
            assert torch.allclose(lg, full[:, t], atol=1e-4, rtol=1e-4), t
    assert dec.position == 20


def test_cached_greedy_generation_matches_recompute():
    m = _model()
    idx = torch.randint(0, 97, (2, 5))
    torch.manual_seed(1)
    a = m.generate(idx, 30, top_k=1)
    torch.manual_seed(1)
    b = m.generate_cached(idx, 30, top_k=1)
    assert torch.equal(a, b)


def test_cached_generation_falls_back_past_block_size():
    m = _model(block_size=16)
    idx = torch.randint(0, 97, (1, 10))
    torch.manual_seed(2)
    a = m.generate(idx, 12, top_k=1)
    torch.manual_seed(2)
    b = m.generate_cached(idx, 12, top_k=1)
    assert torch.equal(a, b) and b.shape == (1, 22)


def test_sample_cli_uses_the_cache(tmp_path, monkeypatch):
    from nanosandbox_amd import sample

    m = _model()
    ck = {"model": m.state_dict(), "model_args": dict(block_size=48, vocab_size=97, n_layer=2, n_head=4, n_embd=64,
                                                      bias=True, dropout=0.0),
          "iter_num": 0, "best_val_loss": 0.0, "config": {}}
    torch.save(ck, tmp_path / "ckpt.pt")
    (tmp_path / "prompt.txt").write_text("1,2,3")
    # raw token-id codec (the tokenizer found offline differs between environments)
    monkeypatch.setattr(sample, "_codec", lambda ck, dd: ((lambda s: [int(t) for t in s.split(",")]),
                                                          (lambda ids: ",".join(map(str, ids)))))
    args = [f"--out_dir={tmp_path}", "--device=cpu", "--num_samples=1", "--max_new_tokens=6",
            f"--start=FILE:{tmp_path / 'prompt.txt'}", "--top_k=1"]
    outs = sample.main(args)
    outs_nc = sample.main(args + ["--kv_cache=False"])
    assert outs == outs_nc and len(outs[0].split(",")) == 9
