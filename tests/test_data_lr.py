"""Data format, samplers (memmap / native C++ / synthetic) and the LR schedule."""

import json
import math
import os
import pickle

import numpy as np
import pytest
import torch

from nanosandbox_amd.data import MemmapBatchSource, NativeBatchSource, SyntheticBatchSource, load_meta
from nanosandbox_amd.data.prepare import synthetic_corpus, write_char_dataset, write_token_dataset
from nanosandbox_amd.utils import get_lr


@pytest.fixture(scope="module")
def char_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("char")
    write_char_dataset(str(d), synthetic_corpus(50_000))
    return str(d)


def test_char_dataset_format(char_dir):
    tr = np.fromfile(os.path.join(char_dir, "train.bin"), dtype=np.uint16)
    va = np.fromfile(os.path.join(char_dir, "val.bin"), dtype=np.uint16)
    assert len(tr) == 45_000 and len(va) == 5_000  # 90/10 split
    meta = load_meta(char_dir)
    assert meta["vocab_size"] == int(max(tr.max(), va.max())) + 1
    text = "".join(meta["itos"][int(i)] for i in tr[:100])
    assert text == synthetic_corpus(50_000)[:100]
    # meta.pkl is the nanoGPT-compatible copy
    with open(os.path.join(char_dir, "meta.pkl"), "rb") as f:
        assert pickle.load(f)["vocab_size"] == meta["vocab_size"]


def test_meta_pkl_safe_loader(tmp_path):
    # without meta.json, meta.pkl is read by a restricted unpickler
    meta = {"vocab_size": 3, "itos": {0: "a", 1: "b", 2: "c"}, "stoi": {"a": 0, "b": 1, "c": 2}}
    with open(tmp_path / "meta.pkl", "wb") as f:
        pickle.dump(meta, f)
    assert load_meta(str(tmp_path))["vocab_size"] == 3

    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))

    with open(tmp_path / "meta.pkl", "wb") as f:
        pickle.dump({"x": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        load_meta(str(tmp_path))


def test_synthetic_corpus_size():
    assert len(synthetic_corpus()) == 1115394


def _check_xy(x, y, data, T):
    assert x.shape == y.shape and x.dtype == torch.int64
    for r in range(x.shape[0]):
        row = x[r].numpy()
        # locate the window: x = data[i:i+T], y = data[i+1:i+1+T]
        assert np.array_equal(row[1:], y[r].numpy()[:-1])


def test_memmap_source(char_dir):
    src = MemmapBatchSource(char_dir, 32, 8, "cpu", seed=1)
    x, y = src.get_batch("train")
    assert x.shape == (8, 32)
    _check_xy(x, y, None, 32)


@pytest.mark.skipif(not NativeBatchSource.available(), reason="native runtime not built")
def test_native_source_windows(char_dir):
    data = np.fromfile(os.path.join(char_dir, "train.bin"), dtype=np.uint16).astype(np.int64)
    src = NativeBatchSource(char_dir, 64, 16, "cpu", seed=3)
    for _ in range(5):
        x, y = src.get_batch("train")
        assert x.shape == (16, 64)
        _check_xy(x, y, data, 64)
        # every window must be a real slice of the file
        for r in range(16):
            seq = x[r].numpy()
            cand = np.nonzero(data[: len(data) - 64] == seq[0])[0]
            assert any(np.array_equal(data[i:i + 64], seq) for i in cand)
    xv, _ = src.get_batch("val")
    assert xv.shape == (16, 64)
    src.close()


@pytest.mark.skipif(not NativeBatchSource.available(), reason="native runtime not built")
def test_native_source_uniform_offsets(tmp_path):
    # token value == position -> x[:, 0] is the sampled offset
    n = 5000
    np.arange(n, dtype=np.uint16).tofile(tmp_path / "train.bin")
    np.arange(n, dtype=np.uint16).tofile(tmp_path / "val.bin")
    src = NativeBatchSource(str(tmp_path), 8, 256, "cpu", seed=7)
    offs = torch.cat([src.get_batch("train")[0][:, 0] for _ in range(40)]).numpy()
    assert offs.min() >= 0 and offs.max() < n - 8
    hist, _ = np.histogram(offs, bins=10, range=(0, n - 8))
    assert hist.min() > 0.7 * hist.mean()
    src.close()


def test_token_dataset(tmp_path):
    write_token_dataset(str(tmp_path), 20000)
    tr = np.fromfile(tmp_path / "train.bin", dtype=np.uint16)
    assert tr.max() < 50257 and len(tr) > 19000


def test_synthetic_source():
    s = SyntheticBatchSource(100, 16, 4, "cpu", seed=0)
    x, y = s.get_batch("train")
    assert x.shape == (4, 16) and int(x.max()) < 100
    assert torch.equal(x[:, 1:], y[:, :-1])


def test_lr_schedule():
    lr, wu, dec, mn = 6e-4, 10, 100, 6e-5
    assert get_lr(0, lr, wu, dec, mn) == pytest.approx(lr * 1 / 11)
    assert get_lr(9, lr, wu, dec, mn) == pytest.approx(lr * 10 / 11)
    assert get_lr(10, lr, wu, dec, mn) == pytest.approx(lr)
    assert get_lr(55, lr, wu, dec, mn) == pytest.approx(mn + 0.5 * (lr - mn))
    assert get_lr(100, lr, wu, dec, mn) == pytest.approx(mn)
    assert get_lr(101, lr, wu, dec, mn) == mn
    # monotone decay after warmup
    vals = [get_lr(i, lr, wu, dec, mn) for i in range(10, 101)]
    assert all(a >= b for a, b in zip(vals, vals[1:]))


def _tiny_bpe(tmp_path):
    """Train a small byte-level BPE in-process (GPT-2's files are not available offline)."""
    from tokenizers import ByteLevelBPETokenizer

    from nanosandbox_amd.data.prepare import synthetic_corpus

    text = synthetic_corpus(n_chars=20000, seed=3)
    tok = ByteLevelBPETokenizer()
    tok.train_from_iterator([text], vocab_size=400, min_frequency=2, special_tokens=["<|endoftext|>"])
    d = tmp_path / "tok"
    d.mkdir()
    tok.save_model(str(d))  # vocab.json + merges.txt, the GPT-2 release layout
    return text, d


def test_bpe_dataset_split_and_roundtrip(tmp_path):
    """nanoGPT data/shakespeare/prepare.py semantics: 90/10 char split, uint16 ids, lossless decode."""
    import numpy as np

    from nanosandbox_amd.data.prepare import load_bpe, main

    text, d = _tiny_bpe(tmp_path)
    inp = tmp_path / "input.txt"
    inp.write_text(text)
    out = tmp_path / "bpe"
    main(["bpe", "--out", str(out), "--input", str(inp), "--tokenizer", str(d)])
    train = np.fromfile(out / "train.bin", dtype=np.uint16)
    val = np.fromfile(out / "val.bin", dtype=np.uint16)
    tok = load_bpe(str(d))
    n = len(text)
    assert tok.decode(train.tolist()) == text[: int(n * 0.9)]
    assert tok.decode(val.tolist()) == text[int(n * 0.9):]


def test_bpe_docs_mode_eot(tmp_path):
    """OWT-style: every document is followed by <|endoftext|> (id 50256 in GPT-2's vocab)."""
    import numpy as np

    from nanosandbox_amd.data.prepare import load_bpe, write_bpe_dataset

    text, d = _tiny_bpe(tmp_path)
    flat = text.replace("\n", " ")
    docs = "\n".join(flat[i:i + 500] for i in range(0, 5000, 500))
    stats = write_bpe_dataset(str(tmp_path / "owt"), docs, load_bpe(str(d)), docs=True, val_frac=0.1, eot=50256)
    train = np.fromfile(tmp_path / "owt" / "train.bin", dtype=np.uint16)
    assert (train == 50256).sum() == 9 and train[-1] == 50256
    assert stats["val"] > 0
