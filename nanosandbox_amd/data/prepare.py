"""Dataset preparation into nanoGPT's on-disk format.

Format (upstream ``data/shakespeare_char/prepare.py`` run by
reference ``notebooks/colab_nanoGPT_companion.ipynb:50-56``): ``train.bin`` and
``val.bin`` are raw ``np.uint16`` token streams, ``meta.pkl`` holds
``{vocab_size, itos, stoi}`` for char-level data.  We also write ``meta.json``
(same content) which our loaders prefer — it needs no unpickling.

There is no network in this environment, so the char dataset is built from a
local text file (``--input``) or, by default, from a deterministic synthetic
English-like corpus of the same size as tinyshakespeare (1,115,394 chars).
``tokens`` writes a GPT-2-vocabulary token stream (the offline stand-in for the
OpenWebText subset job, reference ``scripts/gh_sync.ps1:145-147``).
``bpe`` is upstream ``data/shakespeare/prepare.py`` / ``data/openwebtext/prepare.py``:
byte-level BPE encoding of a local text (tiktoken's GPT-2 ``encode_ordinary``
there; here the HF ``tokenizers`` library with a local GPT-2 ``tokenizer.json``
or ``vocab.json`` + ``merges.txt`` — no network, tiktoken is not installed), a
90/10 split (``--docs``: one document per line, each followed by <|endoftext|>
50256, split by ``--val_frac`` as the OWT script does).  Parity with tiktoken's
ids holds for the same GPT-2 vocab/merges files; it is not pinned by a test here.

CLI::

    python -m nanosandbox_amd.data.prepare char   --out data/shakespeare_char [--input input.txt]
    python -m nanosandbox_amd.data.prepare tokens --out data/openwebtext --n_tokens 10000000
    python -m nanosandbox_amd.data.prepare bpe    --out data/shakespeare --input input.txt --tokenizer gpt2/
"""

from __future__ import annotations

import argparse
import json
import os
import pickle

import numpy as np

TINYSHAKESPEARE_CHARS = 1115394

_WORDS = (
    "the of and to in that is was he for it with as his on be at by i this had not are but from or have an "
    "they which one you were her all she there would their we him been has when who will more no if out so "
    "said what up its about into than them can only other new some could time these two may then do first any "
    "my now such like our over man me even most made after also did many before must through back years where "
    "much your way well down should because each just those people mr how too little state good very make world "
    "still own see men work long get here between both life being under never day same another know while last "
    "might us great old year off come since against go came right used take three king lord thou thee love "
    "sweet death night heart blood crown honour grace fair speak"
).split()
_NAMES = ["KING", "QUEEN", "ROMEO", "JULIET", "HAMLET", "MERCUTIO", "DUKE", "CLOWN", "First Citizen", "GLOUCESTER"]


def synthetic_corpus(n_chars: int = TINYSHAKESPEARE_CHARS, seed: int = 1337) -> str:
    """Deterministic play-like text (speaker lines, punctuation, newlines)."""
    rng = np.random.default_rng(seed)
    # Zipf-ish word frequencies give the text realistic, learnable statistics
    w = 1.0 / np.arange(1, len(_WORDS) + 1) ** 1.1
    w /= w.sum()
    out = []
    n = 0
    while n < n_chars:
        speaker = _NAMES[rng.integers(len(_NAMES))]
        block = [f"{speaker}:\n"]
        for _ in range(int(rng.integers(1, 5))):
            k = int(rng.integers(4, 12))
            words = rng.choice(_WORDS, size=k, p=w)
            line = " ".join(words)
            line = line[0].upper() + line[1:]
            line += [",", ".", ";", "!", "?", ":"][int(rng.integers(6))]
            block.append(line + "\n")
        block.append("\n")
        s = "".join(block)
        out.append(s)
        n += len(s)
    return "".join(out)[:n_chars]


def write_char_dataset(out_dir: str, text: str) -> dict:
    os.makedirs(out_dir, exist_ok=True)
    print(f"length of dataset in characters: {len(text):,}")
    chars = sorted(list(set(text)))
    vocab_size = len(chars)
    print("all the unique characters:", "".join(chars))
    print(f"vocab size: {vocab_size:,}")
    stoi = {ch: i for i, ch in enumerate(chars)}
    itos = {i: ch for i, ch in enumerate(chars)}
    n = len(text)
    train_data = text[: int(n * 0.9)]
    val_data = text[int(n * 0.9):]
    train_ids = np.array([stoi[c] for c in train_data], dtype=np.uint16)
    val_ids = np.array([stoi[c] for c in val_data], dtype=np.uint16)
    print(f"train has {len(train_ids):,} tokens")
    print(f"val has {len(val_ids):,} tokens")
    train_ids.tofile(os.path.join(out_dir, "train.bin"))
    val_ids.tofile(os.path.join(out_dir, "val.bin"))
    meta = {"vocab_size": vocab_size, "itos": itos, "stoi": stoi}
    with open(os.path.join(out_dir, "meta.pkl"), "wb") as f:
        pickle.dump(meta, f)
    with open(os.path.join(out_dir, "meta.json"), "w") as f:
        json.dump({"vocab_size": vocab_size, "itos": {str(k): v for k, v in itos.items()}, "stoi": stoi}, f)
    return meta


def write_token_dataset(out_dir: str, n_tokens: int, vocab: int = 50257, seed: int = 1337, val_frac: float = 0.0005):
    """GPT-2-vocab token stream with Zipfian unigram statistics and EOT separators."""
    os.makedirs(out_dir, exist_ok=True)
    rng = np.random.default_rng(seed)
    ranks = rng.zipf(1.2, size=n_tokens).astype(np.int64)
    ids = np.where(ranks < vocab, ranks, rng.integers(0, vocab, size=n_tokens)).astype(np.uint16)
    doc_ends = rng.integers(0, n_tokens, size=max(1, n_tokens // 1000))
    ids[doc_ends] = 50256  # <|endoftext|>
    n_val = max(1, int(n_tokens * val_frac))
    ids[:-n_val].tofile(os.path.join(out_dir, "train.bin"))
    ids[-n_val:].tofile(os.path.join(out_dir, "val.bin"))
    print(f"train has {n_tokens - n_val:,} tokens, val has {n_val:,} tokens")


def load_bpe(path: str):
    """A byte-level BPE tokenizer from a ``tokenizer.json`` or a dir with it / vocab.json + merges.txt."""
    from tokenizers import Tokenizer
    from tokenizers.implementations import ByteLevelBPETokenizer

    if os.path.isdir(path):
        tj = os.path.join(path, "tokenizer.json")
        if os.path.exists(tj):
            return Tokenizer.from_file(tj)
        return ByteLevelBPETokenizer(os.path.join(path, "vocab.json"), os.path.join(path, "merges.txt"))
    return Tokenizer.from_file(path)


def write_bpe_dataset(out_dir: str, text: str, tokenizer, docs: bool = False, val_frac: float = 0.0005,
                      eot: int = 50256) -> dict:
    """Encode ``text`` (nanoGPT shakespeare: 90/10 split; ``docs``: OWT-style EOT after each line)."""
    os.makedirs(out_dir, exist_ok=True)
    if docs:
        lines = [ln for ln in text.splitlines() if ln.strip()]
        enc = tokenizer.encode_batch(lines)
        n_val_docs = max(1, int(round(len(lines) * val_frac))) if len(lines) > 1 else 0
        split_at = len(lines) - n_val_docs
        ids = [[*e.ids, eot] for e in enc]
        train = np.array([t for d in ids[:split_at] for t in d], dtype=np.uint16)
        val = np.array([t for d in ids[split_at:] for t in d], dtype=np.uint16)
    else:
        n = len(text)
        train = np.array(tokenizer.encode(text[: int(n * 0.9)]).ids, dtype=np.uint16)
        val = np.array(tokenizer.encode(text[int(n * 0.9):]).ids, dtype=np.uint16)
    train.tofile(os.path.join(out_dir, "train.bin"))
    val.tofile(os.path.join(out_dir, "val.bin"))
    print(f"train has {len(train):,} tokens")
    print(f"val has {len(val):,} tokens")
    return {"train": len(train), "val": len(val)}


def _download(url: str, timeout: float = 30.0):
    import urllib.request

    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:  # honours HTTP(S)_PROXY
            return r.read().decode("utf-8")
    except Exception as e:  # no network: keep the pipeline usable
        print(f"download of {url} failed ({e}); using the synthetic corpus instead")
        return None


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["char", "tokens", "bpe"])
    ap.add_argument("--out", required=True)
    ap.add_argument("--input", default="")
    ap.add_argument("--url", default="", help="download the text (through HTTP(S)_PROXY); falls back to "
                                              "the synthetic corpus when unreachable (air-gapped clusters)")
    ap.add_argument("--n_tokens", type=int, default=10_000_000)
    ap.add_argument("--seed", type=int, default=1337)
    ap.add_argument("--tokenizer", default="", help="bpe: tokenizer.json, or a dir with it / vocab.json + merges.txt")
    ap.add_argument("--docs", action="store_true", help="bpe: one document per line, EOT-separated (OWT style)")
    ap.add_argument("--val_frac", type=float, default=0.0005)
    a = ap.parse_args(argv)
    if a.kind == "bpe":
        if not a.input or not a.tokenizer:
            ap.error("bpe needs --input and --tokenizer (no network: tiktoken's GPT-2 files must be local)")
        with open(a.input) as f:
            write_bpe_dataset(a.out, f.read(), load_bpe(a.tokenizer), docs=a.docs, val_frac=a.val_frac)
        return
    if a.kind == "char":
        text = None
        if a.input:
            with open(a.input) as f:
                text = f.read()
        elif a.url:
            text = _download(a.url)
        if text is None:
            text = synthetic_corpus(seed=a.seed)
        write_char_dataset(a.out, text)
    else:
        write_token_dataset(a.out, a.n_tokens, seed=a.seed)


if __name__ == "__main__":
    main()
