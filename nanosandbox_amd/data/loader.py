"""Batch sources for training and evaluation.

``get_batch(split)`` semantics follow nanoGPT: uniform random
windows ``ix ~ U[0, len(data) - block_size)``, ``x = data[i:i+T]``,
``y = data[i+1:i+1+T]`` as int64, every rank sampling independently (seeded
1337 + rank, no DistributedSampler), host->device copy from pinned memory with
``non_blocking=True`` so it overlaps the running step.

Three implementations:

* ``MemmapBatchSource`` — the reference behaviour (re-creates ``np.memmap``
  every call to dodge the memmap leak).
* ``NativeBatchSource`` — our C++ runtime loader (``csrc/runtime/dataloader.cpp``):
  the token file is mmapped once, a background thread samples windows with its
  own PRNG and fills a ring of ready batches, so the training thread only does
  one memcpy into a pinned buffer plus the async H2D copy.
* ``SyntheticBatchSource`` — random tokens generated directly on the device
  (the benchmark's ``data: synthetic``): no host work at all.
"""

from __future__ import annotations

import ctypes
import json
import os
import pickle

import numpy as np
import torch

_RUNTIME_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                            "libnsa_runtime.so")


class _SafeUnpickler(pickle.Unpickler):
    """meta.pkl only ever holds dicts of ints/strs; refuse anything that would execute code."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from meta.pkl")


def load_meta(data_dir: str):
    jp = os.path.join(data_dir, "meta.json")
    if os.path.exists(jp):
        with open(jp) as f:
            meta = json.load(f)
        meta["itos"] = {int(k): v for k, v in meta["itos"].items()}
        return meta
    pp = os.path.join(data_dir, "meta.pkl")
    if os.path.exists(pp):
        with open(pp, "rb") as f:
            return _SafeUnpickler(f).load()
    return None


def resolve_data_dir(dataset: str, data_dir: str = "") -> str:
    root = data_dir or "data"
    return os.path.join(root, dataset)


def _to_device(x, y, device):
    if device.type == "cuda":
        return x.pin_memory().to(device, non_blocking=True), y.pin_memory().to(device, non_blocking=True)
    return x.to(device), y.to(device)


class MemmapBatchSource:
    def __init__(self, data_dir, block_size, batch_size, device, seed=1337):
        self.data_dir = data_dir
        self.block_size = block_size
        self.batch_size = batch_size
        self.device = torch.device(device)
        self.gen = torch.Generator().manual_seed(seed)

    def get_batch(self, split):
        # We recreate np.memmap every batch to avoid a memory leak, as per
        # https://stackoverflow.com/questions/45132940/numpy-memmap-memory-usage-want-to-iterate-once/61472122#61472122
        fname = "train.bin" if split == "train" else "val.bin"
        data = np.memmap(os.path.join(self.data_dir, fname), dtype=np.uint16, mode="r")
        T = self.block_size
        ix = torch.randint(len(data) - T, (self.batch_size,), generator=self.gen)
        x = torch.stack([torch.from_numpy((data[i:i + T]).astype(np.int64)) for i in ix])
        y = torch.stack([torch.from_numpy((data[i + 1:i + 1 + T]).astype(np.int64)) for i in ix])
        return _to_device(x, y, self.device)


class NativeBatchSource:
    """C++ prefetching loader; one background sampler thread per split."""

    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            L = ctypes.CDLL(_RUNTIME_LIB)
            L.nsa_loader_create.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                            ctypes.c_int]
            L.nsa_loader_create.restype = ctypes.c_void_p
            L.nsa_loader_next.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            L.nsa_loader_next.restype = ctypes.c_int
            L.nsa_loader_num_tokens.argtypes = [ctypes.c_void_p]
            L.nsa_loader_num_tokens.restype = ctypes.c_int64
            L.nsa_loader_destroy.argtypes = [ctypes.c_void_p]
            L.nsa_loader_destroy.restype = None
            cls._lib = L
        return cls._lib

    @staticmethod
    def available():
        return os.path.exists(_RUNTIME_LIB)

    def __init__(self, data_dir, block_size, batch_size, device, seed=1337, prefetch=4):
        self.device = torch.device(device)
        self.block_size = block_size
        self.batch_size = batch_size
        L = self.lib()
        self._h = {}
        for i, split in enumerate(("train", "val")):
            path = os.path.join(data_dir, f"{split}.bin").encode()
            h = L.nsa_loader_create(path, block_size, batch_size, seed * 2 + i, prefetch)
            if not h:
                raise RuntimeError(f"native loader failed to open {path!r}")
            self._h[split] = h
        pin = self.device.type == "cuda"
        # two pinned staging slots per split so the H2D copy of batch k can be in
        # flight while batch k+1 is being staged
        self._slots = {s: [(torch.empty(batch_size, block_size, dtype=torch.int64).pin_memory() if pin else
                            torch.empty(batch_size, block_size, dtype=torch.int64),
                            torch.empty(batch_size, block_size, dtype=torch.int64).pin_memory() if pin else
                            torch.empty(batch_size, block_size, dtype=torch.int64)) for _ in range(2)]
                       for s in self._h}
        self._events = {s: [None, None] for s in self._h}
        self._turn = {s: 0 for s in self._h}

    def get_batch(self, split):
        k = self._turn[split]
        self._turn[split] ^= 1
        ev = self._events[split][k]
        if ev is not None:
            ev.synchronize()  # the H2D copy that last used this staging slot is done
        xs, ys = self._slots[split][k]
        rc = self.lib().nsa_loader_next(self._h[split], ctypes.c_void_p(xs.data_ptr()),
                                        ctypes.c_void_p(ys.data_ptr()))
        if rc != 0:
            raise RuntimeError("native loader failed")
        if self.device.type == "cuda":
            x = xs.to(self.device, non_blocking=True)
            y = ys.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._events[split][k] = ev
            return x, y
        return xs.clone(), ys.clone()

    def close(self):
        for h in self._h.values():
            self.lib().nsa_loader_destroy(h)
        self._h = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SyntheticBatchSource:
    """Uniform random tokens in [0, vocab) generated on the device (benchmarks)."""

    def __init__(self, vocab_size, block_size, batch_size, device, seed=1337):
        self.device = torch.device(device)
        self.vocab_size = vocab_size
        self.block_size = block_size
        self.batch_size = batch_size
        self.gen = torch.Generator(device=self.device).manual_seed(seed)

    def get_batch(self, split):
        d = torch.randint(0, self.vocab_size, (self.batch_size, self.block_size + 1), device=self.device,
                          generator=self.gen)
        return d[:, :-1].contiguous(), d[:, 1:].contiguous()


def make_batch_source(dataset, data_dir, block_size, batch_size, device, seed, vocab_size=50304, impl="auto"):
    if dataset == "synthetic":
        return SyntheticBatchSource(vocab_size, block_size, batch_size, device, seed)
    path = resolve_data_dir(dataset, data_dir)
    if impl == "native" or (impl == "auto" and NativeBatchSource.available()):
        return NativeBatchSource(path, block_size, batch_size, device, seed)
    return MemmapBatchSource(path, block_size, batch_size, device, seed)
