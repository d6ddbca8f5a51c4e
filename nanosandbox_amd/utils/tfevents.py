"""Minimal TensorBoard event-file writer (scalars only), no tensorboard dependency.

The reference claims TensorBoard logs under ``/data/runs`` (README.md:74-87,
notebooks/colab_nanoGPT_companion.ipynb:127) but upstream nanoGPT never writes
any.  tensorboard is not installed in this image, so we
emit the on-disk format directly:

record := uint64 len | uint32 masked_crc32c(len) | bytes data | uint32 masked_crc32c(data)
data   := serialized ``tensorflow.Event`` {1: wall_time double, 2: step int64,
          3: file_version string | 5: Summary{1: repeated Value{1: tag, 2: simple_value float}}}
"""

from __future__ import annotations

import os
import socket
import struct
import time

_CRC_TABLE = []


def _make_table():
    poly = 0x82F63B78  # CRC-32C (Castagnoli), reflected
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        _CRC_TABLE.append(c)


_make_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _CRC_TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field_bytes(num: int, payload: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def _event(wall_time: float, step: int, *, file_version: str = None, summary: bytes = None) -> bytes:
    out = _varint((1 << 3) | 1) + struct.pack("<d", wall_time)
    out += _varint((2 << 3) | 0) + _varint(step)
    if file_version is not None:
        out += _field_bytes(3, file_version.encode())
    if summary is not None:
        out += _field_bytes(5, summary)
    return out


def _scalar_summary(tag: str, value: float) -> bytes:
    val = _field_bytes(1, tag.encode()) + _varint((2 << 3) | 5) + struct.pack("<f", float(value))
    return _field_bytes(1, val)


class EventWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        fname = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}"
        self.path = os.path.join(logdir, fname)
        self._f = open(self.path, "wb")
        self._write(_event(time.time(), 0, file_version="brain.Event:2"))

    def _write(self, data: bytes):
        header = struct.pack("<Q", len(data))
        self._f.write(header + struct.pack("<I", masked_crc32c(header)) + data +
                      struct.pack("<I", masked_crc32c(data)))

    def add_scalar(self, tag: str, value: float, step: int):
        self._write(_event(time.time(), int(step), summary=_scalar_summary(tag, value)))

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


def read_events(path: str):
    """Decode scalar events written by EventWriter (used by tests): [(step, tag, value)]."""
    out = []
    with open(path, "rb") as f:
        buf = f.read()
    pos = 0
    while pos < len(buf):
        (n,) = struct.unpack_from("<Q", buf, pos)
        hcrc = struct.unpack_from("<I", buf, pos + 8)[0]
        assert hcrc == masked_crc32c(buf[pos:pos + 8]), "header crc mismatch"
        data = buf[pos + 12:pos + 12 + n]
        dcrc = struct.unpack_from("<I", buf, pos + 12 + n)[0]
        assert dcrc == masked_crc32c(data), "data crc mismatch"
        pos += 16 + n
        out.extend(_decode_event(data))
    return out


def _read_varint(b, i):
    shift = 0
    val = 0
    while True:
        c = b[i]
        i += 1
        val |= (c & 0x7F) << shift
        if not c & 0x80:
            return val, i
        shift += 7


def _fields(b):
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        else:
            raise ValueError(f"wire type {wt}")
        yield num, wt, v


def _decode_event(data):
    step = 0
    res = []
    for num, wt, v in _fields(data):
        if num == 2:
            step = v
        elif num == 5:
            for vn, _, val in _fields(v):
                if vn != 1:
                    continue
                tag, sv = None, None
                for fn, _, fv in _fields(val):
                    if fn == 1:
                        tag = fv.decode()
                    elif fn == 2:
                        sv = struct.unpack("<f", fv)[0]
                res.append((tag, sv))
    return [(step, t, v) for t, v in res]
