"""Box calibration for the bench record: GPU clocks and a fixed calibration GEMM.

Two boxes running the same tree differ by a few percent (MI355X_MICROARCH.md 'DVFS
give-back' item 5: devices hold different clocks under load), which is as large as one
round's code gains.  bench.py therefore records, beside its timed steps:

* ``read_clocks()``: the current / top shader (sclk) and memory (mclk) clock levels from
  the amdgpu sysfs DPM tables (``pp_dpm_sclk`` / ``pp_dpm_mclk``, the ``*`` line is the
  level in use), read before and after the timed loop.  sysfs is what an unprivileged
  process can read on the box; ``amd-smi`` / ``rocm-smi`` are tried only as a fallback.
  These are DPM levels, not the in-kernel clock (the guide: up to ~10 % above it).
* ``calibration_gemm(seconds)``: our own persistent NT GEMM (``gemm_nt4.hip``) on one fixed
  shape (M = 16384, N = K = 4096, gaussian bf16 operands) launched back to back for a fixed
  wall time; TF/s of that loop.  The same binary on the same shape on every box, so the
  ratio of two boxes' calibration TF/s separates box speed from code speed.
"""

from __future__ import annotations

import glob
import json
import os
import re
import shutil
import subprocess
import time

CAL_SHAPE = (16384, 4096, 4096)  # M, N, K


def _dpm(path: str) -> dict | None:
    """Parse one pp_dpm_* table: {'cur_mhz': level marked '*', 'max_mhz': top level}."""
    try:
        with open(path) as f:
            lines = f.read().splitlines()
    except OSError:
        return None
    levels, cur = [], None
    for ln in lines:
        m = re.match(r"\s*\d+:\s*(\d+)\s*[Mm]hz\s*(\*)?", ln)
        if m:
            v = int(m.group(1))
            levels.append(v)
            if m.group(2):
                cur = v
    if not levels:
        return None
    return {"cur_mhz": cur, "max_mhz": max(levels)}


def _card_for_device(index: int) -> str | None:
    """sysfs device directory of the index-th amdgpu card that has DPM tables (the same
    order as HIP's device enumeration on a box with one visible GPU; with several it is
    the PCI order, which HIP also uses by default)."""
    cards = sorted(d for d in glob.glob("/sys/class/drm/card*/device") if os.path.exists(os.path.join(d, "pp_dpm_sclk")))
    if not cards:
        return None
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis and len(cards) > 1:
        try:
            index = [int(v) for v in vis.split(",") if v.strip()][index]
        except (ValueError, IndexError):
            pass
    return cards[index] if index < len(cards) else cards[0]


def _smi_clocks() -> dict | None:
    """Fallback: amd-smi's current clocks (JSON), when sysfs has no DPM table."""
    exe = shutil.which("amd-smi")
    if not exe:
        return None
    try:
        r = subprocess.run([exe, "metric", "-c", "--json"], capture_output=True, text=True, timeout=10)
        data = json.loads(r.stdout)
    except (OSError, ValueError, subprocess.TimeoutExpired):
        return None
    try:
        clk = (data[0] if isinstance(data, list) else data)["clock"]
        out = {}
        for key, name in (("gfx_0", "sclk"), ("mem_0", "mclk")):
            c = clk.get(key, {})
            v = c.get("clk", {}).get("value") if isinstance(c.get("clk"), dict) else c.get("clk")
            if v is not None:
                out[name] = {"cur_mhz": int(float(v)), "max_mhz": None}
        return out or None
    except (KeyError, TypeError, ValueError, IndexError):
        return None


def read_clocks(device_index: int = 0) -> dict:
    """{'sclk': {'cur_mhz', 'max_mhz'}, 'mclk': {...}, 'source': ...}; fields None when the
    box exposes nothing (the record then says so instead of guessing)."""
    card = _card_for_device(device_index)
    if card:
        out = {"sclk": _dpm(os.path.join(card, "pp_dpm_sclk")), "mclk": _dpm(os.path.join(card, "pp_dpm_mclk")),
               "source": "sysfs:" + os.path.basename(os.path.dirname(card))}
        if out["sclk"] is not None:
            return out
    smi = _smi_clocks()
    if smi:
        return {"sclk": smi.get("sclk"), "mclk": smi.get("mclk"), "source": "amd-smi"}
    return {"sclk": None, "mclk": None, "source": None}


def calibration_gemm(seconds: float = 2.0, device=None) -> dict:
    """TF/s of our NT GEMM on CAL_SHAPE, launched back to back for ``seconds`` of wall time
    (a few untimed launches first).  Random gaussian operands: zeros run at a higher clock
    (MI355X_MICROARCH.md 'DVFS give-back' item 1).  The kernel configuration is pinned (the
    overlapped epilogue off, as in every record before it existed), so the figure measures the
    box and stays comparable across code changes."""
    import torch

    from ..ops import gemm as _gemm

    M, N, K = CAL_SHAPE
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(1234)
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
    b = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        _gemm.nt(a, b, out=out, ovl=2)
    torch.cuda.synchronize(dev)
    # size a batch of launches to ~0.1 s so the host loop is not what is timed
    t0 = time.perf_counter()
    for _ in range(5):
        _gemm.nt(a, b, out=out, ovl=2)
    torch.cuda.synchronize(dev)
    per = max((time.perf_counter() - t0) / 5, 1e-6)
    batch = max(1, int(0.1 / per))
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(batch):
            _gemm.nt(a, b, out=out, ovl=2)
        n += batch
        torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    del a, b, out
    return {"kernel": "gemm_nt4", "ovl": "off", "shape_mnk": [M, N, K], "launches": n, "seconds": round(dt, 3),
            "tflops": round(2.0 * M * N * K * n / dt / 1e12, 1)}
