"""Load pre-tuned hipBLASLt / rocBLAS solution picks for the library GEMMs.

The plain forward / input-grad GEMMs stay on the vendor library (the autotuner in
``gemm_tune`` keeps them there where our MFMA kernel is slower).  torch's default
heuristic pick is not always the fastest solution for GPT-2's tall-skinny shapes
(M = 61k-123k tokens, N/K = 768-50304), so ``scripts/tune_blas.py`` searches the
solutions with PyTorch TunableOp, keeps only the shapes where the tuned pick
measured faster in the same process, and writes them to ``tuned/*.csv``.

``enable()`` loads that file with tuning OFF: shapes in the file use the recorded
solution, every other GEMM keeps torch's default (TunableOp falls back to it when
a shape has no entry).  The file carries TunableOp's validator lines (torch /
HIP / hipBLASLt / rocBLAS versions, gfx arch); on a mismatch TunableOp ignores it.
Set ``NSA_TUNED_BLAS=0`` to disable, ``NSA_TUNED_BLAS_FILE`` to load another table.
"""

from __future__ import annotations

import os

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_FILE = os.path.join(_HERE, "tuned", "gfx950_gpt2.csv")
_enabled = False


def enable(path: str | None = None) -> bool:
    """Turn on TunableOp in replay-only mode with the in-tree solution table."""
    global _enabled
    if _enabled:
        return True
    if os.environ.get("NSA_TUNED_BLAS", "1") == "0":
        return False
    path = path or os.environ.get("NSA_TUNED_BLAS_FILE") or DEFAULT_FILE
    if not os.path.exists(path):
        return False
    import torch

    if not torch.cuda.is_available() or torch.version.hip is None:
        return False
    import torch.cuda.tunable as tn

    with open(path) as f:
        if not any(not line.startswith("Validator") for line in f if line.strip()):
            return False  # validators only: nothing to replay
    tn.enable(True)
    tn.tuning_enable(False)
    tn.record_untuned_enable(False)
    tn.set_filename(os.path.join("/tmp", f"nsa_tunableop_{os.getpid()}.csv"))
    ok = tn.read_file(path)
    if not ok:
        tn.enable(False)
        return False
    _enabled = True
    return True
