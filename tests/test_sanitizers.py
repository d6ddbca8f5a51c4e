"""Host-code sanitizers: the native prefetching data loader
(csrc/runtime/dataloader.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer and
under ThreadSanitizer, driven by csrc/runtime/tests/loader_stress.cpp (window contents,
shutdown while the producer thread is mid-fill or blocked, loaders on several threads).

GPU code is not sanitized here: device ASan / XNACK runs are not available on the
MI355X pool; kernels are checked against fp32 references instead (tests/*_gpu.py).
"""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "csrc", "runtime", "dataloader.cpp"),
       os.path.join(ROOT, "csrc", "runtime", "tests", "loader_stress.cpp")]


def _build_and_run(tmp_path, flags, env=None):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "loader_stress")
    r = subprocess.run([cxx, "-O1", "-g", "-std=c++17", "-pthread", *flags, *SRC, "-o", exe],
                       capture_output=True, text=True)
    if r.returncode != 0:
        if "cannot find" in r.stderr or "unrecognized" in r.stderr:
            pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-200:]}")
        raise AssertionError(r.stderr)
    run = subprocess.run([exe, str(tmp_path / "tokens.bin")], capture_output=True, text=True, timeout=300,
                         env={**os.environ, **(env or {})})
    assert run.returncode == 0, run.stdout + run.stderr
    assert "loader_stress: ok" in run.stdout
    return run


def test_loader_asan_ubsan(tmp_path):
    run = _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                                    "-fno-sanitize-recover=undefined"],
                         env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1"})
    assert "ERROR: AddressSanitizer" not in run.stderr


def test_loader_tsan(tmp_path):
    run = _build_and_run(tmp_path, ["-fsanitize=thread"], env={"TSAN_OPTIONS": "halt_on_error=1"})
    assert "WARNING: ThreadSanitizer" not in run.stderr
