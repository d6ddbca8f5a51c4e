"""Build the native libraries in-tree (no JIT cache, so they travel with the repo).

* ``lib/libnsa_kernels.so`` — every ``csrc/kernels/*.hip`` compiled by
  ``hipcc --offload-arch=gfx950 -O3`` (CDNA4 only; no CUDA / multi-arch paths)
* ``lib/libnsa_runtime.so`` — the C++ host runtime (``csrc/runtime/*.cpp``:
  prefetching data loader), built with g++
* ``bin/rccl_bench`` — RCCL collective micro-benchmark (``csrc/comm/rccl_bench.cpp``)
  used to size DDP gradient buckets over xGMI

Usage: ``python -m nanosandbox_amd.build [--force] [--jobs N]``.
Objects are rebuilt only when a source or header is newer than the library.
"""

from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
LIB_DIR = os.path.join(ROOT, "nanosandbox_amd", "lib")
BUILD_DIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("NSA_OFFLOAD_ARCH", "gfx950")

KERNEL_LIB = os.path.join(LIB_DIR, "libnsa_kernels.so")
RUNTIME_LIB = os.path.join(LIB_DIR, "libnsa_runtime.so")
BIN_DIR = os.path.join(ROOT, "nanosandbox_amd", "bin")
RCCL_BENCH = os.path.join(BIN_DIR, "rccl_bench")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise FileNotFoundError("hipcc not found (ROCm 7.x expected under /opt/rocm)")


def _newer(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


# per-source compiler flags.  The attention kernels without the SLP vectorizer: it packed the
# softmax's adjacent f32 multiplies / adds into v_pk_*_f32, an anti-lever beside MFMAs
# (MI355X_MICROARCH.md 'price of one filler'; A/B: scripts/attn_ab.py against a variant
# library built with file_flags={}).
FILE_FLAGS = {"flash_attn.hip": ["-fno-slp-vectorize"], "flash_attn_f16.hip": ["-fno-slp-vectorize"]}


def build_kernels(force=False, jobs=8, verbose=True, defines=(), lib_path=KERNEL_LIB, obj_dir=BUILD_DIR,
                  file_flags=None):
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    if not force and not _newer(lib_path, srcs + headers + [os.path.abspath(__file__)]):
        return lib_path
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(lib_path), exist_ok=True)
    hipcc = _hipcc()
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
             "-munsafe-fp-atomics", "-I", os.path.join(CSRC, "kernels"), *[f"-D{d}" for d in defines]]

    def deps(src):
        # sources a kernel file #includes from this directory (flash_attn_f16.hip is
        # flash_attn.hip compiled again for fp16)
        out = []
        for line in open(src):
            if line.startswith('#include "') and line.rstrip().endswith('.hip"'):
                out.append(os.path.join(os.path.dirname(src), line.split('"')[1]))
        return out

    ff = FILE_FLAGS if file_flags is None else file_flags

    def compile_one(src):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if force or _newer(obj, [src] + headers + deps(src) + [os.path.abspath(__file__)]):
            _run([hipcc, *flags, *ff.get(os.path.basename(src), []), "-c", src, "-o", obj])
            if verbose:
                print(f"  [hipcc {ARCH}] {os.path.relpath(src, ROOT)}")
        return obj

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = lib_path + ".tmp"
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp])
    os.replace(tmp, lib_path)
    if verbose:
        print(f"built {os.path.relpath(lib_path, ROOT)}")
    return lib_path


def build_variant(name, defines, force=False, jobs=8, verbose=True, file_flags=None):
    """Build the kernel library with extra -D flags into ``build/variants/<name>/``.

    Used for A/B probes (``NSA_KERNEL_LIB=<path>`` selects it at import time), e.g.
    ``NSA_PROBE_DQ_STORE`` replaces the attention backward's dQ atomics by plain
    stores to measure what the atomics cost (wrong results; timing only).
    """
    vdir = os.path.join(ROOT, "build", "variants", name)
    return build_kernels(force=force, jobs=jobs, verbose=verbose, defines=defines,
                         lib_path=os.path.join(vdir, "libnsa_kernels.so"), obj_dir=os.path.join(vdir, "obj"),
                         file_flags=file_flags)


def build_runtime(force=False, verbose=True):
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return None
    if not force and not _newer(RUNTIME_LIB, srcs):
        return RUNTIME_LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    tmp = RUNTIME_LIB + ".tmp"
    _run([cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", *srcs, "-o", tmp])
    os.replace(tmp, RUNTIME_LIB)
    if verbose:
        print(f"built {os.path.relpath(RUNTIME_LIB, ROOT)}")
    return RUNTIME_LIB


def build_tools(force=False, verbose=True):
    """Native command-line tools (host code linked against RCCL / the HIP runtime)."""
    src = os.path.join(CSRC, "comm", "rccl_bench.cpp")
    if not os.path.exists(src):
        return None
    if not force and not _newer(RCCL_BENCH, [src]):
        return RCCL_BENCH
    os.makedirs(BIN_DIR, exist_ok=True)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    tmp = RCCL_BENCH + ".tmp"
    _run([_hipcc(), "-O2", "-std=c++17", "-I", os.path.join(rocm, "include"), src, "-L", os.path.join(rocm, "lib"),
          "-lrccl", f"-Wl,-rpath,{os.path.join(rocm, 'lib')}", "-o", tmp])
    os.replace(tmp, RCCL_BENCH)
    if verbose:
        print(f"built {os.path.relpath(RCCL_BENCH, ROOT)}")
    return RCCL_BENCH


def build_all(force=False, jobs=8, verbose=True):
    build_runtime(force=force, verbose=verbose)
    build_tools(force=force, verbose=verbose)
    return build_kernels(force=force, jobs=jobs, verbose=verbose)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--variant", nargs="+", metavar=("NAME", "DEFINE"),
                    help="build an A/B probe variant: NAME followed by preprocessor defines")
    ap.add_argument("--no-file-flags", action="store_true",
                    help="with --variant: compile every source with the common flags only (no FILE_FLAGS)")
    a = ap.parse_args(argv)
    if a.variant:
        print(build_variant(a.variant[0], a.variant[1:], force=a.force, jobs=a.jobs,
                            file_flags={} if a.no_file_flags else None))
        return 0
    build_all(force=a.force, jobs=a.jobs)


if __name__ == "__main__":
    sys.exit(main())
