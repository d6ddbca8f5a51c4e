#!/usr/bin/env bash
# Build stand-alone copies of an NT GEMM source with compile-time knobs, for A/B timing in
# one process (scripts/gemm_nt_ab.py --alt NAME=PATH; the script calls nsa_gemm_nt4 when the
# library exports it, else nsa_gemm_nt).
#   usage: [SRC=csrc/kernels/gemm_nt4.hip] scripts/build_nt_variants.sh NAME "-DFLAG=V ..." [NAME FLAGS ...]
set -eu
cd "$(dirname "$0")/.."
SRC=${SRC:-csrc/kernels/gemm_nt.hip}
mkdir -p build/ntvar
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags -Icsrc/kernels \
    "$SRC" -o build/ntvar/libnt_$name.so &
done
wait
ls -la build/ntvar
