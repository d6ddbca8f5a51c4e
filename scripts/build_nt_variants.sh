#!/usr/bin/env bash
# Build stand-alone copies of the NT GEMM (csrc/kernels/gemm_nt.hip) with compile-time
# knobs, for A/B timing in one process (scripts/gemm_nt_ab.py --alt NAME=PATH).
#   usage: scripts/build_nt_variants.sh NAME "-DNSA_NT_DEF=2 -DNSA_NT_RPP=1" [NAME FLAGS ...]
set -eu
cd "$(dirname "$0")/.."
mkdir -p build/ntvar
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags -Icsrc/kernels \
    csrc/kernels/gemm_nt.hip -o build/ntvar/libnt_$name.so &
done
wait
ls -la build/ntvar
