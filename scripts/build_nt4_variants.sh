#!/usr/bin/env bash
# Stand-alone builds of csrc/kernels/gemm_nt4.hip with compile-time knobs (A/B in one
# process: scripts/gemm_nt_ab.py --alt4 NAME=PATH).
#   usage: scripts/build_nt4_variants.sh NAME "-DNT4_DMA_EARLY=0" [NAME FLAGS ...]
set -eu
cd "$(dirname "$0")/.."
mkdir -p build/ntvar
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags -Icsrc/kernels \
    csrc/kernels/gemm_nt4.hip -o build/ntvar/libnt4_$name.so &
done
wait
