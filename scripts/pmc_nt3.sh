#!/usr/bin/env bash
# PMC groups (scripts/pmc_nt.sh) for the NT kernel, its no-DMA probe and torch's matmul (yardstick) on one shape.
# usage: scripts/pmc_nt3.sh <outdir> <gemm_nt_prof.py shape args...>
set -u
out="$1"; shift
R="${GRAFT_REPO_ROOT:-/root/repo}"
bash "$R/scripts/pmc_nt.sh" "$out/nt" --probe 0 "$@" || exit $?
bash "$R/scripts/pmc_nt.sh" "$out/nodma" --probe 1 "$@" || exit $?
bash "$R/scripts/pmc_nt.sh" "$out/lib" --lib "$@" || exit $?
exit 0
