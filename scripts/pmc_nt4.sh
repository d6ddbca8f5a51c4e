#!/usr/bin/env bash
# PMC groups (scripts/pmc_nt.sh) for the four-wave NT kernel and its no-DMA probe on one shape.
# usage: scripts/pmc_nt4.sh <outdir> <gemm_nt_prof.py shape args...>
set -u
out="$1"; shift
R="${GRAFT_REPO_ROOT:-/root/repo}"
bash "$R/scripts/pmc_nt.sh" "$out/nt4" --w4 --probe 0 "$@" || exit $?
bash "$R/scripts/pmc_nt.sh" "$out/nt4nodma" --w4 --probe 1 "$@" || exit $?
exit 0
