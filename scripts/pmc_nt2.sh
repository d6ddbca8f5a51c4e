#!/usr/bin/env bash
# Two PMC passes (cycles + MFMA busy, memory pipe) for several NT-GEMM probes.
# usage: scripts/pmc_nt2.sh <outdir> "<probe list>" <gemm_nt_prof.py args...>
set -u
out="$1"; probes="$2"; shift 2
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
for pr in $probes; do
  d="$R/$out/probe$pr"
  mkdir -p "$d"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$d/p1" -o pmc -- python3 "$R/scripts/gemm_nt_prof.py" --probe "$pr" "$@" > "$d/p1.log" 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$d/p2" -o pmc -- python3 "$R/scripts/gemm_nt_prof.py" --probe "$pr" "$@" > "$d/p2.log" 2>&1 || exit $?
  echo "probe $pr done"
done
