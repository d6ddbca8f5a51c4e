#!/usr/bin/env bash
# PMC passes over the NT GEMM: one rocprofv3 run per counter group, each under its own
# time limit (rocprofv3 does not split counters over passes; per-block slot limits:
# SQ 8, TA 2, TD 2, TCP 4, GRBM 2).
# usage: scripts/pmc_nt.sh <outdir> <gemm_nt_prof.py args...>
set -u
out="$1"; shift
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/$out"
groups=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT"
  "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU SQ_VALU_MFMA_COEXEC_CYCLES"
)
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$R/$out/p$i" -o pmc -- python3 "$R/scripts/gemm_nt_prof.py" "$@" > "$R/$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
