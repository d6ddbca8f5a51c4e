#!/usr/bin/env bash
# Kernel traces of one optimizer step for several bench configurations (rocprofv3
# --kernel-trace --stats), each under its own time limit, plus the per-step breakdown
# (scripts/step_breakdown.py) and the count of vendor-library (Cijk_*) dispatches.
#   usage: scripts/prof_models.sh "<label>|<seconds>|<bench.py args>" ...
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  label="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; args="${rest#*|}"
  out="$R/gpurun_out/prof_$label"
  echo "=== [$label] bench.py $args"
  timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
    python3 "$R/bench.py" $args > "$out.log" 2>&1
  rc=$?
  echo "=== [$label] rc=$rc"
  tail -n 2 "$out.log" | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  trace=$(ls "$out"/*/*/run_kernel_trace.csv "$out"/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 "$R/scripts/step_breakdown.py" "$trace" --top 40 > "$out.md" || exit 1
  echo "Cijk dispatches in the whole trace: $(grep -c Cijk_ "$trace" || true)" | tee -a "$out.md"
  head -n 3 "$out.md"
done
exit 0
