#!/usr/bin/env bash
# Run a sequence of GPU steps on the gpurun box, each under its own time limit.
# A step that fails an assertion (exit 1-127 from pytest/python) lets the session
# continue; a timeout (124/137), abort (134), segfault (139) or any signal exit
# stops the session so nothing else touches a possibly-faulted GPU.
#   usage: scripts/gpu_session.sh "<label>|<seconds>|<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  label="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$label] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== [$label] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$label.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping session after [$label] (rc=$rc)"
    exit $rc
  fi
done
exit 0
