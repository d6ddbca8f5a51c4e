#!/usr/bin/env bash
# Memory-side PMC of the whole GPT-2 124M step (one warm-up + one timed step): FETCH_SIZE and
# WRITE_SIZE per dispatch, in two passes (TCC block: at most 4 counters; FETCH_SIZE uses 3,
# WRITE_SIZE 2), for the LayerNorm bytes-per-element accounting.
#   summaries: python scripts/pmc_summary.py gpurun_out/pmcl/**/*_counter_collection.csv --match ln_
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pmcl
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcl -o f -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pmcl1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcl -o w -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pmcl2.log 2>&1
