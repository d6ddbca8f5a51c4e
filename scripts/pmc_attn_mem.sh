#!/usr/bin/env bash
# Memory-side PMC passes for the flash-attention kernels at the GPT-2 training shape:
# FETCH_SIZE (L2 -> fabric reads: Infinity-Cache hits and HBM), L2 hit/miss, kernel clock.
# Each pass is its own rocprofv3 run (TCC block: at most 4 counters; FETCH_SIZE uses 3).
#   usage: PMC_ATTN_ARGS="..." scripts/pmc_attn_mem.sh
# summaries: python scripts/pmc_summary.py gpurun_out/pmcm/**/*_counter_collection.csv --match flash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pmcm
ARGS=${PMC_ATTN_ARGS:---rounds 1 --iters 2}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcm -o m1 -- python3 scripts/attn_ab.py $ARGS > gpurun_out/pmcm1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmcm -o m2 -- python3 scripts/attn_ab.py $ARGS > gpurun_out/pmcm2.log 2>&1
