#!/usr/bin/env bash
# PMC counters for weight-gradient GEMM kernels (two passes within the per-block counter
# limits); WGRAD_ARGS selects shapes / candidates of scripts/wgrad_ab.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pmcg
ARGS=${WGRAD_ARGS:---shapes c_fc --only nsa7/s7,nsa11/s7 --rounds 1 --reps 2}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcg -o p1 -- python3 scripts/wgrad_ab.py $ARGS > gpurun_out/pmcg1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcg -o p2 -- python3 scripts/wgrad_ab.py $ARGS > gpurun_out/pmcg2.log 2>&1
