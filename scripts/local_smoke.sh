#!/usr/bin/env bash
# The reference's Colab companion without Colab or k8s (P2-P6, nb:27-119):
# prepare the char dataset, 1-process CPU smoke, then an N-process gloo run on
# one machine through the same container entrypoint the pods use.
#   bash scripts/local_smoke.sh [NPROC]
set -euo pipefail
cd "$(dirname "$0")/.."
NPROC="${1:-2}"
WORK="${WORK:-/tmp/disttrain-smoke}"
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
python3 -m nanosandbox_amd.data.prepare char --out "$WORK/datasets/shakespeare_char"
python3 train.py config/smoke_cpu.py --data_dir="$WORK/datasets" --out_dir="$WORK/cpu"
NPROC_PER_NODE="$NPROC" container/entrypoint.sh train.py config/smoke_cpu.py \
  --data_dir="$WORK/datasets" --out_dir="$WORK/ddp" --gradient_accumulation_steps="$NPROC" --max_iters=20
