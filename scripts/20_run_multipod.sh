#!/usr/bin/env bash
# Topology B: StatefulSet of 8 single-GPU pods + headless Service (quick-start step 6, D5).
#   scripts/20_run_multipod.sh          RCCL SHM through host memory (40-train-multipod.yaml)
#   scripts/20_run_multipod.sh xgmi     every pod mounts all GPUs of the node, RCCL P2P over
#                                       xGMI (42-train-multipod-xgmi.yaml; docs/rccl.md)
set -euo pipefail
cd "$(dirname "$0")/.."
if [[ "${1:-shm}" == "xgmi" ]]; then
  kubectl -n disttrain apply -f k8s/statefulset/42-train-multipod-xgmi.yaml
  kubectl -n disttrain rollout status sts/train-multipod-xgmi --timeout=15m
  kubectl -n disttrain logs -f pod/train-multipod-xgmi-0
else
  kubectl -n disttrain apply -f k8s/services/41-train-mp-headless.yaml
  kubectl -n disttrain apply -f k8s/statefulset/40-train-multipod.yaml
  kubectl -n disttrain rollout status sts/train-multipod --timeout=15m
  kubectl -n disttrain logs -f pod/train-multipod-0
fi
