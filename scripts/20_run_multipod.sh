#!/usr/bin/env bash
# Topology B: StatefulSet of 8 single-GPU pods + headless Service (quick-start step 6, D5).
set -euo pipefail
cd "$(dirname "$0")/.."
kubectl -n disttrain apply -f k8s/services/41-train-mp-headless.yaml
kubectl -n disttrain apply -f k8s/statefulset/40-train-multipod.yaml
kubectl -n disttrain rollout status sts/train-multipod --timeout=15m
kubectl -n disttrain logs -f pod/train-multipod-0
