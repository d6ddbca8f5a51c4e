#!/usr/bin/env bash
# Topology A: single pod, 8 GPUs, torchrun --standalone (quick-start step 5).
set -euo pipefail
cd "$(dirname "$0")/.."
kubectl -n disttrain apply -f k8s/jobs/30-train-singlepod.yaml
kubectl -n disttrain logs -f job/train-singlepod
