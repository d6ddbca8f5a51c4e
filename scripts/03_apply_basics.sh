#!/usr/bin/env bash
# Namespace, proxy ConfigMap, storage, dataset job (quick-start steps 3-4, D5).
set -euo pipefail
cd "$(dirname "$0")/.."
kubectl apply -f k8s/00-namespace.yaml
kubectl -n disttrain apply -f k8s/01-proxy-config.yaml
kubectl apply -f k8s/storage/
kubectl -n disttrain apply -f k8s/jobs/20-download-tiny-shakespeare.yaml
kubectl -n disttrain wait --for=condition=complete job/download-tiny-shakespeare --timeout=10m
