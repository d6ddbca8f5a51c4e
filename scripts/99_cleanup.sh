#!/usr/bin/env bash
# Ordered teardown (D18, README.md:105-114).
set -uo pipefail
cd "$(dirname "$0")/.."
kubectl -n disttrain delete job/download-tiny-shakespeare --ignore-not-found
kubectl -n disttrain delete job/prepare-owt-subset --ignore-not-found
kubectl -n disttrain delete job/train-singlepod --ignore-not-found
kubectl -n disttrain delete sts/train-multipod --ignore-not-found
kubectl -n disttrain delete -f k8s/statefulset/42-train-multipod-xgmi.yaml --ignore-not-found
kubectl -n disttrain delete -f k8s/services/41-train-mp-headless.yaml --ignore-not-found
kubectl delete -f k8s/storage/ --ignore-not-found
kubectl delete ns disttrain --ignore-not-found
