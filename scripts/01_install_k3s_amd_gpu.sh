#!/usr/bin/env bash
# Install k3s and expose the node's MI355X GPUs as `amd.com/gpu`.
# Reference: k3s + NVIDIA GPU Operator (README.md:28-32).  Here: the ROCm k8s
# device plugin (DaemonSet) on a host that already has the amdgpu driver + ROCm.
#   sudo -E bash scripts/01_install_k3s_amd_gpu.sh
set -euo pipefail
K3S_VERSION="${K3S_VERSION:-v1.30.4+k3s1}"
PLUGIN_MANIFEST="${PLUGIN_MANIFEST:-https://raw.githubusercontent.com/ROCm/k8s-device-plugin/master/k8s-ds-amdgpu-dp.yaml}"

command -v rocm-smi >/dev/null || { echo "ROCm driver stack not found (rocm-smi)"; exit 1; }
rocm-smi --showproductname | grep -qi "MI355" || echo "warning: no MI355X reported by rocm-smi"
if ! command -v k3s >/dev/null; then
  curl -sfL https://get.k3s.io | INSTALL_K3S_VERSION="$K3S_VERSION" sh -s - --write-kubeconfig-mode 644
fi
export KUBECONFIG=/etc/rancher/k3s/k3s.yaml
kubectl apply -f "$PLUGIN_MANIFEST"
kubectl -n kube-system rollout status ds/amdgpu-device-plugin-daemonset --timeout=300s
kubectl get nodes -o jsonpath='{.items[*].status.allocatable.amd\.com/gpu}'; echo " amd.com/gpu allocatable"
