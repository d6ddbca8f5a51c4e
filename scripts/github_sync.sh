#!/usr/bin/env bash
# Upsert the project's labels and backlog issues on GitHub with the `gh` CLI
# (reference P7 is a PowerShell script doing the same; this is the bash form).
#   scripts/github_sync.sh            # apply
#   DRY_RUN=1 scripts/github_sync.sh  # print what would be done
set -euo pipefail
cd "$(dirname "$0")/.."

slug() {
  local url
  url="$(git config --get remote.origin.url)" || { echo "no origin remote" >&2; exit 1; }
  url="${url%.git}"
  echo "${url#*github.com[:/]}"
}

run() { if [[ -n "${DRY_RUN:-}" ]]; then echo "+ $*"; else "$@"; fi; }

REPO="${REPO:-$(slug)}"

ensure_label() {  # name color description
  if gh api "repos/$REPO/labels/$(printf '%s' "$1" | jq -sRr @uri)" >/dev/null 2>&1; then
    run gh api -X PATCH "repos/$REPO/labels/$(printf '%s' "$1" | jq -sRr @uri)" -f color="$2" -f description="$3" >/dev/null
  else
    run gh api -X POST "repos/$REPO/labels" -f name="$1" -f color="$2" -f description="$3" >/dev/null
  fi
}

ensure_issue() {  # title labels body
  if gh issue list -R "$REPO" --state all --search "in:title \"$1\"" --json title -q '.[].title' | grep -Fxq "$1"; then
    echo "exists: $1"
  else
    run gh issue create -R "$REPO" --title "$1" --label "$2" --body "$3"
  fi
}

while IFS='|' read -r name color desc; do
  [[ -z "$name" ]] && continue
  ensure_label "$name" "$color" "$desc"
done <<'LABELS'
type:bug|d73a4a|Something is broken
type:feature|a2eeef|New capability
type:task|c5def5|Scoped work item
type:docs|0075ca|Documentation
status:triage|fbca04|Needs triage
status:blocked|b60205|Blocked
status:in-progress|0e8a16|Being worked on
priority:P0|b60205|Drop everything
priority:P1|d93f0b|Next up
priority:P2|fbca04|Planned
priority:P3|c2e0c6|Nice to have
size:S|ededed|< 1 day
size:M|d4c5f9|1-3 days
size:L|bfd4f2|1-2 weeks
size:XL|5319e7|Multi-week
area:kernels|1d76db|gfx950 HIP kernels (attention, GEMM, LN, GELU, xent, AdamW)
area:model|0052cc|GPT model / training loop
area:distributed|5319e7|RCCL, reducer, rendezvous
area:data|006b75|Datasets, loaders
area:k8s|0e8a16|Manifests, StatefulSet, Jobs
area:docker|c2e0c6|Training image
area:docs|0075ca|Docs and playbook
area:ci|bfdadc|Lint and CI
area:perf|e99695|Throughput / MFU / scaling
area:storage|f9d0c4|PV/PVC, checkpoints
area:observability|fef2c0|Metrics, tfevents, profiling
area:security|b60205|Secrets, proxy
good-first-issue|7057ff|Small and well scoped
LABELS

ensure_issue "Bring up k3s with the AMD GPU device plugin" "type:task,area:k8s,priority:P0,size:M" \
  "Acceptance: scripts/01_install_k3s_amd_gpu.sh leaves amd.com/gpu allocatable on the node."
ensure_issue "ROCm training image (gfx950)" "type:task,area:docker,priority:P0,size:M" \
  "Acceptance: docker/Dockerfile builds, kernels compile for gfx950, image imported into k3s containerd."
ensure_issue "PV/PVC for datasets, checkpoints and runs" "type:task,area:storage,priority:P0,size:S" \
  "Acceptance: disttrain-pvc Bound and mounted at /data in every Pod."
ensure_issue "tiny-shakespeare download Job" "type:task,area:data,priority:P1,size:S" \
  "Acceptance: /data/datasets/shakespeare_char/{train,val}.bin and meta.pkl written; kubectl wait succeeds."
ensure_issue "Single-Pod 8-GPU training Job" "type:task,area:k8s,priority:P0,size:M" \
  "Acceptance: torchrun --standalone --nproc_per_node=8 trains GPT-2 124M; logs via kubectl logs."
ensure_issue "Multi-Pod StatefulSet (8 x 1 GPU)" "type:task,area:distributed,priority:P1,size:L" \
  "Acceptance: ordinal -> NODE_RANK, c10d rendezvous through the headless Service, rank-0 logs."
ensure_issue "TensorBoard events under /data/runs" "type:feature,area:observability,priority:P2,size:S" \
  "Acceptance: tfevents written by the trainer; tensorboard --logdir /data/runs shows loss/lr/mfu."
ensure_issue "OpenWebText subset dataset Job" "type:feature,area:data,priority:P2,size:M" \
  "Acceptance: configurable-size tokenized subset written to the PVC."
ensure_issue "RCCL presets and bucket sizing over xGMI" "type:task,area:perf,priority:P1,size:M" \
  "Acceptance: docs/rccl.md presets; rccl_bench recommendation used as ddp_bucket_mb."
ensure_issue "CI: lint manifests and scripts" "type:task,area:ci,priority:P2,size:S" \
  "Acceptance: .github/workflows/lint.yml runs manifest tests, bash -n and the CPU test-suite."
ensure_issue "Playbook: architecture, runbook, pitfalls" "type:docs,area:docs,priority:P2,size:S" \
  "Acceptance: docs/playbook.md covers both topologies, the runbook and known pitfalls."
