#!/usr/bin/env bash
# Pod entrypoint: derive the node rank and launch torchrun.
#
# Reference behaviour (README.md:21,102): in the multi-Pod StatefulSet the pod
# ordinal becomes NODE_RANK (train-multipod-3 -> 3) and every pod rendezvouses
# with pod 0 through the headless Service.  Single-Pod jobs use --standalone.
#
# Environment (all optional):
#   NNODES          number of pods (1 = single-Pod topology)          [1]
#   NPROC_PER_NODE  processes (= GPUs) per pod                         [1]
#   NODE_RANK       explicit rank; default: ordinal suffix of POD_NAME/HOSTNAME
#   MASTER_ADDR     rendezvous host, e.g. train-multipod-0.train-mp-headless
#   MASTER_PORT     rendezvous port                                    [29500]
#   RDZV_BACKEND    static (MASTER_ADDR/PORT + node_rank) | c10d         [static]
#   RDZV_ID         c10d job id                                        [disttrain]
#   MAX_RESTARTS    torchrun --max-restarts (elastic recovery)         [0]
#   NSA_RCCL_PRESET xgmi (single node, P2P) | xgmi-pods (one GPU per pod, every GPU of
#                   the node mounted: P2P) | shm | socket (pods without shared IPC)
#   NSA_DEVICE_SELECT ordinal: this pod's GPU is NODE_RANK mod NSA_GPUS_PER_NODE
#                   (exported as NSA_LOCAL_DEVICE, read by init_distributed) instead of
#                   LOCAL_RANK; for pods that see every GPU of the node (xgmi-pods)
#   NSA_DRY_RUN=1   print the torchrun command instead of running it
# Arguments: the training command after torchrun, e.g. train.py config/x.py --k=v
set -euo pipefail

NNODES="${NNODES:-1}"
NPROC_PER_NODE="${NPROC_PER_NODE:-1}"
MASTER_PORT="${MASTER_PORT:-29500}"
RDZV_BACKEND="${RDZV_BACKEND:-static}"
RDZV_ID="${RDZV_ID:-disttrain}"
MAX_RESTARTS="${MAX_RESTARTS:-0}"

ordinal_of() {
  local host="$1"
  if [[ "$host" =~ -([0-9]+)$ ]]; then
    echo "${BASH_REMATCH[1]}"
  else
    echo ""
  fi
}

if [[ -z "${NODE_RANK:-}" ]]; then
  host="${POD_NAME:-${HOSTNAME:-$(hostname)}}"
  NODE_RANK="$(ordinal_of "$host")"
  if [[ -z "$NODE_RANK" ]]; then
    if [[ "$NNODES" != "1" ]]; then
      echo "entrypoint: cannot derive NODE_RANK from hostname '$host' (expected <name>-<ordinal>)" >&2
      exit 2
    fi
    NODE_RANK=0
  fi
fi
export NODE_RANK

# RCCL transport preset: xGMI P2P inside one pod; socket fallback across pods
# that do not share IPC (the reference's NCCL_IB_DISABLE/NCCL_SOCKET_IFNAME).
#   xgmi   all ranks in one pod: RCCL P2P over xGMI
#   shm    pods of one node sharing the host /dev/shm (hostIPC + hostPath) and one
#          NCCL_HOSTID: RCCL SHM through host memory (no peer GPU access across pods)
#   socket pods that share nothing: TCP (the reference's NCCL_IB_DISABLE / SOCKET_IFNAME)
case "${NSA_RCCL_PRESET:-xgmi}" in
  socket)
    export NCCL_IB_DISABLE="${NCCL_IB_DISABLE:-1}"
    export NCCL_SOCKET_IFNAME="${NCCL_SOCKET_IFNAME:-eth0}"
    ;;
  shm|xgmi-pods)
    export NCCL_SHM_DISABLE="${NCCL_SHM_DISABLE:-0}"
    if [[ -z "${NCCL_HOSTID:-}" ]]; then
      echo "entrypoint: WARNING NSA_RCCL_PRESET=${NSA_RCCL_PRESET} without NCCL_HOSTID: RCCL will see each pod as its own host (NET transport)" >&2
    fi
    ;;
esac
# the pod's GPU by ordinal (Topology B over xGMI: every pod sees all GPUs of the node)
if [[ "${NSA_DEVICE_SELECT:-}" == "ordinal" ]]; then
  gpn="${NSA_GPUS_PER_NODE:-8}"
  if (( NPROC_PER_NODE != 1 )); then
    echo "entrypoint: NSA_DEVICE_SELECT=ordinal needs NPROC_PER_NODE=1 (got $NPROC_PER_NODE)" >&2
    exit 2
  fi
  export NSA_LOCAL_DEVICE=$(( NODE_RANK % gpn ))
  echo "entrypoint: device by ordinal: NSA_LOCAL_DEVICE=${NSA_LOCAL_DEVICE} (of ${gpn})" >&2
fi
# the transport facts that decide what RCCL can pick, for kubectl logs
shm_fs="$(stat -f -c %T /dev/shm 2>/dev/null || echo '?')"
echo "entrypoint: rccl preset=${NSA_RCCL_PRESET:-xgmi} NCCL_HOSTID=${NCCL_HOSTID:-<unset>} /dev/shm=${shm_fs}" >&2
export HSA_ENABLE_IPC_MODE_LEGACY="${HSA_ENABLE_IPC_MODE_LEGACY:-0}"
export TORCH_NCCL_HIGH_PRIORITY="${TORCH_NCCL_HIGH_PRIORITY:-1}"

args=()
if [[ "$NNODES" == "1" ]]; then
  args+=(--standalone --nnodes=1 --nproc-per-node="$NPROC_PER_NODE")
else
  : "${MASTER_ADDR:?MASTER_ADDR must be set for NNODES > 1}"
  if [[ "$RDZV_BACKEND" == "c10d" ]]; then
    args+=(--nnodes="$NNODES" --nproc-per-node="$NPROC_PER_NODE" --rdzv-backend=c10d
           --rdzv-endpoint="${MASTER_ADDR}:${MASTER_PORT}" --rdzv-id="$RDZV_ID" --node-rank="$NODE_RANK")
  else
    args+=(--nnodes="$NNODES" --nproc-per-node="$NPROC_PER_NODE" --node-rank="$NODE_RANK"
           --master-addr="$MASTER_ADDR" --master-port="$MASTER_PORT")
  fi
fi
if [[ "$MAX_RESTARTS" != "0" ]]; then
  args+=(--max-restarts="$MAX_RESTARTS")
fi

PY="${PYTHON:-python3}"
cmd=("$PY" -m torch.distributed.run "${args[@]}" "$@")
echo "entrypoint: NODE_RANK=$NODE_RANK NNODES=$NNODES NPROC_PER_NODE=$NPROC_PER_NODE rdzv=$RDZV_BACKEND" >&2
if [[ "${NSA_DRY_RUN:-0}" == "1" ]]; then
  printf '%q ' "${cmd[@]}"
  echo
  exit 0
fi
exec "${cmd[@]}"
