#!/usr/bin/env bash
# Build the ROCm/gfx950 training image and import it into k3s containerd (D4, README.md:34-38,103).
set -euo pipefail
cd "$(dirname "$0")/.."
IMAGE="${IMAGE:-disttrain-mi355x:latest}"
docker build -f docker/Dockerfile -t "$IMAGE" \
  ${HTTP_PROXY:+--build-arg HTTP_PROXY="$HTTP_PROXY"} ${HTTPS_PROXY:+--build-arg HTTPS_PROXY="$HTTPS_PROXY"} .
docker save "$IMAGE" | sudo k3s ctr images import -
sudo k3s ctr images ls | grep -q "${IMAGE%%:*}" && echo "imported $IMAGE into k3s containerd"
