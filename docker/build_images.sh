#!/bin/bash
# Build (and optionally push) the three images (reference build_image.sh /
# examples/mnist/Makefile).  Usage: docker/build_images.sh [REGISTRY] [TAG]
set -euo pipefail
REG=${1:-pto}
TAG=${2:-$(git rev-parse --short HEAD 2>/dev/null || echo dev)}
cd "$(dirname "$0")/.."
docker build -f docker/Dockerfile.operator -t "$REG/operator:$TAG" .
docker build -f docker/Dockerfile.trainer -t "$REG/pytorch-mnist:rocm" -t "$REG/pytorch-mnist:$TAG" .
docker build -f docker/Dockerfile.sendrecv -t "$REG/pytorch-sendrecv:rocm" .
if [[ "${PUSH:-0}" == 1 ]]; then
  for i in operator:$TAG pytorch-mnist:rocm pytorch-mnist:$TAG pytorch-sendrecv:rocm; do docker push "$REG/$i"; done
fi
