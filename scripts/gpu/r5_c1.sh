#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5m
timeout -k 10 300 python tools/conv1x1_bench.py > gpurun_out/r5m/conv1x1.jsonl 2> gpurun_out/r5m/conv1x1.err || { tail -5 gpurun_out/r5m/conv1x1.err; exit 1; }
cat gpurun_out/r5m/conv1x1.jsonl
