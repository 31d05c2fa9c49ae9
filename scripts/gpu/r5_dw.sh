#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5l2
timeout -k 10 400 python tools/dw_layout_bench.py > gpurun_out/r5l2/dw.txt 2>&1 || { tail -20 gpurun_out/r5l2/dw.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r5l2/dw.txt
