#!/bin/bash
# DDP numerics (2 ranks on one GPU) + the multi-rank bench rehearsal.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py tests/test_ddp_gpu.py tests/test_graph_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_ddp.log 2>&1 || { grep -E "PASS|FAIL" gpurun_out/pytest_ddp.log | tail; tail -40 gpurun_out/pytest_ddp.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_ddp.log | tail -16
bash scripts/gpu/multirank_rehearsal.sh
