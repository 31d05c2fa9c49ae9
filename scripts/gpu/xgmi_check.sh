#!/bin/bash
# xGMI peer all-reduce protocol tests (W ranks sharing the one GPU), then the
# 2-rank fused DDP test that now runs over it.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_xgmi_gpu.py -x -q -s > gpurun_out/xgmi.log 2>&1 || { tail -60 gpurun_out/xgmi.log; exit 1; }
tail -5 gpurun_out/xgmi.log
timeout -k 10 400 python -m pytest tests/test_ddp_gpu.py tests/test_graph_gpu.py -x -q > gpurun_out/ddp.log 2>&1 || { tail -60 gpurun_out/ddp.log; exit 1; }
tail -3 gpurun_out/ddp.log
