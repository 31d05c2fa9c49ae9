#!/bin/bash
# fc role without its first barrier (coherent protocol): DDP / graph / xGMI
# tests incl. the exchange pair at world 3 and 8 (ranks sharing the GPU),
# world-1 schedule costs, then the self-launched bench.py rehearsal (N = 2, 4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/s2
timeout -k 10 700 python -u -m pytest tests/test_xgmi_gpu.py tests/test_ddp_gpu.py tests/test_graph_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/s2/pytest_world.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/s2/pytest_world.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/s2/pytest_world.log | head -20; exit 1; }
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/s2/ddp_step_nobar0.json 2> gpurun_out/s2/ddp_step_nobar0.err || { tail -20 gpurun_out/s2/ddp_step_nobar0.err; exit 1; }
tail -1 gpurun_out/s2/ddp_step_nobar0.json
bash scripts/gpu/rehearsal_r4.sh
