#!/bin/bash
# SGD operands of the xGMI one-shot / role epilogues loaded before the
# barriers: DDP / graph / xGMI tests, world-1 schedule costs (2 runs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pf
timeout -k 10 700 python -u -m pytest tests/test_xgmi_gpu.py tests/test_ddp_gpu.py tests/test_graph_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pf/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pf/pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pf/pytest.log | head -20; exit 1; }
for i in 1 2; do
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/pf/ddp_step_$i.json 2> gpurun_out/pf/ddp_step_$i.err || { tail -20 gpurun_out/pf/ddp_step_$i.err; exit 1; }
tail -1 gpurun_out/pf/ddp_step_$i.json
done
