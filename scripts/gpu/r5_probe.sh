#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 120 python tools/exchange_phases_probe.py --steps 60 > $O/phases.json 2> $O/phases.err || { tail -20 $O/phases.err; exit 1; }
cat $O/phases.json
timeout -k 10 300 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > $O/ddp_step.json 2> $O/ddp_step.err || { tail -20 $O/ddp_step.err; exit 1; }
cat $O/ddp_step.json
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_ddp_gpu.py tests/test_graph_gpu.py -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2; grep FAILED $O/pytest.log | head
exit $rc
