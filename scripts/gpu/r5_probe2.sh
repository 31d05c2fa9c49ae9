#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5p2
mkdir -p $O
timeout -k 10 120 python tools/exchange_phases_probe.py --steps 60 > $O/phases_uc.json 2> $O/phases.err || { tail -20 $O/phases.err; exit 1; }
cat $O/phases_uc.json
PTO_AR_FLAGS_CACHED=1 timeout -k 10 120 python tools/exchange_phases_probe.py --steps 60 > $O/phases_cached.json 2> $O/phases2.err || { tail -20 $O/phases2.err; exit 1; }
cat $O/phases_cached.json
PTO_AR_FLAGS_CACHED=1 timeout -k 10 300 python tools/ddp_step_bench.py --steps 2000 --warmup 200 --only xgmi > $O/ddp_step_cached.json 2> $O/ddp_step.err || { tail -20 $O/ddp_step.err; exit 1; }
cat $O/ddp_step_cached.json
PTO_AR_FLAGS_CACHED=1 timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -v --timeout 150 --timeout-method thread > $O/pytest_cached.log 2>&1
echo "cached-flags xgmi tests rc=$?"; grep -E "passed|failed" $O/pytest_cached.log | tail -2; grep FAILED $O/pytest_cached.log | head
