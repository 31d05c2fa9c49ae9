#!/bin/bash
# Early barrier-0 arrival (k_bwd_all sends the conv role's arrival): xGMI /
# graph / DDP GPU tests, the world-1 step of every schedule with and without
# it, and the F12 phase probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_xgmi_gpu.py tests/test_graph_gpu.py tests/test_ddp_gpu.py -v -s --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2; grep FAILED $O/pytest.log | head
case $rc in 0) ;; *) echo "pytest rc=$rc"; exit 1;; esac
for ea in 1 0 1; do
PTO_EARLY_ARRIVAL=$ea timeout -k 10 300 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > $O/ddp_step_ea$ea.json 2> $O/ddp_step_ea$ea.err || { tail -20 $O/ddp_step_ea$ea.err; exit 1; }
echo "early_arrival=$ea $(cat $O/ddp_step_ea$ea.json)"
done
timeout -k 10 300 python tools/exchange_phases_probe.py > $O/phases.json 2> $O/phases.err || { tail -20 $O/phases.err; exit 1; }
cat $O/phases.json | head -40
