#!/bin/bash
# Closing fc exchange zeroes the conv grads: the DDP/graph/xGMI GPU tests,
# world-1 DDP schedule costs, kernel stats of the overlapped step, then the
# dW1-in-dgrad-blocks A/B (PTO_BWD_D_IN_B).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_graph_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/s2/pytest_fix.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/s2/pytest_fix.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/s2/pytest_fix.log | head; exit 1; }
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/s2/ddp_step.json 2> gpurun_out/s2/ddp_step.err || { tail -20 gpurun_out/s2/ddp_step.err; exit 1; }
cat gpurun_out/s2/ddp_step.json
cd /tmp
for only in xgmi xgmi_noov; do
rm -rf /tmp/ktr_$only
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktr_$only -o run -- python3 "$R/tools/ddp_step_bench.py" --only $only --steps 400 --warmup 40 > "$R/gpurun_out/s2/trace_$only.log" 2>&1 || exit 1
f=$(find /tmp/ktr_$only -name "*kernel_stats.csv" | head -1)
echo "== $only"; python3 "$R/tools/kstats_table.py" "$f" | tee "$R/gpurun_out/s2/kstats_$only.txt"
f=$(find /tmp/ktr_$only -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/trace_gaps.py" "$f" --last 24 > "$R/gpurun_out/s2/gaps_$only.txt"
done
cd "$R"
for v in 1 0 1 0; do
  PTO_BWD_D_IN_B=$v timeout -k 10 200 python bench.py --no-latency > gpurun_out/s2/dinb_$v.json 2> gpurun_out/s2/dinb_$v.err || { tail -5 gpurun_out/s2/dinb_$v.err; exit 1; }
  echo "d_in_b=$v $(cut -c1-140 gpurun_out/s2/dinb_$v.json)"
done
