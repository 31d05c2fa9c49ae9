#!/bin/bash
# kill-test probe (overlap on/off), bucketer xGMI hook tests, world-1 step
# costs of every schedule, the sync/launch/plan probe, and the overlapped
# step's kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu/r4_killprobe.sh
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -k bucketer -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_bucketer.log 2>&1
echo "bucketer rc=$?"; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_bucketer.log | tail -8
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/ddp_step_ov.json 2> gpurun_out/ddp_step_ov.err || { tail -20 gpurun_out/ddp_step_ov.err; exit 1; }
cat gpurun_out/ddp_step_ov.json
timeout -k 10 200 python tools/sync_latency_probe.py > gpurun_out/sync_latency2.json || exit 1
head -c 1500 gpurun_out/sync_latency2.json; echo
cd /tmp
rm -rf /tmp/ktr_ov
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktr_ov -o run -- python3 "$R/tools/ddp_step_bench.py" --only xgmi --steps 400 --warmup 40 > "$R/gpurun_out/ov_trace.log" 2>&1 || exit 1
f=$(find /tmp/ktr_ov -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/trace_gaps.py" "$f" --last 30 | tee "$R/gpurun_out/ov_trace_last.txt"
f=$(find /tmp/ktr_ov -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" | tee "$R/gpurun_out/ov_kstats.txt"
