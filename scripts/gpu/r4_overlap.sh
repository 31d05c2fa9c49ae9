#!/bin/bash
# The overlapped ddp-xgmi schedule: DDP/xGMI GPU tests, the world-1 step
# costs of every schedule (tools/ddp_step_bench.py) and the kernel trace of
# a few overlapped steps.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ddp_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_overlap.log 2>&1 || { tail -60 gpurun_out/pytest_overlap.log; exit 1; }
grep -E "passed|failed|PASS|FAIL" gpurun_out/pytest_overlap.log | tail -24
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/ddp_step_ov.json 2> gpurun_out/ddp_step_ov.err || { tail -20 gpurun_out/ddp_step_ov.err; exit 1; }
cat gpurun_out/ddp_step_ov.json
cd /tmp
rm -rf /tmp/ktr_ov
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktr_ov -o run -- python3 "$R/tools/ddp_step_bench.py" --only xgmi --steps 400 --warmup 40 > "$R/gpurun_out/ov_trace.log" 2>&1
f=$(find /tmp/ktr_ov -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/trace_gaps.py" "$f" --last 30 | tee "$R/gpurun_out/ov_trace_last.txt"
f=$(find /tmp/ktr_ov -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" | tee "$R/gpurun_out/ov_kstats.txt"
