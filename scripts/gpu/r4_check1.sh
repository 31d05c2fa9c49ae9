#!/bin/bash
# Round 4, first check: the bench window trace (scripts/gpu/window_trace.sh),
# then the rewritten xGMI all-reduce (coherent protocol): its protocol
# tests, the 2-rank DDP numerics, the world-1 step cost
# (tools/ddp_step_bench.py) and rocprof kernel stats of the ddp-xgmi step.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu/window_trace.sh
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py tests/test_ddp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_xgmi.log 2>&1 || { tail -60 gpurun_out/pytest_xgmi.log; exit 1; }
grep -E "passed|failed|PASS|FAIL" gpurun_out/pytest_xgmi.log | tail -20
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/ddp_step.json 2> gpurun_out/ddp_step.err || { tail -20 gpurun_out/ddp_step.err; exit 1; }
cat gpurun_out/ddp_step.json
cd /tmp
rm -rf /tmp/kst_x
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kst_x -o run -- python3 "$R/tools/ddp_step_bench.py" --only xgmi --steps 400 --warmup 50 > "$R/gpurun_out/xgmi_prof.log" 2>&1
f=$(find /tmp/kst_x -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" | tee "$R/gpurun_out/xgmi_kstats.txt"
