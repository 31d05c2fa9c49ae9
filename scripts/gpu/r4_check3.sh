#!/bin/bash
# overlapped ddp-xgmi after the one-barrier conv exchange: DDP + xGMI GPU
# tests, world-1 step costs, kernel trace of the overlapped step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_ov3.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_ov3.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_ov3.log | head; tail -40 gpurun_out/pytest_ov3.log; exit 1; }
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/ddp_step_ov3.json 2> gpurun_out/ddp_step_ov3.err || { tail -20 gpurun_out/ddp_step_ov3.err; exit 1; }
cat gpurun_out/ddp_step_ov3.json
cd /tmp
rm -rf /tmp/ktr_ov3
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktr_ov3 -o run -- python3 "$R/tools/ddp_step_bench.py" --only xgmi --steps 400 --warmup 40 > "$R/gpurun_out/ov3_trace.log" 2>&1 || exit 1
f=$(find /tmp/ktr_ov3 -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" | tee "$R/gpurun_out/ov3_kstats.txt"
