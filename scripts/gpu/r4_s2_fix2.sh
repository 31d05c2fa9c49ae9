#!/bin/bash
# conv-grad zeroing in F12's all-reduce role (F4dx spare block idle): DDP /
# graph / xGMI GPU tests, world-1 schedule costs, kernel stats of the
# overlapped step; then BASELINE configs 3/4 on HEAD (scripts/gpu/r4_models.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_graph_gpu.py tests/test_xgmi_gpu.py tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/s2/pytest_fix2.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/s2/pytest_fix2.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/s2/pytest_fix2.log | head; exit 1; }
timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/s2/ddp_step2.json 2> gpurun_out/s2/ddp_step2.err || { tail -20 gpurun_out/s2/ddp_step2.err; exit 1; }
cat gpurun_out/s2/ddp_step2.json
cd /tmp
rm -rf /tmp/ktr_ov
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktr_ov -o run -- python3 "$R/tools/ddp_step_bench.py" --only xgmi --steps 400 --warmup 40 > "$R/gpurun_out/s2/trace_ov2.log" 2>&1 || exit 1
f=$(find /tmp/ktr_ov -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" | tee "$R/gpurun_out/s2/kstats_ov2.txt"
cd "$R"
bash scripts/gpu/r4_models.sh
