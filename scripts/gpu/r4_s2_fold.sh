#!/bin/bash
# conv exchange folded into k_bwd_all (PTO_XGMI_BWD_FOLD): DDP / graph /
# xGMI / kernel GPU tests, world-1 schedule costs with and without the fold,
# kernel stats of the folded overlapped step; then BASELINE configs 3/4
# (scripts/gpu/r4_models.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s2
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_graph_gpu.py tests/test_xgmi_gpu.py tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/s2/pytest_fold.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/s2/pytest_fold.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/s2/pytest_fold.log | head; exit 1; }
for fold in 1 0; do
PTO_XGMI_BWD_FOLD=$fold timeout -k 10 200 python tools/ddp_step_bench.py --steps 2000 --warmup 200 > gpurun_out/s2/ddp_step_fold$fold.json 2> gpurun_out/s2/ddp_step_fold$fold.err || { tail -20 gpurun_out/s2/ddp_step_fold$fold.err; exit 1; }
echo "fold=$fold $(cat gpurun_out/s2/ddp_step_fold$fold.json)"
done
cd /tmp
rm -rf /tmp/ktr_ov
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktr_ov -o run -- python3 "$R/tools/ddp_step_bench.py" --only xgmi --steps 400 --warmup 40 > "$R/gpurun_out/s2/trace_fold.log" 2>&1 || exit 1
f=$(find /tmp/ktr_ov -name "*kernel_stats.csv" | head -1)
python3 "$R/tools/kstats_table.py" "$f" | tee "$R/gpurun_out/s2/kstats_fold.txt"
f=$(find /tmp/ktr_ov -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/trace_gaps.py" "$f" --last 24 > "$R/gpurun_out/s2/gaps_fold.txt"
cd "$R"
bash scripts/gpu/r4_models.sh
