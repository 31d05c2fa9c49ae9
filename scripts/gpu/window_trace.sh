#!/bin/bash
# The driver's short bench window under a kernel + HIP-API trace
# (tools/window_trace.py), the graph-replay fixed costs
# (tools/graph_launch_probe.py), and the driver's bench command 3x.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-latency 2>/dev/null | cut -c1-120
done
for m in first rewarm rewarm_last upload_last first rewarm; do
  timeout -k 10 90 python tools/bench_window_probe.py --mode $m 2>/dev/null
done | tee gpurun_out/bwp_modes.txt
timeout -k 10 120 python tools/graph_launch_probe.py > gpurun_out/graph_launch_probe.json
cat gpurun_out/graph_launch_probe.json
cd /tmp
rm -rf /tmp/wtr
timeout -s KILL 180 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/wtr -o run -- \
  python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-latency > "$R/gpurun_out/wtr_bench.log" 2>&1
python3 "$R/tools/window_trace.py" /tmp/wtr | tee "$R/gpurun_out/window_trace.json"
mkdir -p "$R/gpurun_out/wtr"
cp $(find /tmp/wtr -name "*kernel_trace.csv" | head -1) "$R/gpurun_out/wtr/kernel_trace.csv"
cp $(find /tmp/wtr -name "*hip_api_trace.csv" | head -1) "$R/gpurun_out/wtr/hip_api_trace.csv"
