#!/bin/bash
# sync/launch latency probe (tools/sync_latency_probe.py) and the kernel
# order of a few ddp-xgmi steps (is there a memset per step?)
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/sync_latency_probe.py | tee gpurun_out/sync_latency.json
cd /tmp
rm -rf /tmp/ktr_x
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/ktr_x -o run -- python3 "$R/tools/ddp_step_bench.py" --only xgmi --steps 64 --warmup 8 > "$R/gpurun_out/xgmi_trace.log" 2>&1
f=$(find /tmp/ktr_x -name "*kernel_trace.csv" | head -1)
python3 "$R/tools/trace_gaps.py" "$f" --last 24 | tee "$R/gpurun_out/xgmi_trace_last.txt"
