#!/bin/bash
# first timed window after a bench-like warmup, per warm-up mode
# (tools/bench_window_probe.py), then the driver's bench command 3x
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in ${MODES:-first rewarm_last upload_last first rewarm_last upload_last first rewarm_last upload_last}; do
  timeout -k 10 60 python tools/bench_window_probe.py --mode $m 2>/dev/null || exit 1
done > gpurun_out/bwp_modes.txt
cat gpurun_out/bwp_modes.txt
for i in 1 2 3; do timeout -k 10 60 python bench.py --gpus 1 --steps 20 --warmup 5 --no-latency 2>/dev/null | cut -c1-110 || exit 1; done
