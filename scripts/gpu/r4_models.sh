#!/bin/bash
# BASELINE configs 3/4 on HEAD: ResNet-50 and Llama-3-8B bf16, 20 timed
# steps each (JSON lines -> gpurun_out/models/), then rocprofv3 kernel
# summaries of both (steady-state windows).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/models
( while sleep 30; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u bench.py --model resnet50 --steps 20 --warmup 3 > gpurun_out/models/resnet50.json 2> gpurun_out/models/resnet50.err || { tail -20 gpurun_out/models/resnet50.err; exit 1; }
cut -c1-300 gpurun_out/models/resnet50.json
timeout -k 10 600 python -u bench.py --model llama3-8b --steps 20 --warmup 3 > gpurun_out/models/llama8b.json 2> gpurun_out/models/llama8b.err || { tail -20 gpurun_out/models/llama8b.err; exit 1; }
cut -c1-300 gpurun_out/models/llama8b.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_resnet -o run -- python3 "$R/bench.py" --model resnet50 --steps 4 --warmup 3 > "$R/gpurun_out/models/resnet_prof.log" 2>&1 || { tail -30 "$R/gpurun_out/models/resnet_prof.log"; exit 1; }
python3 "$R/tools/rocprof_window.py" /tmp/prof_resnet --marker sgd --steps 3 --top 40 > "$R/gpurun_out/models/resnet_window.md"
head -30 "$R/gpurun_out/models/resnet_window.md"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof_llama8b -o run -- python3 "$R/bench.py" --model llama3-8b --steps 3 --warmup 1 > "$R/gpurun_out/models/llama8b_prof.log" 2>&1 || { tail -30 "$R/gpurun_out/models/llama8b_prof.log"; exit 1; }
python3 "$R/tools/rocprof_summary.py" /tmp/prof_llama8b --steps 4 --top 40 > "$R/gpurun_out/models/llama8b_summary.md"
head -40 "$R/gpurun_out/models/llama8b_summary.md"
