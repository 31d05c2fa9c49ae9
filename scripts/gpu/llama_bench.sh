#!/bin/bash
# Llama-3-8B bench (config 4) with a heartbeat (model init + warmup are silent).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/llama
( while sleep 20; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u bench.py --model llama3-8b --steps 5 --warmup 2 "$@" > gpurun_out/llama/bench.json 2> gpurun_out/llama/bench.err
rc=$?
cat gpurun_out/llama/bench.json
tail -3 gpurun_out/llama/bench.err
exit $rc
