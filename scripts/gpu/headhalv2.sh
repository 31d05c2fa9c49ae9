#!/bin/bash
# Head-halving A/B, reversed order, with a kernel profile of each variant on the same box.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
for rep in 1 2; do
for ng in 1 0; do
PTO_HEAD_HALVING=$ng timeout -k 10 200 python bench.py --steps 4000 --warmup 400 > gpurun_out/hh2_$ng.json 2>/dev/null
echo "ng=$ng $(python -c "import json;d=json.load(open('gpurun_out/hh2_$ng.json'));print(d['value'],d['ms_per_step']*1000)")"
done
done
cd /tmp
for ng in 0 1; do
PTO_HEAD_HALVING=$ng timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_hh2_$ng" -o run -- python3 "$R/bench.py" --steps 200 --warmup 20 > "$R/gpurun_out/hh2_prof_$ng.log" 2>&1
echo "== ng=$ng"; python3 "$R/tools/rocprof_summary.py" "$R/gpurun_out/prof_hh2_$ng" --top 5
done
