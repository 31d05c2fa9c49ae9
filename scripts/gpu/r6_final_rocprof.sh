#!/bin/bash
# Final tree: rocprofv3 kernel statistics of the MNIST step (bench.py, 300
# timed steps) -- per-kernel time of the four launches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_final_rocprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 300 --warmup 20 --no-latency > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1e3:8.2f} pct {float(r["Percentage"]):6.2f}')
PY
