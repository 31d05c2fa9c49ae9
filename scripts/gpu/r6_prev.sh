#!/bin/bash
# run(20) timed right after different replays / launches (what the replay
# just before the driver's region does to it).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_prev
mkdir -p $O
timeout -k 10 200 python tools/driver_overhead_probe.py --reps 10 > $O/prev.json 2> $O/prev.err || { tail -5 $O/prev.err; exit 1; }
python -c "
import json; d=json.load(open('$O/prev.json'))
for k, v in d['run20_after_us'].items(): print(k, v)
"
