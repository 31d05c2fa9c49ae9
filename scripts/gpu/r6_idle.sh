#!/bin/bash
# Does an idle GPU before the driver's 20-step region slow it?  run(20) after
# the host sleeps 0..1000 ms (then the warm-up steps), and two bench.py
# driver commands back to back.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_idle
mkdir -p $O
timeout -k 10 200 python tools/driver_overhead_probe.py --reps 10 > $O/idle.json 2> $O/idle.err || { tail -5 $O/idle.err; exit 1; }
python -c "import json; d=json.load(open('$O/idle.json')); print(d['bench_like_run20_us']); print(d['after_idle_ms_run20_us'])"
for r in 1 2 3; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-latency > $O/b20_$r.json 2>/dev/null || exit 1
python -c "import json; b=json.load(open('$O/b20_$r.json')); print('driver cmd', b['value'], b['ms_per_step'])"
done
