#!/bin/bash
# Fixed cost of the driver's 20-step MNIST command: sync / graph round trips,
# run(n) for several n, and bench.py's own sequence (the first replay of the
# 20-step closing graph after capture, then repeats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_overhead
mkdir -p $O
timeout -k 10 200 python tools/driver_overhead_probe.py > $O/seq.json 2> $O/seq.err || { tail -5 $O/seq.err; exit 1; }
cat $O/seq.json
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20.json 2>/dev/null || exit 1
python -c "import json; b=json.load(open('$O/b20.json')); print('driver cmd', b['value'], b['ms_per_step'])"
