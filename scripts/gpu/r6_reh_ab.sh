#!/bin/bash
# Round 6: 2-rank partitioned rehearsal, A/B on one box: warm-up on a second
# masked queue ("own") vs on the rank's one masked stream ("main"), twice
# each interleaved, plus the unpartitioned (colocated) reference.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6ab
mkdir -p $O
show() {
python - $1 <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
g = d["config"]["grad_allreduce"]
r = g.get("schedule_autotune", {})
print(sys.argv[1], d["value"], d["ms_per_step"], "identical", d.get("ranks_bit_identical"), "kept", r.get("kept"), "race_s", r.get("seconds"))
print("  ", {k: (v.get("step_us"), v.get("exchange")) for k, v in r.get("candidates", {}).items()})
PY
}
i=0
for v in own main own main none; do
i=$((i+1))
if [ $v = none ]; then P=0; else P=1; fi
PTO_CU_SIDE_STREAM=$v PTO_BACKEND=gloo PTO_CU_PARTITION=$P timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 5 --no-latency > $O/reh2_${v}_$i.json 2> $O/reh2_${v}_$i.err || { tail -30 $O/reh2_${v}_$i.err; exit 1; }
show $O/reh2_${v}_$i.json
done
