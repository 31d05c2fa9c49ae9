#!/bin/bash
# Round 6: world-4 partitioned rehearsal with the shipped side stream,
# default hardware queues vs GPU_MAX_HW_QUEUES=1 (queue oversubscription?).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6reh4b
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
for cfg in "4 1" "4 d" "2 1"; do
set -- $cfg
n=$1; q=$2
if [ $q = d ]; then unset GPU_MAX_HW_QUEUES; else export GPU_MAX_HW_QUEUES=$q; fi
PTO_BACKEND=gloo PTO_CU_PARTITION=1 timeout -k 10 300 python bench.py --gpus $n --steps 200 --warmup 5 --no-latency > $O/reh${n}_q$q.json 2> $O/reh${n}_q$q.err || { tail -30 $O/reh${n}_q$q.err; exit 1; }
show $O/reh${n}_q$q.json
done
