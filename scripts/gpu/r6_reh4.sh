#!/bin/bash
# Round 6: world-4 rehearsal on one GPU -- is the 30 ms/step of the first
# try hardware-queue oversubscription?  Default vs GPU_MAX_HW_QUEUES=1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6reh4
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
for q in 1 default; do
for n in 2 4; do
if [ $q = default ]; then unset GPU_MAX_HW_QUEUES; else export GPU_MAX_HW_QUEUES=$q; fi
PTO_BACKEND=gloo PTO_CU_PARTITION=1 timeout -k 10 300 python bench.py --gpus $n --steps 200 --warmup 5 --no-latency > $O/reh${n}_q$q.json 2> $O/reh${n}_q$q.err || { tail -30 $O/reh${n}_q$q.err; exit 1; }
show $O/reh${n}_q$q.json
done
done
