#!/bin/bash
# Final tree: the multi-GPU step at world 1 (every schedule, 2000 steps) and
# the N>1 default rehearsed with two / four CU-partitioned ranks on the one
# GPU (bench.py --gpus 2 / 4, gloo for the host side).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_final_ddp
mkdir -p $O
timeout -k 10 300 python tools/ddp_step_bench.py --steps 2000 > $O/ddp_step.json 2> $O/ddp_step.err || { tail -20 $O/ddp_step.err; exit 1; }
cat $O/ddp_step.json | cut -c1-600
for n in 2 4; do
  PTO_BACKEND=gloo PTO_CU_PARTITION=1 timeout -k 10 300 python bench.py --gpus $n --steps 200 --warmup 5 --no-latency > $O/reh$n.json 2> $O/reh$n.err || { tail -30 $O/reh$n.err; exit 1; }
  python - $O/reh$n.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
g = d["config"]["grad_allreduce"]
r = g.get("schedule_autotune", {})
print(sys.argv[1], d["value"], d["ms_per_step"], "identical", d.get("ranks_bit_identical"), "overlap", g.get("overlap"), "kept", r.get("kept"))
print("  ", {k: (v.get("step_us"), v.get("exchange")) for k, v in r.get("candidates", {}).items()})
PY
done
