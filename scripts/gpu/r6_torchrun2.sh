#!/bin/bash
# The driver's N>1 launch line (torch.distributed.run, 2 ranks) rehearsed on
# the one GPU: gloo for the host-side group, CU-partitioned ranks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_torchrun2
mkdir -p $O
PTO_BACKEND=gloo PTO_CU_PARTITION=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 200 --warmup 5 > $O/tr2.json 2> $O/tr2.err || { tail -30 $O/tr2.err; exit 1; }
python - $O/tr2.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
g = d["config"]["grad_allreduce"]
print(d["value"], d["ms_per_step"], "n_gpus", d["n_gpus"], "identical", d.get("ranks_bit_identical"), "overlap", g.get("overlap"), "kept", g.get("schedule_autotune", {}).get("kept"), "latency", d.get("submit_to_first_step_s"))
PY
