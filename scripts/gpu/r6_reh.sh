#!/bin/bash
# Round 6: the driver's N>1 path rehearsed on one GPU with CU-partitioned
# ranks (PTO_CU_PARTITION=1): self-verify hash tests (shared and partitioned),
# then bench.py --gpus 2 / 4 over gloo with its race table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6reh
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -v -x --timeout 150 --timeout-method thread -k "self_verify" > $O/pytest_hash.log 2>&1 || { tail -40 $O/pytest_hash.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_hash.log | tail -6
for n in 2 4; do
PTO_BACKEND=gloo PTO_CU_PARTITION=1 timeout -k 10 400 python bench.py --gpus $n --steps 200 --warmup 5 > $O/reh$n.json 2> $O/reh$n.err || { tail -30 $O/reh$n.err; exit 1; }
python - $O/reh$n.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
g = d["config"]["grad_allreduce"]
print(sys.argv[1], d["value"], d["ms_per_step"], "identical", d.get("ranks_bit_identical"), "overlap:", g.get("overlap"))
print("  partition", g.get("cu_partition"))
print("  race", json.dumps(g.get("schedule_autotune")))
PY
done
