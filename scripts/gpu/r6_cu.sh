#!/bin/bash
# Round 6: is a stream's CU mask honoured (eager + graph replay)?  Then the
# inline exchange schedule with co-located ranks on disjoint CU partitions:
# 2-rank parity, self-verify hash, race, 200 steps, 4 and 8 ranks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6cu
mkdir -p $O
timeout -k 10 120 python -u tools/cu_partition_probe.py --out $O/cu_probe.json > $O/probe.log 2>&1 || { tail -30 $O/probe.log; exit 1; }
python - <<'EOF'
import json
d = json.load(open("gpurun_out/r6cu/cu_probe.json"))
print("unmasked", d["unmasked"])
for r in d["partitions"]:
    print({k: v for k, v in r.items() if "per_xcc" not in k})
EOF
timeout -k 10 200 python -u -m pytest tests/test_cu_partition_gpu.py -v -x --timeout 120 --timeout-method thread > $O/pytest_cu.log 2>&1 || { tail -30 $O/pytest_cu.log; exit 1; }
grep -E "passed|failed" $O/pytest_cu.log | tail -1
timeout -k 10 200 python -u -m pytest tests/test_ddp_gpu.py -v -x --timeout 150 --timeout-method thread -k "matches_reference and xgmi-inline" > $O/pytest_inline2.log 2>&1 || { tail -40 $O/pytest_inline2.log; exit 1; }
grep -E "passed|failed" $O/pytest_inline2.log | tail -1
timeout -k 10 700 python -u -m pytest tests/test_ddp_gpu.py -v -x --timeout 150 --timeout-method thread -k "inline" > $O/pytest_inline_all.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/pytest_inline_all.log | tail -12
exit $rc
