#!/bin/bash
# k_bwd_all D role: one dW1 tile per wave (PTO_BWD_DPAIR=0, 400 blocks) vs a
# pair of tiles side by side (=1, 200 blocks; the grid then fits the
# resident slots).  Bitwise check (deterministic mode), role probe, the
# step bench interleaved, numerics tests.  Output: gpurun_out/dpair/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/dpair
mkdir -p $O
chk() {
  PTO_DETERMINISTIC=1 PTO_BWD_DPAIR=$1 timeout -k 10 120 python -c "
import os, torch
from pytorch_operator_1_amd.train.fused_step import FusedMnistTrainer
tr = FusedMnistTrainer(torch.device('cuda', 0), batch_size=64, dataset_size=64 * 16, graph='none')
for _ in range(30): tr.step()
tr.flush(); torch.cuda.synchronize()
p = tr._params.double()
print('dpair', os.environ['PTO_BWD_DPAIR'], 'sum', repr(p.sum().item()), 'sumsq', repr((p * p).sum().item()))
"
}
{ chk 0 && chk 1; } > $O/bitwise.txt 2>&1 || { cat $O/bitwise.txt; exit 1; }
cat $O/bitwise.txt
timeout -k 10 240 python tools/bwd_roles_probe.py --dpair 0 1 > $O/roles.txt 2>&1 || { tail -20 $O/roles.txt; exit 1; }
grep -E "==|all|D dW1|C\+F" $O/roles.txt
for r in 1 2; do
  for d in 0 1; do
    PTO_BWD_DPAIR=$d timeout -k 10 200 python bench.py > $O/bench2000_d${d}_$r.json 2> $O/bench_err || { tail $O/bench_err; exit 1; }
    PTO_BWD_DPAIR=$d timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench20_d${d}_$r.json 2> $O/bench_err || { tail $O/bench_err; exit 1; }
    python -c "import json; a=json.load(open('$O/bench2000_d${d}_$r.json')); b=json.load(open('$O/bench20_d${d}_$r.json')); print('dpair $d run $r', a['value'], a['ms_per_step']*1000, '| 20 steps', b['value'])"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_parity_long_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
exit $rc
