#!/bin/bash
# N = 2, 4, 8 ranks sharing cuda:0 through the driver's launcher (bench.py
# under torch.distributed.run; gloo for host collectives, xGMI kernels over
# same-device IPC): exercises the N>1 path end to end (xGMI autotune against
# the host all-reduce, schedule autotune, power-of-two step graphs, timing,
# JSON).  Time-sliced processes on one GPU: NOT a scaling measurement, hence
# the long barrier timeout.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4 8; do
  PTO_BACKEND=gloo PTO_XGMI_TIMEOUT_MS=20000 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 > gpurun_out/reh_$n.json 2> gpurun_out/reh_$n.err || { tail -30 gpurun_out/reh_$n.err; exit 1; }
  grep '^{"metric"' gpurun_out/reh_$n.json > gpurun_out/reh_$n.line
  python - "$n" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/reh_{sys.argv[1]}.line"))
print(f"n={sys.argv[1]} ms/step={d['ms_per_step']} loss={d['config']['final_loss']} ar={d['config']['grad_allreduce']}")
PY
done
