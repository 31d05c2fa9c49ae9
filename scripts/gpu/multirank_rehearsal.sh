#!/bin/bash
# Multi-rank bench rehearsal on a one-GPU box: N ranks share cuda:0, gloo
# carries the host collectives, the xGMI kernels run over same-device IPC
# mappings.  Exercises the N>1 code path end to end (autotune, whole-step
# graph with cross-process all-reduce kernels, timing, JSON); the numbers
# are not a scaling measurement.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
  PTO_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 400 --warmup 40 > gpurun_out/rehearsal_$n.json 2> gpurun_out/rehearsal_$n.err || { tail -30 gpurun_out/rehearsal_$n.err; exit 1; }
  grep '^{"metric"' gpurun_out/rehearsal_$n.json > gpurun_out/rehearsal_$n.line
  echo "n=$n $(cut -c1-220 gpurun_out/rehearsal_$n.line)"
  python - "$n" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/rehearsal_{sys.argv[1]}.line"))
print("  grad_allreduce:", d["config"]["grad_allreduce"], "final_loss:", d["config"]["final_loss"])
PY
done
