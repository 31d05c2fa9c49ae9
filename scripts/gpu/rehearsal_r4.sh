#!/bin/bash
# N = 2 and 4 ranks sharing cuda:0, started by bench.py ITSELF (no
# launcher: `bench.py --gpus N` spawns the ranks), host collectives on gloo,
# the xGMI kernels over same-device IPC.  Exercises the N>1 path end to end
# (self-launch, xGMI verification + protocol, schedule race, overlapped
# step graphs, world evidence, JSON).  Time-sliced processes on one GPU:
# NOT a scaling measurement, hence the long barrier timeout.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
  PTO_BACKEND=gloo PTO_XGMI_TIMEOUT_MS=20000 timeout -k 10 300 python bench.py --gpus $n --steps 20 --warmup 5 > gpurun_out/reh4_$n.json 2> gpurun_out/reh4_$n.err || { tail -30 gpurun_out/reh4_$n.err; exit 1; }
  grep '^{"metric"' gpurun_out/reh4_$n.json > gpurun_out/reh4_$n.line
  python - "$n" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/reh4_{sys.argv[1]}.line"))
ar = d["config"]["grad_allreduce"]
print(f"n={sys.argv[1]} n_gpus={d['n_gpus']} ms/step={d['ms_per_step']} loss={d['config']['final_loss']} "
      f"schedule={ar.get('schedule')} race={ar.get('schedule_autotune')} pg_world={ar.get('pg_world_size')} "
      f"devices={ar.get('distinct_devices')}")
PY
done
