#!/bin/bash
# Round 4 session 3 (prepare(), eager first step): N = 2 (warm-up 5 and 1) and 4 ranks sharing cuda:0, started by bench.py ITSELF (no
# launcher: `bench.py --gpus N` spawns the ranks), host collectives on gloo,
# the xGMI kernels over same-device IPC.  Exercises the N>1 path end to end
# (self-launch, xGMI verification + protocol, schedule race, overlapped
# step graphs, world evidence, JSON).  Time-sliced processes on one GPU:
# NOT a scaling measurement, hence the long barrier timeout.
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in 2:5 2:1 4:5; do
  n=${cfg%%:*}; w=${cfg##*:}
  PTO_BACKEND=gloo PTO_XGMI_TIMEOUT_MS=20000 timeout -k 10 300 python bench.py --gpus $n --steps 20 --warmup $w > gpurun_out/reh4_${n}_$w.json 2> gpurun_out/reh4_${n}_$w.err || { tail -30 gpurun_out/reh4_${n}_$w.err; exit 1; }
  grep '^{"metric"' gpurun_out/reh4_${n}_$w.json > gpurun_out/reh4_${n}_$w.line
  python - "$n" "$w" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/reh4_{sys.argv[1]}_{sys.argv[2]}.line"))
ar = d["config"]["grad_allreduce"]
print(f"n={sys.argv[1]} w={sys.argv[2]} n_gpus={d['n_gpus']} ms/step={d['ms_per_step']} loss={d['config']['final_loss']} "
      f"schedule={ar.get('schedule')} race={ar.get('schedule_autotune')} pg_world={ar.get('pg_world_size')} "
      f"devices={ar.get('distinct_devices')}")
PY
done
