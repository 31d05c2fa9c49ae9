#!/bin/bash
# ResNet-50 bench A/B of env settings (heartbeat keeps the run visibly alive
# through MIOpen's first-run solver search): rn_ab.sh "A=1" "A=0 B=2" ...
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/rn
( while sleep 20; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
i=0
rc=0
for setting in "$@"; do
  i=$((i+1))
  ( export $setting; timeout -k 10 600 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/rn/b_$i.json 2> gpurun_out/rn/b_$i.err ) || { rc=$?; echo "run $i failed rc=$rc"; tail -5 gpurun_out/rn/b_$i.err; break; }
  echo "== $setting: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rn/b_$i.json)"
done
exit $rc
