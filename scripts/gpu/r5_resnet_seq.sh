#!/bin/bash
# ResNet-50 step under a kernel trace: window summary + the last step's
# dispatch sequence (which library kernels sit next to which convs).
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
O=$R/gpurun_out/rseq
mkdir -p $O
cd /tmp
( while sleep 30; do echo "[prof] $(date +%T) running"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_rs -o run -- python3 "$R/bench.py" --model resnet50 --steps 3 --warmup 3 --no-latency > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
grep '^{' $O/prof.log | cut -c1-200
python3 "$R/tools/rocprof_window.py" /tmp/prof_rs --marker sgd --steps 2 --top 45 --seq > $O/window.md
head -30 $O/window.md
cd "$R"
timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 --no-latency --force-ddp > $O/bench_ddp.json 2> $O/bench_ddp.err || { tail -20 $O/bench_ddp.err; exit 1; }
cut -c1-300 $O/bench_ddp.json
