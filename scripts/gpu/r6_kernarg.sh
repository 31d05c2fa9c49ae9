#!/bin/bash
# Is the slow first replay of a graph (and the close[5] -> close[20]
# alternation) the kernel-argument fetch?  Same probe with kernargs forced
# to device memory and forced off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6_kernarg
mkdir -p $O
for v in 1 0; do
HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python tools/driver_overhead_probe.py --reps 10 > $O/k$v.json 2> $O/k$v.err || { tail -5 $O/k$v.err; exit 1; }
python -c "import json; d=json.load(open('$O/k$v.json')); print('devkernarg=$v', d['bench_like_run20_us'], d['after_idle_ms_run20_us'], d['run_us'])"
HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-latency > $O/b20_$v.json 2>/dev/null || exit 1
python -c "import json; b=json.load(open('$O/b20_$v.json')); print('driver cmd devkernarg=$v', b['value'], b['ms_per_step'])"
done
