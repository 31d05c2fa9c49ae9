set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --impl eager --steps 500 --warmup 50 > gpurun_out/eager_bench.json 2> gpurun_out/eager_bench.err
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof_eager -o run -- python3 /root/repo/bench.py --impl eager --steps 100 --warmup 10 > /root/repo/gpurun_out/eager_prof.log 2>&1
