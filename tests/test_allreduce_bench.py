"""tools/allreduce_bench.py plumbing on CPU (gloo, 2 ranks): sweep records
and the bucket stress pass verify every element of the summed buffer."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_allreduce_bench_two_ranks_cpu():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port),
                          os.path.join(ROOT, "tools", "allreduce_bench.py"), "--cpu", "--sizes-mb", "0.01,0.2",
                          "--iters", "2", "--stress-gb", "0.004", "--bucket-mb", "0.5"],
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    recs = [json.loads(line) for line in out.stdout.splitlines() if line.startswith("{")]
    sweep = [r for r in recs if r["op"] == "all_reduce"]
    assert len(sweep) == 2 and all(r["world"] == 2 and r["us"] > 0 for r in sweep)
    (st,) = [r for r in recs if r["op"] == "bucket_stress"]
    assert st["mismatched_elements"] == 0 and st["buckets"] == 8
