"""bench.py output contract on CPU (gloo, 2 ranks): exactly one JSON line
from rank 0 with the fields the driver reads, both data modes."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("sampler", [False, True])
def test_bench_two_ranks_cpu_json_line(sampler):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6",
           "--warmup", "2", "--cpu", "--dataset-size", "1280"] + (["--sampler"] if sampler else [])
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [line for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["steps"] == 6 and d["warmup"] == 2 and d["scaling"] == "weak"
    assert d["value"] > 0 and d["config"]["global_batch"] == 128 and d["config"]["parallelism"] == "dp2"
    assert ("DistributedSampler" in d["config"]["sampler"]) == sampler
    # the replicas were compared after the timed steps (DDP keeps them identical)
    assert d["ranks_bit_identical"] is True
    # submit -> first step of a Master + Worker job through the operator stack
    lat = d["config"]["submit_to_first_step"]
    assert lat["replicas"] == "Master=1, Worker=1" and lat.get("job_state") == "Succeeded", lat
    assert 0 < d["submit_to_first_step_s"] < 120, lat


def test_bench_single_rank_reports_submit_to_first_step():
    """World size 1: after the timed run, bench.py submits a 1-replica job
    through the operator stack (fresh child agent + zygote) and reports
    submit -> first optimizer step in the same JSON line."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "1", "--cpu",
           "--dataset-size", "1280"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [line for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    lat = d["config"]["submit_to_first_step"]
    assert "error" not in lat, lat
    assert lat["job_state"] == "Succeeded" and lat["zygote_warm"] is True
    assert 0 < d["submit_to_first_step_s"] < 60


def test_pto_bench_scaling_sweep_cpu():
    """`pto bench --scale 1,2` launches bench.py the driver's way (direct at
    N=1, torch.distributed.run at N>1), prints each JSON line and a
    weak-scaling table."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, "-m", "pytorch_operator_1_amd", "bench", "--scale", "1,2", "--", "--cpu", "--steps", "4",
           "--warmup", "1", "--dataset-size", "640", "--no-latency"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith('{"metric"')]
    assert [d["n_gpus"] for d in lines] == [1, 2]
    assert "efficiency" in out.stdout and "100.0%" in out.stdout


def test_bench_gpus_n_without_launcher_starts_n_ranks():
    """`bench.py --gpus 2` with no torchrun must not measure one rank and
    call it two: it starts 2 child ranks itself and reports n_gpus 2 with
    the process group's own world size as evidence."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                                                            "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--dataset-size", "640", "--no-latency"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [line for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    world = d["config"]["grad_allreduce"]
    assert world["pg_world_size"] == 2 and len(world["ranks"]) == 2


def test_bench_world_size_mismatch_is_an_error():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(WORLD_SIZE="3")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2", "--steps", "2", "--warmup", "1"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert out.returncode == 2 and "WORLD_SIZE=3" in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_params_fingerprint_is_bit_exact():
    """The replica check's fingerprint: equal for equal bits, different for
    a one-ulp change or a permutation, dtype-agnostic."""
    import torch

    from pytorch_operator_1_amd.utils.dist import params_fingerprint

    a = [torch.randn(1000), torch.randn(37, 5).to(torch.bfloat16)]
    b = [t.clone() for t in a]
    assert params_fingerprint(a) == params_fingerprint(b)
    b[0][17] = torch.nextafter(b[0][17], torch.tensor(float("inf")))
    assert params_fingerprint(a) != params_fingerprint(b)
    c = [a[0].flip(0), a[1]]
    assert params_fingerprint(a) != params_fingerprint(c)
    assert params_fingerprint(a, chunk=64) == params_fingerprint(a)


def test_bench_falls_back_to_rccl_when_xgmi_fails():
    """N > 1: when the peer-memory exchange times out (a bounded spin giving
    up -- seen by every rank, since the peers wait on each other; injected
    here on all ranks), the
    ranks agree through the status all-reduces that double as the timing
    barriers, the job is re-measured on the RCCL schedule and the JSON says
    so instead of losing the data point."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                                                            "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="2", PTO_BENCH_INJECT_XGMI_FAILURE="all")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--dataset-size", "640", "--no-latency"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([line for line in out.stdout.splitlines() if line.startswith("{")][0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert "injected" in d["config"]["grad_allreduce"]["xgmi_failed_fell_back_to_rccl"]
    assert "re-measuring on the RCCL schedule" in out.stderr


def test_bench_fallback_only_on_timeouts():
    """Only a timed-out exchange is re-measured on the RCCL schedule; diverged
    replicas (XgmiDivergence) and unrelated errors whose message merely names
    xGMI are not: they fail the bench."""
    sys.path.insert(0, ROOT)
    import bench
    from pytorch_operator_1_amd.parallel.xgmi import XgmiDivergence, XgmiTimeout

    assert bench._xgmi_failure(XgmiTimeout("barrier timed out"))
    assert not bench._xgmi_failure(XgmiDivergence("ranks diverged"))
    assert not bench._xgmi_failure(RuntimeError("xgmi_allreduce failed with hipError 1"))


def test_partitioned_rehearsal_overrides_inherited_hw_queues(monkeypatch):
    """Stacked CU-partitioned ranks (PTO_CU_PARTITION=1, host backend) get one
    pooled hardware queue each even when the environment already exports
    GPU_MAX_HW_QUEUES (GPU boxes export HIP's default, 4: the world-4
    rehearsal then ran ~200x slower); PTO_CU_HW_QUEUES picks another count.
    One-rank-per-GPU launches leave the environment alone."""
    import importlib.util
    import subprocess as sp

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    seen = []
    monkeypatch.setattr(sp, "call", lambda cmd, env=None: seen.append(env) or 0)
    for k in ("WORLD_SIZE", "RANK", "PTO_CU_HW_QUEUES"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    monkeypatch.setenv("PTO_BACKEND", "gloo")
    args = bench.parse_args(["--gpus", "4"])
    monkeypatch.setenv("PTO_CU_PARTITION", "1")
    assert bench._launch_ranks(args, []) == 0 and seen[-1]["GPU_MAX_HW_QUEUES"] == "1"
    monkeypatch.setenv("PTO_CU_HW_QUEUES", "2")
    assert bench._launch_ranks(args, []) == 0 and seen[-1]["GPU_MAX_HW_QUEUES"] == "2"
    monkeypatch.setenv("PTO_CU_PARTITION", "0")
    assert bench._launch_ranks(args, []) == 0 and seen[-1] is None
