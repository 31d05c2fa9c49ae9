"""Backend resolution of the trainer's --backend flag (reference choices
gloo|nccl|mpi, examples/mnist/mnist.py:99-102, plus rccl)."""
import pytest
import torch.distributed as dist

from pytorch_operator_1_amd.utils.dist import resolve_backend


def test_aliases():
    assert resolve_backend("rccl", True) == "nccl"
    assert resolve_backend("NCCL", True) == "nccl"
    assert resolve_backend("gloo", True) == "gloo"
    assert resolve_backend(None, True) == "nccl"
    assert resolve_backend(None, False) == "gloo"
    with pytest.raises(ValueError):
        resolve_backend("ucc", False)


def test_mpi_falls_back_without_mpi_support(capsys):
    if dist.is_mpi_available():
        assert resolve_backend("mpi", False) == "mpi"
        return
    assert resolve_backend("mpi", True) == "nccl"
    assert resolve_backend("mpi", False) == "gloo"
    assert "no MPI support" in capsys.readouterr().err


def test_generation_store_defers_to_torchrun_agent_store():
    """under torchrun inside a pod (agent store on MASTER_PORT),
    PTO_RESTART_GENERATION must not make rank 0 host a second TCPStore;
    init goes through torchrun's own env:// store."""
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    prog = ("import sys; sys.path.insert(0, %r)\n"
            "from pytorch_operator_1_amd.utils import dist as pdist\n"
            "import torch.distributed as dist\n"
            "env, _ = pdist.init_distributed('gloo', use_gpu=False)\n"
            "dist.barrier()\n"
            "print('OK', env.rank, dist.get_world_size(), flush=True)\n"
            "pdist.cleanup()\n") % root
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(PTO_RESTART_GENERATION="3", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "--no-python", sys.executable, "-c", prog]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    assert sorted(ln for ln in out.stdout.splitlines() if ln.startswith("OK")) == ["OK 0 2", "OK 1 2"]


def test_generation_store_none_under_agent_env(monkeypatch):
    from pytorch_operator_1_amd.utils.dist import DistEnv, generation_store

    monkeypatch.setenv("PTO_RESTART_GENERATION", "1")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "abc")
    assert generation_store(DistEnv(0, 2, 0, "127.0.0.1", 1), 5.0) is None


RCCL_LOG = """\
host:1:1 [0] NCCL INFO RCCL version 2.26.6-HEAD:abc
host:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC/read
host:1:1 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC/read
host:1:1 [0] NCCL INFO Channel 00/0 : 1[1] -> 0[0] via SHM/direct/direct
host:1:1 [0] NCCL INFO Channel 02 : 0[0] -> 1[1] [send] via NET/Socket/0
host:1:1 [0] NCCL INFO 16 coll channels, 0 collnet channels, 0 nvls channels, 32 p2p channels, 32 p2p channels per peer
"""


def test_parse_rccl_transports():
    from pytorch_operator_1_amd.utils.dist import parse_rccl_transports

    d = parse_rccl_transports(RCCL_LOG)
    assert d["via"] == {"P2P/IPC/read": 2, "SHM/direct/direct": 1, "NET/Socket/0": 1}
    assert d["coll_channels"] == 16 and d["p2p_channels"] == 32
    assert d["version"].startswith("2.26.6")


def test_describe_world_single_process_cpu():
    import torch

    from pytorch_operator_1_amd.utils.dist import describe_world

    d = describe_world(torch.device("cpu"))
    assert d["pg_world_size"] == 1 and d["ranks"] == [{"device": "cpu"}]


def test_gpu_count_without_a_gpu_and_no_amdsmi(monkeypatch):
    """gpu_count() is the HIP runtime's count: 0 here, and it never calls
    torch.cuda.device_count() (whose amdsmi probe costs ~0.11 s on the
    MI355X box, profiles/startup_latency_r4.md)."""
    import torch

    from pytorch_operator_1_amd.utils import dist as pdist

    def boom():
        raise AssertionError("torch.cuda.device_count() called")

    monkeypatch.setattr(torch.cuda, "device_count", boom)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    assert pdist.gpu_count() == 0
    env, device = pdist.init_distributed(None, use_gpu=False)
    assert device.type == "cpu" and env.world_size >= 1


def _fake_kfd(tmp_path, versions):
    root = tmp_path / "nodes"
    for i, v in enumerate(versions):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {0 if v else 64}\nsimd_count 1024\ngfx_target_version {v}\n")
    return str(root)


def test_visible_gpu_count_from_kfd_sysfs(tmp_path):
    """The launcher's GPU count: KFD topology nodes with a non-zero
    gfx_target_version (node 0 is the CPU), restricted by the visibility
    env lists -- no HIP, no amdsmi."""
    from pytorch_operator_1_amd.utils.dist import visible_gpu_count_no_hip

    topo = _fake_kfd(tmp_path, [0] + [90500] * 8)
    assert visible_gpu_count_no_hip({}, topo) == 8
    assert visible_gpu_count_no_hip({"HIP_VISIBLE_DEVICES": "0,1"}, topo) == 2
    assert visible_gpu_count_no_hip({"ROCR_VISIBLE_DEVICES": "3,4,5", "HIP_VISIBLE_DEVICES": "0"}, topo) == 1
    assert visible_gpu_count_no_hip({"CUDA_VISIBLE_DEVICES": "0,1,2,3"}, topo) == 4
    assert visible_gpu_count_no_hip({"HIP_VISIBLE_DEVICES": ""}, topo) == 0
    # more indices than GPUs: only the GPUs that exist
    assert visible_gpu_count_no_hip({"HIP_VISIBLE_DEVICES": ",".join(map(str, range(12)))}, topo) == 8
    # no KFD (this container): nothing but the env lists
    assert visible_gpu_count_no_hip({}, str(tmp_path / "missing")) == 0
    assert visible_gpu_count_no_hip({"HIP_VISIBLE_DEVICES": "0,1"}, str(tmp_path / "missing")) == 2


def test_bench_launcher_never_touches_torch_cuda(monkeypatch, tmp_path):
    """bench.py --gpus N (no WORLD_SIZE) counts GPUs without torch.cuda and
    refuses to measure fewer ranks than asked for."""
    import importlib.util
    import os

    import torch

    def boom(*a, **k):
        raise AssertionError("the launcher initialised HIP")

    for name in ("device_count", "is_available", "init", "synchronize"):
        monkeypatch.setattr(torch.cuda, name, boom)
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", boom, raising=False)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("PTO_BACKEND", raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    from pytorch_operator_1_amd.utils import dist as pdist

    monkeypatch.setattr(pdist, "KFD_TOPOLOGY", _fake_kfd(tmp_path, [0, 90500]))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    args = bench.parse_args(["--gpus", "4"])
    assert bench._launch_ranks(args, ["--gpus", "4"]) == 2


def test_bucket_timing_plan_is_bounded():
    """GradBucketer's startup timing: one timed bucket
    per power-of-two size class, at most ``max_classes`` classes, every
    other bucket mapped to the nearest timed class -- 35 Llama-sized
    buckets cost 4 timings, not 35."""
    from pytorch_operator_1_amd.parallel.ddp import plan_bucket_timing

    mb = 2**20
    sizes = [256 * mb] * 33 + [100 * mb, 3 * mb]
    plan = plan_bucket_timing(sizes, 4)
    timed = sorted(set(plan))
    assert timed == [0, 33, 34] and plan[:33] == [0] * 33
    assert all(plan[j] == j for j in timed)
    many = [2**k for k in range(10, 30)]  # 20 classes
    plan = plan_bucket_timing(many, 4)
    assert len(set(plan)) == 4 and set(plan) == {16, 17, 18, 19}  # the four largest classes
    assert plan[0] == 16 and plan[19] == 19
    assert plan_bucket_timing([5], 4) == [0]
    assert plan_bucket_timing([8, 9, 1000], 1) == [2, 2, 2]
