"""Sharded checkpoint / auto-resume of the large-model trainer
(train/lm.py, BASELINE configs 3-5): kill mid-run, restart, and the resumed
run ends exactly where the uninterrupted one does (CPU, deterministic)."""
import os
import re
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--no-cuda", "--model", "llama3-tiny", "--seq-len", "64", "--steps", "8", "--log-interval", "2"]


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    return env


def _final(out: str) -> float:
    return float(re.search(r"final_loss=([0-9.]+)", out).group(1))


def _run(extra, cwd):
    return subprocess.run([sys.executable, "-m", "pytorch_operator_1_amd.train.lm"] + ARGS + extra,
                          capture_output=True, text=True, timeout=300, env=_env(), cwd=cwd)


def test_kill_and_resume_matches_uninterrupted(tmp_path):
    ref = _run([], tmp_path)
    assert ref.returncode == 0, ref.stderr[-2000:]
    ck = str(tmp_path / "ck")
    extra = ["--checkpoint-dir", ck, "--checkpoint-interval", "4", "--fail-at-step", "6"]
    a = _run(extra, tmp_path)
    assert a.returncode == -9, a.stdout[-2000:] + a.stderr[-2000:]
    b = _run(extra, tmp_path)
    assert b.returncode == 0, b.stderr[-2000:]
    assert "Resumed from" in b.stdout and "at step 4" in b.stdout
    assert _final(b.stdout) == _final(ref.stdout)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(extra, cwd):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "-m", "pytorch_operator_1_amd.train.lm"] + ARGS + [
               "--backend", "gloo"] + extra
    return subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=_env(), cwd=cwd)


def test_two_rank_sharded_checkpoint_resume(tmp_path):
    """world 2 (gloo): each tensor is written once by its owner, the manifest
    names both shards, and a restart after rank 1 is killed resumes both
    ranks from the committed step and ends on the uninterrupted loss."""
    ref = _torchrun([], tmp_path)
    assert ref.returncode == 0, ref.stderr[-3000:]
    ck = tmp_path / "ck"
    extra = ["--checkpoint-dir", str(ck), "--checkpoint-interval", "4", "--fail-at-step", "6", "--fail-rank", "1"]
    a = _torchrun(extra, tmp_path)
    assert a.returncode != 0
    b = _torchrun(extra, tmp_path)
    assert b.returncode == 0, b.stderr[-3000:]
    assert b.stdout.count("Resumed from") == 2 and b.stdout.count("at step 4") == 2, b.stdout
    assert _final(b.stdout) == _final(ref.stdout)
    import json

    steps = sorted(p.name for p in ck.iterdir() if (p / "manifest.json").exists())
    man = json.load(open(ck / steps[-1] / "manifest.json"))
    assert man["world"] == 2 and len(man["shards"]) == 2
    owners = {t["owner"] for t in man["tensors"].values()}
    assert owners == {0, 1}
    s0 = torch.load(ck / steps[-1] / man["shards"][0], weights_only=True)
    s1 = torch.load(ck / steps[-1] / man["shards"][1], weights_only=True)
    assert not (set(s0) & set(s1)) and set(s0) | set(s1) == set(man["tensors"])


def test_shard_owners_balance_and_roundtrip(tmp_path):
    from pytorch_operator_1_amd.train.checkpoint import ShardedCheckpointer, shard_owners, tensor_layout

    ts = {f"t{i}": torch.randn(100 * (i + 1)) for i in range(9)}
    own = shard_owners(tensor_layout(ts), 3)
    load = [sum(ts[k].numel() for k in own if own[k] == r) for r in range(3)]
    assert max(load) - min(load) <= 900  # greedy bound: one largest tensor
    ck = ShardedCheckpointer(str(tmp_path), async_write=True)
    ck.save(5, ts, {"x": 1})
    ck.close()
    dst = {k: torch.zeros_like(v) for k, v in list(ts.items())[:5]}
    made = {}

    def create(name, shape, dtype):
        made[name] = torch.zeros(shape, dtype=dtype)
        return made[name]

    man = ck.load_into(dst, create=create)
    assert man["step"] == 5 and man["meta"] == {"x": 1}
    assert set(made) == {f"t{i}" for i in range(5, 9)}
    for k, v in ts.items():
        assert torch.equal(dst[k], v)


@pytest.mark.parametrize("keep", [1, 2])
def test_keep_prunes_old_steps(tmp_path, keep):
    from pytorch_operator_1_amd.train.checkpoint import ShardedCheckpointer, list_sharded

    ck = ShardedCheckpointer(str(tmp_path), keep=keep)
    for step in (1, 2, 3):
        ck.save(step, {"a": torch.full((4,), float(step))})
    ck.close()
    assert [int(p.rsplit("-", 1)[1]) for p in list_sharded(str(tmp_path))] == [3 - i for i in range(keep)][::-1]


def test_orphaned_uncommitted_step_is_deleted(tmp_path):
    """A save killed before its manifest leaves a step directory nobody
    resumes from; the next committed save deletes it (older steps only)."""
    import os

    from pytorch_operator_1_amd.train.checkpoint import ShardedCheckpointer, list_sharded

    ck = ShardedCheckpointer(str(tmp_path), keep=2)
    ck.save(1, {"a": torch.ones(4)})
    ck.commit()
    crashed = tmp_path / "step-000000002"
    crashed.mkdir()
    (crashed / "shard-00000-of-00001.pt").write_bytes(b"partial")
    ck.save(3, {"a": torch.ones(4)})
    ck.close()
    assert not crashed.exists()
    assert [os.path.basename(p) for p in list_sharded(str(tmp_path))] == ["step-000000001", "step-000000003"]


def _agree_worker(rank, port, dirs, out):
    import torch.distributed as dist

    from pytorch_operator_1_amd.train.checkpoint import ShardedCheckpointer

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    try:
        ck = ShardedCheckpointer(dirs[rank], rank, 2)
        dst = {"a": torch.zeros(4)}
        man = ck.load_into(dst)
        out.put((rank, man["step"], ck.resumed_from, dst["a"].tolist()))
    finally:
        dist.destroy_process_group()


def test_resume_point_is_rank0s_choice(tmp_path):
    """Ranks whose view of the checkpoint directory differs (rank 1 sees
    only an older committed step) still resume from ONE step: rank 0's."""
    import multiprocessing as mp

    from pytorch_operator_1_amd.train.checkpoint import ShardedCheckpointer

    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    for d, steps in ((a, (1, 2)), (b, (1,))):
        for r in range(2):
            ck = ShardedCheckpointer(d, r, 2, async_write=False, barrier=lambda step: None)
            for s in steps:
                ck.save(s, {"a": torch.full((4,), float(s))})
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_agree_worker, args=(r, port, [a, b], q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [2, 2]
    assert res[0][2] == res[1][2] and res[0][2].startswith(a)
    assert res[1][3] == [2.0] * 4
