"""Checkpoint / resume.

The reference only has ``--save-model`` (``examples/mnist/mnist.py:146-147``,
DDP-prefixed keys, no optimizer state, no resume).  Here rank 0 writes
periodic checkpoints containing model, optimizer, step, epoch and RNG
state atomically (write to a temp file in the same directory, fsync,
``os.replace``) into a job-scoped directory; on start the trainer resumes
from the newest complete one.  Files are plain ``torch.save`` dicts of
tensors/ints and are read back with ``weights_only=True``.

Large models (Llama-3-8B: ~112 GB of fp32 master + Adam state) use
:func:`save_sharded`: every rank writes its own shard file and rank 0
writes the manifest last, so a crash mid-write never produces a manifest
that names missing shards.
"""
from __future__ import annotations

import glob
import json
import os
import re
import tempfile
import threading

import torch

_CKPT_RE = re.compile(r"ckpt-(\d+)\.pt$")


def _atomic_save(obj, path: str):
    d = os.path.dirname(path) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".tmp-", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            torch.save(obj, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def rng_state() -> dict:
    st = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st: dict):
    if "cpu" in st:
        torch.set_rng_state(st["cpu"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


def save(ckpt_dir: str, step: int, state: dict, keep: int = 3) -> str:
    path = os.path.join(ckpt_dir, f"ckpt-{step:09d}.pt")
    _atomic_save(dict(state, step=step), path)
    for old in list_checkpoints(ckpt_dir)[:-keep]:
        try:
            os.unlink(old)
        except OSError:
            pass
    return path


def list_checkpoints(ckpt_dir: str) -> list[str]:
    files = [f for f in glob.glob(os.path.join(ckpt_dir, "ckpt-*.pt")) if _CKPT_RE.search(f)]
    return sorted(files, key=lambda f: int(_CKPT_RE.search(f).group(1)))


def latest(ckpt_dir: str | None) -> str | None:
    if not ckpt_dir or not os.path.isdir(ckpt_dir):
        return None
    files = list_checkpoints(ckpt_dir)
    return files[-1] if files else None


def load(path: str, map_location="cpu") -> dict:
    return torch.load(path, map_location=map_location, weights_only=True)


class AsyncSaver:
    """Snapshot to host memory on the training thread, write on a
    background thread (keeps large checkpoints off the step's critical
    path)."""

    def __init__(self):
        self._t = None

    def save(self, ckpt_dir, step, state, keep=3):
        self.wait()
        host = _to_cpu(state)
        self._t = threading.Thread(target=save, args=(ckpt_dir, step, host, keep), daemon=True)
        self._t.start()

    def wait(self):
        if self._t is not None:
            self._t.join()
            self._t = None


def _to_cpu(o):
    if isinstance(o, torch.Tensor):
        return o.detach().to("cpu", copy=True)
    if isinstance(o, dict):
        return {k: _to_cpu(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return type(o)(_to_cpu(v) for v in o)
    return o


def save_sharded(ckpt_dir: str, step: int, shard: dict, rank: int, world: int, barrier=None) -> str:
    d = os.path.join(ckpt_dir, f"step-{step:09d}")
    _atomic_save(shard, os.path.join(d, f"shard-{rank:05d}-of-{world:05d}.pt"))
    if barrier is not None:
        barrier()
    if rank == 0:
        man = {"step": step, "world": world, "shards": [f"shard-{r:05d}-of-{world:05d}.pt" for r in range(world)]}
        tmp = os.path.join(d, ".manifest.tmp")
        with open(tmp, "w") as f:
            json.dump(man, f)
        os.replace(tmp, os.path.join(d, "manifest.json"))
    return d


def latest_sharded(ckpt_dir: str) -> str | None:
    ds = sorted(glob.glob(os.path.join(ckpt_dir, "step-*", "manifest.json")))
    return os.path.dirname(ds[-1]) if ds else None


def load_shard(d: str, rank: int, map_location="cpu") -> dict:
    man = json.load(open(os.path.join(d, "manifest.json")))
    return torch.load(os.path.join(d, man["shards"][rank]), map_location=map_location, weights_only=True)
