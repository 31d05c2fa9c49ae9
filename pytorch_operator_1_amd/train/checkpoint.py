"""Checkpoint / resume.

The reference only has ``--save-model`` (``examples/mnist/mnist.py:146-147``,
DDP-prefixed keys, no optimizer state, no resume).  Here rank 0 writes
periodic checkpoints containing model, optimizer, step, epoch and RNG
state atomically (write to a temp file in the same directory, fsync,
``os.replace``) into a job-scoped directory; on start the trainer resumes
from the newest complete one.  Files are plain ``torch.save`` dicts of
tensors/ints and are read back with ``weights_only=True``.

Large models (Llama-3-8B: ~128 GB of bf16 params + fp32 master + Adam
state per replica) use :class:`ShardedCheckpointer`: each tensor is
written once by its owner rank (in parallel, off the training thread),
rank 0 commits a manifest last, and resume reads one shard per rank and
broadcasts (``train/lm.py``).
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


def _to_cpu(o):
    if isinstance(o, torch.Tensor):
        return o.detach().to("cpu", copy=True)
    if isinstance(o, dict):
        return {k: _to_cpu(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return type(o)(_to_cpu(v) for v in o)
    return o


# ---------------------------------------------------------------------------
# Sharded checkpoints for the large DDP configs (Llama-3-8B: bf16 params +
# fp32 master + Adam m/v = 16 B/param = 128 GB on every replica).  Every
# replica holds the same state (DDP), so each tensor is written ONCE, by its
# owner rank (size-balanced assignment), in parallel; on resume every rank
# reads only its own shard and the owners broadcast over the process group
# (RCCL over xGMI on the node: ~16 GB per rank instead of 128 GB of file
# reads per rank).  Layout on disk:
#   <dir>/step-<N>/shard-<r>-of-<W>.pt   plain tensors, weights_only loads
#   <dir>/step-<N>/manifest.json         written by rank 0 LAST, after every
#                                        shard is durable (barrier): a crash
#                                        mid-save never yields a manifest
#                                        naming missing shards.

def shard_owners(layout: dict[str, tuple], world: int) -> dict[str, int]:
    """Deterministic size-balanced owner per tensor name: largest first onto
    the least-loaded rank (ties: lower rank), names sorted for stability."""
    load = [0] * world
    own = {}
    for name in sorted(layout, key=lambda n: (-_numel(layout[n][0]) * _esize(layout[n][1]), n)):
        r = min(range(world), key=lambda i: (load[i], i))
        own[name] = r
        load[r] += _numel(layout[name][0]) * _esize(layout[name][1])
    return own


def _numel(shape) -> int:
    n = 1
    for d in shape:
        n *= int(d)
    return n


def _esize(dtype: str) -> int:
    return torch.empty((), dtype=getattr(torch, dtype)).element_size()


def tensor_layout(tensors: dict[str, torch.Tensor]) -> dict[str, tuple]:
    return {k: (list(v.shape), str(v.dtype).replace("torch.", "")) for k, v in tensors.items()}


class ShardedCheckpointer:
    """Periodic sharded, atomic, asynchronous checkpoints of a dict of named
    tensors (parameters + optimizer state) plus JSON metadata.

    ``save`` snapshots this rank's shard to host memory on the calling
    thread (so training can overwrite the device tensors right away); a
    background thread writes the shard, waits until every rank's shard of
    that step is durable (a barrier over the rendezvous TCPStore -- no
    collective on the GPU streams, nothing the training thread waits for),
    and rank 0 then commits the manifest.  A kill at any point leaves either
    a complete committed step or none (resume falls back to the previous
    one)."""

    def __init__(self, ckpt_dir: str, rank: int = 0, world: int = 1, async_write: bool = True, keep: int = 2,
                 barrier=None, barrier_timeout_s: float = 1800.0):
        self.dir, self.rank, self.world, self.keep = ckpt_dir, rank, world, keep
        self.async_write = async_write
        self._barrier = barrier or (lambda step: _store_barrier(f"pto/ckpt/{step}", rank, world,
                                                                barrier_timeout_s))
        self._thread = None
        self._error = None
        self.resumed_from = None

    # ---------------------------------------------------------------- save
    def save(self, step: int, tensors: dict[str, torch.Tensor], meta: dict | None = None):
        self.commit()  # one save in flight at a time
        layout = tensor_layout(tensors)
        owners = shard_owners(layout, self.world)
        mine = {k: v.detach().to("cpu", copy=True) for k, v in tensors.items() if owners[k] == self.rank}
        args = (step, mine, layout, owners, dict(meta or {}))
        if self.async_write:
            self._thread = threading.Thread(target=self._write_and_commit, args=args, daemon=True)
            self._thread.start()
        else:
            self._write_and_commit(*args)
            self.commit()

    def _write_and_commit(self, step, mine, layout, owners, meta):
        try:
            d = os.path.join(self.dir, f"step-{step:09d}")
            _atomic_save(mine, os.path.join(d, f"shard-{self.rank:05d}-of-{self.world:05d}.pt"))
            if self.world > 1:
                self._barrier(step)  # every shard of this step is durable
            if self.rank == 0:
                man = {"step": step, "world": self.world, "meta": meta,
                       "shards": [f"shard-{r:05d}-of-{self.world:05d}.pt" for r in range(self.world)],
                       "tensors": {k: {"shape": layout[k][0], "dtype": layout[k][1], "owner": owners[k]}
                                   for k in sorted(layout)}}
                tmp = os.path.join(d, ".manifest.tmp")
                with open(tmp, "w") as f:
                    json.dump(man, f)
                    f.flush()
                    os.fsync(f.fileno())
                os.replace(tmp, os.path.join(d, "manifest.json"))
                for old in list_sharded(self.dir)[:-self.keep]:
                    _rmtree(old)
                for orphan in list_uncommitted(self.dir, before=step):
                    _rmtree(orphan)  # a save killed before its manifest (~128 GB per crash at 8B)
        except BaseException as e:  # noqa: BLE001 - re-raised on the training thread by commit()
            self._error = e

    def commit(self):
        """Wait for the save in flight (shard written, manifest committed)."""
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise e

    def close(self):
        self.commit()

    # ---------------------------------------------------------------- load
    def latest(self) -> str | None:
        steps = list_sharded(self.dir)
        return steps[-1] if steps else None

    def load_into(self, tensors: dict[str, torch.Tensor], path: str | None = None, create=None) -> dict | None:
        """Restore the newest committed step (or ``path``) into ``tensors``
        in place.  Names missing from ``tensors`` are materialised through
        ``create(name, shape, dtype) -> tensor`` (optimizer state that does
        not exist before the first step).  Every rank reads its own shard;
        each tensor is then broadcast from its owner.  Returns the manifest
        (``step``, ``meta``) or None when there is nothing to resume."""
        import torch.distributed as dist

        dist_on = self.world > 1 and dist.is_available() and dist.is_initialized()
        if path is None:
            path = self.latest()
            if dist_on:
                # rank 0's choice for everyone: a replica restarted early can
                # otherwise see an older committed step than one whose save
                # was still committing, and the ranks would resume at
                # different steps (mismatched collectives)
                box = [path]
                dist.broadcast_object_list(box, src=0)
                path = box[0]
        self.resumed_from = path
        if path is None:
            return None
        with open(os.path.join(path, "manifest.json")) as f:
            man = json.load(f)
        if man["world"] != self.world:
            raise ValueError(f"checkpoint {path} was written by {man['world']} ranks, this job has {self.world} "
                             f"(re-shard offline or run with the same world size)")
        shard = {}
        if self.world == 1 or any(t["owner"] == self.rank for t in man["tensors"].values()):
            shard = torch.load(os.path.join(path, man["shards"][self.rank]), map_location="cpu",
                               weights_only=True)
        for name in sorted(man["tensors"]):
            info = man["tensors"][name]
            dst = tensors.get(name)
            if dst is None:
                if create is None:
                    raise KeyError(f"checkpoint tensor {name} has no destination")
                dst = create(name, info["shape"], getattr(torch, info["dtype"]))
                tensors[name] = dst
            if list(dst.shape) != list(info["shape"]):
                raise ValueError(f"{name}: checkpoint shape {info['shape']} != {list(dst.shape)}")
            with torch.no_grad():
                if info["owner"] == self.rank or not dist_on:
                    dst.copy_(shard[name])
                if dist_on:
                    # contiguous staging so NCCL/gloo can broadcast any layout
                    buf = dst if dst.is_contiguous() else dst.contiguous()
                    dist.broadcast(buf, src=info["owner"])
                    if buf is not dst:
                        dst.copy_(buf)
        return man


def _store_barrier(key: str, rank: int, world: int, timeout_s: float):
    """Barrier over the default process group's TCPStore (safe from a side
    thread: no device work, no collective)."""
    import datetime

    import torch.distributed as dist

    store = dist.distributed_c10d._get_default_store()
    store.set(f"{key}/{rank}", "1")
    store.wait([f"{key}/{r}" for r in range(world)], datetime.timedelta(seconds=timeout_s))


def list_sharded(ckpt_dir: str) -> list[str]:
    """Committed (manifest present) sharded steps, oldest first."""
    ds = glob.glob(os.path.join(ckpt_dir, "step-*", "manifest.json"))
    return sorted((os.path.dirname(d) for d in ds), key=lambda p: int(p.rsplit("-", 1)[1]))


def list_uncommitted(ckpt_dir: str, before: int) -> list[str]:
    """Step directories older than ``before`` that never got a manifest: a
    save that was killed mid-write.  Saves are sequential and the restart
    gate ends every process of the previous incarnation before the next one
    starts, so none of them can still be in flight."""
    out = []
    for d in glob.glob(os.path.join(ckpt_dir, "step-*")):
        try:
            n = int(d.rsplit("-", 1)[1])
        except ValueError:
            continue
        if n < before and not os.path.exists(os.path.join(d, "manifest.json")):
            out.append(d)
    return sorted(out)


def _rmtree(d: str):
    import shutil

    shutil.rmtree(d, ignore_errors=True)
