"""Rendezvous / process-group helpers for one-process-per-GPU training.

The operator injects the same env contract as the reference
(``pkg/controller.v1/pytorch/pod.go:234-281``): ``MASTER_ADDR``,
``MASTER_PORT``, ``WORLD_SIZE``, ``RANK``.  torchrun additionally provides
``LOCAL_RANK``; the node agent provides ``LOCAL_RANK=0`` plus
``HIP_VISIBLE_DEVICES`` pinning, so device selection always goes through
``LOCAL_RANK``.

Backend names: ``rccl`` is accepted as an alias of torch's ``nccl`` (which
*is* RCCL on ROCm builds); ``gloo`` is kept for the CPU configuration.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

BACKEND_ALIASES = {"rccl": "nccl", "nccl": "nccl", "gloo": "gloo", "mpi": "mpi"}


@dataclass
class DistEnv:
    rank: int
    world_size: int
    local_rank: int
    master_addr: str
    master_port: int

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_master(self) -> bool:
        return self.rank == 0


def read_env() -> DistEnv:
    return DistEnv(
        rank=int(os.environ.get("RANK", "0")),
        world_size=int(os.environ.get("WORLD_SIZE", "1")),
        local_rank=int(os.environ.get("LOCAL_RANK", "0")),
        master_addr=os.environ.get("MASTER_ADDR", "127.0.0.1"),
        master_port=int(os.environ.get("MASTER_PORT", "23456")),
    )


def resolve_backend(name: str | None, use_gpu: bool) -> str:
    """Torch backend for a reference ``--backend`` value.  ``mpi`` (reference
    ``examples/mnist/v1/pytorch_job_mnist_mpi.yaml``, an MPI-built PyTorch
    image) falls back to the collective backend of the device when this
    PyTorch has no MPI support (the ROCm wheels do not): RCCL on a GPU,
    gloo on CPU — same env:// world, same DDP semantics."""
    if not name:
        return "nccl" if use_gpu else "gloo"
    try:
        be = BACKEND_ALIASES[name.lower()]
    except KeyError as e:
        raise ValueError(f"unknown backend {name!r}; choose from {sorted(BACKEND_ALIASES)}") from e
    if be == "mpi" and not dist.is_mpi_available():
        be = "nccl" if use_gpu else "gloo"
        import sys

        print(f"[pto] --backend mpi: this PyTorch has no MPI support, using {be}", file=sys.stderr, flush=True)
    return be


def init_distributed(backend: str | None = None, use_gpu: bool | None = None,
                     timeout_s: float = 300.0) -> tuple[DistEnv, torch.device]:
    """Initialise the default process group from the env contract and pick
    this rank's device.  Safe to call with ``WORLD_SIZE`` unset (single
    process, no process group).

    RCCL failures must surface as a retryable exit instead of a hang
    (SURVEY §5.3), so async error handling is switched on and a finite
    timeout is used.
    """
    env = read_env()
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    if use_gpu:
        n = torch.cuda.device_count()
        device = torch.device("cuda", env.local_rank % max(n, 1))
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")
    if env.is_distributed and not dist.is_initialized():
        be = resolve_backend(backend, use_gpu)
        # 2 = clean up the communicator and raise in the caller instead of
        # abort() (SIGABRT = exit 134, which the operator treats as
        # permanent); the trainer maps the exception to a retryable exit.
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
        timeout_s = float(os.environ.get("PTO_PG_TIMEOUT", timeout_s))
        kwargs = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kwargs["device_id"] = device
        store = generation_store(env, timeout_s)
        if store is not None:
            kwargs.update(store=store, rank=env.rank, world_size=env.world_size)
        dist.init_process_group(**kwargs)
    return env, device


class StaleRendezvous(RuntimeError):
    """This replica reached the rendezvous store of another restart
    generation (an old incarnation's master still serving the port)."""


GENERATION_KEY = "pto/restart-generation"


def generation_store(env: DistEnv, timeout_s: float):
    """Rendezvous store of one restart generation, or None outside the
    operator (no ``PTO_RESTART_GENERATION``: plain ``env://``).

    The node manager tags every restart wave of a job with
    ``PTO_RESTART_GENERATION`` (node/kubelet.py, "Restarts").  Rank 0 hosts
    the TCPStore and publishes its generation; every other rank connects,
    reads it, and refuses a store of a different generation
    (:class:`StaleRendezvous`, which the trainers turn into the retryable
    exit) instead of joining an old world.  Every key of the process group
    and of the trainers (resume path, host barriers) lives under the
    generation's prefix, so nothing of an earlier wave is ever read."""
    gen = os.environ.get("PTO_RESTART_GENERATION")
    if gen is None or not env.is_distributed:
        return None
    store = dist.TCPStore(env.master_addr, env.master_port, env.world_size, env.is_master,
                          timeout=datetime.timedelta(seconds=timeout_s), wait_for_workers=False,
                          use_libuv=os.environ.get("USE_LIBUV", "1") == "1")
    if env.is_master:
        store.set(GENERATION_KEY, gen)
    else:
        theirs = store.get(GENERATION_KEY).decode()
        if theirs != gen:
            raise StaleRendezvous(f"rendezvous at {env.master_addr}:{env.master_port} belongs to restart "
                                  f"generation {theirs}, this replica is generation {gen}")
    return dist.PrefixStore(f"pto/g{gen}", store)


def barrier(device: torch.device | None = None) -> None:
    if dist.is_available() and dist.is_initialized():
        if device is not None and device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


_host_barrier_seq = 0


def host_barrier(timeout_s: float | None = None, tag: str = "hb") -> None:
    """Bounded barrier over the rendezvous TCPStore (no device work, no
    collective on the GPU streams).  Used after long host-side work
    (checkpoint, evaluation) by trainers whose device collectives have
    short spin timeouts (the xGMI all-reduce): no rank launches its next
    chunk of steps before every rank is back.  A rank that died makes the
    others raise after ``timeout_s`` (``PTO_HOST_BARRIER_TIMEOUT``, default
    30 s) instead of blocking until the process-group timeout; the caller
    maps that to the retryable exit."""
    global _host_barrier_seq
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    if timeout_s is None:
        timeout_s = float(os.environ.get("PTO_HOST_BARRIER_TIMEOUT", "30"))
    store = dist.distributed_c10d._get_default_store()
    _host_barrier_seq += 1
    key = f"pto/{tag}/{_host_barrier_seq}"
    store.set(f"{key}/{dist.get_rank()}", "1")
    keys = [f"{key}/{r}" for r in range(dist.get_world_size())]
    try:
        store.wait(keys, datetime.timedelta(seconds=timeout_s))
    except Exception as e:  # noqa: BLE001 - store errors differ by backend/version
        raise TimeoutError(f"host barrier {key} timed out after {timeout_s} s: a peer rank died or stalled "
                           f"({type(e).__name__}: {e})") from e


def all_reduce_max(value: float, device: torch.device) -> float:
    """MAX of a host scalar over ranks (bench reports the slowest rank)."""
    if not (dist.is_available() and dist.is_initialized()):
        return value
    dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cleanup() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
