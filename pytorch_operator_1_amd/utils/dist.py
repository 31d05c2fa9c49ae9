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


def gpu_count() -> int:
    """Visible GPUs as the HIP runtime counts them (honours
    ``HIP_VISIBLE_DEVICES``).  ``torch.cuda.device_count()`` on ROCm asks
    amdsmi first, and its first ``amdsmi_init`` costs ~0.11 s on the MI355X
    box, on a fresh job's submit -> first step path
    (profiles/startup_latency_r4.md)."""
    return int(torch._C._cuda_getDeviceCount()) if torch.cuda.is_available() else 0


KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def _visible_list(value: str | None) -> list[str] | None:
    if value is None:
        return None
    return [v for v in (s.strip() for s in value.split(",")) if v]


def visible_gpu_count_no_hip(env: dict | None = None, topology: str | None = None) -> int:
    """GPUs a child process will see, counted WITHOUT the HIP runtime or
    amdsmi (a launcher that starts rank processes must never initialise the
    GPU itself -- on this pool a process that did may not start GPU
    children).  Physical GPUs are the KFD topology nodes whose
    ``gfx_target_version`` is non-zero (CPU nodes report 0); the
    ``ROCR_VISIBLE_DEVICES`` list restricts them, and ``HIP_VISIBLE_DEVICES``
    (or ``CUDA_VISIBLE_DEVICES``) indexes into what ROCr left."""
    env = os.environ if env is None else env
    topology = KFD_TOPOLOGY if topology is None else topology
    n = 0
    try:
        for node in os.listdir(topology):
            try:
                with open(os.path.join(topology, node, "properties")) as f:
                    for line in f:
                        k, _, v = line.partition(" ")
                        if k == "gfx_target_version":
                            n += int(v.strip() or "0") != 0
                            break
            except (OSError, ValueError):
                continue
    except OSError:
        n = 0
    rocr = _visible_list(env.get("ROCR_VISIBLE_DEVICES"))
    if rocr is not None:
        n = min(n, len(rocr)) if n else len(rocr)
    hip = _visible_list(env.get("HIP_VISIBLE_DEVICES"))
    if hip is None:
        hip = _visible_list(env.get("CUDA_VISIBLE_DEVICES"))
    if hip is not None:
        n = min(n, len(hip)) if n else len(hip)
    return n


def gpu_name(index: int = 0) -> str:
    """Marketing name of a visible GPU, without ``torch.cuda.device_count()``
    (see :func:`gpu_count`)."""
    torch.cuda.init()  # defines torch.cuda._get_device_properties (C++ binding)
    props = getattr(torch.cuda, "_get_device_properties", None)
    return props(index).name if props is not None else torch.cuda.get_device_name(index)


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
        n = gpu_count()
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
    if use_gpu and env.is_distributed and os.environ.get("PTO_CU_PARTITION") == "1":
        # ranks that share a GPU (a rehearsal on fewer GPUs than ranks):
        # each on its own CU partition, so they run the schedules of one
        # rank per GPU (utils/cu_partition.py)
        from . import cu_partition

        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", env.world_size))
        cu_partition.activate_for_rank(env.local_rank, local_world, device)
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
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") or os.environ.get("TORCHELASTIC_RUN_ID"):
        # torchrun inside the pod: MASTER_PORT is the elastic agent's own
        # TCPStore, and the agent already scopes every rendezvous to its run
        # -- hosting a second store there would fail with EADDRINUSE
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


def params_fingerprint(tensors, chunk: int = 1 << 22) -> int:
    """Exact 64-bit fingerprint of the BITS of ``tensors`` (any float
    dtype): sum over elements of (raw bits) x (a position weight), in int64
    arithmetic, so it is bit-exact and independent of reduction order.  Two
    replicas of a data-parallel model agree iff (up to a negligible
    collision chance) their parameters are bit-identical."""
    h = 0
    pos = 0
    for t in tensors:
        v = t.detach().contiguous().view(-1)
        iv = {4: torch.int32, 2: torch.int16, 8: torch.int64, 1: torch.uint8}[v.element_size()]
        v = v.view(iv)
        for i in range(0, v.numel(), chunk):
            c = v[i:i + chunk].to(torch.int64)
            w = (torch.arange(c.numel(), device=c.device, dtype=torch.int64) + (pos + i)) % 1_000_003 + 1
            h = (h + int((c * w).sum().item())) & 0xFFFFFFFFFFFFFFFF
        pos += v.numel()
    return h


def ranks_bit_identical(tensors, device: torch.device) -> bool | None:
    """Whether every rank holds bit-identical ``tensors`` (the data-parallel
    replicas after a run): their fingerprints all-gathered and compared.
    Collective; None without a process group of more than one rank."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return None
    fp = params_fingerprint(tensors)
    allfp = [None] * dist.get_world_size()
    dist.all_gather_object(allfp, fp)
    return len(set(allfp)) == 1


def rccl_log_setup() -> str | None:
    """Route RCCL's INFO log (communicator init and transport selection
    only: no per-collective lines) to a per-process file, so the transport
    RCCL picked for each peer (P2P/IPC over xGMI, SHM, NET) can be reported.
    Must run before the process group is created; a user-set NCCL_DEBUG is
    left alone (returns None)."""
    if os.environ.get("NCCL_DEBUG") or os.environ.get("NCCL_DEBUG_FILE"):
        return None
    import tempfile

    path = os.path.join(tempfile.gettempdir(), f"pto-rccl-{os.getpid()}.log")
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT,P2P,SHM,NET,GRAPH"
    os.environ["NCCL_DEBUG_FILE"] = path
    return path


_CHANNEL_RE = None


def parse_rccl_transports(text: str) -> dict:
    """Transport summary from an RCCL/NCCL INFO log: how many ring/tree
    channel connections use each transport (``via P2P/IPC``, ``via SHM``,
    ``via NET/...``), plus the channel/ring counts RCCL reports."""
    import re

    global _CHANNEL_RE
    if _CHANNEL_RE is None:
        _CHANNEL_RE = re.compile(r"Channel \d+(?:/\d+)? ?: ?\d+\[[^\]]*\] -> \d+\[[^\]]*\] (?:\[\w+\] )?via (\S+)")
    via: dict[str, int] = {}
    for m in _CHANNEL_RE.finditer(text):
        via[m.group(1)] = via.get(m.group(1), 0) + 1
    out: dict = {"via": via}
    m = re.search(r"(\d+) coll channels,[^\n]*?(\d+) p2p channels", text)
    if m:
        out["coll_channels"], out["p2p_channels"] = int(m.group(1)), int(m.group(2))
    m = re.search(r"RCCL version\s*(\S+)|NCCL version\s*(\S+)", text)
    if m:
        out["version"] = m.group(1) or m.group(2)
    return out


def describe_world(device: torch.device, rccl_log: str | None = None) -> dict:
    """What the measured world really was (bench.py evidence): the world
    size the process group reports, every rank's device (PCI bus id / UUID),
    and -- with an RCCL log from :func:`rccl_log_setup` -- the transports
    RCCL chose.  Collective over the default group (call it on every rank,
    outside timed regions); world size 1 returns the local entry."""
    me: dict = {"device": str(device)}
    if device.type == "cuda":
        props = torch.cuda.get_device_properties(device)
        me["name"] = props.name
        bus = [getattr(props, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id")]
        if None not in bus:
            me["pci"] = "%04x:%02x:%02x" % tuple(bus)
        uuid = getattr(props, "uuid", None)
        if uuid is not None:
            me["uuid"] = str(uuid)
        me["visible"] = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if rccl_log and os.path.exists(rccl_log):
        with open(rccl_log, errors="replace") as f:
            me["rccl"] = parse_rccl_transports(f.read())
    pg = dist.is_available() and dist.is_initialized()
    ranks = [me]
    if pg and dist.get_world_size() > 1:
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, me)
    out = {"pg_world_size": dist.get_world_size() if pg else 1, "ranks": ranks}
    devs = [r.get("pci") or r.get("uuid") for r in ranks]
    if None not in devs:
        out["distinct_devices"] = len(set(devs))
    via: dict[str, int] = {}
    for r in ranks:
        for k, v in (r.get("rccl") or {}).get("via", {}).items():
            via[k] = via.get(k, 0) + v
    if via:
        out["rccl_transport"] = via
    return out


def cleanup() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
