"""MNIST DDP trainer — the workload container of a PyTorchJob.

CLI-compatible with the reference trainer (``examples/mnist/mnist.py:78-103``:
``--batch-size 64 --test-batch-size 1000 --epochs 1 --lr 0.01
--momentum 0.5 --no-cuda --seed 1 --log-interval 10 --save-model --dir logs
--backend gloo|nccl|mpi``), same log lines (``Train Epoch: ...
loss=...``, ``accuracy=...``), same env:// rendezvous from the operator's
``MASTER_ADDR/MASTER_PORT/WORLD_SIZE/RANK``.

MI355X additions: ``--backend rccl`` (alias of torch's ``nccl`` = RCCL),
``--impl fused`` (hand-written gfx950 kernels + HIP graph, default on GPU)
or ``eager`` (stock PyTorch DDP), synthetic HBM-resident data (no
network), ``--sampler`` for true global throughput, periodic atomic
checkpoints with auto-resume (``--checkpoint-dir``), ``--max-steps``,
and a metrics stream (``$PTO_METRICS_FILE``: first optimizer step time and
samples/s) that the node agent turns into pod annotations for the
submit -> first-step latency metric.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import time

import torch
import torch.distributed as dist

from ..models.mnist import synthetic_mnist
from ..utils import dist as pdist
from ..utils.profiling import torch_trace
from . import checkpoint as ckpt


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="PyTorch MNIST Example (MI355X)")
    p.add_argument("--batch-size", type=int, default=64, metavar="N")
    p.add_argument("--test-batch-size", type=int, default=1000, metavar="N")
    p.add_argument("--epochs", type=int, default=1, metavar="N")
    p.add_argument("--lr", type=float, default=0.01, metavar="LR")
    p.add_argument("--momentum", type=float, default=0.5, metavar="M")
    p.add_argument("--no-cuda", action="store_true", default=False)
    p.add_argument("--seed", type=int, default=1, metavar="S")
    p.add_argument("--log-interval", type=int, default=10, metavar="N")
    p.add_argument("--save-model", action="store_true", default=False)
    p.add_argument("--dir", default="logs", metavar="L")
    p.add_argument("--backend", type=str, default="gloo", choices=["gloo", "nccl", "rccl", "mpi"])
    # MI355X runtime extensions
    p.add_argument("--impl", choices=["fused", "eager"], default=None)
    p.add_argument("--synthetic", action="store_true", default=True)
    p.add_argument("--data", default=None, help="optional .npz with x_train/y_train/x_test/y_test (no pickle)")
    p.add_argument("--data-root", default=os.environ.get("PTO_DATA_ROOT", "../data"),
                   help="IDX files in torchvision's layout (<root>/<dataset>/raw/*-ubyte[.gz]), read if present")
    p.add_argument("--dataset", default="FashionMNIST", help="dataset directory name under --data-root")
    p.add_argument("--train-size", type=int, default=60000)
    p.add_argument("--test-size", type=int, default=10000)
    p.add_argument("--sampler", action="store_true", help="DistributedSampler: shard the data over ranks")
    p.add_argument("--no-shuffle", action="store_true",
                   help="keep the training order fixed (default: reshuffle every epoch like DataLoader(shuffle=True))")
    p.add_argument("--max-steps", type=int, default=0, help="stop after N optimizer steps (0 = full epochs)")
    p.add_argument("--no-test", action="store_true")
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--checkpoint-interval", type=int, default=0)
    p.add_argument("--fail-at-step", type=int, default=int(os.environ.get("PTO_FAIL_AT_STEP", "0")),
                   help="fault injection: SIGKILL self at this step (once)")
    p.add_argument("--fail-rank", type=int, default=int(os.environ.get("PTO_FAIL_RANK", "1")))
    p.add_argument("--profile", default=os.environ.get("PTO_PROFILE_DIR"),
                   help="torch.profiler Chrome trace (HIP kernels + host) of 10 steps into this directory")
    p.add_argument("--comm", choices=["auto", "rccl", "xgmi"], default=None,
                   help="fused trainer gradient all-reduce transport (default: auto = measured at startup)")
    return p.parse_args(argv)


class Metrics:
    def __init__(self):
        self.path = os.environ.get("PTO_METRICS_FILE")
        self.f = open(self.path, "a", buffering=1) if self.path else None

    def emit(self, **rec):
        if self.f:
            self.f.write(json.dumps(rec) + "\n")


def load_data(args, device, rank):
    """Real data when available (``--data`` .npz, or the reference's
    FashionMNIST IDX files under ``--data-root``), normalised like the
    reference (``ToTensor`` + ``Normalize((0.1307,), (0.3081,))``,
    examples/mnist/mnist.py:119-131); synthetic HBM-resident data otherwise."""
    mean, std = 0.1307, 0.3081

    def prep(x):
        t = torch.from_numpy(x.astype("float32"))
        if t.max() > 1.5:
            t = t / 255.0
        return ((t - mean) / std).reshape(-1, 1, 28, 28).to(device)

    if args.data:
        import numpy as np

        z = np.load(args.data, allow_pickle=False)
        return (prep(z["x_train"]), torch.from_numpy(z["y_train"]).long().to(device),
                prep(z["x_test"]), torch.from_numpy(z["y_test"]).long().to(device))
    if args.data_root:
        from ..utils import idx

        d = idx.find_dataset(args.data_root, args.dataset)
        if d is not None:
            (xtr, ytr), (xte, yte) = idx.load_split(d, True), idx.load_split(d, False)
            if rank == 0:
                print(f"[pto] {args.dataset} from {d}: {len(ytr)} train / {len(yte)} test", flush=True)
            return (prep(xtr), torch.from_numpy(ytr).to(device), prep(xte), torch.from_numpy(yte).to(device))
    # reference-equivalent: every rank uses the same seed/order (no sampler)
    # generated on the GPU by one HIP launch (synthetic_mnist source="hash"):
    # a fresh job reaches its first step without host-side data generation
    src = "hash" if device.type == "cuda" else "torch"
    xtr, ytr = synthetic_mnist(args.train_size, device, seed=args.seed, source=src)
    xte, yte = synthetic_mnist(args.test_size, device, seed=args.seed + 7, source=src)
    return xtr, ytr, xte, yte


# Exit code for "a peer died under me": 138 (128+SIGUSR1) is retryable in
# the operator's exit-code table (train_util.go:18-53), so with
# restartPolicy ExitCode the survivors are recreated too and every rank
# resumes from the latest checkpoint (kill/rejoin).
RETRYABLE_EXIT = 138
_COMM_ERRORS = ("XgmiTimeout", "XgmiDivergence", "StaleRendezvous", "host barrier", "Connection closed by peer", "Connection reset by peer", "NCCL", "RCCL", "Broken pipe",
                "timed out", "Timeout", "DistBackendError", "ProcessGroup", "Gloo", "gloo")


def run_with_retryable_exit(fn, *a, **kw):
    """Run a trainer main; a collective/transport failure (dead or stalled
    peer) ends the process with the retryable exit code 138 instead of a
    traceback exit 1, so the ExitCode restart policy recreates it."""
    try:
        return fn(*a, **kw)
    except Exception as e:  # noqa: BLE001
        msg = f"{type(e).__name__}: {e}"
        if any(k in msg for k in _COMM_ERRORS) or isinstance(e, getattr(dist, "DistError", ())):
            print(f"[pto] collective failed ({msg.splitlines()[0][:200]}); exiting {RETRYABLE_EXIT} for restart",
                  flush=True)
            os._exit(RETRYABLE_EXIT)
        raise


def main(argv=None):
    if os.environ.get("PTO_FAULTHANDLER"):  # debugging: SIGUSR2 dumps every thread's stack (exec'd replicas too)
        import faulthandler

        faulthandler.register(signal.SIGUSR2, all_threads=True)
    return run_with_retryable_exit(_main, argv)


def resume_state(ckpt_dir: str | None, rank: int, world: int):
    """Checkpoint to resume from, agreed by every rank: rank 0 picks the
    newest complete checkpoint in ``ckpt_dir`` and broadcasts its path;
    every rank loads THAT file (a rank that cannot read it raises, so no
    two ranks ever resume from different steps).  Returns ``(path, state)``
    or ``(None, None)``."""
    if not ckpt_dir:
        return None, None
    if world > 1 and dist.is_initialized():
        # agreed through the rendezvous store (no device collective): rank
        # 0 publishes its choice, the others block on the key
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            store.set("pto/resume_path", ckpt.latest(ckpt_dir) or "")
        path = store.get("pto/resume_path").decode() or None
    else:
        path = ckpt.latest(ckpt_dir)
    if not path:
        return None, None
    if not os.path.exists(path):
        raise FileNotFoundError(f"rank {rank}: checkpoint {path} chosen by rank 0 is not visible here "
                                f"(--checkpoint-dir must be shared by all replicas)")
    return path, ckpt.load(path, map_location="cpu")


class EpochShuffler:
    """Per-epoch reshuffle of the training set, like the reference's
    ``DataLoader(shuffle=True)`` (examples/mnist/mnist.py:118-124): epoch e
    trains on ``orig[perm(seed, e)]``.  The permutation is a function of
    (seed, epoch) only, so a resumed run sees the same order.  The working
    buffer is updated in place (stream-ordered after the previous steps),
    so the fused trainer's graph-captured data pointer stays valid."""

    def __init__(self, x, y, seed: int, enabled: bool = True):
        self.enabled = enabled
        self.seed = seed
        self.orig_x, self.orig_y = (x.clone(), y.clone()) if enabled else (x, y)
        self.x, self.y = x, y
        self.epoch = None

    def set_epoch(self, epoch: int):
        if not self.enabled or epoch == self.epoch:
            return
        self.epoch = epoch
        g = torch.Generator().manual_seed(self.seed * 100003 + epoch)
        perm = torch.randperm(self.orig_x.shape[0], generator=g).to(self.orig_x.device)
        self.x.copy_(self.orig_x.index_select(0, perm))
        self.y.copy_(self.orig_y.index_select(0, perm))


def _main(argv=None):
    t_main = time.time()
    args = parse_args(argv)
    use_cuda = not args.no_cuda and torch.cuda.is_available() and os.environ.get("PTO_NO_GPU") != "1"
    if use_cuda:
        print("Using CUDA (HIP) on", pdist.gpu_name(0))
    impl = args.impl or ("fused" if use_cuda else "eager")
    if impl == "fused":
        # the fused trainer draws only from the CPU generator (init weights,
        # epoch shuffles); seeding the GPU generators too, as
        # torch.manual_seed does, costs ~0.11 s of submit -> first step
        torch.default_generator.manual_seed(args.seed)
    else:
        torch.manual_seed(args.seed)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rccl_log = (pdist.rccl_log_setup() if use_cuda and world_env > 1 and
                pdist.resolve_backend(args.backend, True) == "nccl" else None)
    env, device = pdist.init_distributed(args.backend, use_gpu=use_cuda)
    t_pg = time.time()
    if env.is_distributed:
        print(f"Using distributed PyTorch with {dist.get_backend()} backend")
    rank, world = env.rank, env.world_size
    metrics = Metrics()
    # TensorBoard scalars like the reference's SummaryWriter(args.dir)
    # (examples/mnist/mnist.py:49,65,108): 'loss' per log interval, 'accuracy' per epoch
    from ..utils.tbevents import SummaryWriter

    writer = SummaryWriter(args.dir) if args.dir else None
    xtr, ytr, xte, yte = load_data(args, device, rank)
    if args.sampler and world > 1:  # DistributedSampler semantics: disjoint shards
        n = xtr.shape[0] // world
        xtr, ytr = xtr[rank * n:(rank + 1) * n].contiguous(), ytr[rank * n:(rank + 1) * n].contiguous()
    dataset_len = xtr.shape[0]
    shuffler = EpochShuffler(xtr, ytr, args.seed, enabled=not args.no_shuffle)

    from .runner import build_trainer

    extra = {"comm": args.comm} if (args.comm and impl == "fused") else {}
    t_data = time.time()
    trainer = build_trainer(impl, device=device, batch_size=args.batch_size, lr=args.lr, momentum=args.momentum,
                            dataset_size=xtr.shape[0], seed=args.seed, rank=rank, data=xtr, target=ytr, **extra)
    t_trainer = time.time()

    def report_world():
        """Evidence, not setup (after the first step): the transport and
        which devices the world spans (RCCL's per-peer transport choice,
        P2P/IPC over xGMI vs SHM)."""
        comm_info = getattr(trainer, "comm_info", None)
        if comm_info and world > 1:
            print(f"[pto] gradient all-reduce: {comm_info}", flush=True)
            metrics.emit(event="comm", rank=rank, **{k: v for k, v in comm_info.items() if not isinstance(v, dict)})
        if world > 1:
            w = pdist.describe_world(device, rccl_log)
            if rank == 0:
                print(f"[pto] world: {json.dumps(w)}", flush=True)
            metrics.emit(event="world", rank=rank, pg_world_size=w["pg_world_size"],
                         rccl_transport=json.dumps(w.get("rccl_transport", {})))

    start_step = 0
    path, st = resume_state(args.checkpoint_dir, rank, world)
    if st is not None:
        trainer.load_state_dict(st["trainer"])
        if st.get("rng"):
            ckpt.set_rng_state(st["rng"])
        start_step = int(st["step"])
        print(f"Resumed from {path} at step {start_step}")
        sys.stdout.flush()

    n_batches = xtr.shape[0] // args.batch_size
    loader_len = -(-dataset_len // args.batch_size)  # len(train_loader): the partial last batch counts
    total_steps = args.epochs * n_batches
    if args.max_steps:
        total_steps = min(total_steps, args.max_steps)
    fail_at = args.fail_at_step if (args.fail_at_step and rank == args.fail_rank and not start_step) else 0
    align = getattr(trainer, "needs_host_barrier", False)
    run = getattr(trainer, "run", None) or (lambda n: [trainer.step() for _ in range(n)])

    def boundary(s: int) -> bool:
        """Host work is due after completing step s (1-based count)."""
        b = (s - 1) % n_batches
        return (s == start_step + 1 or b % args.log_interval == 0 or s % n_batches == 0 or s >= total_steps
                or (args.checkpoint_interval and s % args.checkpoint_interval == 0) or s == fail_at
                or bool(args.profile))

    step = start_step
    t_epoch = time.time()
    samples_since = 0
    t_last = time.time()
    first = True
    trace = torch_trace(args.profile, rank)
    prof_step = trace.__enter__()
    # Log lines are pipelined on the fused trainer: the loss of a log chunk
    # is copied to pinned memory without waiting, the next chunk is
    # enqueued, and only then is the line printed (its copy is done by then
    # and the device is already running the next chunk), so logging every
    # 10 steps costs no device idle time.  samples/s is measured between
    # consecutive resolved log points.
    loss_async = getattr(trainer, "loss_async", None) if device.type == "cuda" else None
    pending = []

    def resolve():
        nonlocal samples_since, t_last
        for rec in pending:
            ep, bi, st, n_samples, lv = rec
            if isinstance(lv, tuple):
                lv[1].synchronize()
                lv = float(lv[0])
            now = time.time()
            samples_since += n_samples
            dt = max(now - t_last, 1e-9)
            sps = samples_since / dt
            step_s = dt * args.batch_size / max(samples_since, 1)
            samples_since, t_last = 0, now
            print("Train Epoch: {} [{}/{} ({:.0f}%)]\tloss={:.4f}".format(
                ep, bi * args.batch_size, dataset_len, 100.0 * bi / loader_len, lv))
            metrics.emit(event="train", step=st, loss=lv, samples_per_sec=round(sps * world, 1),
                         step_seconds=step_s, rank=rank)
            if writer:
                writer.add_scalar("loss", lv, ep * n_batches + bi)
        pending.clear()

    unlogged = 0  # samples run since the last queued log record
    while step < total_steps:
        if fail_at and step == fail_at:
            resolve()
            print(f"[fault-injection] rank {rank} SIGKILL at step {step}", flush=True)
            os.kill(os.getpid(), signal.SIGKILL)
        epoch = step // n_batches + 1
        shuffler.set_epoch(epoch)
        # steps up to the next log / checkpoint / epoch / fault boundary in
        # one call: the fused trainer replays its multi-step HIP graphs and
        # checks the gradient transport's error word once per chunk (without
        # waiting for the chunk when a log line is all that follows it)
        k = 1
        while step + k < total_steps and not boundary(step + k):
            k += 1
        s_next = step + k
        hard = (s_next >= total_steps or s_next % n_batches == 0 or s_next == fail_at or bool(args.profile)
                or bool(args.checkpoint_dir and args.checkpoint_interval and s_next % args.checkpoint_interval == 0))
        if loss_async is not None and not first and not hard:
            run(k, blocking_check=False)
        else:
            run(k)
        resolve()  # the previous chunk's log line: its loss copy finished before this chunk started
        prof_step()
        step += k
        unlogged += args.batch_size * k
        batch_idx = (step - 1) % n_batches
        if first:
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            t_first = time.time()
            metrics.emit(event="first_step", t=t_first, rank=rank)
            try:
                import psutil

                t_proc = psutil.Process().create_time()
            except Exception:  # noqa: BLE001 - timing evidence only
                t_proc = t_main
            # where a replica's submit -> first step went (process start is
            # the fork of the node's warm interpreter)
            zt = [float(v) for v in os.environ.get("PTO_ZYGOTE_T", "").split(",") if v]
            zyg = ({"fork_to_setup_s": round(zt[0] - t_proc, 4), "zygote_setup_s": round(zt[1] - zt[0], 4),
                    "runpy_to_main_s": round(t_main - zt[1], 4)} if len(zt) == 2 else {})
            metrics.emit(event="startup", rank=rank, process_to_main_s=round(t_main - t_proc, 4), **zyg,
                         pg_init_s=round(t_pg - t_main, 4), data_s=round(t_data - t_pg, 4),
                         trainer_s=round(t_trainer - t_data, 4), first_step_s=round(t_first - t_trainer, 4))
            first = False
            report_world()
            t_last = time.time()
        if batch_idx % args.log_interval == 0:
            lv = loss_async() if loss_async is not None else trainer.last_loss()
            pending.append((epoch, batch_idx, step, unlogged, lv))
            unlogged = 0
            if hard or loss_async is None:
                resolve()
        ckpt_due = bool(args.checkpoint_dir and args.checkpoint_interval and step % args.checkpoint_interval == 0)
        if ckpt_due and rank == 0:
            ckpt.save(args.checkpoint_dir, step, {"trainer": trainer.state_dict(), "rng": ckpt.rng_state()})
        end_of_epoch = step % n_batches == 0 or step == total_steps
        if end_of_epoch and not args.no_test:
            if hasattr(trainer, "evaluate"):
                test_loss, acc = trainer.evaluate(xte, yte, args.test_batch_size)
            else:
                test_loss, acc = evaluate_module(trainer.model, xte, yte, args.test_batch_size)
            print("\naccuracy={:.4f}\n".format(acc))
            if writer:
                writer.add_scalar("accuracy", acc, epoch)
                writer.flush()
            metrics.emit(event="test", epoch=epoch, accuracy=acc, loss=test_loss, rank=rank,
                         epoch_seconds=round(time.time() - t_epoch, 3))
            t_epoch = time.time()
        if align and (ckpt_due or (end_of_epoch and not args.no_test)) and step < total_steps:
            # xGMI barriers spin with a short timeout: nobody starts the next
            # chunk until every rank is done with its host work
            pdist.host_barrier()
        sys.stdout.flush()
    resolve()
    trace.__exit__(None, None, None)
    if writer:
        writer.close()
    if args.checkpoint_dir and rank == 0:
        ckpt.save(args.checkpoint_dir, step, {"trainer": trainer.state_dict(), "rng": ckpt.rng_state()})
    if args.save_model and rank == 0:
        sd = trainer.state_dict()["model"]
        prefix = "module." if world > 1 else ""
        torch.save({prefix + k: v.cpu() for k, v in sd.items()}, "mnist_cnn.pt")
    pdist.cleanup()
    return 0


@torch.no_grad()
def evaluate_module(model, x, y, bs):
    import torch.nn.functional as F

    model.eval()
    loss, correct = 0.0, 0
    for i in range(0, x.shape[0], bs):
        out = model(x[i:i + bs])
        loss += F.nll_loss(out, y[i:i + bs], reduction="sum").item()
        correct += (out.argmax(1) == y[i:i + bs]).sum().item()
    model.train()
    return loss / x.shape[0], correct / x.shape[0]


if __name__ == "__main__":
    sys.exit(main())
