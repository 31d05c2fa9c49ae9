#!/usr/bin/env python3
"""Headline benchmark: MNIST DDP training samples/sec (BASELINE.json).

Config (reference ``examples/mnist/mnist.py``): the reference ``Net``
(431,080 fp32 params), batch 64 per rank, SGD lr=0.01 momentum=0.5,
NLL loss on log-softmax, DDP gradient averaging, fp32 compute.  One
process per GPU; for N>1 the driver launches this file under
``torch.distributed.run`` and ranks talk RCCL (torch backend ``nccl``).

Weak scaling: per-rank batch is fixed at 64, ``value`` is the aggregate
samples/s over all ranks (reference-equivalent mode: no sampler, every
rank runs its own batch stream, exactly like the reference's mnist.py).

Other configs of BASELINE.json (same contract, same timing bracket):
``--model resnet50`` (config 3: ResNet-50 224x224 bf16 DDP, images/s) and
``--model llama3-8b`` (config 4: Llama-3-8B bf16 DDP, tokens/s + MFU).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--impl fused|eager]
                        [--model mnist|resnet50|llama3-8b|llama3-1b]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

# Reference-derived per-rank throughput lower bound (60,000
# samples / 286 s on the CPU cluster, gloo, 2 ranks).
BASELINE_SAMPLES_PER_SEC_PER_RANK = 210.0


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="timed steps (default 2000 mnist, 20 others)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (default 200 mnist, 3 others)")
    p.add_argument("--model", default=os.environ.get("BENCH_MODEL", "mnist"),
                   choices=["mnist", "resnet50", "llama3-8b", "llama3-1b", "llama3-tiny"])
    p.add_argument("--batch-size", type=int, default=None, help="per-rank batch (64 mnist, 256 resnet50, 4 x seq-len llama: 191 GB of the 288 GB HBM)")
    p.add_argument("--seq-len", type=int, default=4096, help="llama sequence length")
    p.add_argument("--checkpoint", choices=["none", "full"], default="none", help="llama activation checkpointing")
    p.add_argument("--breakdown", action="store_true",
                   help="large models: time forward/backward/allreduce-wait/optimizer with HIP events "
                        "(extra pass after the timed steps; printed to stderr)")
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.5)
    p.add_argument("--impl", choices=["fused", "eager"], default=os.environ.get("BENCH_IMPL", "fused"))
    p.add_argument("--dataset-size", type=int, default=60000)
    p.add_argument("--sampler", action="store_true",
                   help="DistributedSampler semantics: one dataset, disjoint per-rank shards (true global "
                        "throughput); default: every rank its own stream (reference-equivalent, no sampler)")
    p.add_argument("--cpu", action="store_true", help="run on CPU with gloo (debug only)")
    p.add_argument("--no-latency", action="store_true",
                   help="skip the submit -> first-step measurement (default: measured at world size 1, after "
                        "the throughput run, through the whole operator stack)")
    p.add_argument("--force-ddp", action="store_true",
                   help="large models at --gpus 1: the whole DDP path (flat buckets, comm stream, per-bucket "
                        "collectives over a 1-rank RCCL group, xGMI hook) -- its cost on one GPU")
    p.add_argument("--verbose", action="store_true")
    return p.parse_args(argv)


def _launch_ranks(args, argv) -> int | None:
    """``--gpus N`` (N > 1) without a launcher: start N fresh rank processes
    under ``torch.distributed.run`` (127.0.0.1 rendezvous) as CHILDREN of
    this one, before anything here touches the GPU, and return their exit
    code.  Never measures fewer ranks than asked for: a world size that
    disagrees with ``--gpus`` is an error.  Returns None when this process
    is itself a rank (or N == 1)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr, flush=True)
            return 2
        return None
    if args.gpus <= 1:
        return None
    host_ranks = args.cpu or os.environ.get("PTO_BACKEND") == "gloo"
    if not host_ranks:
        # counted from KFD sysfs + the visibility env, never through torch:
        # this parent starts the GPU ranks, so it must not initialise HIP
        from pytorch_operator_1_amd.utils.dist import visible_gpu_count_no_hip

        n_dev = visible_gpu_count_no_hip()
        if n_dev < args.gpus:
            print(f"[bench] error: --gpus {args.gpus} but only {n_dev} GPU(s) visible; refusing to measure fewer "
                  f"ranks (PTO_BACKEND=gloo rehearses several ranks on one GPU)", file=sys.stderr, flush=True)
            return 2
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    argv = list(sys.argv[1:] if argv is None else argv)
    env = None
    if host_ranks and os.environ.get("PTO_CU_PARTITION") == "1":
        # several ranks stacked on one GPU, each on its own CU partition: one
        # pooled hardware queue per rank, or with 4+ ranks the queues outnumber
        # what the scheduler maps at once and it time-slices them (~22 ms/step
        # at 4 ranks vs 0.10 ms, profiles/cu_partition_r6.md).  Overrides an
        # inherited GPU_MAX_HW_QUEUES (GPU boxes export HIP's default, 4);
        # PTO_CU_HW_QUEUES picks another count
        env = dict(os.environ, GPU_MAX_HW_QUEUES=os.environ.get("PTO_CU_HW_QUEUES", "1"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    print(f"[bench] starting {args.gpus} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


_RESULT_FD = None


def _reserve_stdout():
    """The contract is ONE JSON line on stdout.  Libraries print banners
    there from C (RCCL's "RCCL version : ..." block at communicator init), so
    the real stdout is kept aside and fd 1 -- C and Python alike -- goes to
    stderr for the rest of the run; :func:`_emit` writes the result line to
    the kept descriptor."""
    global _RESULT_FD
    if _RESULT_FD is None:
        sys.stdout.flush()
        _RESULT_FD = os.dup(1)
        os.dup2(2, 1)


def _emit(line: str):
    sys.stdout.flush()
    fd = _RESULT_FD if _RESULT_FD is not None else 1
    os.write(fd, (line + "\n").encode())


def _xgmi_failure(e: BaseException) -> bool:
    """A peer-memory exchange that timed out (a bounded spin gave up: a peer
    stalled) -- the one failure the RCCL schedule may stand in for.  Matched
    on the exception TYPE only.  A divergence of the ranks' parameters
    (XgmiDivergence, a subclass) is a correctness failure: it is re-raised
    and the bench exits non-zero instead of reporting another schedule's
    number."""
    from pytorch_operator_1_amd.parallel.xgmi import XgmiDivergence, XgmiTimeout

    return isinstance(e, XgmiTimeout) and not isinstance(e, XgmiDivergence)


def main(argv=None):
    args = parse_args(argv)
    rc = _launch_ranks(args, argv)
    if rc is not None:
        return rc
    _reserve_stdout()
    mnist = args.model == "mnist"
    if args.steps is None:
        args.steps = 2000 if mnist else 20
    if args.warmup is None:
        args.warmup = 200 if mnist else 3
    if args.batch_size is None:
        args.batch_size = 64 if mnist else (256 if args.model == "resnet50" else 4)
    from pytorch_operator_1_amd.utils import dist as pdist

    use_gpu = torch.cuda.is_available() and not args.cpu
    # PTO_BACKEND=gloo: rehearse the multi-rank path with several ranks on
    # one GPU (RCCL refuses duplicate devices); default nccl (= RCCL) on GPU
    rccl_log = pdist.rccl_log_setup() if (use_gpu and args.gpus > 1 and
                                          os.environ.get("PTO_BACKEND", "nccl") in ("nccl", "rccl")) else None
    env, device = pdist.init_distributed(os.environ.get("PTO_BACKEND"), use_gpu=use_gpu)
    if env.world_size != args.gpus:  # unreachable after _launch_ranks; never report a mislabelled world
        raise SystemExit(f"[bench] --gpus {args.gpus} but the process group has {env.world_size} ranks")

    if not mnist:
        return run_model_bench(args, env, device, pdist, rccl_log)

    from pytorch_operator_1_amd.train.runner import build_trainer

    data_kw = {}
    if args.sampler and env.world_size > 1:
        from pytorch_operator_1_amd.models.mnist import synthetic_mnist

        x, y = synthetic_mnist(args.dataset_size, device, seed=1)  # the same dataset on every rank
        data_kw = dict(data=x[env.rank::env.world_size].contiguous(), target=y[env.rank::env.world_size].contiguous())
    trainer = build_trainer(args.impl, device=device, batch_size=args.batch_size, lr=args.lr,
                            momentum=args.momentum, dataset_size=args.dataset_size,
                            seed=1, rank=env.rank, **data_kw)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    injected = []

    def measure(trainer):
        """Warm-up, then EXACTLY K timed steps; (elapsed, None), or (None,
        reason) when the peer-memory exchange failed.  Its failures reach
        every rank (a rank whose peer stopped times out waiting for it; the
        parameter-hash check runs on all of them), and the status all-reduces
        double as the timing barriers, so the ranks leave together."""
        run = getattr(trainer, "run", None) or (lambda n: [trainer.step() for _ in range(n)])
        status, reason = 0.0, None
        try:
            if os.environ.get("PTO_BENCH_INJECT_XGMI_FAILURE") in ("all", str(env.rank)) and not injected:
                injected.append(1)  # test hook: the exchange "times out" once
                from pytorch_operator_1_amd.parallel.xgmi import XgmiTimeout

                raise XgmiTimeout("injected by PTO_BENCH_INJECT_XGMI_FAILURE")
            run(args.warmup)
            # graph capture is setup, never timed: a warm-up of 0 or 1 step (the
            # first step runs eagerly) would otherwise leave it to the timed run()
            getattr(trainer, "prepare", lambda: None)()
            sync()
        except Exception as e:  # noqa: BLE001 - only comm failures are handled
            if not _xgmi_failure(e):
                raise
            status, reason = 1.0, f"warm-up: {type(e).__name__}: {e}"[:300]
        if pdist.all_reduce_max(status, device):  # also the barrier before the timed region
            return None, reason or "a peer rank's exchange failed"
        sync()
        t0 = time.perf_counter()
        try:
            run(args.steps)  # exactly K optimizer steps
            # the fused-optimizer schedule applies conv1's update of step i inside
            # step i+1's launches: commit the last one inside the timed region so it
            # holds K complete updates
            getattr(trainer, "flush", lambda: None)()
            sync()
        except Exception as e:  # noqa: BLE001
            if not _xgmi_failure(e):
                raise
            status, reason = 1.0, f"timed run: {type(e).__name__}: {e}"[:300]
        if pdist.all_reduce_max(status, device):  # the barrier after it
            return None, reason or "a peer rank's exchange failed"
        sync()
        elapsed = time.perf_counter() - t0
        return pdist.all_reduce_max(elapsed, device), None

    def make():
        return build_trainer(args.impl, device=device, batch_size=args.batch_size, lr=args.lr,
                             momentum=args.momentum, dataset_size=args.dataset_size,
                             seed=1, rank=env.rank, **data_kw)

    elapsed, failed = measure(trainer)
    if elapsed is None:
        # the xGMI schedule failed mid-run (bounded spin timed out, or the
        # in-graph parameter hashes of the ranks diverged): report the RCCL
        # schedule's number instead of none, and say so in the JSON
        print(f"[bench] xGMI exchange failed ({failed}); re-measuring on the RCCL schedule", file=sys.stderr)
        os.environ["PTO_COMM"] = "rccl"
        trainer = make()
        elapsed, again = measure(trainer)
        if elapsed is None:
            raise SystemExit(f"[bench] the RCCL schedule failed too: {again}")
    run = None
    loss = trainer.last_loss()
    # evidence of the world that was measured (outside the timed region):
    # the ranks, their devices and transports, and whether the replicas
    # still hold bit-identical parameters after the timed steps
    world = pdist.describe_world(device, rccl_log)
    identical = pdist.ranks_bit_identical(_param_tensors(trainer), device)
    comm = dict(getattr(trainer, "comm_info", None) or {})
    comm.update(world)
    if failed:
        comm["xgmi_failed_fell_back_to_rccl"] = failed

    n = env.world_size
    ms_per_step = elapsed / args.steps * 1e3
    value = args.batch_size * n * args.steps / elapsed
    out = None
    if env.rank == 0:
        out = {
            "metric": "samples/sec MNIST DDP",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (BASELINE_SAMPLES_PER_SEC_PER_RANK * n), 1),
            "dtype": "fp32",
            "data": ("synthetic (MNIST-shaped 1x28x28, resident in HBM), random-init weights" if device.type == "cuda"
                     else "synthetic (MNIST-shaped 1x28x28, in host memory), random-init weights"),
            "config": {
                "model": "mnist-cnn (reference examples/mnist/mnist.py Net, 431,080 params)",
                "global_batch": args.batch_size * n,
                "per_rank_batch": args.batch_size,
                "seq_len": None,
                "input_shape": [1, 28, 28],
                "optimizer": f"SGD lr={args.lr} momentum={args.momentum}",
                "parallelism": f"dp{n}",
                "impl": args.impl,
                "sampler": ("DistributedSampler (disjoint shards of one dataset)" if args.sampler and n > 1
                            else "none (every rank its own batch stream, reference-equivalent)"),
                "backend": (torch.distributed.get_backend() if n > 1 else "none"),
                "baseline": "210 samples/s/rank (BASELINE.md, derived lower bound); vs_baseline = value/(210*n_gpus)",
                "final_loss": round(loss, 4) if loss is not None else None,
                "grad_allreduce": comm,
            },
        }
        if identical is not None:
            out["ranks_bit_identical"] = identical
    pdist.cleanup()
    if out is not None and not args.no_latency and os.environ.get("BENCH_LATENCY", "1") == "1":
        # second half of the BASELINE metric, outside the timed region, on
        # rank 0 after the process group is gone: a job of n replicas
        # (Master=1, Worker=n-1) submitted through the whole operator stack.
        # The trainer's buffers are released first (the job runs on these
        # GPUs); the other ranks have nothing left to do and exit.
        del trainer, run
        if device.type == "cuda":
            torch.cuda.synchronize(device)
            torch.cuda.empty_cache()
        lat = measure_submit_to_first_step(gpu=device.type == "cuda", replicas=n)
        out["submit_to_first_step_s"] = lat.get("submit_to_first_step_s")
        out["config"]["submit_to_first_step"] = lat
    if out is not None:
        _emit(json.dumps(out))
    if identical is False:
        print("[bench] error: the data-parallel replicas diverged (parameters not bit-identical across ranks)",
              file=sys.stderr, flush=True)
        return 3


def _param_tensors(trainer) -> list:
    """The parameters whose replicas must agree across ranks."""
    p = getattr(trainer, "params", None)
    if isinstance(p, torch.Tensor):
        return [p]
    m = getattr(trainer, "model", None)
    return [t for t in m.parameters()] if m is not None else []


def measure_submit_to_first_step(gpu: bool, replicas: int = 1, timeout: float = 240.0) -> dict:
    """CRD-submit -> first optimizer step through the whole local stack:
    in-process API store + PyTorchJob controller + node manager, whose C++
    node agent and warm interpreter (zygote) are fresh CHILD processes of
    this one (nothing is exec'ed in place), then the trainer processes they
    start.  ``replicas`` = 1 Master + (replicas - 1) Workers, each with
    ``amd.com/gpu: 1`` and the fused HIP trainer over RCCL (the reference's
    GPU figure is for a Master + Worker job), or the eager trainer over
    gloo with ``--cpu``.  With fewer GPUs than replicas (a rehearsal on a
    one-GPU box) the node offers each GPU to several replicas and the job
    uses gloo.  The first step is the Master's.  The node is up before the
    job arrives (the zygote's imports are done), like the reference's
    cluster, whose submit -> Running was 121 s (CPU) / 334 s (GPU)
    (BASELINE.md)."""
    import math
    import tempfile

    from pytorch_operator_1_amd.api.types import new_job
    from pytorch_operator_1_amd.cluster import LocalCluster
    from pytorch_operator_1_amd.utils.dist import visible_gpu_count_no_hip

    share = 1
    if gpu and replicas > 1:
        share = max(1, math.ceil(replicas / max(1, visible_gpu_count_no_hip())))
    res = {"replicas": "Master=1" + (f", Worker={replicas - 1}" if replicas > 1 else ""),
           "trainer": "fused (HIP graphs)" if gpu else "eager (gloo, CPU)"}
    if share > 1:
        res["gpu_share"] = share
    os.environ.setdefault("PTO_ZYGOTE", "1")
    # this process may be a torchrun rank: the node agent and its pods must
    # not inherit the launcher's rendezvous (TORCHELASTIC_USE_AGENT_STORE
    # would make every replica a client of a store nobody hosts)
    scrub = [k for k in os.environ if k.startswith(("TORCHELASTIC_", "NCCL_DEBUG")) or k in
             ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK",
              "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT", "TORCH_NCCL_ASYNC_ERROR_HANDLING")]
    saved_env = {k: os.environ.pop(k) for k in scrub}
    t_start = time.time()
    try:
        with tempfile.TemporaryDirectory(prefix="pto-bench-") as d, \
                LocalCluster(gpus=None if gpu else 0, log_dir=d, serve_http=False, gpu_share=share) as c:
            res["zygote_warm"] = bool(c.kubelet.agent.wait_warm(120))
            res["node_startup_s"] = round(time.time() - t_start, 3)
            backend = "gloo" if (not gpu or share > 1) else "rccl"
            margs = (["--backend", backend, "--impl", "fused"] if gpu else ["--backend", "gloo", "--no-cuda",
                                                                           "--train-size", "2560"])
            margs += ["--max-steps", "20", "--log-interval", "10", "--no-test", "--dir", ""]
            job = new_job("bench-latency", image="pto/pytorch-mnist:rocm", master_args=margs,
                          workers=replicas - 1, gpus=1 if gpu else 0)
            t0 = time.time()
            c.submit(job)
            j = c.wait_for_condition("bench-latency", timeout=timeout)
            pod = c.store.get("pods", "default", "bench-latency-master-0")
            ann = pod["metadata"].get("annotations") or {}
            first = ann.get("pto.amd.com/first-step-unix")
            if ann.get("pto.amd.com/startup-phases"):
                res["master_phases_s"] = json.loads(ann["pto.amd.com/startup-phases"])
            res["job_state"] = j["status"]["conditions"][-1]["type"]
            if first is not None:
                res["submit_to_first_step_s"] = round(float(first) - t0, 3)
            else:
                res["error"] = "no first-step annotation"
                res["log_tail"] = c.pod_log("default", "bench-latency-master-0")[-500:]
    except Exception as e:  # noqa: BLE001 - the throughput result still stands
        res["error"] = f"{type(e).__name__}: {e}"[:500]
    finally:
        os.environ.update(saved_env)
    return res


# Dense bf16 MFMA peak of one MI355X (no sparsity), for MFU reporting.
MI355X_BF16_DENSE_FLOPS = 2.5e15


def run_model_bench(args, env, device, pdist, rccl_log=None):
    """BASELINE configs 3/4: ResNet-50 / Llama-3 DDP, full optimizer steps."""
    from pytorch_operator_1_amd.train.bench_models import LlamaTrainer, ResNetTrainer

    if device.type != "cuda":
        raise SystemExit(f"--model {args.model} needs a GPU")
    force = bool(args.force_ddp)
    if force and env.world_size == 1 and not torch.distributed.is_initialized():
        # a real 1-rank RCCL group on 127.0.0.1, so every bucket's collective is issued
        import socket

        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                             device_id=device)
    if args.model == "resnet50":
        trainer = ResNetTrainer(device, batch_size=args.batch_size, seed=env.rank, force_ddp=force)
    else:
        trainer = LlamaTrainer(device, model=args.model, batch_size=args.batch_size, seq_len=args.seq_len,
                               seed=env.rank, checkpoint=args.checkpoint, force_ddp=force)
    trainer.run(args.warmup)
    torch.cuda.synchronize(device)
    pdist.barrier(device)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    trainer.run(args.steps)
    torch.cuda.synchronize(device)
    pdist.barrier(device)
    torch.cuda.synchronize(device)
    elapsed = pdist.all_reduce_max(time.perf_counter() - t0, device)
    identical = pdist.ranks_bit_identical(_param_tensors(trainer), device)
    breakdown = None
    if args.breakdown:  # separate, untimed pass so event records do not perturb the measurement
        trainer.timer.enabled = True
        trainer.run(max(2, min(args.steps, 5)))
        breakdown = trainer.timer.summary()
        trainer.timer.enabled = False
        print(f"[bench] phase ms/step: {breakdown}", file=sys.stderr)
    n = env.world_size
    per_step = trainer.samples_per_step()
    value = per_step * n * args.steps / elapsed
    world = pdist.describe_world(device, rccl_log)
    if env.rank == 0:
        cfg = {"model": args.model, "global_batch": args.batch_size * n, "per_rank_batch": args.batch_size,
               "seq_len": args.seq_len if args.model.startswith("llama") else None,
               "parallelism": f"dp{n}" + (" (DDP path forced: 1-rank RCCL group)" if force and n == 1 else ""),
               "backend": (torch.distributed.get_backend() if (n > 1 or force) else "none"),
               "bucket_mb": round(max((b["hi"] - b["lo"]) * trainer.bucketer.flat[b["dtype"]].element_size()
                                      for b in trainer.bucketer.buckets) / 2**20, 1)
               if trainer.bucketer.buckets else None,
               "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 1e9, 1),
               "final_loss": trainer.last_loss()}
        cfg.update(trainer.describe())
        cfg["world"] = world
        cfg["grad_allreduce"] = dict(getattr(trainer.bucketer, "comm_info", {}) or {})
        if identical is not None:
            cfg["ranks_bit_identical"] = identical
        if breakdown:
            cfg["phase_ms"] = breakdown
        if args.model.startswith("llama") and n == 1:
            # what one rank of the N=8 run holds: this run's peak plus, when it
            # ran without buckets, the flat bf16 gradient buffer DDP adds
            extra = 0 if trainer.bucketer.flat else sum(p.numel() * p.element_size()
                                                        for p in trainer.model.parameters())
            cfg["projected_dp8_peak_gb"] = round((torch.cuda.max_memory_allocated(device) + extra) / 1e9, 1)
            cfg["hbm_gb"] = round(torch.cuda.get_device_properties(device).total_memory / 1e9, 1)
        if hasattr(trainer, "flops_per_step"):
            cfg["mfu"] = round(trainer.flops_per_step() * args.steps / elapsed / MI355X_BF16_DENSE_FLOPS, 4)
        unit = "images/s" if args.model == "resnet50" else "tokens/s"
        metric = "images/sec ResNet-50 DDP bf16" if args.model == "resnet50" else f"tokens/sec {args.model} DDP bf16"
        _emit(json.dumps({"metric": metric, "value": round(value, 1), "unit": unit, "n_gpus": n,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
                          "data": "synthetic (random tokens / ImageNet-shaped images), random-init weights",
                          "config": cfg}))
    pdist.cleanup()
    if identical is False:
        print("[bench] error: the data-parallel replicas diverged", file=sys.stderr, flush=True)
        return 3


if __name__ == "__main__":
    sys.exit(main() or 0)
