"""Large-model DDP trainer CLI (BASELINE configs 3-5 as PyTorchJob
workloads): Llama-3 (``llama3-tiny`` / ``-1b`` / ``-8b``) or ResNet-50,
synthetic data, with periodic sharded checkpoints and automatic resume.

The reference's only workload is the MNIST example, which saves a final
``state_dict`` and cannot resume (``examples/mnist/mnist.py:146-147``); its
operator restarts failed replicas (``pkg/controller.v1/pytorch/pod.go:91-109``)
but a restarted replica starts from step 0.  Here:

* every ``--checkpoint-interval`` steps the full training state (params,
  BN buffers, fp32 master weights, optimizer moments, step counters) is
  written by :class:`~.checkpoint.ShardedCheckpointer`: each tensor once, by
  its owner rank, snapshotted to host memory and written on a background
  thread, the manifest committed last;
* on start the newest committed step is restored (own shard read, owners
  broadcast) and training continues from it ("Resumed from <dir> at step N");
* a collective failure exits 138 (retryable for ``restartPolicy: ExitCode``)
  exactly like the MNIST trainer, so kill/rejoin works for these models too.

Example (one replica per GPU, through the operator or torchrun)::

    python -m pytorch_operator_1_amd.train.lm --model llama3-8b --steps 1000 \\
        --checkpoint-dir /ckpt/job --checkpoint-interval 100 --backend rccl
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import time

import torch

from ..utils import dist as pdist
from . import checkpoint as ckpt
from .mnist import Metrics, run_with_retryable_exit


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Llama-3 / ResNet-50 DDP trainer (MI355X)")
    p.add_argument("--model", default="llama3-tiny",
                   choices=["llama3-tiny", "llama3-1b", "llama3-8b", "resnet50"])
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--batch-size", type=int, default=None, help="per rank (default 2 llama, 64 resnet50)")
    p.add_argument("--seq-len", type=int, default=512)
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--lr", type=float, default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--log-interval", type=int, default=10)
    p.add_argument("--backend", default=None, help="rccl|nccl|gloo (default: rccl on GPU, gloo on CPU)")
    p.add_argument("--no-cuda", action="store_true")
    p.add_argument("--activation-checkpoint", choices=["none", "full"], default="none")
    p.add_argument("--checkpoint-dir", default=None)
    p.add_argument("--checkpoint-interval", type=int, default=0)
    p.add_argument("--sync-checkpoint", action="store_true", help="write shards on the training thread")
    p.add_argument("--fail-at-step", type=int, default=int(os.environ.get("PTO_FAIL_AT_STEP", "0")),
                   help="fault injection: SIGKILL self before this step (first incarnation only)")
    p.add_argument("--fail-rank", type=int, default=int(os.environ.get("PTO_FAIL_RANK", "0")))
    return p.parse_args(argv)


def build(args, device):
    from .bench_models import LlamaTrainer, ResNetTrainer

    if args.model == "resnet50":
        kw = {} if args.lr is None else {"lr": args.lr}
        return ResNetTrainer(device, batch_size=args.batch_size or 64, image_size=args.image_size, seed=args.seed,
                             **kw)
    kw = {} if args.lr is None else {"lr": args.lr}
    return LlamaTrainer(device, model=args.model, batch_size=args.batch_size or 2, seq_len=args.seq_len,
                        seed=args.seed, checkpoint=args.activation_checkpoint, **kw)


def _main(argv=None):
    args = parse_args(argv)
    use_gpu = not args.no_cuda and torch.cuda.is_available() and os.environ.get("PTO_NO_GPU") != "1"
    env, device = pdist.init_distributed(args.backend, use_gpu=use_gpu)
    rank, world = env.rank, env.world_size
    metrics = Metrics()
    trainer = build(args, device)
    saver = None
    start = 0
    if args.checkpoint_dir:
        saver = ckpt.ShardedCheckpointer(args.checkpoint_dir, rank, world, async_write=not args.sync_checkpoint)
        man = saver.load_into(trainer.checkpoint_tensors(), create=trainer.create_state)
        if man is not None:
            trainer.after_load(man["meta"])
            start = int(man["step"])
            print(f"Resumed from {saver.resumed_from} at step {start}", flush=True)
    fail = args.fail_at_step if (args.fail_at_step and rank == args.fail_rank and start == 0) else 0
    t_last, steps_since = time.time(), 0
    for step in range(start, args.steps):
        if fail and step == fail:
            # deterministic injection: the kill lands after the checkpoint in
            # flight is durable (a real crash may lose it; resume then falls
            # back to the previous committed step)
            if saver:
                saver.commit()
            print(f"[fault-injection] rank {rank} SIGKILL at step {step}", flush=True)
            os.kill(os.getpid(), signal.SIGKILL)
        trainer.step()
        steps_since += 1
        done = step + 1
        if done == start + 1:
            if device.type == "cuda":
                torch.cuda.synchronize(device)
            metrics.emit(event="first_step", t=time.time(), rank=rank)
        if done % args.log_interval == 0 or done == args.steps:
            loss = trainer.last_loss()
            now = time.time()
            sps = steps_since * trainer.samples_per_step() * world / max(now - t_last, 1e-9)
            print(f"step {done}/{args.steps}\tloss={loss:.6f}\t{sps:.1f} samples/s", flush=True)
            metrics.emit(event="train", step=done, loss=loss, samples_per_sec=round(sps, 1),
                         step_seconds=(now - t_last) / steps_since, rank=rank)
            t_last, steps_since = now, 0
        if saver and args.checkpoint_interval and done % args.checkpoint_interval == 0 and done < args.steps:
            saver.save(done, trainer.checkpoint_tensors(), trainer.checkpoint_meta())
    if saver:
        saver.save(args.steps, trainer.checkpoint_tensors(), trainer.checkpoint_meta())
        saver.close()
    print(f"final_loss={trainer.last_loss():.8f}", flush=True)
    pdist.cleanup()
    return 0


def main(argv=None):
    return run_with_retryable_exit(_main, argv)


if __name__ == "__main__":
    sys.exit(main())
