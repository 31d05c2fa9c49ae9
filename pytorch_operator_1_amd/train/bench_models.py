"""Large-model DDP training steps for BASELINE configs 3 and 4.

* :class:`ResNetTrainer` — ResNet-50, ImageNet-shaped 224x224 synthetic
  batches, channels_last + bf16 autocast, fp32 master params, SGD
  momentum 0.9 / wd 1e-4 as one HIP launch (``FusedSGD``).
* :class:`LlamaTrainer` — Llama-3-8B (or a smaller preset), bf16 params,
  mixed-precision AdamW (fp32 master/m/v) as one HIP launch
  (``FusedAdamW``), HIP kernels between the hipBLASLt GEMMs.

Both use :class:`..parallel.ddp.GradBucketer`: grads accumulate straight
into flat buckets that are all-reduced over RCCL/xGMI on a comm stream
while backward continues; the 1/world average and grad zeroing are folded
into the optimizer's single pass.  Each ``step()`` is a complete optimizer
step (forward, backward, all-reduce, update) — nothing is skipped.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ..ops.conv1x1 import GradStash
from ..ops.optim import FusedAdamW, FusedSGD
from ..parallel.ddp import GradBucketer
from ..utils.profiling import StepTimer


class _TorchOpt:
    """Stock ``torch.optim`` behind the fused optimizers' ``step(grad_scale,
    zero_grad)`` call (CPU runs: the HIP optimizers need a GPU)."""

    def __init__(self, opt):
        self.opt = opt
        self.state = opt.state
        self.param_groups = opt.param_groups

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, zero_grad: bool = False):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None and grad_scale != 1.0:
                    p.grad.mul_(grad_scale)
        self.opt.step()
        if zero_grad:
            self.opt.zero_grad(set_to_none=False)


class CheckpointMixin:
    """Named tensors of the full training state (parameters, buffers,
    optimizer state) for :class:`..train.checkpoint.ShardedCheckpointer`,
    and the inverse.  DDP replicas hold identical copies, so the sharded
    checkpointer writes each tensor once (its owner rank)."""

    def _param_names(self):
        return {p: n for n, p in self.model.named_parameters()}

    def checkpoint_tensors(self) -> dict:
        t = {f"model.{n}": p.data for n, p in self.model.named_parameters()}
        t.update({f"buffer.{n}": b for n, b in self.model.named_buffers()})
        names = self._param_names()
        for p, st in self.opt.state.items():
            for k, v in st.items():
                if torch.is_tensor(v):
                    t[f"opt.{names[p]}.{k}"] = v
        return t

    def checkpoint_meta(self) -> dict:
        return {"steps_done": self.steps_done, "opt_step": getattr(self.opt, "_step", None)}

    def create_state(self, name: str, shape, dtype):
        """Destination for optimizer state that does not exist yet (resume
        before the first step): same layout as the parameter."""
        if not name.startswith("opt."):
            raise KeyError(name)
        pname, key = name[4:].rsplit(".", 1)
        p = dict(self.model.named_parameters())[pname]
        if list(p.shape) == list(shape):
            v = torch.zeros_like(p, dtype=dtype)
        else:
            v = torch.zeros(shape, dtype=dtype, device=p.device if key != "step" else "cpu")
        self.opt.state[p][key] = v
        return v

    def after_load(self, meta: dict):
        self.steps_done = int(meta.get("steps_done", 0))
        if meta.get("opt_step") is not None and hasattr(self.opt, "_step"):
            self.opt._step = int(meta["opt_step"])
        if hasattr(self.opt, "_tables"):
            self.opt._tables = None  # launch tables point at the old state tensors
        if getattr(self, "_graph", None) is not None:  # a captured step holds the old addresses too
            self._graph = None
            self._eager_done = 0
        refresh = getattr(self.model, "refresh_transposed", None)
        if refresh is not None and getattr(self, "transposed_dgrad", False):
            refresh()


class ResNetTrainer(CheckpointMixin):
    """``graph`` (``PTO_STEP_GRAPH=1``): replay the whole step (forward,
    loss, backward, FusedSGD) as ONE captured HIP graph after
    ``EAGER_STEPS`` eager steps (MIOpen's solver search, library handles and
    the optimizer state are created eagerly); single-process runs only
    (``GradBucketer`` mode ``none``).  Off by default: at batch 256 the GPU
    is never starved by the ~1,400 eager launches per step (26.74 vs 26.73
    ms/step measured, profiles/resnet50_r5.md), so the graph buys nothing
    here -- it is for smaller per-GPU batches, where launch latency shows."""

    EAGER_STEPS = 2

    def __init__(self, device, batch_size: int = 256, image_size: int = 224, lr: float = 0.1,
                 momentum: float = 0.9, weight_decay: float = 1e-4, seed: int = 0, bucket_mb: float | None = None,
                 force_ddp: bool = False, graph: bool | None = None):
        from ..models.resnet import resnet50, synthetic_images

        torch.manual_seed(seed)
        # MIOpen find: benchmark the conv solvers once per shape (warmup) and
        # keep the fastest instead of the heuristic pick
        torch.backends.cudnn.benchmark = True
        self.device = device
        self.batch_size = batch_size
        self.model = resnet50().to(device=device, memory_format=torch.channels_last)
        self.model.train()
        self.bucketer = GradBucketer(self.model, bucket_mb=bucket_mb, force_ddp=force_ddp)
        if device.type == "cuda":
            self.opt = FusedSGD(self.model.parameters(), lr=lr, momentum=momentum, weight_decay=weight_decay)
        else:
            self.opt = _TorchOpt(torch.optim.SGD(self.model.parameters(), lr=lr, momentum=momentum,
                                                 weight_decay=weight_decay))
        # images arrive in the compute dtype on the GPU (what a GPU-side
        # decode/normalise stage hands over); the model casts nothing per step
        self.x, self.y = synthetic_images(batch_size, device, image_size, seed=seed,
                                          dtype=torch.bfloat16 if device.type == "cuda" else torch.float32)
        self._loss = None
        self.steps_done = 0
        self.timer = StepTimer(device, enabled=False)
        if graph is None:
            graph = os.environ.get("PTO_STEP_GRAPH", "0") == "1"
        self.use_graph = bool(graph) and device.type == "cuda" and self.bucketer.mode == "none"
        self._graph = None
        self._eager_done = 0

    def step(self):
        if not self.use_graph or self._eager_done < self.EAGER_STEPS:
            self._eager_step()
            self._eager_done += 1
            return
        if self._graph is None:
            self._capture()
        self.opt.sync_lr()
        self._graph.replay()
        self.steps_done += 1

    def _capture(self):
        """Record one whole step into a HIP graph (nothing executes while
        capturing: :meth:`step` replays it right after)."""
        torch.cuda.synchronize(self.device)
        self.bucketer.release()  # grads None: the captured backward allocates them in the graph's pool
        self.opt.prepare_capture()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
                out = self.model(self.x)
            loss = F.cross_entropy(out.float(), self.y)
            loss.backward()
            GradStash.assert_drained()
            self.bucketer.finish()
            self.opt.step(grad_scale=self.bucketer.grad_scale, zero_grad=self.bucketer.optimizer_zeroes_grads)
        self.opt.finish_capture()  # the launch table of the graph's gradients
        self._loss = loss.detach()
        self._graph = g

    def _eager_step(self):
        t = self.timer
        with t.phase("forward"), torch.autocast(device_type=self.device.type, dtype=torch.bfloat16):
            out = self.model(self.x)
        with t.phase("forward"):
            loss = F.cross_entropy(out.float(), self.y)
        with t.phase("backward"):
            loss.backward()
            GradStash.assert_drained()  # host counter: no sibling conv1x1 gradient left parked
        with t.phase("allreduce_wait"):
            self.bucketer.finish()
        with t.phase("optimizer"):
            self.opt.step(grad_scale=self.bucketer.grad_scale, zero_grad=self.bucketer.optimizer_zeroes_grads)
            self.bucketer.release()
        self._loss = loss.detach()
        self.steps_done += 1

    def run(self, n: int):
        for _ in range(n):
            self.step()

    def last_loss(self):
        return None if self._loss is None else float(self._loss)

    def samples_per_step(self) -> int:
        return self.batch_size

    def describe(self) -> dict:
        return {"model": "resnet50 (v1.5, 25.6M params)", "input_shape": [3, 224, 224],
                "optimizer": "SGD momentum=0.9 wd=1e-4 (FusedSGD HIP)", "amp": "bf16 autocast, fp32 master",
                "step": (f"whole step replayed as one HIP graph (after {self.EAGER_STEPS} eager steps)"
                         if self.use_graph else "eager")}


class LlamaTrainer(CheckpointMixin):
    def __init__(self, device, model: str = "llama3-8b", batch_size: int = 2, seq_len: int = 4096,
                 lr: float = 3e-4, weight_decay: float = 0.1, seed: int = 0, checkpoint: str = "none",
                 impl: str | None = None, bucket_mb: float | None = None, force_ddp: bool = False):
        from ..models.llama import CONFIGS, Llama, synthetic_tokens

        torch.manual_seed(seed)
        impl = impl or ("hip" if device.type == "cuda" else "torch")
        self.cfg = CONFIGS[model]
        self.name = model
        self.device = device
        self.batch_size, self.seq_len = batch_size, seq_len
        self.model = Llama(self.cfg, impl=impl, device=device, checkpoint=checkpoint)
        self.model.train()
        # W^T copies for K-contiguous dgrad GEMMs (PTO_WT=0: plain F.linear backward)
        self.transposed_dgrad = impl == "hip" and os.environ.get("PTO_WT", "1") == "1"
        if self.transposed_dgrad:
            self.model.enable_transposed_dgrad()
        self.bucketer = GradBucketer(self.model, bucket_mb=bucket_mb, force_ddp=force_ddp)
        if device.type == "cuda":
            self.opt = FusedAdamW(self.model.parameters(), lr=lr, betas=(0.9, 0.95), eps=1e-8,
                                  weight_decay=weight_decay)
        else:  # CPU: stock AdamW on the bf16 params (tests of the checkpoint/resume path)
            self.opt = _TorchOpt(torch.optim.AdamW(self.model.parameters(), lr=lr, betas=(0.9, 0.95), eps=1e-8,
                                                   weight_decay=weight_decay))
        self.tokens, self.labels = synthetic_tokens(batch_size, seq_len, self.cfg.vocab_size, device, seed=seed)
        self._loss = None
        self.steps_done = 0
        self.timer = StepTimer(device, enabled=False)

    def step(self):
        t = self.timer
        with t.phase("forward"):
            loss = self.model(self.tokens, self.labels)
        with t.phase("backward"):
            loss.backward()
        with t.phase("allreduce_wait"):
            self.bucketer.finish()
        with t.phase("optimizer"):
            self.opt.step(grad_scale=self.bucketer.grad_scale, zero_grad=self.bucketer.optimizer_zeroes_grads)
            self.bucketer.release()
            if self.transposed_dgrad:
                self.model.refresh_transposed()
        self._loss = loss.detach()
        self.steps_done += 1

    def run(self, n: int):
        for _ in range(n):
            self.step()

    def last_loss(self):
        return None if self._loss is None else float(self._loss)

    def samples_per_step(self) -> int:
        return self.batch_size * self.seq_len  # tokens

    def flops_per_step(self) -> float:
        return self.cfg.train_flops_per_token(self.seq_len) * self.samples_per_step()

    def describe(self) -> dict:
        return {"model": f"{self.name} ({self.cfg.num_params() / 1e9:.2f}B params)",
                "optimizer": "AdamW betas=(0.9,0.95) wd=0.1 (FusedAdamW HIP, fp32 master/m/v)",
                "amp": "bf16 params/activations, fp32 optimizer state",
                "checkpoint": self.model.checkpoint,
                "dgrad": "W^T copies (K-contiguous dX GEMMs)" if self.transposed_dgrad else "F.linear"}
