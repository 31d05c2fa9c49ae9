"""Trainer factory shared by ``bench.py``, the ``mnist`` trainer CLI and
the tests.

* ``eager`` — stock-PyTorch DDP path, the behavioural twin of the
  reference workload (``examples/mnist/mnist.py:35-49``): ``zero_grad`` →
  forward → ``nll_loss`` → ``backward`` (DDP bucket all-reduce hooks) →
  ``SGD.step``.  Used as the numerics/throughput baseline and for CPU/gloo.
* ``fused`` — :class:`~pytorch_operator_1_amd.train.fused_step.FusedMnistTrainer`:
  flat parameter/gradient/momentum buffers, hand-written gfx950 kernels,
  single-bucket all-reduce, whole step replayed from a HIP graph.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..models.mnist import MnistNet, synthetic_mnist


class EagerMnistTrainer:
    def __init__(self, device, batch_size=64, lr=0.01, momentum=0.5, dataset_size=60000, seed=1,
                 impl="torch", rank=0, data=None, target=None, weight_decay=0.0):
        torch.manual_seed(seed)
        self.device = device
        self.batch_size = batch_size
        self.module = MnistNet(impl=impl).to(device)
        self.model = self.module
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            kw = {"device_ids": [device.index]} if device.type == "cuda" else {}
            self.model = torch.nn.parallel.DistributedDataParallel(self.module, **kw)
        self.opt = torch.optim.SGD(self.model.parameters(), lr=lr, momentum=momentum, weight_decay=weight_decay)
        if data is None:
            data, target = synthetic_mnist(dataset_size, device, seed=seed + 1000 * rank)
        self.data, self.target = data, target
        self.n_batches = data.shape[0] // batch_size
        self.it = 0
        self._loss = None

    def step(self):
        b = self.it % self.n_batches
        self.it += 1
        x = self.data[b * self.batch_size:(b + 1) * self.batch_size]
        y = self.target[b * self.batch_size:(b + 1) * self.batch_size]
        self.opt.zero_grad(set_to_none=True)
        out = self.model(x)
        loss = F.nll_loss(out, y)
        loss.backward()
        self.opt.step()
        self._loss = loss.detach()
        return self._loss

    def last_loss(self):
        return None if self._loss is None else float(self._loss.item())

    def state_dict(self):
        mom = {}
        names = dict(self.module.named_parameters())
        for name, p in names.items():
            st = self.opt.state.get(p, {})
            if "momentum_buffer" in st and st["momentum_buffer"] is not None:
                mom[name] = st["momentum_buffer"].detach().clone()
        return {"model": {k: v.detach().clone() for k, v in self.module.state_dict().items()}, "momentum": mom,
                "batch_idx": self.it % self.n_batches, "steps_done": self.it}

    def load_state_dict(self, sd):
        self.module.load_state_dict({k: v.to(self.device) for k, v in sd["model"].items()})
        names = dict(self.module.named_parameters())
        for name, buf in sd.get("momentum", {}).items():
            self.opt.state[names[name]]["momentum_buffer"] = buf.to(self.device).clone()
        self.it = int(sd.get("steps_done", 0))


def build_trainer(impl: str, device, **kw):
    if impl == "eager":
        return EagerMnistTrainer(device, **kw)
    if impl == "fused":
        if device.type != "cuda":
            # The fused path is HIP-only; CPU runs (gloo tests) use eager.
            return EagerMnistTrainer(device, **kw)
        from .fused_step import build_fused_trainer

        return build_fused_trainer(device, **kw)
    raise ValueError(f"unknown impl {impl!r}")
