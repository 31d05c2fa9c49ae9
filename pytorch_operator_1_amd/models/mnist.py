"""MNIST CNN — the reference's benchmark workload, rebuilt for MI355X.

Architecture parity: ``examples/mnist/mnist.py:17-33`` of the reference
(conv(1→20,5) → ReLU → maxpool2 → conv(20→50,5) → ReLU → maxpool2 →
fc(800→500) → ReLU → fc(500→10) → log_softmax).  431,080 fp32 parameters.

Two implementations live here:

* :class:`MnistNet` — an ``nn.Module`` whose forward dispatches either to
  stock PyTorch ops (``impl="torch"``, the numerics reference) or to this
  package's HIP kernels (``impl="hip"``) through autograd Functions in
  :mod:`pytorch_operator_1_amd.ops`.
* :class:`pytorch_operator_1_amd.train.fused_step.FusedMnistStep` (in
  ``train/``) — the production training step: parameters, gradients and
  momentum in ONE flat fp32 buffer (so the DDP all-reduce is a single
  1.72 MB bucket), every op a hand-written gfx950 kernel, the whole step
  captured in a HIP graph.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

# Parameter table in the flat-buffer order used by the fused trainer.  The
# order is reverse-of-backward so that the fc grads (produced first in
# backward) occupy the front of the buffer and can be all-reduced first.
PARAM_SHAPES = (
    ("fc2.weight", (10, 500)),
    ("fc2.bias", (10,)),
    ("fc1.weight", (500, 800)),
    ("fc1.bias", (500,)),
    ("conv2.weight", (50, 20, 5, 5)),
    ("conv2.bias", (50,)),
    ("conv1.weight", (20, 1, 5, 5)),
    ("conv1.bias", (20,)),
)
NUM_PARAMS = sum(math.prod(s) for _, s in PARAM_SHAPES)  # 431,080
IMAGE_SHAPE = (1, 28, 28)
NUM_CLASSES = 10


def param_offsets(align: int = 64):
    """Offsets (in elements) of each parameter inside the flat buffer.

    Each tensor starts on a ``align``-element boundary (256 B for fp32) so
    every kernel can use 16-byte vector loads on any parameter view.
    Returns ``(dict name -> (offset, shape), total_padded_elems)``.
    """
    out, off = {}, 0
    for name, shape in PARAM_SHAPES:
        out[name] = (off, shape)
        off += math.prod(shape)
        off = (off + align - 1) // align * align
    return out, off


def init_params_(named: dict[str, torch.Tensor], seed: int = 1) -> None:
    """PyTorch-default init (kaiming-uniform(a=sqrt(5)) weights, fan-in
    uniform biases) so loss curves match a stock ``nn.Conv2d``/``nn.Linear``
    model with the same seed."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    for name, t in named.items():
        if name.endswith("weight"):
            fan_in = math.prod(t.shape[1:])
        else:
            wname = name.replace("bias", "weight")
            fan_in = math.prod(named[wname].shape[1:])
        bound = 1.0 / math.sqrt(fan_in)  # kaiming_uniform(a=sqrt(5)) == U(-1/sqrt(fan_in), ...)
        vals = torch.empty(t.shape, dtype=torch.float32).uniform_(-bound, bound, generator=g)
        with torch.no_grad():
            t.copy_(vals.to(t.device, t.dtype))


class MnistNet(nn.Module):
    """``nn.Module`` form of the reference ``Net``.

    ``impl="torch"``: stock ops (used as the fp32 numerics reference and
    for the CPU/gloo path).  ``impl="hip"``: fused HIP kernels from
    :mod:`pytorch_operator_1_amd.ops` (conv+bias+ReLU+pool, linear+bias+ReLU,
    log-softmax).  Both produce log-probabilities, like the reference.
    """

    def __init__(self, impl: str = "torch"):
        super().__init__()
        self.impl = impl
        self.conv1 = nn.Conv2d(1, 20, 5, 1)
        self.conv2 = nn.Conv2d(20, 50, 5, 1)
        self.fc1 = nn.Linear(4 * 4 * 50, 500)
        self.fc2 = nn.Linear(500, 10)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.impl == "hip":
            from .. import ops

            x = ops.conv2d_bias_relu_maxpool(x, self.conv1.weight, self.conv1.bias)
            x = ops.conv2d_bias_relu_maxpool(x, self.conv2.weight, self.conv2.bias)
            x = x.reshape(x.shape[0], 4 * 4 * 50)
            x = ops.linear(x, self.fc1.weight, self.fc1.bias, relu=True)
            x = ops.linear(x, self.fc2.weight, self.fc2.bias, relu=False)
            return ops.log_softmax(x)
        x = F.relu(self.conv1(x))
        x = F.max_pool2d(x, 2, 2)
        x = F.relu(self.conv2(x))
        x = F.max_pool2d(x, 2, 2)
        x = x.view(-1, 4 * 4 * 50)
        x = F.relu(self.fc1(x))
        x = self.fc2(x)
        return F.log_softmax(x, dim=1)


# class -> top-left corner of its 6x6 blob (k_synth_mnist hard-codes the same table)
BLOB_ROWS = (2, 2, 2, 11, 11, 11, 20, 20, 20, 11)
BLOB_COLS = (2, 11, 20, 2, 11, 20, 2, 11, 20, 8)
_GOLD = 0x9E3779B97F4A7C15
_M64 = (1 << 64) - 1


def _smix64_int(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _synth_key(seed: int) -> int:
    return _smix64_int((int(seed) + _GOLD) & _M64)


def synthetic_mnist(n: int, device, seed: int = 1, dtype=torch.float32, source: str = "torch"):
    """Synthetic MNIST-shaped data (normalised like ``Normalize((0.1307,),
    (0.3081,))``) with a learnable label rule, resident on ``device``.

    There is no network in this environment, so real MNIST cannot be
    downloaded; the label is a deterministic function of the image (which
    quadrant holds the brightest blob) so training visibly converges.

    ``source="torch"`` (default): drawn from the torch CPU generator and
    copied to ``device`` -- the same values on every device, the set the
    numerics tests and the benchmark use.  ``source="hash"`` on a GPU: one
    HIP launch (``k_synth_mnist``, common_kernels.hip) writes the set in
    place from a counter-based hash of (seed, image, pixel), same
    distribution, different values: no host generation, no host->device
    copy and none of the framework's lazily loaded RNG kernels, which
    together were ~0.4 s of a fresh job's submit -> first step (the
    operator's training image uses it; train/mnist.py).
    """
    dev = torch.device(device)
    key = _synth_key(seed)
    if dev.type == "cuda" and source == "hash":
        from ..ops import _lib

        x = torch.empty((n, 1, 28, 28), device=dev, dtype=torch.float32)
        y = torch.empty(n, device=dev, dtype=torch.int64)
        _lib.check(_lib.lib().pto_synth_mnist(x.data_ptr(), y.data_ptr(), n, key, _lib.stream_ptr(dev)),
                   "synth_mnist")
        return x.to(dtype), y
    g = torch.Generator(device="cpu").manual_seed(seed)
    labels = torch.randint(0, NUM_CLASSES, (n,), generator=g)
    imgs = torch.rand((n, 1, 28, 28), generator=g) * 0.3
    # Paint a class-dependent 6x6 blob: 10 classes -> 10 fixed positions.
    ys = torch.tensor(BLOB_ROWS)
    xs = torch.tensor(BLOB_COLS)
    # one broadcast mask instead of per-class fancy indexing (same values)
    r = torch.arange(28)
    y0, x0 = ys[labels][:, None], xs[labels][:, None]
    rows = (r >= y0) & (r < y0 + 6)
    cols = (r >= x0) & (r < x0 + 6)
    imgs[:, 0].add_((rows[:, :, None] & cols[:, None, :]).to(imgs.dtype), alpha=0.7)
    imgs = (imgs.clamp_(0, 1) - 0.1307) / 0.3081
    return imgs.to(device=dev, dtype=dtype), labels.to(dev)
