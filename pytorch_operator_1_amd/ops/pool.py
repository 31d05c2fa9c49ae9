"""Max pooling over channels-last bf16 activations (the ResNet-50 stem's
3x3 / stride-2 / pad-1 pool) on the package's HIP kernels
(``csrc/kernels/bn_kernels.hip``: ``k_maxpool_fwd`` / ``k_maxpool_bwd``).

The forward keeps one uint8 argmax code per output element; the backward
gathers dy through those codes into every input element (no atomics, no
zero-fill).  Same results as ``F.max_pool2d`` (ties: first maximum; NaN
propagates).  CPU / other dtypes: the stock op.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

_CL = torch.channels_last


def _out(n: int, k: int, s: int, p: int) -> int:
    return (n + 2 * p - k) // s + 1


def maxpool_supported(x: torch.Tensor, k: int, s: int, p: int) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0 and k * k <= 255
            and 2 * p <= k and os.environ.get("PTO_MAXPOOL", "1") == "1")


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        x = x.contiguous(memory_format=_CL)
        N, C, H, W = x.shape
        OH, OW = _out(H, k, s, p), _out(W, k, s, p)
        y = torch.empty(N, C, OH, OW, device=x.device, dtype=x.dtype, memory_format=_CL)
        code = torch.empty(N * OH * OW * C, device=x.device, dtype=torch.uint8)
        _lib.check(_lib.lib().pto_maxpool_fwd(x.data_ptr(), y.data_ptr(), code.data_ptr(), N, H, W, C, OH, OW, k, s,
                                              p, _lib.stream_ptr(x.device)), "maxpool_fwd")
        ctx.save_for_backward(code)
        ctx.geom = (N, C, H, W, OH, OW, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (code,) = ctx.saved_tensors
        N, C, H, W, OH, OW, k, s, p = ctx.geom
        dy = dy.to(torch.bfloat16).contiguous(memory_format=_CL)
        dx = torch.empty(N, C, H, W, device=dy.device, dtype=torch.bfloat16, memory_format=_CL)
        _lib.check(_lib.lib().pto_maxpool_bwd(dy.data_ptr(), code.data_ptr(), dx.data_ptr(), N, H, W, C, OH, OW, k,
                                              s, p, _lib.stream_ptr(dy.device)), "maxpool_bwd")
        return dx, None, None, None


def max_pool2d(x: torch.Tensor, k: int, s: int, p: int) -> torch.Tensor:
    """``F.max_pool2d(x, k, s, p)``; the HIP path for channels-last bf16."""
    if maxpool_supported(x, k, s, p):
        return _MaxPool.apply(x, k, s, p)
    return F.max_pool2d(x, k, s, p)


class MaxPool2d(nn.MaxPool2d):
    """``nn.MaxPool2d`` (square kernel, no dilation / ceil mode) whose forward
    takes :func:`max_pool2d`."""

    def forward(self, x):
        k, s, p = self.kernel_size, self.stride, self.padding
        if (isinstance(k, int) and isinstance(s, int) and isinstance(p, int) and self.dilation == 1
                and not self.ceil_mode and not self.return_indices):
            return max_pool2d(x, k, s, p)
        return super().forward(x)
