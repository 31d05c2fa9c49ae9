"""ResNet-50's stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels,
224 -> 112) on the package's MFMA implicit-GEMM kernel
(``csrc/kernels/bn_kernels.hip``: ``k_stem_fwd``), channels-last bf16 in and
out.  MIOpen ran it as an asm implicit GEMM after zero-filling its 411 MB
output (0.36 + 0.09 ms per step at batch 256).  The weight gradient stays
MIOpen's (the image needs no input gradient).  CPU / other shapes: stock.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

_CL = torch.channels_last


def stem_supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and tuple(x.shape[1:]) == (3, 224, 224) and conv.in_channels == 3
            and conv.out_channels == 64 and conv.kernel_size == (7, 7) and conv.stride == (2, 2)
            and conv.padding == (3, 3) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.weight.dtype == torch.float32 and os.environ.get("PTO_STEM", "1") == "1")


class _Stem(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, wp=None):
        x = x.to(torch.bfloat16).contiguous(memory_format=_CL)
        N = x.shape[0]
        y = torch.empty(N, 64, 112, 112, device=x.device, dtype=torch.bfloat16, memory_format=_CL)
        if wp is None:
            wp = torch.empty(64 * 176, device=x.device, dtype=torch.bfloat16)
        _lib.check(_lib.lib().pto_stem_fwd(x.data_ptr(), weight.data_ptr(), *weight.stride(), wp.data_ptr(),
                                           y.data_ptr(), N, _lib.stream_ptr(x.device)), "stem_fwd")
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=_CL)
        wb = weight.to(torch.bfloat16)
        _, dw, _ = torch.ops.aten.convolution_backward(dy, x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                       [False, True, False])
        dw = dw.to(weight.dtype)
        if dw.stride() != weight.stride():
            dw = torch.empty_strided(weight.shape, weight.stride(), dtype=dw.dtype, device=dw.device).copy_(dw)
        return None, dw, None


def stem_conv(x: torch.Tensor, conv: nn.Conv2d) -> torch.Tensor:
    """``conv(x)`` for ResNet's stem conv: the HIP kernel on supported
    shapes (bf16 output, as under autocast), the stock module otherwise."""
    if stem_supported(x, conv):
        # the bf16 GEMM image of the weights, rebuilt in place every call
        # (one buffer per module: no allocator churn around the step)
        wp = getattr(conv, "_pto_stem_wp", None)
        if wp is None or wp.device != x.device:
            wp = conv._pto_stem_wp = torch.empty(64 * 176, device=x.device, dtype=torch.bfloat16)
        with torch.autocast("cuda", enabled=False):
            return _Stem.apply(x, conv.weight, wp)
    return conv(x)
