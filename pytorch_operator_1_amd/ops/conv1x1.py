"""The residual gradient of a ResNet identity bottleneck folded into conv1's
input-gradient GEMM.

In an identity bottleneck the block input ``x`` feeds both ``conv1`` and the
identity path (``bn3(..., residual=x)``), so autograd adds the two input
gradients with a separate elementwise kernel (16 of them per ResNet-50 step,
1.33 ms of a 30 ms step: profiles/resnet50_window_r4.md).  Here the fused
BatchNorm backward of ``bn3`` hands its residual gradient to a
:class:`GradStash` instead of returning it, and ``conv1``'s backward computes
``dX = g_res + dY W`` as ONE hipBLASLt GEMM with beta = 1, in place on the
residual gradient: a 1x1 stride-1 convolution over NHWC memory is exactly
``Y[M, Co] = X[M, Ci] W[Co, Ci]^T`` (M = N*H*W), so its input gradient is
``dY[M, Co] W[Co, Ci]`` with no layout change.  The forward and the weight
gradient stay MIOpen's (tools/conv1x1_bench.py: a GEMM with K = N*H*W is
4-10x slower than MIOpen's weight-gradient solvers on these shapes, while
the data-gradient GEMM with the accumulation beats MIOpen's data-gradient
conv plus the add it replaces on all four identity-block shapes).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

_CL = torch.channels_last


class GradStash:
    """One gradient handed from a later backward node to an earlier one of
    the same bottleneck (bn3's residual gradient -> conv1's input GEMM)."""

    __slots__ = ("g",)

    def __init__(self):
        self.g = None

    def put(self, g):
        if self.g is not None:
            raise RuntimeError("GradStash: gradient already stashed (backward ran twice without a forward?)")
        self.g = g

    def take(self):
        g, self.g = self.g, None
        return g


def gemm_supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    return (x.is_cuda and x.dim() == 4 and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.groups == 1 and conv.bias is None
            and os.environ.get("PTO_CONV1X1_GEMM", "1") == "1")


class _Conv1x1Res(torch.autograd.Function):
    """A 1x1 stride-1 convolution whose INPUT gradient also carries a
    stashed residual gradient: forward and weight gradient stay MIOpen's
    (its weight-gradient solvers beat a hipBLASLt GEMM with K = N*H*W by
    4-10x on these shapes, profiles/resnet50_r5.md); the input gradient is
    ONE hipBLASLt GEMM accumulating into the residual gradient in place
    (beta = 1), which is faster than MIOpen's data-gradient conv + the
    separate add it replaces on every ResNet-50 identity block."""

    @staticmethod
    def forward(ctx, x, weight, stash, dtype):
        x = x.to(dtype).contiguous(memory_format=_CL)
        wb = weight.to(dtype)
        if wb.dim() == 4 and not wb.is_contiguous(memory_format=_CL):
            wb = wb.contiguous(memory_format=_CL)
        ctx.save_for_backward(x, wb)
        ctx.stash, ctx.wdtype = stash, weight.dtype
        ctx.wshape, ctx.wstride = weight.shape, weight.stride()
        return F.conv2d(x, wb)

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        N, ci, H, W = x.shape
        co = wb.shape[0]
        dy = dy.to(wb.dtype).contiguous(memory_format=_CL)
        _, dw, _ = torch.ops.aten.convolution_backward(dy, x, wb, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                       [False, True, False])
        dw = dw.to(ctx.wdtype)
        if dw.stride() != ctx.wstride:
            dw = torch.empty_strided(ctx.wshape, ctx.wstride, dtype=dw.dtype, device=dw.device).copy_(dw)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, co)
        w2 = wb.reshape(co, ci)
        extra = ctx.stash.take() if ctx.stash is not None else None
        if extra is not None:
            g = extra.to(dy2.dtype).contiguous(memory_format=_CL)
            dx2 = g.permute(0, 2, 3, 1).reshape(-1, ci).addmm_(dy2, w2)  # dX = g_res + dY W, in place
        else:
            dx2 = torch.mm(dy2, w2)
        return dx2.view(N, H, W, ci).permute(0, 3, 1, 2), dw, None, None


def conv1x1_res(x: torch.Tensor, conv: nn.Conv2d, stash: GradStash) -> torch.Tensor:
    """``conv(x)`` for a 1x1 stride-1 bias-free conv whose input gradient
    also receives ``stash``'s residual gradient (see :class:`_Conv1x1Res`).
    Dtype: the autocast dtype when autocast is on, else x's."""
    if not gemm_supported(x, conv):
        raise ValueError("conv1x1_res: needs a 1x1 stride-1 bias-free conv on a HIP tensor")
    dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    with torch.autocast("cuda", enabled=False):
        return _Conv1x1Res.apply(x, conv.weight, stash, dtype)
