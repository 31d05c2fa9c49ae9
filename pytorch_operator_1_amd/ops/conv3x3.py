"""ResNet-50's 3x3 convolutions on the package's MFMA implicit-GEMM kernel
(``csrc/kernels/conv3x3.hip``), channels-last bf16, pad 1, stride 1 or 2.

Forward: ``k_conv3x3_fwd`` -- and, when the consumer is a fused BatchNorm
(``ops/bn.py``), the per-channel sums / sums of squares of the rounded
outputs come out of the conv epilogue (:class:`ConvStats`), so the BN
forward skips its statistics pass (a full read of the conv output).
Backward: the input gradient of a stride-1 conv is the SAME kernel run on dY
with the filter flipped and transposed (``k_conv3x3_wflip``); the stride-2
input gradient and every weight gradient stay MIOpen's
(``aten.convolution_backward``).  CPU / unsupported shapes: the stock conv.

Reference parity: the reference's workload is the MNIST ``Net``
(``examples/mnist/mnist.py:17-33``); ResNet-50 is BASELINE.json config 3,
whose convolutions SURVEY §2.9 K3 asks to own as an implicit GEMM with a
fused epilogue.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

_CL = torch.channels_last


class ConvStats:
    """Holder for the BN statistics partials a conv epilogue produced:
    ``part`` ([tiles][2][C] fp32: per-tile channel sums, sums of squares)
    and ``nblk`` (tiles).  Filled by :func:`conv3x3` in the forward, read
    (and cleared) by ``BatchNormAct``."""

    __slots__ = ("part", "nblk")

    def __init__(self):
        self.part, self.nblk = None, 0

    def take(self):
        p, n = self.part, self.nblk
        self.part, self.nblk = None, 0
        return p, n


def _compute_dtype(x):
    return torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype


def conv3x3_supported(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    """Shapes and dtypes the kernel takes: bf16 compute (autocast or a bf16
    input), 3x3 / pad 1 / stride 1 or 2, channels multiples of the tiles,
    fp32 channels-last filter."""
    if not (x.is_cuda and x.dim() == 4 and _compute_dtype(x) == torch.bfloat16 and conv.kernel_size == (3, 3)
            and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.stride in ((1, 1), (2, 2)) and os.environ.get("PTO_CONV3X3", "1") == "1"):
        return False
    C, K = conv.in_channels, conv.out_channels
    if C % 64 or K % 64 or (K > 64 and K % 128) or (K > 256 and K % 256):
        return False
    w = conv.weight
    return w.dtype == torch.float32 and w.is_contiguous(memory_format=_CL)


def _out_hw(h: int, s: int) -> int:
    return (h + 2 - 3) // s + 1


def _fwd(L, x, wb, stride, part=None):
    N, C, H, W = x.shape
    K = wb.shape[0]
    OH, OW = _out_hw(H, stride), _out_hw(W, stride)
    y = torch.empty(N, K, OH, OW, device=x.device, dtype=torch.bfloat16, memory_format=_CL)
    _lib.check(L.pto_conv3x3_fwd(x.data_ptr(), wb.data_ptr(), y.data_ptr(), None if part is None else part.data_ptr(),
                                 N, H, W, C, K, stride, _lib.stream_ptr(x.device)), "conv3x3_fwd")
    return y


def stats_tiles(N: int, OH: int, OW: int, K: int) -> int:
    tm = _lib.lib().pto_conv3x3_tile_m(K)
    return (N * OH * OW + tm - 1) // tm


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, wb, stride, stats):
        L = _lib.lib()
        x = x.to(torch.bfloat16).contiguous(memory_format=_CL)
        # the bf16 image of the fp32 master filter (same channels-last layout),
        # rebuilt every call into the module's persistent buffer
        _lib.check(L.pto_conv3x3_wcast(weight.data_ptr(), wb.data_ptr(), wb.numel(), _lib.stream_ptr(x.device)),
                   "conv3x3_wcast")
        part = None
        if stats is not None:
            N, _, H, W = x.shape
            K = weight.shape[0]
            nblk = stats_tiles(N, _out_hw(H, stride), _out_hw(W, stride), K)
            part = torch.empty(nblk * 2 * K, device=x.device, dtype=torch.float32)
            stats.part, stats.nblk = part, nblk
        y = _fwd(L, x, wb, stride, part)
        ctx.save_for_backward(x, wb)
        ctx.stride = stride
        ctx.wshape, ctx.wstride, ctx.wdtype = weight.shape, weight.stride(), weight.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        s = ctx.stride
        dy = dy.to(torch.bfloat16).contiguous(memory_format=_CL)
        dx = None
        if ctx.needs_input_grad[0] and s == 1:
            L = _lib.lib()
            K, C = wb.shape[0], wb.shape[1]
            wf = torch.empty(C, K, 3, 3, device=x.device, dtype=torch.bfloat16, memory_format=_CL)
            _lib.check(L.pto_conv3x3_wflip(None, wb.data_ptr(), wf.data_ptr(), K, C, _lib.stream_ptr(x.device)),
                       "conv3x3_wflip")
            dx = _fwd(L, dy, wf, 1)
        need_dx_lib = ctx.needs_input_grad[0] and dx is None
        dxl, dw, _ = torch.ops.aten.convolution_backward(dy, x, wb, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                         [need_dx_lib, bool(ctx.needs_input_grad[1]), False])
        if need_dx_lib:
            dx = dxl
        if dw is not None:
            dw = dw.to(ctx.wdtype)
            if dw.stride() != ctx.wstride:
                dw = torch.empty_strided(ctx.wshape, ctx.wstride, dtype=dw.dtype, device=dw.device).copy_(dw)
        return dx, dw, None, None, None


def conv3x3(x: torch.Tensor, conv: nn.Conv2d, stats: ConvStats | None = None) -> torch.Tensor:
    """``conv(x)`` for a 3x3 / pad-1 / bias-free conv: the HIP kernel on
    supported shapes (bf16 channels-last output, as under autocast; with
    ``stats`` the BN partials of the output too), the stock module otherwise
    (``stats`` then stays empty and the BN computes its own)."""
    if not conv3x3_supported(x, conv):
        return conv(x)
    wb = getattr(conv, "_pto_c3_wb", None)
    if wb is None or wb.device != x.device or wb.shape != conv.weight.shape:
        wb = torch.empty(conv.weight.shape, device=x.device, dtype=torch.bfloat16, memory_format=_CL)
        conv._pto_c3_wb = wb
    with torch.autocast("cuda", enabled=False):
        return _Conv3x3.apply(x, conv.weight, wb, conv.stride[0], stats)


def reference_conv3x3(x: torch.Tensor, w: torch.Tensor, stride: int) -> torch.Tensor:
    """fp32 reference of the kernel's math: bf16 operands, fp32 sums."""
    return F.conv2d(x.float(), w.to(torch.bfloat16).float(), stride=stride, padding=1)
