"""Fused training-mode BatchNorm (+ residual add) (+ ReLU) over channels-last
bf16 activations (``csrc/kernels/bn_kernels.hip``), as used by the ResNet-50
bottlenecks: ``relu(bn(x))``, ``relu(bn(x) + identity)`` and ``bn(x)``.

:class:`BatchNormAct` is an ``nn.BatchNorm2d`` (same parameters, buffers and
state-dict keys) whose ``forward(x, residual=None, relu=False)`` takes the
fused HIP path in training mode on bf16 channels-last HIP tensors and the
stock module (+ add / ReLU) everywhere else (CPU, eval, other dtypes).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

_CL = torch.channels_last


def fused_supported(x: torch.Tensor) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
        return False
    C = x.shape[1]
    tpr = C // 8
    return C % 8 == 0 and 8 <= C <= 2048 and (tpr & (tpr - 1)) == 0 and os.environ.get("PTO_FUSED_BN", "1") == "1"


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, residual, relu, momentum, eps, stash,
                part=None, nblk=0):
        L = _lib.lib()
        x = x.contiguous(memory_format=_CL)
        N, C, H, W = x.shape
        M = N * H * W
        dev = x.device
        y = torch.empty_like(x, memory_format=_CL)
        stat = torch.empty(4 * C, device=dev, dtype=torch.float32)
        scratch = (torch.empty(L.pto_bn_scratch_floats(M, C), device=dev, dtype=torch.float32) if part is None
                   else None)
        res = None
        if residual is not None:
            res = residual.contiguous(memory_format=_CL)
            if res.shape != x.shape or res.dtype != x.dtype:
                raise ValueError("BatchNormAct: residual must match the input")
        ctx.mode = 2 if (residual is not None and relu) else (1 if relu else 0)
        ctx.has_res = residual is not None
        ctx.stash = stash  # residual gradient handed to the block's conv1 GEMM (ops/conv1x1.py)
        # relu(bn(x) + res): the backward's ReLU mask cannot be recomputed
        # from x alone; one bit per element (bit j of byte i = y[8i + j] > 0)
        # instead of re-reading y
        mask = torch.empty(M * C // 8, device=dev, dtype=torch.uint8) if ctx.mode == 2 else None
        rm = None if running_mean is None else running_mean.data_ptr()
        rv = None if running_var is None else running_var.data_ptr()
        nb = None if nbt is None else nbt.data_ptr()
        rp = None if res is None else res.data_ptr()
        mp = None if mask is None else mask.data_ptr()
        if part is not None:  # statistics from the producing conv's epilogue (ops/conv3x3.py): no stats pass
            _lib.check(L.pto_bn_fwd_part(part.data_ptr(), nblk, x.data_ptr(), rp, y.data_ptr(), M, C,
                                         weight.data_ptr(), bias.data_ptr(), eps, momentum, rm, rv, nb,
                                         stat.data_ptr(), int(relu), mp, _lib.stream_ptr(dev)), "bn_fwd_part")
        else:
            _lib.check(L.pto_bn_fwd(x.data_ptr(), rp, y.data_ptr(), M, C, weight.data_ptr(), bias.data_ptr(), eps,
                                    momentum, rm, rv, nb, stat.data_ptr(), scratch.data_ptr(), int(relu), mp,
                                    _lib.stream_ptr(dev)), "bn_fwd")
        ctx.save_for_backward(x, mask, weight, stat)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        x, mask, weight, stat = ctx.saved_tensors
        dy = dy.contiguous(memory_format=_CL)
        N, C, H, W = x.shape
        M = N * H * W
        dev = x.device
        dx = torch.empty_like(x, memory_format=_CL)
        g = torch.empty_like(x, memory_format=_CL) if ctx.mode == 2 else None
        dgamma = torch.empty(C, device=dev, dtype=torch.float32)
        dbeta = torch.empty(C, device=dev, dtype=torch.float32)
        coef = torch.empty(3 * C, device=dev, dtype=torch.float32)
        scratch = torch.empty(L.pto_bn_scratch_floats(M, C), device=dev, dtype=torch.float32)
        _lib.check(L.pto_bn_bwd(dy.data_ptr(), x.data_ptr(), None if mask is None else mask.data_ptr(), dx.data_ptr(),
                                None if g is None else g.data_ptr(), M, C, weight.data_ptr(), stat.data_ptr(),
                                dgamma.data_ptr(), dbeta.data_ptr(), coef.data_ptr(), scratch.data_ptr(), ctx.mode,
                                _lib.stream_ptr(dev)), "bn_bwd")
        dres = (g if ctx.mode == 2 else dy) if ctx.has_res else None
        if dres is not None and ctx.stash is not None:
            ctx.stash.put(dres)  # accumulated by conv1's input-gradient GEMM instead of an autograd add
            dres = None
        return (dx, dgamma.to(weight.dtype), dbeta.to(weight.dtype), None, None, None, dres, None, None, None, None,
                None, None)


def bn_act(x, weight, bias, running_mean=None, running_var=None, num_batches_tracked=None, residual=None,
           relu=False, momentum: float = 0.1, eps: float = 1e-5, stash=None, part=None, nblk: int = 0):
    """Training-mode ``[relu](batch_norm(x) [+ residual])`` on a bf16
    channels-last HIP tensor; running statistics updated in place.
    ``stash``: the residual's gradient goes there instead of to autograd.
    ``part``/``nblk``: x's per-channel partial sums and sums of squares,
    already computed by its producer ([nblk][2][C] fp32)."""
    return _BNAct.apply(x, weight, bias, running_mean, running_var, num_batches_tracked, residual, relu,
                        float(momentum), float(eps), stash, part, int(nblk))


class BatchNormAct(nn.BatchNorm2d):
    def can_fuse(self, x) -> bool:
        return bool(self.training and self.momentum is not None and self.affine and fused_supported(x))

    def forward(self, x, residual=None, relu: bool = False, stash=None, stats=None):  # noqa: D102
        """``stats``: an ``ops.conv3x3.ConvStats`` the producing conv filled
        (its epilogue's partial sums of x): the fused path then skips its
        statistics pass."""
        part, nblk = stats.take() if stats is not None else (None, 0)
        if self.can_fuse(x):
            nbt = self.num_batches_tracked if self.track_running_stats else None
            rm = self.running_mean if self.track_running_stats else None
            rv = self.running_var if self.track_running_stats else None
            return bn_act(x, self.weight, self.bias, rm, rv, nbt, residual, relu, self.momentum, self.eps, stash,
                          part, nblk)
        if stash is not None:
            raise ValueError("BatchNormAct: a gradient stash needs the fused path")
        y = super().forward(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y
