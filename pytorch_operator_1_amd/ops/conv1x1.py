"""ResNet's 1x1 stride-1 convolutions with their backward on hipBLASLt,
and the residual gradient of an identity bottleneck folded into conv1's
input-gradient GEMM.

A 1x1 stride-1 convolution over NHWC memory is exactly
``Y[M, Co] = X[M, Ci] W[Co, Ci]^T`` (M = N*H*W), so:

* input gradient ``dX = dY W`` is one GEMM with no layout change.  In an
  identity bottleneck the block input ``x`` feeds both ``conv1`` and the
  identity path (``bn3(..., residual=x)``), so autograd would add the two
  input gradients with a separate elementwise kernel (16 per ResNet-50
  step, 1.33 ms of a 30 ms step: profiles/resnet50_window_r4.md).  Here the
  fused BatchNorm backward of ``bn3`` hands its residual gradient to a
  :class:`GradStash` and ``conv1``'s GEMM accumulates onto it in place
  (beta = 1).
* weight gradient ``dW = dY^T X`` has K = N*H*W (up to 800k) and a tiny
  output (down to 64 x 64): one GEMM has a single output tile and ran 4-10x
  slower than MIOpen.  It is split over K instead: S batched GEMMs of
  ~3,136 rows each with fp32 outputs (``bmm(out_dtype=float32)``), then
  their sum -- as fast as or faster than MIOpen's weight-gradient solvers on
  every ResNet-50 shape (profiles/raw/r5/conv1x1_splitk.jsonl), and the
  gradient comes out in fp32 directly (no bf16 round trip, no cast kernel).
* the strided 1x1 convs (the downsample of layers 2-4) take the same
  GEMMs on the stride-2 sub-grid; their input gradient is scattered into a
  zeroed full-size tensor.

This is also what lets the whole ResNet step be captured in a HIP graph:
MIOpen's GEMM-based 1x1 backward solvers zero their outputs with a memset
that a captured graph does not replay (from the second replay on, the stale
contents of the graph's pool leaked into the gradients of layer 1 and the
stem: tools/probes/graph_alias_probe.py).

Forward: the 3x3 implicit-GEMM kernel of ``csrc/kernels/conv3x3.hip``
instantiated with one tap (``pto_conv1x1_fwd``; hipBLASLt's ``mm`` was
slower than MIOpen on most of these shapes, profiles/raw/r5/conv1x1_bench.jsonl),
so the next BatchNorm's batch statistics come out of its epilogue as for
the 3x3 convs (``stats``) and the BN skips its full statistics read of the
output.  Opt-in (``PTO_CONV1X1_FWD=1``); MIOpen's forward is the default.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .conv3x3 import stats_tiles

_CL = torch.channels_last


class GradStash:
    """One gradient handed from a later backward node to an earlier one of
    the same bottleneck (bn3's residual gradient -> conv1's input GEMM).

    Constraint (merge mode, a downsample block's two sibling 1x1 convs):
    BOTH siblings must run their backward in the same pass.  The first one
    parks its input gradient here and returns None; the second adds its own
    part and returns the sum.  If autograd prunes one branch (e.g.
    ``torch.autograd.grad`` restricted to one branch's inputs, or a detached
    downsample) the parked gradient would be lost, so every parked gradient
    is counted (:attr:`parked`) and :meth:`assert_drained` -- called by the
    ResNet trainer after each backward -- raises if one was never taken."""

    __slots__ = ("g",)
    parked = 0  # gradients put and not yet taken, over every stash

    def __init__(self):
        self.g = None

    def put(self, g):
        if self.g is not None:
            raise RuntimeError("GradStash: gradient already stashed (backward ran twice without a forward?)")
        self.g = g
        GradStash.parked += 1

    def take(self):
        g, self.g = self.g, None
        if g is not None:
            GradStash.parked -= 1
        return g

    @classmethod
    def assert_drained(cls):
        """Raise if a parked gradient was never consumed (a pruned sibling
        branch: its input gradient would silently be missing)."""
        if cls.parked:
            n, cls.parked = cls.parked, 0
            raise RuntimeError(f"GradStash: {n} parked input gradient(s) never consumed -- a conv1x1 merge pair "
                               "whose sibling branch did not run backward (pruned / detached branch)")


def gemm_supported(x: torch.Tensor, conv: nn.Conv2d, stride1: bool = False) -> bool:
    """1x1 bias-free conv, stride 1 (or equal strides, unless ``stride1``)."""
    st = conv.stride
    return (x.is_cuda and x.dim() == 4 and conv.kernel_size == (1, 1) and st[0] == st[1]
            and (st == (1, 1) or not stride1) and conv.padding == (0, 0) and conv.dilation == (1, 1)
            and conv.groups == 1 and conv.bias is None and os.environ.get("PTO_CONV1X1_GEMM", "1") == "1")


def _splitk(m: int) -> int:
    """Batches of the split-K weight gradient: ~3,136 rows each, dividing M."""
    s = max(1, m // 3136)
    while m % s:
        s -= 1
    return s


def weight_grad_1x1(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """``dY^T X`` in fp32 for ``dy2`` [M, Co], ``x2`` [M, Ci] (bf16)."""
    m, co = dy2.shape
    ci = x2.shape[1]
    s = _splitk(m)
    kw = {} if dy2.dtype == torch.float32 else {"out_dtype": torch.float32}
    if s == 1:
        return torch.mm(dy2.t(), x2, **kw)
    part = torch.bmm(dy2.view(s, m // s, co).transpose(1, 2), x2.view(s, m // s, ci), **kw)
    return part.sum(0)


def owned_fwd_supported(x: torch.Tensor, weight: torch.Tensor, dtype) -> bool:
    """The package's MFMA kernel (``pto_conv1x1_fwd``: the 3x3 implicit GEMM
    with one tap) takes the forward: bf16 compute, channel counts on its
    tiles, an fp32 filter, and ``PTO_CONV1X1_FWD=1`` (default off: measured
    slower than MIOpen's on the expanding shapes, profiles/resnet50_r6.md)."""
    C, K = weight.shape[1], weight.shape[0]
    return (dtype == torch.bfloat16 and weight.dtype == torch.float32 and x.dim() == 4 and C % 64 == 0
            and K % 64 == 0 and (K <= 64 or K % 128 == 0) and (K <= 256 or K % 256 == 0)
            and weight.is_contiguous() and os.environ.get("PTO_CONV1X1_FWD", "0") == "1")


class _Conv1x1(torch.autograd.Function):
    """A 1x1 bias-free convolution (stride s): forward on the package's MFMA
    kernel where :func:`owned_fwd_supported` (with the next BatchNorm's
    statistics from its epilogue when ``stats`` is given) else MIOpen; GEMM
    input gradient (accumulating a stashed residual gradient, if any; at
    s > 1 scattered into a zeroed full-size gradient), split-K GEMM weight
    gradient in fp32 (from the strided sub-grid of x at s > 1)."""

    @staticmethod
    def forward(ctx, x, weight, stash, dtype, stride=1, merge=None, stats=None, wbuf=None):
        x = x.to(dtype).contiguous(memory_format=_CL)
        ctx.stash, ctx.wdtype, ctx.stride, ctx.merge = stash, weight.dtype, stride, merge
        ctx.wshape, ctx.wstride = weight.shape, weight.stride()
        if wbuf is not None:
            # bf16 image of the fp32 master filter in the module's persistent
            # buffer (one cast launch), then the MFMA kernel
            L = _lib.lib()
            dev = _lib.stream_ptr(x.device)
            _lib.check(L.pto_conv3x3_wcast(weight.data_ptr(), wbuf.data_ptr(), wbuf.numel(), dev), "conv1x1 wcast")
            N, C, H, W = x.shape
            K = weight.shape[0]
            OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
            part = None
            if stats is not None:
                nblk = stats_tiles(N, OH, OW, K)
                part = torch.empty(nblk * 2 * K, device=x.device, dtype=torch.float32)
                stats.part, stats.nblk = part, nblk
            y = torch.empty(N, K, OH, OW, device=x.device, dtype=torch.bfloat16, memory_format=_CL)
            _lib.check(L.pto_conv1x1_fwd(x.data_ptr(), wbuf.data_ptr(), y.data_ptr(),
                                         None if part is None else part.data_ptr(), N, H, W, C, K, stride, dev),
                       "conv1x1_fwd")
            ctx.save_for_backward(x, wbuf)
            return y
        wb = weight.to(dtype)
        if wb.dim() == 4 and not wb.is_contiguous(memory_format=_CL):
            wb = wb.contiguous(memory_format=_CL)
        ctx.save_for_backward(x, wb)
        return F.conv2d(x, wb, stride=stride)

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        s = ctx.stride
        xfull = x
        if s > 1:  # the pixels a strided 1x1 conv reads
            x = x[:, :, ::s, ::s].contiguous(memory_format=_CL)
        N, ci, H, W = x.shape
        co = wb.shape[0]
        dy = dy.to(wb.dtype).contiguous(memory_format=_CL)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, co)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
        dw = None
        if ctx.needs_input_grad[1]:
            dw = weight_grad_1x1(dy2, x2).to(ctx.wdtype)
            # the parameter's own layout (channels_last [Co, Ci, 1, 1] and
            # contiguous share strides only up to the size-1 dims)
            dw = dw.view(co, ci, 1, 1).as_strided(ctx.wshape, ctx.wstride) if dw.is_contiguous() else dw
        dx = None
        if ctx.needs_input_grad[0]:
            w2 = wb.reshape(co, ci)
            base = ctx.stash.take() if ctx.stash is not None else None
            first = False
            if ctx.merge is not None:  # a sibling conv reads the same x (downsample block)
                sib = ctx.merge.take()
                first = sib is None
                base = base if first else sib
            if base is not None:
                base = base.to(dy2.dtype).contiguous(memory_format=_CL)
            if s == 1 and base is not None:
                dx2 = base.permute(0, 2, 3, 1).reshape(-1, ci).addmm_(dy2, w2)  # dX = base + dY W, in place
                dx = dx2.view(N, H, W, ci).permute(0, 3, 1, 2)
            else:
                dx = torch.mm(dy2, w2).view(N, H, W, ci).permute(0, 3, 1, 2)
                if s > 1:
                    full = base if base is not None else torch.zeros_like(xfull, memory_format=_CL)
                    if base is not None:
                        full[:, :, ::s, ::s] += dx
                    else:
                        full[:, :, ::s, ::s] = dx
                    dx = full
            if first:  # the sibling's backward adds its own part onto this one
                ctx.merge.put(dx)
                dx = None
        elif ctx.stash is not None:
            ctx.stash.take()
        return dx, dw, None, None, None, None, None, None


def _dtype(x):
    return torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype


def _wbuf(conv: nn.Conv2d, x: torch.Tensor, dtype):
    """The module's persistent bf16 filter image for the owned forward, or
    None when that forward does not apply."""
    if not owned_fwd_supported(x, conv.weight, dtype):
        return None
    wb = getattr(conv, "_pto_c1_wb", None)
    if wb is None or wb.device != x.device or wb.shape != conv.weight.shape:
        wb = torch.empty(conv.weight.shape, device=x.device, dtype=torch.bfloat16, memory_format=_CL)
        conv._pto_c1_wb = wb
    return wb


def conv1x1(x: torch.Tensor, conv: nn.Conv2d, merge: GradStash | None = None, stats=None) -> torch.Tensor:
    """``conv(x)`` for a 1x1 bias-free conv, any equal stride (see
    :class:`_Conv1x1`).  ``merge``: shared with the one other conv1x1 that
    reads the same ``x`` (a downsample block's conv1 and downsample conv):
    whichever backward runs second accumulates its input gradient onto the
    first one's (GEMM beta = 1, or a strided in-place add) instead of
    autograd adding the two.  ``stats``: an ``ops.conv3x3.ConvStats`` the
    owned forward fills with the next BatchNorm's statistics partials (left
    empty on the MIOpen path).  Dtype: the autocast dtype when autocast is
    on, else x's."""
    if not gemm_supported(x, conv):
        raise ValueError("conv1x1: needs a 1x1 bias-free conv on a HIP tensor")
    dtype = _dtype(x)
    wb = _wbuf(conv, x, dtype)
    with torch.autocast("cuda", enabled=False):
        return _Conv1x1.apply(x, conv.weight, None, dtype, conv.stride[0], merge, stats if wb is not None else None,
                              wb)


def conv1x1_res(x: torch.Tensor, conv: nn.Conv2d, stash: GradStash, stats=None) -> torch.Tensor:
    """:func:`conv1x1` whose input gradient also receives ``stash``'s
    residual gradient."""
    if not gemm_supported(x, conv, stride1=True):
        raise ValueError("conv1x1_res: needs a 1x1 stride-1 bias-free conv on a HIP tensor")
    dtype = _dtype(x)
    wb = _wbuf(conv, x, dtype)
    with torch.autocast("cuda", enabled=False):
        return _Conv1x1.apply(x, conv.weight, stash, dtype, 1, None, stats if wb is not None else None, wb)
