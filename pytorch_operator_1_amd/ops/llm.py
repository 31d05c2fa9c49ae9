"""Autograd wrappers over the bf16 transformer kernels
(``csrc/kernels/llm_kernels.hip``) used by :mod:`..models.llama`.

The ops take bf16 HIP tensors and raise on anything else (no silent
fallback): :func:`add_rmsnorm` (residual add + RMSNorm, the residual
gradient add fused into the RMSNorm backward), :func:`swiglu`,
:func:`rope_` (in place on the fused QKV projection), and
:func:`cross_entropy` (vocab-wide CE on bf16 logits, gradient written in
place into the logits buffer so no fp32 ``[tokens, 128256]`` tensor ever
exists).
"""
from __future__ import annotations

import torch

from . import _lib


def _req(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"{name}: HIP device tensor required")
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name}: bf16 only (got {t.dtype})")
    return t.contiguous()


def _p(t):
    return None if t is None else t.data_ptr()


class _AddRMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, w, eps):
        x = _req(x, "add_rmsnorm")
        w = _req(w, "add_rmsnorm")
        D = x.shape[-1]
        M = x.numel() // D
        y = torch.empty_like(x)
        rstd = torch.empty(M, device=x.device, dtype=torch.float32)
        if r is not None:
            r = _req(r, "add_rmsnorm")
            h = torch.empty_like(x)
        else:
            h = x
        _lib.check(_lib.lib().pto_add_rmsnorm_fwd(x.data_ptr(), _p(r), w.data_ptr(), _p(h if r is not None else None),
                                                   y.data_ptr(), rstd.data_ptr(), M, D, float(eps),
                                                   _lib.stream_ptr(x.device)), "add_rmsnorm_fwd")
        ctx.save_for_backward(h, w, rstd)
        ctx.has_res = r is not None
        ctx.set_materialize_grads(False)  # an unused h output costs no zero tensor
        if r is None:
            return y
        return h, y

    @staticmethod
    def backward(ctx, *grads):
        h, w, rstd = ctx.saved_tensors
        if ctx.has_res:
            dh, dy = grads
        else:
            dh, dy = None, grads[0]
        D = h.shape[-1]
        M = h.numel() // D
        L = _lib.lib()
        dy = torch.zeros_like(h) if dy is None else dy.contiguous()
        if dh is not None:
            dh = dh.contiguous()
        dx = torch.empty_like(h)
        dw = torch.empty_like(w)
        part = torch.empty(L.pto_rmsnorm_bwd_groups(M), D, device=h.device, dtype=torch.float32)
        _lib.check(L.pto_rmsnorm_bwd(dy.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr(), _p(dh), dx.data_ptr(),
                                     dw.data_ptr(), part.data_ptr(), M, D, _lib.stream_ptr(h.device)), "rmsnorm_bwd")
        return dx, (dx if ctx.has_res else None), dw, None


def add_rmsnorm(x, residual, weight, eps: float = 1e-5):
    """``h = x + residual; y = rmsnorm(h) * weight`` -> ``(h, y)``."""
    return _AddRMSNorm.apply(x, residual, weight, eps)


def rmsnorm(x, weight, eps: float = 1e-5):
    return _AddRMSNorm.apply(x, None, weight, eps)


class TStash:
    """A gradient handed TRANSPOSED from one backward node to the next: the
    SwiGLU backward writes d(gate|up)^T while it computes d(gate|up), and the
    gate|up projection's K-contiguous weight gradient (:class:`_LinearTW`)
    takes it instead of transposing the [tokens x 2F] gradient itself."""

    __slots__ = ("t",)

    def __init__(self):
        self.t = None

    def take(self):
        t, self.t = self.t, None
        return t


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, tstash=None):
        gu = _req(gu, "swiglu")
        F2 = gu.shape[-1]
        M = gu.numel() // F2
        out = torch.empty(*gu.shape[:-1], F2 // 2, device=gu.device, dtype=gu.dtype)
        _lib.check(_lib.lib().pto_swiglu_fwd(gu.data_ptr(), out.data_ptr(), M, F2 // 2, _lib.stream_ptr(gu.device)),
                   "swiglu_fwd")
        ctx.save_for_backward(gu)
        ctx.tstash = tstash
        return out

    @staticmethod
    def backward(ctx, dout):
        (gu,) = ctx.saved_tensors
        F2 = gu.shape[-1]
        M = gu.numel() // F2
        dout = dout.contiguous()
        dgu = torch.empty_like(gu)
        st = ctx.tstash
        if st is not None and M % 8 == 0 and (F2 // 2) % 64 == 0:
            dgu_t = torch.empty(F2, M, device=gu.device, dtype=gu.dtype)
            _lib.check(_lib.lib().pto_swiglu_bwd_t(gu.data_ptr(), dout.data_ptr(), dgu.data_ptr(), dgu_t.data_ptr(),
                                                   M, F2 // 2, _lib.stream_ptr(gu.device)), "swiglu_bwd_t")
            st.t = dgu_t
        else:
            _lib.check(_lib.lib().pto_swiglu_bwd(gu.data_ptr(), dout.data_ptr(), dgu.data_ptr(), M, F2 // 2,
                                                 _lib.stream_ptr(gu.device)), "swiglu_bwd")
        return dgu, None


def swiglu(gu, tstash: TStash | None = None):
    """``silu(gu[..., :F]) * gu[..., F:]`` for the fused gate|up projection.
    ``tstash``: also hand the transposed input gradient to the producer of
    ``gu`` (see :class:`TStash`)."""
    return _SwiGLU.apply(gu, tstash)


class _RoPE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, seq_len, n_rot, head_dim):
        if not qkv.is_contiguous():
            raise ValueError("rope_: qkv must be contiguous")
        _req(qkv, "rope_")
        M = qkv.numel() // qkv.shape[-1]
        _lib.check(_lib.lib().pto_rope(qkv.data_ptr(), None, cos.data_ptr(), sin.data_ptr(), M, seq_len, n_rot, 0,
                                       head_dim, qkv.shape[-1], 0, _lib.stream_ptr(qkv.device)), "rope_fwd")
        ctx.mark_dirty(qkv)
        ctx.save_for_backward(cos, sin)
        ctx.cfg = (seq_len, n_rot, head_dim)
        return qkv

    @staticmethod
    def backward(ctx, g):
        cos, sin = ctx.saved_tensors
        S, n_rot, D = ctx.cfg
        # out of place: the incoming gradient may be referenced elsewhere
        g = g.contiguous()
        dg = torch.empty_like(g)
        M = g.numel() // g.shape[-1]
        _lib.check(_lib.lib().pto_rope(g.data_ptr(), dg.data_ptr(), cos.data_ptr(), sin.data_ptr(), M, S, n_rot,
                                       g.shape[-1] // D, D, g.shape[-1], 1, _lib.stream_ptr(g.device)), "rope_bwd")
        return dg, None, None, None, None, None


def rope_(qkv, cos, sin, seq_len: int, n_rot: int, head_dim: int):
    """Rotate (HF rotate_half convention) the first ``n_rot`` heads of every
    ``[.., heads*head_dim]`` row of ``qkv`` in place; rows are ordered
    ``(batch, position)`` and ``cos``/``sin`` are fp32 ``[seq_len, head_dim/2]``."""
    return _RoPE.apply(qkv, cos, sin, seq_len, n_rot, head_dim)


def rope_tables(seq_len: int, head_dim: int, theta: float, device, scaling: dict | None = None):
    """fp32 cos/sin tables ``[seq_len, head_dim/2]`` (Llama-3 frequency
    scaling applied when ``scaling`` is given, as in the Llama-3.1 recipe)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling:
        import math

        factor, lo, hi, old = (scaling["factor"], scaling["low_freq_factor"], scaling["high_freq_factor"],
                               scaling["original_max_position_embeddings"])
        wl = 2 * math.pi / inv
        smooth = ((old / wl) - lo) / (hi - lo)
        scaled = torch.where(wl > old / lo, inv / factor, inv)
        mid = (wl <= old / lo) & (wl >= old / hi)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    ang = torch.outer(torch.arange(seq_len, dtype=torch.float64), inv)
    return ang.cos().float().to(device), ang.sin().float().to(device)


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        logits = _req(logits, "cross_entropy")
        V = logits.shape[-1]
        M = logits.numel() // V
        labels = labels.reshape(M).to(torch.int64).contiguous()
        lse = torch.empty(M, device=logits.device, dtype=torch.float32)
        rows = torch.empty(M, device=logits.device, dtype=torch.float32)
        _lib.check(_lib.lib().pto_ce_fwd(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), rows.data_ptr(), M, V,
                                         ignore_index, _lib.stream_ptr(logits.device)), "ce_fwd")
        count = (labels != ignore_index).sum().clamp_min(1).float()
        ctx.save_for_backward(logits, labels, lse, count)
        ctx.ignore_index = ignore_index
        return rows.sum() / count

    @staticmethod
    def backward(ctx, gout):
        logits, labels, lse, count = ctx.saved_tensors
        V = logits.shape[-1]
        M = logits.numel() // V
        scale = (gout.float() / count).reshape(1)
        # logits is an intermediate owned by this op (the producing GEMM's
        # backward needs only its inputs), so the gradient overwrites it.
        _lib.check(_lib.lib().pto_ce_bwd(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), scale.data_ptr(), M, V,
                                         ctx.ignore_index, _lib.stream_ptr(logits.device)), "ce_bwd")
        return logits, None, None


def cross_entropy(logits, labels, ignore_index: int = -100):
    """Mean token cross-entropy over non-ignored labels on bf16 logits."""
    return _CrossEntropy.apply(logits, labels, ignore_index)


def flash_attention_supported(S: int, H: int, Hkv: int, head_dim: int) -> bool:
    """Shapes the HIP kernels cover: head_dim 128, S % 128 == 0, H % Hkv == 0."""
    return head_dim == 128 and S % 128 == 0 and H % Hkv == 0 and ((S // 32) * (H // Hkv)) % 4 == 0


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B, S, H, Hkv):
        qkv = _req(qkv, "flash_attention")
        D = 128
        rs = qkv.shape[-1]
        if rs != (H + 2 * Hkv) * D or qkv.numel() != B * S * rs:
            raise ValueError("flash_attention: qkv must be [B*S, (H + 2*Hkv)*128]")
        o = torch.empty(B * S, H * D, device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty(B, H, S, device=qkv.device, dtype=torch.float32)
        base = qkv.data_ptr()
        esz = qkv.element_size()
        _lib.check(_lib.lib().pto_attn_fwd(base, base + H * D * esz, base + (H + Hkv) * D * esz, o.data_ptr(),
                                           lse.data_ptr(), B, S, H, Hkv, rs, rs, rs, H * D, D ** -0.5,
                                           _lib.stream_ptr(qkv.device)), "attn_fwd")
        ctx.save_for_backward(qkv, o, lse)
        ctx.shape = (B, S, H, Hkv)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        B, S, H, Hkv = ctx.shape
        D = 128
        rs = qkv.shape[-1]
        do = do.contiguous()
        dqkv = torch.empty_like(qkv)
        delta = torch.empty(B, H, S, device=qkv.device, dtype=torch.float32)
        base, dbase, esz = qkv.data_ptr(), dqkv.data_ptr(), qkv.element_size()
        _lib.check(_lib.lib().pto_attn_bwd(base, base + H * D * esz, base + (H + Hkv) * D * esz, o.data_ptr(),
                                           do.data_ptr(), lse.data_ptr(), delta.data_ptr(), dbase,
                                           dbase + H * D * esz, dbase + (H + Hkv) * D * esz, rs, B, S, H, Hkv,
                                           rs, rs, rs, H * D, D ** -0.5, _lib.stream_ptr(qkv.device)), "attn_bwd")
        return dqkv, None, None, None, None


def flash_attention(qkv, B: int, S: int, H: int, Hkv: int):
    """Causal GQA attention straight from the fused QKV projection
    ``[B*S, (H + 2*Hkv)*128]`` (q heads, then k, then v heads per row) to
    ``O [B*S, H*128]`` — the layout the output projection consumes."""
    return _FlashAttention.apply(qkv, B, S, H, Hkv)


def transpose_into(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """``dst[:] = src.t()`` for 2-D bf16 HIP matrices (LDS-tiled kernel);
    plain copy on CPU tensors (tests)."""
    if src.dim() != 2 or dst.shape != (src.shape[1], src.shape[0]):
        raise ValueError(f"transpose_into: {tuple(src.shape)} -> {tuple(dst.shape)}")
    if not src.is_cuda:
        dst.copy_(src.t())
        return dst
    src, dst_c = _req(src, "transpose_into"), dst
    if not dst.is_contiguous() or dst.dtype != torch.bfloat16:
        raise ValueError("transpose_into: contiguous bf16 destination required")
    _lib.check(_lib.lib().pto_transpose_bf16(src.data_ptr(), dst_c.data_ptr(), src.shape[0], src.shape[1],
                                             src.stride(0), dst_c.stride(0), _lib.stream_ptr(src.device)),
               "transpose_bf16")
    return dst


class _LinearTW(torch.autograd.Function):
    """``y = x W^T`` whose input gradient is computed from the transposed
    copy ``Wt = W^T`` (``dX = dY Wt^T``): both dgrad operands are then
    K-contiguous, the layout the forward GEMM already uses.  hipBLASLt's
    pick for the usual ``dY W`` (B operand N-contiguous) ran at ~1.0
    PFLOP/s in the Llama-3-8B step vs ~1.5 for the K-contiguous one
    (profiles/llama8b_step_rocprof.md)."""

    @staticmethod
    def forward(ctx, x, w, wt, dw_kcontig, tstash=None):
        ctx.save_for_backward(x, wt)
        ctx.dw_kcontig, ctx.tstash = dw_kcontig, tstash
        return torch.nn.functional.linear(x, w)

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        dx = torch.nn.functional.linear(dy, wt) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            dy2 = dy.reshape(-1, dy.shape[-1])
            if ctx.dw_kcontig and x2.is_cuda:
                # dW = (dY^T)(X^T)^T from transposed activations: both operands
                # K(token)-contiguous.  Pays for w13/wo only
                # (tools/dw_layout_bench.py: 3.21 -> 2.39 + 0.51 ms, 0.58 ->
                # 0.38 + 0.14 ms at 4x4096 tokens)
                xt = transpose_into(x2.contiguous(), torch.empty(x2.shape[1], x2.shape[0], device=x2.device,
                                                                  dtype=x2.dtype))
                dyt = ctx.tstash.take() if ctx.tstash is not None else None  # written by the SwiGLU backward
                if dyt is None or dyt.shape != (dy2.shape[1], dy2.shape[0]):
                    dyt = transpose_into(dy2.contiguous(), torch.empty(dy2.shape[1], dy2.shape[0],
                                                                        device=dy2.device, dtype=dy2.dtype))
                dw = dyt.mm(xt.t())
            else:
                dw = dy2.t().mm(x2)
        return dx, dw, None, None, None


def linear_tw(x, w, wt, dw_kcontig: bool = False, tstash: TStash | None = None):
    """``F.linear(x, w)`` with the dgrad taken from ``wt`` (== ``w.t()``,
    kept current by the caller after every weight update); ``dw_kcontig``:
    weight gradient from transposed activations (``tstash``: the output
    gradient's transpose, if the next op's backward provides it)."""
    return _LinearTW.apply(x, w, wt, dw_kcontig, tstash)
