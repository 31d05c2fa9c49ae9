"""Fused multi-tensor SGD (momentum / weight decay / nesterov) on gfx950.

One launch updates every parameter tensor: a device-resident table of
``(param, grad, momentum, numel)`` records plus a block-prefix array lets
each workgroup find its tensor with a binary search.  The table is built
once and reused, so the launch is HIP-graph capturable.  The learning rate
may live in device memory (``lr_dev``) so LR schedules keep working under
graph replay.

Semantics: ``torch.optim.SGD`` with ``dampening=0`` (the reference uses
``SGD(lr, momentum)``, ``examples/mnist/mnist.py:140``), plus an optional
gradient pre-scale (DDP 1/world) and gradient zeroing after the update
(``zero_grad`` folded into the step).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


class _SgdTensor(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p), ("n", ctypes.c_longlong)]


def _same_dense_layout(*ts) -> bool:
    """Elementwise multi-tensor kernels walk the raw storage, so every tensor
    of a record must be dense (contiguous or channels_last) with equal strides."""
    t0 = ts[0]
    dense = t0.is_contiguous() or (t0.dim() == 4 and t0.is_contiguous(memory_format=torch.channels_last))
    return dense and all(t is None or (t.shape == t0.shape and t.stride() == t0.stride()) for t in ts)


def _grad_ptrs(groups):
    return tuple(p.grad.data_ptr() for g in groups for p in g["params"])


class _TableMixin:
    """Rebuild the device launch table when any gradient tensor changed
    (grads handed over fresh each step by autograd, GradBucketer "none")."""

    def _refresh(self):
        if self._tables is not None and all(p.grad is not None for g in self.param_groups for p in g["params"]):
            if _grad_ptrs(self.param_groups) == self._gptrs:
                return
        self._build()  # also materialises missing grads as zeros
        self._gptrs = _grad_ptrs(self.param_groups)


def _upload(host: torch.Tensor, device) -> torch.Tensor:
    """Host -> device copy of a launch table that never blocks the host: a
    table is rebuilt whenever autograd hands over gradients at new addresses
    (allocator churn), and a pageable copy would stall the CPU for a whole
    step (0.37 ms of idle GPU per ResNet-50 step when the stem's weight
    gradient alternated between two blocks).  The pinned staging block is
    kept by the caching host allocator until the copy has run."""
    if torch.device(device).type != "cuda":
        return host.to(device)
    return host.pin_memory().to(device, non_blocking=True)


def _to_device(host: torch.Tensor, device, pending: list | None, reserved: list | None = None):
    """``host.to(device)``; while a HIP graph is being captured the copy is
    deferred (``pending``, see :meth:`FusedSGD.finish_capture`): the launch
    recorded into the graph only needs the device address, and a host->device
    copy cannot be captured.  The destination must come from ``reserved``
    (allocated before the capture): a tensor allocated DURING the capture
    lives in the graph's private pool, whose blocks the captured kernels
    reuse for their own temporaries -- a replay would overwrite the table."""
    if pending is None or not torch.cuda.is_current_stream_capturing():
        return _upload(host, device)
    for i, t in enumerate(reserved or []):
        if t.shape == host.shape and t.dtype == host.dtype:
            dev = reserved.pop(i)
            break
    else:
        raise RuntimeError("FusedSGD: call prepare_capture() before capturing step() into a HIP graph")
    pending.append((dev, host))
    return dev


class SgdTable:
    @staticmethod
    def table_shapes(ntensors: int):
        """(bytes of the record table, entries of the block-start array)."""
        return ctypes.sizeof(_SgdTensor) * ntensors, ntensors

    def __init__(self, triples, device, keep_grads: bool = True, pending: list | None = None,
                 reserved: list | None = None):
        L = _lib.lib()
        self.L = L
        recs, starts, nb = [], [], 0
        self._keep = []
        for p, g, m in triples:
            if p.dtype != torch.float32 or not _same_dense_layout(p, g, m):
                raise ValueError("SgdTable: fp32 params with grads/momentum of the same dense layout required")
            recs.append((p.data_ptr(), g.data_ptr(), 0 if m is None else m.data_ptr(), p.numel()))
            starts.append(nb)
            nb += L.pto_sgd_block_count(p.numel())
            # the fused trainer owns its flat buffers; an Optimizer must not pin
            # gradients autograd will replace (pointers re-checked every step)
            self._keep.append((p, g if keep_grads else None, m))
        self.nblocks = nb
        self.ntensors = len(recs)
        raw = (_SgdTensor * len(recs))(*[_SgdTensor(*r) for r in recs])
        host = torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(raw), ctypes.sizeof(raw))),
                                dtype=torch.uint8)
        self.table = _to_device(host, device, pending, reserved)
        self.starts = _to_device(torch.tensor(starts, dtype=torch.int32), device, pending, reserved)

    def step(self, lr_dev, lr, momentum, weight_decay, grad_scale, nesterov, zero_grad=True, stream=None,
             batch_cursor=None, n_batches=1):
        """``batch_cursor``: optional int64 device scalar advanced modulo
        ``n_batches`` by the same launch (fused trainer data cursor)."""
        s = stream if stream is not None else _lib.stream_ptr()
        _lib.check(self.L.pto_sgd_multi(self.table.data_ptr(), self.starts.data_ptr(), self.ntensors, self.nblocks,
                                        None if lr_dev is None else lr_dev.data_ptr(), float(lr), float(momentum),
                                        float(weight_decay), float(grad_scale), int(bool(nesterov)),
                                        int(bool(zero_grad)), _lib.ptr(batch_cursor), int(n_batches), s),
                   "sgd_multi")


class FusedSGD(_TableMixin, torch.optim.Optimizer):
    """Drop-in ``torch.optim.SGD`` (dampening=0) backed by one HIP launch.

    Grads are consumed and zeroed in the same launch when ``zero_grad=True``
    is passed to :meth:`step` (set_to_none semantics are emulated by zeros).
    """

    def __init__(self, params, lr=0.01, momentum=0.0, weight_decay=0.0, nesterov=False):
        if nesterov and momentum <= 0:
            raise ValueError("Nesterov momentum requires a momentum")
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, nesterov=nesterov))
        self._tables = None
        self._gptrs = None
        self._pending: list = []
        self._reserved: list = []
        self._lr_dev: list | None = None  # per-group device learning rates of a captured step
        self._lr_host: list = []

    def _build(self):
        self._tables = []
        for group in self.param_groups:
            triples = []
            for p in group["params"]:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                st = self.state[p]
                if group["momentum"] != 0 and "momentum_buffer" not in st:
                    st["momentum_buffer"] = torch.zeros_like(p)
                triples.append((p.data, p.grad, st.get("momentum_buffer")))
            dev = group["params"][0].device
            self._tables.append(SgdTable(triples, dev, keep_grads=False, pending=self._pending,
                                         reserved=self._reserved))

    def prepare_capture(self):
        """Before capturing :meth:`step` into a HIP graph: allocate (outside
        the graph's memory pool) the launch tables the captured step will use."""
        self._reserved = []
        self._lr_dev, self._lr_host = [], []
        for group in self.param_groups:
            nbytes, nstarts = SgdTable.table_shapes(len(group["params"]))
            dev = group["params"][0].device
            self._reserved.append(torch.empty(nbytes, dtype=torch.uint8, device=dev))
            self._reserved.append(torch.empty(nstarts, dtype=torch.int32, device=dev))
            # the captured launch reads lr from device memory: LR schedules keep working
            self._lr_dev.append(torch.full((1,), float(group["lr"]), dtype=torch.float32, device=dev))
            self._lr_host.append(float(group["lr"]))

    def sync_lr(self):
        """Before replaying a captured step: push changed learning rates to
        the device scalars the graph reads (momentum / weight decay / nesterov
        are fixed at capture)."""
        for i, group in enumerate(self.param_groups):
            if self._lr_dev is not None and float(group["lr"]) != self._lr_host[i]:
                self._lr_dev[i].fill_(float(group["lr"]))
                self._lr_host[i] = float(group["lr"])

    def finish_capture(self):
        """After capturing :meth:`step` into a HIP graph: upload the launch
        tables built during the capture (the graph's gradient tensors)."""
        for dev, host in self._pending:
            dev.copy_(host)
        self._pending = []
        self._reserved = []

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0, zero_grad: bool = False):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._refresh()
        capturing = self._lr_dev is not None and torch.cuda.is_current_stream_capturing()
        for i, (group, table) in enumerate(zip(self.param_groups, self._tables)):
            table.step(self._lr_dev[i] if capturing else None, group["lr"], group["momentum"],
                       group["weight_decay"], grad_scale, group["nesterov"], zero_grad=zero_grad)
        return loss

    def zero_grad(self, set_to_none: bool = False):
        # keep grad tensors alive: the launch table holds their pointers
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    p.grad.zero_()


class _AdamTensor(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("master", ctypes.c_void_p), ("m", ctypes.c_void_p),
                ("v", ctypes.c_void_p), ("n", ctypes.c_longlong)]


class FusedAdamW(_TableMixin, torch.optim.Optimizer):
    """Multi-tensor AdamW in one HIP launch (csrc/kernels/optim_kernels.hip).

    bf16 parameters get fp32 master weights and fp32 moments inside the
    optimizer (``mixed``); fp32 parameters are updated in place.  Matches
    ``torch.optim.AdamW`` (decoupled weight decay, bias correction) up to
    the bf16 rounding of the exported parameter.  ``grad_scale`` folds a
    DDP 1/world (or loss-scale) factor into the same pass.
    """

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._tables = None
        self._gptrs = None
        self._step = 0

    def _build(self):
        L = _lib.lib()
        self._tables = []
        for group in self.param_groups:
            recs, starts, nb, keep = [], [], 0, []
            mixed = None
            for p in group["params"]:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                st = self.state[p]
                is_mixed = p.dtype == torch.bfloat16
                if mixed is None:
                    mixed = is_mixed
                if mixed != is_mixed:
                    raise ValueError("FusedAdamW: a param group must be all-bf16 or all-fp32")
                if "exp_avg" not in st:
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)  # keeps p's layout
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                    if is_mixed:
                        st["master"] = p.detach().float()
                master = st.get("master")
                if not _same_dense_layout(p, p.grad, master, st["exp_avg"], st["exp_avg_sq"]):
                    raise ValueError("FusedAdamW: param, grad and state must share one dense layout")
                recs.append(_AdamTensor(p.data_ptr(), p.grad.data_ptr(), 0 if master is None else master.data_ptr(),
                                        st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), p.numel()))
                starts.append(nb)
                nb += L.pto_adamw_block_count(p.numel())
                keep.append((p, master, st["exp_avg"], st["exp_avg_sq"]))  # not the grad: see _grad_ptrs
            raw = (_AdamTensor * len(recs))(*recs)
            dev = group["params"][0].device
            table = _upload(torch.frombuffer(bytearray(ctypes.string_at(ctypes.addressof(raw), ctypes.sizeof(raw))),
                                             dtype=torch.uint8), dev)
            self._tables.append((table, _upload(torch.tensor(starts, dtype=torch.int32), dev), len(recs), nb,
                                 int(bool(mixed)), keep))

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0, zero_grad: bool = False):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._refresh()
        self._step += 1
        L = _lib.lib()
        for group, (table, starts, nt, nb, mixed, _) in zip(self.param_groups, self._tables):
            b1, b2 = group["betas"]
            _lib.check(L.pto_adamw_multi(table.data_ptr(), starts.data_ptr(), nt, nb, mixed, None,
                                         float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                                         float(group["weight_decay"]), self._step, float(grad_scale),
                                         int(bool(zero_grad)), _lib.stream_ptr()), "adamw_multi")
        return loss

    def zero_grad(self, set_to_none: bool = False):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    p.grad.zero_()
