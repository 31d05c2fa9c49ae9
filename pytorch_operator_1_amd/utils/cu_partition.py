"""Disjoint CU partitions for ranks that share one GPU.

The multi-GPU MNIST step (``train/fused_step.py``) runs its gradient
exchange as extra workgroups of the next step's forward launch: the
forward's conv workgroups wait on a counter that the exchange workgroups of
the SAME launch publish, and those wait on the peers' exchange workgroups.
On a node with one rank per GPU that is safe (the exchange workgroups are
first in the grid and the dispatcher places them first).  Ranks that share
one GPU (a rehearsal on a one-GPU box) could starve each other instead: one
rank's spinning conv workgroups may hold the CUs its peer needs to start its
own exchange (``XgmiAllReduce.colocated``).

A :class:`Partition` gives each co-located rank its own CUs: a HIP stream
created with ``hipExtStreamCreateWithCUMask`` (``pto_stream_create_cu_mask``)
whose hardware queue may only dispatch to the CUs of this rank's mask,
wrapped in ``torch.cuda.ExternalStream`` and made the current stream, so
every launch of the rank -- eager or HIP-graph replay, which launches on the
current stream -- stays inside the mask.  With disjoint masks a co-located
rank can no longer hold a peer's CUs, and the trainer runs the schedule a
one-rank-per-GPU node runs.  Whether the hardware honours the mask (eagerly
and under graph replay) is measured, not assumed: :func:`probe_cus` reads
each workgroup's ``HW_REG_XCC_ID`` / ``HW_REG_HW_ID`` (tests/test_cu_partition_gpu.py,
profiles/cu_partition_r6.md).

Mask layout: bit ``i`` of the mask is "CU ``i``" of the device's flat CU
numbering.  ``layout="block"`` (the default) gives partition ``k`` of ``n``
the bits ``[k*C/n, (k+1)*C/n)``; measured on the MI355X, the runtime deals
those bits over the 8 XCDs, so the partition gets 32/n CUs of EVERY XCD
(each rank keeps all eight L2s).  ``"stride"`` (bits ``i % n == k``) is
accepted by the runtime but not applied: its kernels still reach all 256
CUs (profiles/cu_partition_r6.md), so it is kept only as the probe's
negative control.
"""
from __future__ import annotations

import ctypes
import os

# HW_ID fields (gfx9 layout, the one gfx950 keeps)
_HW_FIELDS = {"wave": (0, 4), "simd": (4, 2), "pipe": (6, 2), "cu": (8, 4), "sh": (12, 1), "se": (13, 3),
              "tg": (16, 4), "vm": (20, 4), "queue": (24, 3), "state": (27, 3), "me": (30, 2)}

_active: dict[int, "Partition"] = {}


def mask_bits(index: int, parts: int, n_cu: int, layout: str = "block") -> list[int]:
    """The CU numbers of partition ``index`` of ``parts`` over ``n_cu`` CUs."""
    if not (0 <= index < parts) or parts < 1 or n_cu < parts:
        raise ValueError(f"bad partition {index} of {parts} over {n_cu} CUs")
    if layout == "block":
        return list(range(index * n_cu // parts, (index + 1) * n_cu // parts))
    if layout == "stride":
        return list(range(index, n_cu, parts))
    raise ValueError(f"layout must be 'block' or 'stride', not {layout!r}")


def mask_words(bits, n_cu: int) -> list[int]:
    """32-bit words of a CU bit mask (word w holds CUs 32w .. 32w+31)."""
    words = [0] * ((n_cu + 31) // 32)
    for b in bits:
        if not 0 <= b < n_cu:
            raise ValueError(f"CU {b} outside 0..{n_cu - 1}")
        words[b // 32] |= 1 << (b % 32)
    return words


def words_bits(words) -> list[int]:
    return [32 * w + i for w, x in enumerate(words) for i in range(32) if (int(x) >> i) & 1]


def decode_hw_id(hw: int) -> dict:
    """Fields of one HW_ID word."""
    return {k: (int(hw) >> lo) & ((1 << n) - 1) for k, (lo, n) in _HW_FIELDS.items()}


def cu_key(xcc: int, hw: int) -> tuple[int, int, int, int]:
    """Physical CU of a wave: (XCD, shader engine, shader array, CU)."""
    f = decode_hw_id(hw)
    return (int(xcc), f["se"], f["sh"], f["cu"])


def summarize(words) -> dict:
    """Per-CU and per-XCD workgroup counts of a :func:`probe_cus` result
    (flat ``[xcc, hw, xcc, hw, ...]``)."""
    cus: dict[tuple, int] = {}
    queues: set[int] = set()
    for i in range(0, len(words), 2):
        k = cu_key(words[i], words[i + 1])
        cus[k] = cus.get(k, 0) + 1
        queues.add(decode_hw_id(words[i + 1])["queue"])
    per_xcc: dict[int, int] = {}
    for k in cus:
        per_xcc[k[0]] = per_xcc.get(k[0], 0) + 1
    return {"cus": cus, "n_cus": len(cus), "cus_per_xcc": dict(sorted(per_xcc.items())), "queues": sorted(queues)}


def probe_cus(stream=None, blocks: int = 8192, spin: int = 400, graph: bool = False) -> dict:
    """Launch ``k_cu_id`` (``blocks`` one-wave workgroups that each idle a
    few µs) on ``stream`` (default: the current one) and return
    :func:`summarize` of where its workgroups ran.  ``graph``: capture the
    launch in a HIP graph and replay it on ``stream`` instead (the path the
    trainer's replays take)."""
    import torch

    from ..ops import _lib

    L = _lib.lib()
    stream = stream or torch.cuda.current_stream()
    out = torch.empty(2 * blocks, dtype=torch.int32, device=stream.device)
    with torch.cuda.stream(stream):
        out.fill_(-1)
        if graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                _lib.check(L.pto_cu_id_probe(blocks, out.data_ptr(), spin, torch.cuda.current_stream().cuda_stream),
                           "cu_id_probe")
            out.fill_(-1)
            g.replay()
        else:
            _lib.check(L.pto_cu_id_probe(blocks, out.data_ptr(), spin, stream.cuda_stream), "cu_id_probe")
    stream.synchronize()
    w = [x & 0xFFFFFFFF for x in out.tolist()]
    if any(x == 0xFFFFFFFF for x in w[0::2]):
        raise RuntimeError("cu_id_probe: some workgroups did not report")
    return summarize(w)


class Partition:
    """CU partition ``index`` of ``parts`` of ``device``: :attr:`stream` (a
    ``torch.cuda.ExternalStream`` on a CU-masked HIP stream) and
    :meth:`new_stream` for more streams with the same mask."""

    def __init__(self, device, index: int, parts: int, layout: str | None = None, n_cu: int | None = None):
        import torch

        self.device = torch.device(device)
        self.index, self.parts = int(index), int(parts)
        self.layout = layout or os.environ.get("PTO_CU_PARTITION_LAYOUT", "block")
        self.n_cu = int(n_cu or torch.cuda.get_device_properties(self.device).multi_processor_count)
        self.bits = mask_bits(self.index, self.parts, self.n_cu, self.layout)
        self.words = mask_words(self.bits, self.n_cu)
        self._raw: list[int] = []
        self._streams = []
        self.stream = self.new_stream()

    def new_stream(self):
        import torch

        from ..ops import _lib

        L = _lib.lib()
        arr = (ctypes.c_uint * len(self.words))(*self.words)
        raw = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(L.pto_stream_create_cu_mask(len(self.words), arr, ctypes.byref(raw)), "stream_create_cu_mask")
        back = (ctypes.c_uint * len(self.words))()
        _lib.check(L.pto_stream_get_cu_mask(raw, len(self.words), back), "stream_get_cu_mask")
        if [int(x) for x in back] != self.words:
            raise RuntimeError(f"CU mask not applied: asked {self.words}, stream has {list(back)}")
        self._raw.append(raw.value)
        s = torch.cuda.ExternalStream(raw.value, device=self.device)
        self._streams.append(s)
        return s

    def owns(self, stream) -> bool:
        return stream is not None and int(stream.cuda_stream) in self._raw

    def activate(self) -> "Partition":
        """Make :attr:`stream` this thread's current stream on the device and
        register the partition (:func:`active`)."""
        import torch

        torch.cuda.set_stream(self.stream)
        _active[self.device.index] = self
        return self

    def describe(self) -> dict:
        return {"index": self.index, "parts": self.parts, "layout": self.layout, "cus": len(self.bits),
                "device_cus": self.n_cu, "mask_words": [f"{w:08x}" for w in self.words]}

    def close(self):
        import torch

        from ..ops import _lib

        torch.cuda.synchronize(self.device)
        if _active.get(self.device.index) is self:
            torch.cuda.set_stream(torch.cuda.default_stream(self.device))
            del _active[self.device.index]
        L = _lib.lib()
        for r in self._raw:
            L.pto_stream_destroy(ctypes.c_void_p(r))
        self._raw, self._streams = [], []


def active(device=None) -> Partition | None:
    """The partition whose stream is the current stream of ``device``
    (None when the rank runs on unmasked streams)."""
    import torch

    if not torch.cuda.is_available():
        return None
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    p = _active.get(dev.index)
    if p is None or not p.owns(torch.cuda.current_stream(dev)):
        return None
    return p


def side_stream(device):
    """A stream for work that runs beside the current one (e.g. a graph
    warm-up): a pool stream normally; with a partition active, a SECOND
    stream carrying the partition's mask (cached on the partition).
    Measured on the 2-rank rehearsal (profiles/cu_partition_r6.md): warming
    up on the partition's own stream instead (``PTO_CU_SIDE_STREAM=main``)
    made every later replay of the inline schedule ~11x slower (728-750 vs
    66 us/step, interleaved on one box), so the warm-up gets its own
    masked queue."""
    import torch

    p = active(device)
    if p is None:
        return torch.cuda.Stream(device)
    if os.environ.get("PTO_CU_SIDE_STREAM", "own") == "main":  # the measured-slower variant, for A/B runs
        return p.stream
    if len(p._streams) < 2:
        p.new_stream()
    return p._streams[1]


def share_of(local_rank: int, local_world: int, n_gpus: int) -> tuple[int, int, int]:
    """``(device index, partition index, partitions)`` of a local rank when
    ``local_world`` ranks are dealt round-robin over ``n_gpus`` GPUs (the
    device choice of ``utils.dist.init_distributed``: local_rank % n_gpus)."""
    n = max(1, n_gpus)
    d = local_rank % n
    parts = len(range(d, local_world, n))
    return d, local_rank // n, parts


def activate_for_rank(local_rank: int, local_world: int, device=None) -> Partition | None:
    """Give this rank its own CUs when it shares its GPU with other local
    ranks (``local_world`` > visible GPUs); None (nothing changed) when it
    has the GPU to itself."""
    import torch

    from .dist import gpu_count

    n = gpu_count()
    d, k, parts = share_of(local_rank, local_world, n)
    if parts <= 1:
        return None
    dev = torch.device(device) if device is not None else torch.device("cuda", d)
    return Partition(dev, k, parts).activate()
