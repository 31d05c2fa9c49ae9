"""Minimal TensorBoard event-file writer (scalars only).

The reference trainer logs ``loss`` every ``--log-interval`` batches and
``accuracy`` per epoch through tensorboardX's ``SummaryWriter(args.dir)``
(``examples/mnist/mnist.py:49,65,108``).  Neither tensorboard nor
tensorboardX is installed in this image, so this module writes the same
on-disk format itself: a ``events.out.tfevents.<time>.<host>`` file of
TFRecords (length, masked CRC32C of the length, payload, masked CRC32C of
the payload), each payload a hand-encoded ``tensorflow.Event`` protobuf:

    Event   { double wall_time = 1; int64 step = 2; string file_version = 3;
              Summary summary = 5; }
    Summary { repeated Value value = 1; }
    Value   { string tag = 1; float simple_value = 2; }

TensorBoard (or ``tbparse``/``tf.data.TFRecordDataset``) reads the files.
:func:`read_scalars` parses them back (tests, tooling).
"""
from __future__ import annotations

import os
import socket
import struct
import time

# ---------------------------------------------------------------- CRC32C --
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# -------------------------------------------------------------- protobuf --
def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _event(wall_time: float, step: int, *, file_version: str | None = None,
           scalars: dict[str, float] | None = None) -> bytes:
    msg = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        msg += _len_field(3, file_version.encode())
    if scalars:
        summary = b"".join(
            _len_field(1, _len_field(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v)))
            for tag, v in scalars.items())
        msg += _len_field(5, summary)
    return msg


def _record(payload: bytes) -> bytes:
    n = struct.pack("<Q", len(payload))
    return n + struct.pack("<I", _masked(n)) + payload + struct.pack("<I", _masked(payload))


class SummaryWriter:
    """``add_scalar(tag, value, step)`` into ``logdir`` (tensorboardX API
    subset used by the reference trainer)."""

    def __init__(self, logdir: str = "logs", filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}"
                                         f"{filename_suffix}")
        self._f = open(self.path, "ab")
        self._f.write(_record(_event(time.time(), 0, file_version="brain.Event:2")))
        self._f.flush()

    def add_scalar(self, tag: str, value: float, global_step: int = 0, walltime: float | None = None):
        self._f.write(_record(_event(walltime or time.time(), global_step, scalars={tag: value})))

    def flush(self):
        self._f.flush()

    def close(self):
        if not self._f.closed:
            self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ---------------------------------------------------------------- reader --
def _read_varint(b: bytes, i: int):
    shift = n = 0
    while True:
        c = b[i]
        i += 1
        n |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return n, i


def _fields(b: bytes):
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _read_varint(b, i)
        elif w == 1:
            v, i = b[i:i + 8], i + 8
        elif w == 5:
            v, i = b[i:i + 4], i + 4
        elif w == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        else:
            raise ValueError(f"unsupported wire type {w}")
        yield f, w, v


def read_scalars(path: str) -> list[tuple[int, str, float]]:
    """[(step, tag, value)] from one event file; CRCs are verified."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        (lc,) = struct.unpack_from("<I", data, i + 8)
        if lc != _masked(data[i:i + 8]):
            raise ValueError("corrupt record length")
        payload = data[i + 12:i + 12 + n]
        (pc,) = struct.unpack_from("<I", data, i + 12 + n)
        if pc != _masked(payload):
            raise ValueError("corrupt record payload")
        i += 16 + n
        step = 0
        for f, _, v in _fields(payload):
            if f == 2:
                step = v
            elif f == 5:
                for _, _, val in _fields(v):
                    tag, sv = None, None
                    for vf, _, vv in _fields(val):
                        if vf == 1:
                            tag = vv.decode()
                        elif vf == 2:
                            sv = struct.unpack("<f", vv)[0]
                    if tag is not None and sv is not None:
                        out.append((step, tag, sv))
    return out
