"""IDX (MNIST / FashionMNIST ``*-idx?-ubyte[.gz]``) reader.

The reference trainer reads FashionMNIST through torchvision with
``download=True`` into ``../data`` (``examples/mnist/mnist.py:119-131``).
There is no network here and torchvision is not a dependency, so the
trainer reads the same files from the same on-disk layout when they are
present (``<root>/FashionMNIST/raw/train-images-idx3-ubyte`` etc., plain or
gzipped) and falls back to synthetic data otherwise.  Pure numpy: nothing
in the file is executed.
"""
from __future__ import annotations

import gzip
import os

import numpy as np

# IDX type codes -> numpy big-endian dtypes
_DTYPES = {0x08: ">u1", 0x09: ">i1", 0x0B: ">i2", 0x0C: ">i4", 0x0D: ">f4", 0x0E: ">f8"}

_FILES = {
    True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
    False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"),
}


def read_idx(path: str) -> np.ndarray:
    """Parse one IDX file (``.gz`` transparently)."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        raw = f.read()
    if len(raw) < 4 or raw[0] != 0 or raw[1] != 0:
        raise ValueError(f"{path}: not an IDX file (bad magic)")
    code, ndim = raw[2], raw[3]
    if code not in _DTYPES:
        raise ValueError(f"{path}: unknown IDX element type 0x{code:02x}")
    dims = np.frombuffer(raw, dtype=">u4", count=ndim, offset=4).astype(np.int64)
    dt = np.dtype(_DTYPES[code])
    n = int(np.prod(dims)) if ndim else 1
    off = 4 + 4 * ndim
    if len(raw) - off < n * dt.itemsize:
        raise ValueError(f"{path}: truncated ({len(raw) - off} bytes, need {n * dt.itemsize})")
    return np.frombuffer(raw, dtype=dt, count=n, offset=off).reshape(tuple(dims)).astype(dt.newbyteorder("="))


def write_idx(path: str, arr: np.ndarray) -> None:
    """Inverse of :func:`read_idx` (used by tests and data-prep scripts)."""
    inv = {np.dtype(v).newbyteorder("="): k for k, v in _DTYPES.items()}
    a = np.ascontiguousarray(arr)
    code = inv[a.dtype.newbyteorder("=")]
    head = bytes([0, 0, code, a.ndim]) + np.asarray(a.shape, dtype=">u4").tobytes()
    body = a.astype(np.dtype(_DTYPES[code])).tobytes()
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "wb") as f:
        f.write(head + body)


def _find(raw_dir: str, stem: str) -> str | None:
    for name in (stem, stem + ".gz"):
        p = os.path.join(raw_dir, name)
        if os.path.exists(p):
            return p
    return None


def find_dataset(root: str, name: str = "FashionMNIST") -> str | None:
    """Directory holding the four IDX files, trying torchvision's
    ``<root>/<name>/raw`` layout, then ``<root>/<name>``, then ``<root>``."""
    for d in (os.path.join(root, name, "raw"), os.path.join(root, name), root):
        if all(_find(d, s) for pair in _FILES.values() for s in pair):
            return d
    return None


def load_split(raw_dir: str, train: bool):
    """(images uint8 [N,28,28], labels int64 [N]) of one split."""
    img_stem, lbl_stem = _FILES[train]
    x = read_idx(_find(raw_dir, img_stem))
    y = read_idx(_find(raw_dir, lbl_stem)).astype(np.int64)
    if x.ndim != 3 or y.ndim != 1 or x.shape[0] != y.shape[0]:
        raise ValueError(f"{raw_dir}: inconsistent split shapes {x.shape} / {y.shape}")
    return x, y
