"""IDX file format reader/writer (the on-disk MNIST format), no torchvision.

The reference loads MNIST through ``torchvision.datasets.MNIST('./data', ...)``
(``mnist_ddp.py:157-160``, ``mnist.py:116-119``), which reads the raw IDX files
under ``./data/MNIST/raw``.  IDX layout: big-endian int32 magic
(``0x00000803`` = uint8 images, ``0x00000801`` = uint8 labels), then one
big-endian int32 per dimension, then the row-major uint8 payload.  Gzipped
files (``.gz``) are read transparently.
"""
from __future__ import annotations

import gzip
import os
import struct

import numpy as np

IDX_UBYTE = 0x08
_DTYPES = {0x08: np.uint8, 0x09: np.int8, 0x0B: np.dtype(">i2"), 0x0C: np.dtype(">i4"),
           0x0D: np.dtype(">f4"), 0x0E: np.dtype(">f8")}


def _open(path: str):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx(path: str) -> np.ndarray:
    """Read an IDX file (optionally gzipped) into a numpy array."""
    with _open(path) as f:
        data = f.read()
    if len(data) < 4:
        raise ValueError(f"{path}: truncated IDX header")
    zero, dtype_code, ndim = struct.unpack(">HBB", data[:4])
    if zero != 0 or dtype_code not in _DTYPES:
        raise ValueError(f"{path}: bad IDX magic {data[:4]!r}")
    dims = struct.unpack(">" + "i" * ndim, data[4:4 + 4 * ndim])
    dt = np.dtype(_DTYPES[dtype_code])
    count = int(np.prod(dims)) if dims else 1
    off = 4 + 4 * ndim
    if len(data) - off < count * dt.itemsize:
        raise ValueError(f"{path}: payload shorter than header dims {dims}")
    arr = np.frombuffer(data, dtype=dt, count=count, offset=off).reshape(dims)
    return arr.astype(dt.newbyteorder("=")) if dt.byteorder == ">" else arr.copy()


def write_idx(path: str, arr: np.ndarray) -> None:
    """Write a uint8 array as an IDX file (``.gz`` suffix -> gzipped)."""
    arr = np.ascontiguousarray(arr)
    if arr.dtype != np.uint8:
        raise TypeError("write_idx only writes uint8 payloads")
    header = struct.pack(">HBB", 0, IDX_UBYTE, arr.ndim) + struct.pack(">" + "i" * arr.ndim, *arr.shape)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with (gzip.open(path, "wb") if path.endswith(".gz") else open(path, "wb")) as f:
        f.write(header)
        f.write(arr.tobytes())


MNIST_FILES = {
    True: ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
    False: ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte"),
}


def find_mnist_file(root: str, stem: str) -> str | None:
    """Locate ``<root>/MNIST/raw/<stem>[.gz]`` (torchvision's layout)."""
    for d in (os.path.join(root, "MNIST", "raw"), root):
        for suffix in ("", ".gz"):
            p = os.path.join(d, stem + suffix)
            if os.path.isfile(p):
                return p
    return None


def load_mnist_idx(root: str, train: bool):
    """Return (images uint8 [N,28,28], labels int64 [N]) or None if absent."""
    img_stem, lbl_stem = MNIST_FILES[train]
    ip, lp = find_mnist_file(root, img_stem), find_mnist_file(root, lbl_stem)
    if ip is None or lp is None:
        return None
    images, labels = read_idx(ip), read_idx(lp)
    if images.ndim != 3 or labels.ndim != 1 or images.shape[0] != labels.shape[0]:
        raise ValueError(f"inconsistent MNIST IDX files: {images.shape} vs {labels.shape}")
    return images.astype(np.uint8, copy=False), labels.astype(np.int64)
