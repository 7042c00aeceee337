"""Loader for the in-tree native extension ``pytorch_mnist_ddp_amd._C`` (hipcc, gfx950).

There is deliberately no silent fallback: on a machine with a GPU the GPU path *is* the
hand-written HIP kernels, so a missing/unbuildable extension raises.  ``torch`` is imported
first so the extension binds to the HIP runtime and RCCL that torch already loaded.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the extension: one libamdhip64 / librccl per process)

_C = None
_err: Exception | None = None


def load(build_if_missing: bool = True):
    """Import (building first if needed) and return the native module."""
    global _C, _err
    if _C is not None:
        return _C
    try:
        _C = importlib.import_module("pytorch_mnist_ddp_amd._C")
        return _C
    except ImportError as e:  # not built yet
        _err = e
    if build_if_missing and os.environ.get("MNIST_AMD_NO_BUILD") != "1":
        from .. import _build
        _build.build()
        _C = importlib.import_module("pytorch_mnist_ddp_amd._C")
        return _C
    raise RuntimeError(f"native extension pytorch_mnist_ddp_amd._C is not available: {_err}")


def available() -> bool:
    try:
        load(build_if_missing=False)
        return True
    except Exception:
        return False


def stream_handle(stream: "torch.cuda.Stream | None" = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else int(t.data_ptr())
