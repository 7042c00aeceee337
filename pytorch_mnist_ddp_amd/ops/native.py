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
    if os.environ.get("MNIST_AMD_EXT_PATH"):      # A/B runs: another build of the same sources
        _C = _load_from(os.environ["MNIST_AMD_EXT_PATH"])
        return _C
    if os.environ.get("MNIST_AMD_TIMELINE") == "1":
        _C = _load_variant("tl", build_if_missing)
        return _C
    if os.environ.get("MNIST_AMD_RACE_WIDEN") == "1":
        _C = _load_variant("rw", build_if_missing)
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


def _load_variant(variant: str, build_if_missing: bool):
    """A debug build (``_build.VARIANTS``: "tl" = in-kernel wave timestamps, csrc/include/timeline.h;
    "rw" = race-window widening, csrc/include/device_utils.h), imported under the module name ``_C``
    (its PyInit symbol) so every caller gets it."""
    import sysconfig
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        f"_C_{variant}" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    if not os.path.exists(path):
        if not build_if_missing:
            raise RuntimeError(f"debug build {path} missing (python -m pytorch_mnist_ddp_amd._build "
                               f"{'--timeline' if variant == 'tl' else '--race-widen'})")
        from .. import _build
        _build.build(variant=variant)
    return _load_from(path)


def _load_from(path: str):
    """The extension file ``path`` imported under the module name ``_C`` (its PyInit symbol)."""
    import importlib.util
    import sys
    if not os.path.exists(path):
        raise RuntimeError(f"native extension {path} missing")
    spec = importlib.util.spec_from_file_location("pytorch_mnist_ddp_amd._C", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["pytorch_mnist_ddp_amd._C"] = mod
    return mod


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


def zeros(shape, dtype: torch.dtype, device) -> torch.Tensor:
    """A zero-filled tensor; on the GPU by hipMemset instead of a torch fill kernel, whose code
    object would otherwise load at first launch inside the reference timer (setup-time only:
    synchronous)."""
    t = torch.empty(shape, dtype=dtype, device=device)
    if t.is_cuda:
        load().memset_sync(t.data_ptr(), 0, t.numel() * t.element_size())
    else:
        t.zero_()
    return t


def host_to_device(values, dtype: torch.dtype, device) -> torch.Tensor:
    """A small device tensor from host values by one H2D copy (no device kernel)."""
    return torch.tensor(values, dtype=dtype).to(device)

