"""Tracing helpers: roctx ranges (visible in rocprofv3 --marker-trace / system traces) and
device-event timers.  Both are no-ops when the native module or a GPU is unavailable."""
from __future__ import annotations

import contextlib
import time

import torch


@contextlib.contextmanager
def roctx_range(name: str, enabled: bool = True):
    C = None
    if enabled and torch.cuda.is_available():
        try:
            from ..ops import native
            C = native.load(build_if_missing=False)
        except Exception:
            C = None
    if C is not None:
        C.roctx_push(name)
    try:
        yield
    finally:
        if C is not None:
            C.roctx_pop()


class Timer:
    """Wall-clock timer that synchronises the GPU at both ends when one is in use."""

    def __init__(self, sync: bool = True):
        self.sync = sync and torch.cuda.is_available()
        self.t0 = 0.0
        self.elapsed = 0.0

    def __enter__(self):
        if self.sync:
            torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.sync:
            torch.cuda.synchronize()
        self.elapsed = time.perf_counter() - self.t0
        return False
