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


class PhaseTimes:
    """Host wall-clock seconds per named setup phase (accumulated; insertion ordered), e.g. the
    startup work that lands inside the reference's ``Total cost time`` (mnist_ddp.py:200-203):
    process group, communicators, xGMI map + self-test, all-reduce probe, validation, capture."""

    def __init__(self, origin: float | None = None):
        self.s: dict[str, float] = {}
        self.info: dict = {}   # seconds spent off the critical path (helper threads; sub-step dicts)
        # wall-clock marks in seconds since `origin` (time.time() of the reference timer's start):
        # where the non-phase time goes (epochs, evaluation, teardown)
        self.origin = time.time() if origin is None else origin
        self.marks: dict[str, float] = {}

    def mark(self, name: str) -> None:
        self.marks[name] = round(time.time() - self.origin, 4)

    @contextlib.contextmanager
    def phase(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.add(name, time.perf_counter() - t0)

    def add(self, name: str, seconds: float) -> None:
        self.s[name] = self.s.get(name, 0.0) + seconds

    def add_info(self, name: str, seconds) -> None:
        """seconds: a number, or a dict of sub-step seconds (kept as is)"""
        if isinstance(seconds, dict):
            self.info[name] = dict(seconds)
        elif seconds is not None:
            self.info[name] = round(float(seconds), 4)

    def update(self, other: "PhaseTimes | dict", prefix: str = "") -> None:
        for k, v in (other.s if isinstance(other, PhaseTimes) else other).items():
            self.add(prefix + k, v)
        if isinstance(other, PhaseTimes):
            self.info.update({prefix + k: v for k, v in other.info.items()})

    def rounded(self, nd: int = 4) -> dict[str, float]:
        return {k: round(v, nd) for k, v in self.s.items()}

    def total(self) -> float:
        return sum(self.s.values())
