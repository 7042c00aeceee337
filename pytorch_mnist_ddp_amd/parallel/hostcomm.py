"""Host-side collectives over the c10d TCPStore (the one ``env://`` already created).

The framework's startup verdicts - "did every rank's xGMI self-test pass", "which transport is
faster (max over ranks)", "are the parameters bitwise equal on every rank", barriers around the
IPC buffer hand-offs - are a few bytes each.  Running them as torch collectives on the default
process group would make ProcessGroupNCCL create its NCCL communicator (a second RCCL communicator
per rank next to the framework's own, ~0.1-0.5 s of bootstrap inside the reference's timer,
mnist_ddp.py:200-203) just to move those bytes.  Here each collective is one ``set`` of this
rank's value and one ``wait`` + ``multi_get`` of every rank's, keyed by a per-process sequence
number (every rank issues the same collectives in the same order, as with any process group).

Keys are garbage-collected two operations later: a rank that starts operation k has seen every
rank's key of operation k-1, so every rank has finished reading operation k-2's keys.

A rank that fails calls :meth:`HostComm.abort`; every rank waiting in a collective sees the abort
key within a second and raises with the failing rank's message (instead of waiting out the timeout).
"""
from __future__ import annotations

import os
import struct
import threading
import time
from datetime import timedelta

import torch.distributed as dist

_PREFIX = "pytorch_mnist_ddp_amd/hc"
DEFAULT_TIMEOUT_S = float(os.environ.get("MNIST_AMD_HOST_TIMEOUT", "300"))


class HostComm:
    def __init__(self, store, rank: int, world: int, prefix: str = _PREFIX):
        self.store, self.rank, self.world, self.prefix = store, int(rank), int(world), prefix
        self.seq = 0

    # ------------------------------------------------------------------ primitives
    def _key(self, seq: int, rank: int) -> str:
        return f"{self.prefix}/{seq}/{rank}"

    def abort(self, msg: str) -> None:
        """Tell every rank's pending and future collectives that this job failed (``msg``) - on
        every channel (one abort key for all prefixes)."""
        if self.world > 1:
            self.store.set(f"{_PREFIX}/abort", str(msg).encode())

    def _wait(self, keys: list[str], timeout_s: float) -> None:
        deadline = time.monotonic() + timeout_s
        abort_key = f"{_PREFIX}/abort"
        while True:
            try:
                self.store.wait(keys, timedelta(seconds=min(1.0, max(0.05, deadline - time.monotonic()))))
                return
            except RuntimeError:
                if self.store.check([abort_key]):
                    raise RuntimeError("job aborted by a peer: " + bytes(self.store.get(abort_key)).decode(
                        "utf-8", "replace")) from None
                if time.monotonic() > deadline:
                    raise RuntimeError(f"host collective timed out after {timeout_s:.0f} s "
                                       f"(ranks missing: {[k for k in keys if not self.store.check([k])]})") from None

    def all_gather_bytes(self, data: bytes, timeout_s: float | None = None) -> list[bytes]:
        """Every rank's ``data`` in rank order."""
        if self.world == 1:
            return [bytes(data)]
        seq = self.seq
        self.seq += 1
        if seq >= 2:
            try:
                self.store.delete_key(self._key(seq - 2, self.rank))
            except Exception:  # noqa: BLE001 - best-effort cleanup
                pass
        self.store.set(self._key(seq, self.rank), bytes(data))
        keys = [self._key(seq, q) for q in range(self.world)]
        self._wait(keys, timeout_s or DEFAULT_TIMEOUT_S)
        if hasattr(self.store, "multi_get"):
            vals = self.store.multi_get(keys)
        else:
            vals = [self.store.get(k) for k in keys]
        return [bytes(v) for v in vals]

    # ------------------------------------------------------------------ collectives
    def barrier(self, timeout_s: float | None = None) -> None:
        self.all_gather_bytes(b".", timeout_s)

    def all_ok(self, flag: bool) -> bool:
        return all(v == b"1" for v in self.all_gather_bytes(b"1" if flag else b"0"))

    def max(self, v: float) -> float:
        return max(struct.unpack("<d", b)[0] for b in self.all_gather_bytes(struct.pack("<d", float(v))))

    def gather_strings(self, msg: str) -> list[str]:
        return [b.decode("utf-8", "replace") for b in self.all_gather_bytes(str(msg).encode())]

    def all_equal(self, data: bytes) -> bool:
        vals = self.all_gather_bytes(data)
        return all(v == vals[0] for v in vals)


class _World1(HostComm):
    def __init__(self):
        super().__init__(None, 0, 1)


_default: HostComm | None = None
_default_pg = None
_tls = threading.local()


_channels: dict[str, int] = {}


def channel(name: str, store=None) -> HostComm:
    """A separate sequence of host collectives (own key prefix) for a helper thread whose collectives
    run concurrently with the main thread's: every rank issues each channel's collectives in the same
    order, but the interleaving ACROSS channels differs between ranks, so the two must never share
    one sequence counter.  Every channel of one name gets a fresh prefix (``name/k``: k-th channel of
    that name in this process, the same on every rank), so a later channel never reads an earlier
    one's leftover keys.  ``store``: the channel's own client (see :func:`own_store_client`), else
    the default store."""
    if store is None:
        store = dist.distributed_c10d._get_default_store()
    k = _channels.get(name, 0)
    _channels[name] = k + 1
    return HostComm(store, dist.get_rank(), dist.get_world_size(), prefix=f"{_PREFIX}/{name}/{k}")


def own_store_client():
    """A second client connection to the rendezvous store for a helper thread: ``clone()`` of the
    default store opens a new socket to the same server under the SAME key prefixes (torchelastic's
    ``/worker/attempt_N`` etc.), so a helper's keys and the abort key are in the namespace every other
    channel uses.  One client serialises its calls on one socket, so a helper's blocking waits on the
    default client stall the main thread's collectives (measured: the DDP wrap's one shape check took
    1.1 s behind the xGMI setup thread's record exchange).  None when the store cannot be cloned:
    callers then share the default client (same namespace either way, so ranks that differ here still
    meet)."""
    try:
        return dist.distributed_c10d._get_default_store().clone()
    except Exception:  # noqa: BLE001 - fall back to the shared client
        return None


class use_channel:
    """``with use_channel(hc):`` - this thread's get_hostcomm() returns ``hc``."""

    def __init__(self, hc: HostComm):
        self.hc = hc

    def __enter__(self):
        self.prev = getattr(_tls, "hc", None)
        _tls.hc = self.hc
        return self.hc

    def __exit__(self, *exc):
        _tls.hc = self.prev


def get_hostcomm(world: int | None = None) -> HostComm:
    """The process's host collectives over the default process group's store (world 1 when no
    process group is initialised, or when the caller's job is a world of 1 - e.g. a single-rank
    reference run inside a multi-rank tool's process group); a thread inside ``use_channel`` gets
    its channel."""
    global _default, _default_pg
    if world == 1 or not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return _World1()
    hc = getattr(_tls, "hc", None)
    if hc is not None:
        return hc
    pg = dist.distributed_c10d._get_default_group()
    if _default is None or _default_pg is not pg:
        store = dist.distributed_c10d._get_default_store()
        _default, _default_pg = HostComm(store, dist.get_rank(), dist.get_world_size()), pg
    return _default


def reset_hostcomm() -> None:
    """Forget the cached instance (after destroy_process_group: a new group has a new store)."""
    global _default, _default_pg
    _default, _default_pg = None, None
