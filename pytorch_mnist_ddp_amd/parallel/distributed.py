"""Process-group bootstrap: reference ``init_distributed_mode`` (mnist_ddp.py:13-37) + the
framework's communicators.

Rank discovery order and printed lines are the reference's:
  (a) ``RANK`` and ``WORLD_SIZE`` in the environment (torchrun / torch.distributed.launch)
      -> rank, world_size, gpu = ``LOCAL_RANK``;
  (b) ``SLURM_PROCID`` -> rank, gpu = rank % device_count, world_size from ``--world-size``;
  (c) an ``args.rank`` attribute set by the caller (unreachable from the reference CLI);
  (d) otherwise "Not using distributed mode".
Then ``set_device(gpu)``, print ``| distributed init (rank r): url, local rank:g, world size:w``
and ``init_process_group``.  The backend is ``"nccl"`` (= RCCL on ROCm) on GPU and ``"gloo"``
for ``--no-cuda`` runs (the reference hardcodes nccl, which cannot work without a GPU).

The process group is created lazily (no ``device_id``): ProcessGroupNCCL builds its RCCL
communicator only on its first collective, and the fused engine never issues one - its gradient
all-reduce runs on the framework's own RCCL communicator (:func:`create_rccl_comm`, uid through the
c10d TCPStore) or on the direct xGMI kernels (:func:`create_xgmi_comm`), and its startup verdicts
are host collectives over the same store (``hostcomm``).  So each rank initialises ONE RCCL
communicator (or none with ``--allreduce xgmi``), and that one is created on a helper thread while
the main thread builds data, model and trainer (:func:`start_rccl_comm`).
"""
from __future__ import annotations

import os
import threading
import time
from datetime import timedelta

import torch
import torch.distributed as dist

from .hostcomm import get_hostcomm


def init_distributed_mode(args) -> None:
    # no runtime call on the main thread (driver.gpu_present: is_available() / device_count() cost
    # ~60 / ~53 ms inside the reference timer)
    from ..driver import gpu_present
    use_cuda = not getattr(args, "no_cuda", False) and gpu_present()
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        args.rank = int(os.environ["RANK"])
        args.world_size = int(os.environ["WORLD_SIZE"])
        args.gpu = int(os.environ.get("LOCAL_RANK", "0"))
    elif "SLURM_PROCID" in os.environ:
        args.rank = int(os.environ["SLURM_PROCID"])
        ndev = torch.cuda.device_count() if use_cuda else 1     # (SLURM launch only)
        args.gpu = args.rank % max(1, ndev)
    elif hasattr(args, "rank"):
        pass
    else:
        print("Not using distributed mode")
        args.distributed = False
        return

    args.distributed = True
    if use_cuda and os.environ.get("MNIST_AMD_ONE_GPU", "0") == "1":
        args.gpu = 0        # rehearsal knob: every rank on GPU 0 (needs --dist-backend gloo --allreduce xgmi)
    if use_cuda:
        # the fused driver selects the device after its HIP prewarm thread has initialised the
        # runtime (args._defer_set_device): the process group itself is lazy and touches no device
        if not getattr(args, "_defer_set_device", False):
            torch.cuda.set_device(args.gpu)
        args.dist_backend = getattr(args, "pg_backend", None) or "nccl"
    else:
        args.dist_backend = "gloo"
    from ..utils.logging import print_line
    print_line(f"| distributed init (rank {args.rank}): {args.dist_url}, local rank:{args.gpu}, "
               f"world size:{args.world_size}")
    dist.init_process_group(backend=args.dist_backend, init_method=args.dist_url, world_size=args.world_size,
                            rank=args.rank, timeout=timedelta(minutes=10))


_UID_KEY = "pytorch_mnist_ddp_amd/rccl_unique_id"
_rccl_seq = 0          # communicators created so far (same order on every rank -> unique store keys)
# ncclCommInitRank's own limit (a peer that never arrives): the communicator is aborted after it
RCCL_INIT_TIMEOUT_S = float(os.environ.get("MNIST_AMD_RCCL_INIT_TIMEOUT", "300"))


def _fault_delay(kind: str, rank: int) -> float:
    """Seconds to hold rank ``rank`` back at fault point ``kind`` (``MNIST_AMD_FAULT=kind:rank:seconds``,
    tests only); 0 when not injected."""
    parts = os.environ.get("MNIST_AMD_FAULT", "").split(":")
    if len(parts) == 3 and parts[0] == kind and int(parts[1]) == rank:
        return float(parts[2])
    return 0.0


def _uid(world_size: int, rank: int, tag: str, store=None, cancelled=None):
    """The communicator's ncclUniqueId: made by rank 0, passed through the store (``store``: the
    caller's client, else the default one).  ``cancelled()`` is polled while waiting (None = never)."""
    from ..ops import native
    C = native.load()
    if store is None:
        store = dist.distributed_c10d._get_default_store()
    key = f"{_UID_KEY}/{tag}"
    if rank == 0:
        uid = C.RcclComm.unique_id()
        store.set(key, uid)
        return uid
    deadline = time.monotonic() + RCCL_INIT_TIMEOUT_S
    while True:
        try:
            store.wait([key], timedelta(seconds=0.25))
            return store.get(key)
        except RuntimeError:
            if cancelled is not None and cancelled():
                raise _Cancelled() from None
            if time.monotonic() > deadline:
                raise RuntimeError(f"rank 0's ncclUniqueId did not arrive within {RCCL_INIT_TIMEOUT_S:.0f} s") from None


class _Cancelled(Exception):
    pass


def create_rccl_comm(world_size: int, rank: int, device: int, tag: str | None = None):
    """Framework-owned RCCL communicator (requires an initialised default process group)."""
    from ..ops import native
    global _rccl_seq
    C = native.load()
    if not C.RcclComm.available():
        raise RuntimeError("RCCL not found in this process")
    if tag is None:
        tag = str(_rccl_seq)
    _rccl_seq += 1
    uid = _uid(world_size, rank, tag)
    return C.RcclComm(bytes(uid), world_size, rank, device, RCCL_INIT_TIMEOUT_S)


class PendingRcclComm:
    """The framework's RCCL communicator, initialised off the critical path: a helper thread fetches the
    ncclUniqueId (its own store client) and starts a NON-BLOCKING ``ncclCommInitRankConfig`` (the
    bootstrap - socket rendezvous, topology detection, channel setup - runs in RCCL's own thread),
    then polls it.  Nothing waits for it unless RCCL is actually needed:

    * ``result(timeout_s)`` joins and returns the communicator, or raises its init error (an init that
      fails - e.g. two ranks on one GPU - or exceeds ``RCCL_INIT_TIMEOUT_S`` is aborted first);
    * ``cancel()`` returns at once: the helper aborts the (pending or finished) communicator and exits
      (``--allreduce auto`` once the xGMI transport has validated on every rank: a collective verdict,
      so every rank cancels, and no rank's bootstrap is left waiting for a peer);
    * ``start=False`` defers even the start (``start()``): RCCL is then touched only if the caller asks.

    ``seconds`` is the helper's time; ``status`` one of "not started", "initialising", "ready",
    "failed: ...", "cancelled".  Fault injection (tests): ``MNIST_AMD_FAULT=rccl_init_delay:R:S`` holds
    rank R's helper S seconds before its init (cancel-aware)."""

    def __init__(self, world_size: int, rank: int, device: int, start: bool = True):
        global _rccl_seq
        self._tag = str(_rccl_seq)          # claimed now: the store keys follow the callers' order
        _rccl_seq += 1
        self._args = (world_size, rank, device)
        self._comm, self._err, self.seconds = None, None, None
        self._cancel = threading.Event()
        self._t = None
        self._taken = False                 # result() handed the communicator out: cancel() leaves it
        self.status = "not started"
        if start:
            self.start()

    @property
    def started(self) -> bool:
        return self._t is not None

    def start(self) -> "PendingRcclComm":
        if self._t is None:
            from .hostcomm import own_store_client
            self._store = own_store_client()             # its own socket (None: share the default)
            self.status = "initialising"
            self._t = threading.Thread(target=self._run, name="rccl-init", daemon=True)
            self._t.start()
        return self

    def _run(self):
        from ..ops import native
        t0 = time.perf_counter()
        world, rank, device = self._args
        comm = None
        try:
            if self._cancel.wait(_fault_delay("rccl_init_delay", rank)):
                raise _Cancelled()
            C = native.load()
            if not C.RcclComm.available():
                raise RuntimeError("RCCL not found in this process")
            torch.cuda.set_device(device)
            uid = _uid(world, rank, self._tag, self._store, self._cancel.is_set)
            comm = C.RcclComm(bytes(uid), world, rank, device, RCCL_INIT_TIMEOUT_S, False)
            deadline = time.monotonic() + RCCL_INIT_TIMEOUT_S
            while True:
                st = comm.init_status()
                if st == 0:
                    break
                if st != 7:                 # ncclInProgress
                    raise RuntimeError(f"ncclCommInitRankConfig failed: {C.RcclComm.error_string(st)}")
                if self._cancel.wait(0.002):
                    raise _Cancelled()
                if time.monotonic() > deadline:
                    raise RuntimeError(f"ncclCommInitRankConfig did not complete within {RCCL_INIT_TIMEOUT_S:.0f} s")
            if self._cancel.is_set():
                raise _Cancelled()
            self._comm, self.status = comm, "ready"
        except _Cancelled:
            if comm is not None:
                comm.abort()
            self._err, self.status = RuntimeError("RCCL communicator init cancelled"), "cancelled"
        except BaseException as e:  # noqa: BLE001 - re-raised in result()
            if comm is not None:
                comm.abort()
            self._err, self.status = e, f"failed: {e}"
        self.seconds = time.perf_counter() - t0

    def result(self, timeout_s: float = RCCL_INIT_TIMEOUT_S + 30.0):
        self.start()
        self._t.join(timeout_s)
        if self._t.is_alive():
            self.cancel()
            raise RuntimeError(f"RCCL communicator init did not finish within {timeout_s:.0f} s (cancelled)")
        if self._err is not None:
            raise self._err
        self._taken = True
        return self._comm

    def cancel(self) -> None:
        """Drop the communicator unless ``result()`` handed it out (non-blocking: the helper thread
        aborts a pending init; a finished, unused one is aborted here)."""
        if self._taken:
            return
        self._cancel.set()
        c, self._comm = self._comm, None
        if c is not None:
            c.abort()
            self.status = "cancelled"

    def close(self, timeout_s: float = 10.0) -> None:
        """Cancel and wait (bounded) for the helper thread: call after training, outside any timer."""
        self.cancel()
        if self._t is not None:
            self._t.join(timeout_s)


def start_rccl_comm(world_size: int, rank: int, device: int, start: bool = True) -> PendingRcclComm:
    return PendingRcclComm(world_size, rank, device, start=start)


def get_rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def barrier(world: int | None = None) -> None:
    """Host barrier of the default group's ranks (TCPStore; never creates a device communicator)."""
    get_hostcomm(world).barrier()


# stage-wait timeout of the startup self-test / schedule validation: long enough that a peer delayed
# by the GPU's queue scheduling (many processes on one GPU in rehearsals) is not mistaken for a hang
STARTUP_TIMEOUT_S = float(os.environ.get("MNIST_AMD_STARTUP_TIMEOUT", "15"))
RUN_TIMEOUT_S = 60.0   # stage-wait timeout while training (covers rank 0's evaluation, host stalls)
_xgmi_seq = 0          # communicators created so far (same order on every rank -> unique store keys)


def _all_ok(flag: bool, device=None, world: int | None = None) -> bool:
    """Every rank's verdict (host collective)."""
    return get_hostcomm(world).all_ok(flag)


def _max_over_ranks(v: float, device=None, world: int | None = None) -> float:
    return get_hostcomm(world).max(v)


def params_fingerprint_equal(t: torch.Tensor, device=None, world: int | None = None) -> bool:
    """True when every rank's fp32 tensor ``t`` is bitwise identical (fingerprints compared on the host)."""
    hc = get_hostcomm(world)
    if hc.world == 1:
        return True
    from .ddp import params_fingerprint_host
    return hc.all_equal(params_fingerprint_host([t]))


def gather_strings(msg: str, world: int | None = None) -> list[str]:
    """Every rank's ``msg`` in rank order (host collective)."""
    return get_hostcomm(world).gather_strings(msg)


def broadcast_(t: torch.Tensor, src: int = 0) -> None:
    """In-place broadcast of a (device) tensor over the default process group; GPU tensors are
    staged through the host when the backend is gloo."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    if t.is_cuda and dist.get_backend() != "nccl":
        host = t.cpu()
        dist.broadcast(host, src=src)
        t.copy_(host)
    else:
        dist.broadcast(t, src=src)


def xgmi_broadcast_(x, t: torch.Tensor, src: int = 0) -> None:
    """``t`` (fp32, on this rank's GPU, at most the communicator's size) from rank ``src`` to every
    rank through the xGMI communicator's IPC-mapped output buffers: ``src`` stages it, every other
    rank copies it out of ``src``'s buffer over xGMI (DDP construction without any RCCL)."""
    from ..ops import native
    hc = get_hostcomm(x.world_size)
    if hc.world == 1:
        return
    n = t.numel()
    s = torch.cuda.current_stream(t.device)
    if hc.rank == src:
        x.stage_out(native.ptr(t), n, s.cuda_stream)
    s.synchronize()
    hc.barrier()
    if hc.rank != src:
        x.read_peer_out(src, native.ptr(t), n, s.cuda_stream)
    s.synchronize()
    hc.barrier()                 # every copy out of src's buffer is done before anyone reuses it
    g = x.grad_out
    native.load().memset_sync(g.data_ptr(), 0, g.numel() * g.element_size())   # (no torch fill kernel)
    s.synchronize()


def _device_identity(device) -> str:
    from ..ops import native
    return native.load().device_identity(torch.device(device).index or 0)


def _node_identity() -> str:
    """This host (hostname + kernel boot id): ranks whose identities differ cannot share IPC memory."""
    import socket
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return f"{socket.gethostname()}/{boot}"


def device_topology(device, world: int | None = None) -> tuple[int, int]:
    """(largest number of ranks of the default process group that drive one physical GPU, number of
    nodes): one host collective.  Ranks per GPU is 1 in the production layout and > 1 in the one-GPU
    multi-process rehearsal; the xGMI kernels wait per workgroup on their peers, so the residency
    planner (``xgmi_plan_grids``) sizes their grids for that many ranks' spinning workgroups on one
    GPU.  The direct xGMI transport needs one node (IPC-mapped peer memory)."""
    hc = get_hostcomm(world)
    if hc.world == 1:
        return 1, 1
    ids = [s.split("|", 1) for s in hc.gather_strings(_node_identity() + "|" + _device_identity(device))]
    devs = [d for _, d in ids]
    return max(devs.count(d) for d in devs), len({n for n, _ in ids})


def ranks_per_device(device, world: int | None = None) -> int:
    """Largest number of ranks of the default process group that drive one physical GPU."""
    return device_topology(device, world)[0]


def ranks_share_a_device(device) -> bool:
    """True when two ranks of the default process group drive the same physical GPU."""
    return ranks_per_device(device) > 1


def create_xgmi_comm(world_size: int, rank: int, device, numel: int, tag: str | None = None, channels: int = 3,
                     verify: bool = True, oneshot_max: int = 32768, co_ranks: int | None = None,
                     timings: dict | None = None):
    """Direct xGMI all-reduce communicator over ``numel`` floats (csrc/runtime/xgmi_comm.h).

    The communicator owns its input / output buffers (``x.grad_in`` / ``x.grad_out``: zero-copy fp32
    torch views through DLPack).  Every rank exports IPC handles of those buffers and its flag blocks
    through the c10d store and maps every peer's.  With ``verify`` each channel is then exercised on a
    rank-dependent pattern whose sum is exact in fp32 (STARTUP_TIMEOUT_S stage timeout), and the ranks
    agree on the outcome.  Returns the communicator, or ``None`` on every rank when any rank failed
    to map its peers or to verify (callers then keep the RCCL all-reduce).  ``co_ranks`` (default:
    measured with :func:`ranks_per_device`) sizes the kernel grids so every rank's spinning
    workgroups are resident.  ``timings`` (optional dict) receives host seconds per sub-step
    (co_ranks, alloc, exchange, connect, verify): the N > 1 startup budget.  The records travel as a
    host collective (the calling thread's channel, see ``hostcomm.use_channel``)."""
    from torch.utils.dlpack import from_dlpack

    from ..ops import native
    global _xgmi_seq
    C = native.load()
    if tag is None:
        tag = str(_xgmi_seq)
    _xgmi_seq += 1
    dev = torch.device(device)
    tm = timings if timings is not None else {}
    t = time.perf_counter()

    def lap(name):
        nonlocal t
        now = time.perf_counter()
        tm[name] = round(tm.get(name, 0.0) + now - t, 4)
        t = now

    if co_ranks is None:
        co_ranks, nodes = device_topology(dev, world_size)
        if nodes > 1:                 # (every rank saw the same gather: all return None together)
            if rank == 0:
                print(f"[xgmi] {nodes} nodes: no direct xGMI transport across nodes", flush=True)
            tm["multi_node"] = nodes
            return None
    lap("co_ranks")
    x = None
    try:
        x = C.XgmiComm(world_size, rank, dev.index or 0, int(numel), channels, oneshot_max, co_ranks)
        x.grad_in = from_dlpack(x.dlpack("in"))
        x.grad_out = from_dlpack(x.dlpack("out"))
        lap("alloc")
        if world_size > 1:
            # (a host collective: a peer's abort ends the wait at once instead of after its timeout)
            recs = get_hostcomm(world_size).all_gather_bytes(x.record())
            lap("exchange")
            x.connect(recs)
            lap("connect")
        ok = True
    except RuntimeError as e:
        print(f"[xgmi] rank {rank}: setup failed ({e})", flush=True)
        ok = False
    if not _all_ok(ok, world=world_size):
        release_xgmi_comm(x, world_size)
        return None
    lap("agree")
    if verify:
        ok = _verify_xgmi(x, world_size, rank, x.grad_in, x.grad_out, channels)
        lap("verify")
        if not _all_ok(ok, world=world_size):
            if rank == 0:
                print("[xgmi] self-test failed: keeping the RCCL all-reduce", flush=True)
            release_xgmi_comm(x, world_size)
            return None
    return x


class PendingXgmiComm:
    """:func:`create_xgmi_comm` on a helper thread (its own host-collective channel), started as soon
    as the HIP runtime is up: the buffer allocation, IPC export / exchange / peer mapping and the
    self-test overlap the model build, the DDP wrap and the trainer's buffers on the main thread
    (the N > 1 startup inside the reference timer).  ``result()`` joins and returns
    the communicator (or None when it could not be built / verified, as create_xgmi_comm);
    ``seconds`` / ``timings`` are the helper's."""

    def __init__(self, world_size: int, rank: int, device, numel: int):
        from .hostcomm import channel, own_store_client
        self._store = own_store_client()                 # its own socket (None: share the default)
        self._hc = channel("xgmi_setup", self._store)
        self._args = (world_size, rank, torch.device(device), int(numel))
        self._comm, self._err, self.seconds, self.timings = None, None, None, {}
        self._t = threading.Thread(target=self._run, name="xgmi-setup", daemon=True)
        self._t.start()

    def _run(self):
        from .hostcomm import use_channel
        t0 = time.perf_counter()
        try:
            world, rank, dev, numel = self._args
            torch.cuda.set_device(dev)
            with use_channel(self._hc):
                self._comm = create_xgmi_comm(world, rank, dev, numel, timings=self.timings)
        except BaseException as e:  # noqa: BLE001 - re-raised in result()
            import traceback
            self._err = e
            self._tb = traceback.format_exc()
        self.seconds = time.perf_counter() - t0

    def result(self, timeout_s: float = 600.0):
        self._t.join(timeout_s)
        if self._t.is_alive():
            raise RuntimeError(f"xGMI communicator setup did not finish within {timeout_s:.0f} s")
        if self._err is not None:
            import sys
            print(f"[xgmi] rank {self._args[1]}: setup thread failed:\n{self._tb}", file=sys.stderr, flush=True)
            raise self._err
        return self._comm


def release_xgmi_comm(x, world: int | None = None) -> None:
    """Collective teardown of an xGMI communicator: every rank unmaps its peers, then (host barrier)
    the buffers may be recycled by a later communicator of the same shape.  Call on every rank;
    ``x`` may be None on some (a failed setup), the barrier still matches."""
    if x is not None:
        x.close_peers()
        world = x.world_size
    get_hostcomm(world).barrier()
    if x is not None:
        x.mark_recyclable()


def _verify_xgmi(x, world: int, rank: int, grad_in: torch.Tensor, grad_out: torch.Tensor, channels: int) -> bool:
    n = grad_in.numel()
    # channel 0: a small range (one-shot kernel), channel 1: the rest (two-shot when large), channel 2
    # (conv-bucket split): another small range - every channel in flight concurrently
    cut = min((n // 2) & ~3, 16384)
    ranges = [(0, cut), (cut, n - 2 * cut), (n - cut, cut)] if channels >= 3 else \
        [(0, cut), (cut, n - cut)] if channels >= 2 else [(0, n)]
    # pattern, fills and checks on the host (H2D / D2H copies): no torch GPU kernel launches here, whose
    # first-use code-object loads would land inside the reference timer at world > 1
    i = torch.arange(n, dtype=torch.float32)
    base = torch.remainder(i, 97.0) * 0.25 - 3.0         # multiples of 1/4 in [-3, 21]: sums are exact
    nan_h = torch.full((n,), float("nan"), dtype=torch.float32)
    s_main = torch.cuda.current_stream(grad_in.device)
    side = torch.cuda.Stream(device=grad_in.device)
    side2 = torch.cuda.Stream(device=grad_in.device)
    x.set_timeout_seconds(STARTUP_TIMEOUT_S)
    ok = True
    try:
        for it in range(2):                              # repeated calls exercise the per-WG counters
            scale = float(it + 1)
            # every rank must be done READING the previous call's output shards before anyone
            # rewrites its buffers from outside the kernel protocol (the fill below): the kernels only
            # protect their own next call (its stage 0), not host-side writes
            barrier(world)
            with torch.no_grad():
                grad_in.copy_(base * (scale * (rank + 1)))
                grad_out.copy_(nan_h)
            torch.cuda.synchronize(grad_in.device)
            streams = [s_main, side, side2]
            t0 = time.perf_counter()
            for c, (off, cnt) in enumerate(ranges):       # every channel in flight concurrently
                x.allreduce(c, off, cnt, streams[c % 3].cuda_stream)
            torch.cuda.synchronize(grad_in.device)
            dt = time.perf_counter() - t0
            expect = base * (scale * world * (world + 1) / 2)
            code = x.error()
            out = grad_out.cpu()
            if code or not torch.equal(out, expect):
                from ..ops import native
                if code:
                    what = native.load().Engine.describe_xgmi_error(code) + " timed out"
                else:
                    bad = out != expect
                    what = f"{int(bad.sum())} wrong sums"
                    # where and what: per-range/shard counts, NaN (never written) / zero / stale share
                    for c, (off, cnt) in enumerate(ranges):
                        b = bad[off:off + cnt]
                        sh = (cnt // 4 + world - 1) // world * 4
                        per = [int(b[q * sh:(q + 1) * sh].sum()) for q in range(world)]
                        what += f"; ch{c} wrong per shard {per}"
                    g = out[bad]
                    e = expect[bad]
                    what += (f"; nan {int(torch.isnan(g).sum())}, zero {int((g == 0).sum())}, "
                             f"ratio to expected (median) {float((g / e).nanmedian()):.4g}")
                print(f"[xgmi] rank {rank}: self-test call {it} failed after {dt:.2f} s: {what}", flush=True)
                ok = False
                break
    except RuntimeError as e:
        print(f"[xgmi] rank {rank}: self-test error ({e})", flush=True)
        ok = False
    finally:
        x.set_timeout_seconds(RUN_TIMEOUT_S)
        # the last call's peers may still be READING this rank's output shard (all-gather phase): the
        # host-side zeroing below is outside the kernels' hand-off protocol, so every rank first waits
        # until all ranks have finished their last call (seen at W = 8 on one GPU: a fast rank zeroed
        # its output under a slow rank's phase-2 reads -> whole shards of zeros)
        barrier(world)
        from ..ops import native
        C = native.load()
        for t in (grad_in, grad_out):                    # hipMemset (no torch fill kernel)
            C.memset_sync(t.data_ptr(), 0, t.numel() * t.element_size())
        torch.cuda.synchronize(grad_in.device)
    return ok
