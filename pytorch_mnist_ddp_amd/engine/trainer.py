"""FusedTrainer: the reference train()/test() loops (mnist_ddp.py:65-105) on the native engine.

What changes versus the reference loop, and why (MI355X-first):

* the whole split lives in HBM as uint8 (47 MB); per epoch only the sampler's index vector is
  uploaded (one 240 KB H2D), the first kernel of each step gathers + normalises its rows -
  no DataLoader worker, no pinned-memory thread, no per-step H2D copy (reference :68);
* a training step is 7-8 kernels enqueued by C++ (``_C.Engine``) and chunks of ``graph_steps``
  steps are captured once into hipGraphs and replayed; the host only syncs where the reference
  prints (rank 0, every ``log_interval`` batches) and at eval;
* DDP: the fc gradient bucket (98.4 % of bytes) is all-reduced on the comm stream while the conv
  backward runs, then its Adadelta update runs on that stream too; the conv bucket follows.  The
  transport - RCCL or the direct xGMI kernels - is chosen by validating and timing each one's
  production schedule at startup.  Averaging (1/W) is folded into the head's loss gradient;
* evaluation (rank 0 only, SequentialSampler over the test set) is one captured graph per epoch
  with per-row losses / hits reduced once on the host side.

Index order, RNG consumption, log lines and the loss values printed follow the reference.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

import torch

from ..data.datasets import MNISTData
from ..ops import native
from ..utils.profiling import PhaseTimes
from .state import FLAG_NO_DROPOUT, ModelState


# startup validation: timed replays of the chunk per candidate transport; host watchdog of the RCCL
# schedule's replays (its first collectives also set up RCCL's channels and proxies)
# with two candidate transports ("auto" at world > 1) the validation replay is followed by this many
# timed replays (the choice's measure, without first-replay costs); a single candidate is timed on
# its validation replay alone (the startup inside the reference timer: each 50-step replay is ~15 ms
# at world 2 in the one-GPU rehearsal)
VALIDATE_TIMED = 1


def rccl_watchdog_s() -> float:
    """Host watchdog of the RCCL schedule's startup replays (``MNIST_AMD_RCCL_WATCHDOG``, s)."""
    return float(os.environ.get("MNIST_AMD_RCCL_WATCHDOG", "120"))


# after ncclCommAbort, how long the streams may take to drain (the engine's own device-counter holds
# time out after 60 s, so a chunk whose RCCL kernels returned always drains within that)
RCCL_DRAIN_S = 90.0


from ..parallel.distributed import _fault_delay  # noqa: E402  (MNIST_AMD_FAULT=kind:rank:seconds, tests)


@dataclass
class EpochStats:
    epoch: int
    steps: int
    samples: int
    train_seconds: float
    losses: dict = field(default_factory=dict)   # batch_idx -> loss for logged steps
    device_seconds: float | None = None          # HIP-event time of the epoch's training work
    events: tuple | None = None                  # (start, end) HIP events of that work (sync=False)

    def device_time(self) -> float | None:
        """Device seconds of the epoch's training work (waits for its end event when needed)."""
        if self.device_seconds is None and self.events is not None:
            self.events[1].synchronize()
            self.device_seconds = self.events[0].elapsed_time(self.events[1]) / 1000.0
        return self.device_seconds


class EvalHandle:
    """An enqueued evaluation (FusedTrainer.evaluate_async): per-row losses / hits land in pinned
    buffers; ``result()`` waits for them and sums in float64 on the host (fixed order)."""

    def __init__(self, event, rows, hits, n: int):
        self.event, self.rows, self.hits, self.n = event, rows, hits, n
        self._res = None

    def result(self) -> tuple[float, int, int]:
        if self._res is None:
            if self.event is None:
                self._res = (0.0, 0, 0)
            else:
                self.event.synchronize()
                self._res = (float(self.rows.double().sum()), int(self.hits.sum()), self.n)
        return self._res


class TransportHang(RuntimeError):
    """A startup replay of the RCCL schedule did not complete within its host watchdog: a collective
    is stuck on the device (a peer never arrived) and cannot be cancelled - the caller reports and
    exits the process (``fatal``) instead of waiting for the process group's 10-minute timeout."""
    fatal = True


class StartupValidationError(RuntimeError):
    """No candidate transport passed: carries every candidate's report and the trainer's setup
    phases so far (bench.py puts both into its failure JSON)."""

    def __init__(self, msg: str, transport_report: dict, setup: PhaseTimes):
        super().__init__(msg)
        self.transport_report = transport_report
        self.setup = setup


_ENGINE_STREAMS: dict[int, tuple] = {}


_STREAM_KIND: dict[int, str] = {}


def under_profiler() -> bool:
    """The process runs under rocprofv3 (its ``ROCPROF_*`` environment)."""
    return any(k.startswith("ROCPROF") for k in os.environ)


def stream_kind(device: int | None = None) -> str:
    if not _STREAM_KIND:
        return "not created"
    return _STREAM_KIND.get(device, next(iter(_STREAM_KIND.values())))


def make_streams(dev) -> tuple:
    """The trainers' compute and comm streams: one process-wide pair per device of NON-BLOCKING
    streams, created before any other stream of the process (the driver's prewarm thread and bench.py
    call this right after the HIP context exists), so each lands on a hardware queue of its own.

    Why both properties (profiles/r6/queues/, profiles/r6/ab/stream_kind/):
    * hardware queues: the HIP runtime maps streams onto a pool of GPU_MAX_HW_QUEUES queues per
      process (4); a stream created after the pool is used up shares a queue with an older one, and a
      trainer whose streams landed on shared queues ran its device-counter-chained step 4.6x slower
      (63 -> 290 us at B = 200, ``tools/queue_mapping.py``) - round 5's bimodal slow mode.  Two
      streams created first (the legacy default stream being the only older one) get queues of their
      own, and every trainer of the process reuses them;
    * non-blocking: CU-masked streams (``_C.create_stream(dedicated=True)``, which the runtime never
      puts on a shared queue) are BLOCKING streams - they synchronise with the legacy default stream,
      which torch uses for its host reads (``.item()`` of a logged loss) and small fills.  With them
      the reference's 20-epoch run (``mnist_ddp.py``) trained at 72.5-73.2 us/step instead of the
      62.1-62.3 it reaches on non-blocking streams (Total cost time 0.66-0.76 -> 0.59-0.60 s), although
      bench.py's timed window, which touches no default-stream op, read 61.2 with either.
    The pair is probed at once (``_C.probe_streams``: device-counter hand-offs both ways, 0.5 s timeout);
    if the two non-blocking streams share a queue anyway - a process with a smaller queue pool
    (GPU_MAX_HW_QUEUES=2 in the one-GPU multi-rank rehearsals) or streams made before them - the pair
    becomes two CU-masked streams instead: dedicated queues, blocking semantics (``stream_kind``) -
    except under rocprofv3, whose exit-time teardown segfaults in a process with CU-masked streams
    (profiles/r6/final/prof_b200_cumask.log): there the pair stays as it is and the trainer's own
    stream probe picks OVERLAP or SERIAL."""
    dev = torch.device(dev)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    pair = _ENGINE_STREAMS.get(key)
    if pair is None:
        C = native.load()
        raw = [C.create_stream(key, False, 0) for _ in range(2)]
        kind = "non-blocking, created first (own hardware queues)"
        if not C.probe_streams(raw[0], raw[1]) and not under_profiler():
            for r in raw:
                C.destroy_stream(r)
            raw = [C.create_stream(key, True, 0) for _ in range(2)]
            kind = "cu_masked (the non-blocking pair shared a hardware queue)"
        pair = tuple(torch.cuda.ExternalStream(r, device=torch.device("cuda", key)) for r in raw)
        _ENGINE_STREAMS[key] = pair
        _STREAM_KIND[key] = kind
    return pair


class FusedTrainer:
    """``allreduce`` (DDP): "rccl", "xgmi", "auto" (default) or "fastest".  A candidate transport's
    PRODUCTION schedule - the captured chunk graph training replays - is validated on this node before
    training (``transport_report``).  "auto" validates the direct xGMI transport first and keeps it
    without ever waiting for RCCL (``rccl_pending``, a ``PendingRcclComm``, is cancelled, or - deferred -
    never started); RCCL is brought up only when xGMI is unavailable or fails.  "fastest" validates and
    times both and keeps the faster (see ``_setup_ddp``).  ``hooks``: engine variants for A/B runs
    (``HOOKS``).
    ``overlap`` (single GPU): the OVERLAP schedule (optimizer work on the comm stream) when the two
    streams pass the hand-off probe, else SERIAL.  ``xgmi_fuse``: the xGMI kernels apply Adadelta
    themselves (False = separate launches: the fused kernels' bitwise oracle).  ``probe_world1``
    (tests, bench --force-comm): at world 1, make the xGMI transport a candidate under "auto" / "fastest" too.
    ``fp32`` (``--dtype fp32``): the fp32 step of ``f32_net.hip`` (f32-input MFMA GEMMs, fp32
    activations and gradient operands) in the OVERLAP (fc update on the comm stream) or SERIAL schedule,
    RCCL or XGMI at world > 1."""

    def __init__(self, mstate: ModelState, train: MNISTData, test: MNISTData | None, batch_size: int,
                 test_batch_size: int, num_samples: int, world_size: int = 1, rank: int = 0,
                 comm=None, seed: int = 1, graph_steps: int = 10, dropout: bool = True,
                 two_buckets: bool = True, allreduce: str | None = None, overlap: bool = True,
                 xgmi_fuse: bool = True, probe_world1: bool = False, fp32: bool = False, xgmi_pending=None,
                 streams=None, rccl_pending=None, hooks: dict | None = None):
        C = native.load()
        self.C, self.ms = C, mstate
        # host seconds per setup phase (engine, xgmi_comm, stream_probe, validate.<transport>,
        # graph_capture): the N > 1 startup budget inside the reference's timer
        self.setup = PhaseTimes()
        _t_init = time.perf_counter()
        dev = mstate.device
        self.device = dev
        self.B, self.TB = int(batch_size), int(test_batch_size)
        self.world, self.rank = world_size, rank
        self.seed = int(seed)
        self.graph_steps = int(graph_steps)
        self.flags = 0 if dropout else FLAG_NO_DROPOUT
        self.num_samples = int(num_samples)                 # per-rank samples per epoch
        self.steps_per_epoch = math.ceil(self.num_samples / self.B)
        self.rng_base = 0
        # (``streams``: created by a caller that starts other stream users first - the xGMI setup
        # thread's self-test - so these two are the process's first and keep their own hardware queues)
        self.compute, self.comm_stream = streams if streams is not None else make_streams(dev)
        # ---- device-resident data
        self.train_u8 = train.device_images(dev)              # (synthetic: rendered on the device)
        self.train_labels = train.targets.to(torch.int32).to(dev)
        z = native.zeros                                     # hipMemset: no torch fill kernel
        self.train_idx = z(self.steps_per_epoch * self.B, torch.int32, dev)
        # device-side DataLoader: each epoch's rows pre-gathered in sampler order (Engine::gather_rows)
        self.epoch_u8 = torch.empty(self.steps_per_epoch * self.B, 784, dtype=torch.uint8, device=dev)
        self.epoch_labels = z(self.steps_per_epoch * self.B, torch.int32, dev)
        self.loss_log = z(max(self.steps_per_epoch, 1), torch.float32, dev)
        self.n_test = len(test) if test is not None else 0
        if test is not None:
            self.test_u8 = test.device_images(dev)
            self.test_labels = test.targets.to(torch.int32).to(dev)
            self.test_idx = torch.arange(self.n_test, dtype=torch.int32).to(dev)
            self.test_loss_rows = z(self.n_test, torch.float32, dev)
            self.test_correct = z(self.n_test, torch.int32, dev)
            # pinned landing buffers of the per-epoch evaluation read-back (allocated once: a pinned
            # allocation is a driver call inside every epoch of the reference's timer otherwise)
            self._eval_rows_h = torch.empty(self.n_test, dtype=torch.float32, pin_memory=True)
            self._eval_hits_h = torch.empty(self.n_test, dtype=torch.int32, pin_memory=True)
        # two pinned staging buffers for the per-epoch index upload (alternating; the event of a
        # buffer's last H2D is waited on before the host rewrites it)
        self._idx_h = [torch.empty(self.steps_per_epoch * self.B, dtype=torch.int32, pin_memory=True)
                       for _ in range(2)]
        self._idx_ev = [None, None]
        self._idx_k = 0
        self._lr_h = [torch.empty(1, dtype=torch.float32, pin_memory=True) for _ in range(2)]   # set_lr
        self._lr_ev = [None, None]
        self._lr_k = 0
        bufs = mstate.buffers()
        p = native.ptr
        bufs.update(loss_log=p(self.loss_log), train_u8=p(self.train_u8), train_labels=p(self.train_labels),
                    train_idx=p(self.train_idx), epoch_u8=p(self.epoch_u8), epoch_labels=p(self.epoch_labels))
        if test is not None:
            bufs.update(test_u8=p(self.test_u8), test_labels=p(self.test_labels), test_idx=p(self.test_idx),
                        test_loss_rows=p(self.test_loss_rows), test_correct=p(self.test_correct))
        torch.cuda.synchronize(dev)
        # evaluation runs the whole test split as ONE batch (per-row results are bitwise the same as
        # with --test-batch-size chunks: every eval kernel computes rows independently and the
        # losses / hits are summed once on the host): 3 launches instead of 3 per 1000 images
        self.eval_batch = self.n_test if 0 < self.n_test <= 16384 else max(self.TB, 1)
        self.fp32 = bool(fp32)
        self.engine = C.Engine(bufs, self.B, max(self.eval_batch, self.TB, 1) if test is not None else 1,
                               int(self.compute.cuda_stream), int(self.comm_stream.cuda_stream),
                               world_size, mstate.rho, mstate.eps, mstate.weight_decay, fp32=self.fp32)
        self.engine.set_bucket_split(two_buckets)
        self.apply_hooks(hooks or {})
        self._graphs: dict[tuple[int, int], int] = {}        # captured chunks of the selected schedule
        self._graph_sets: dict[str, dict] = {}               # per transport (validation captures)
        self._eval_graph: int | None = None
        # steps still to run in the profiling window (Engine.profile_steps; bitwise the graph path)
        self.profile_left = 0
        self.use_graphs = self.graph_steps > 0
        self.comm = comm
        if comm is not None:
            self.engine.attach_comm(comm)                    # also the parameter broadcast's transport
        if allreduce is None:
            allreduce = "auto"
        if allreduce not in ("rccl", "xgmi", "auto", "fastest"):
            raise ValueError(f"allreduce must be 'rccl', 'xgmi', 'auto' or 'fastest', got {allreduce!r}")
        if allreduce == "xgmi" and not two_buckets:
            raise ValueError("the xGMI all-reduce runs the engine's two-bucket schedule (two_buckets=True)")
        self.xgmi, self.grad_out = None, None
        self.xgmi_fuse = bool(xgmi_fuse)
        self.engine.set_xgmi_fuse_update(self.xgmi_fuse)
        self.transport_report: dict[str, dict] = {}           # candidate -> validation / us per step
        self._fault_stall, self._fault_stream = False, None   # MNIST_AMD_FAULT=rccl_stall (tests)
        self.allreduce_timings: dict[str, float] = {}
        self.xgmi_validation = None
        self.allreduce = None
        import torch.distributed as _dist
        ddp = (comm is not None or rccl_pending is not None or world_size > 1
               or (allreduce == "xgmi" and _dist.is_initialized()))
        self._xgmi_pending = xgmi_pending        # distributed.PendingXgmiComm started by the caller
        self._rccl_pending = rccl_pending        # distributed.PendingRcclComm (maybe not started)
        if not ddp:
            self._setup_single_gpu(overlap)
        else:
            self._setup_ddp(comm, allreduce, two_buckets, probe_world1, train)
        self.setup.add("engine", time.perf_counter() - _t_init - self.setup.total())

    # engine variants for A/B measurements and tests (tools/ab_*.sh through bench.py --hook), set before
    # any graph is captured: name -> (setter, what it changes)
    HOOKS = {
        # B > 1024 side schedules: fc_bwd's fc1 weight gradient on the comm stream beside the conv
        # backward (default 1; 0 = inside the compute-stream fc_bwd launch)
        "fc_dw1_side": "fc_bwd's weight-gradient roles on the comm stream (1) or in the compute launch (0)",
        # persistent conv2_dgrad grid (0 = the default sizing; n > 0 workgroups)
        "dgrad_grid": "persistent conv2_dgrad grid override in workgroups (0 = default)",
        # the second w1t copy; 0 = the fc update overwrites the w1t fc_bwd role B reads (a known race,
        # for the race-window widening check only - never a product setting)
        "w1t_pingpong": "fc update writes the other w1t copy (1) or the one role B reads (0: the old race)",
        # single-GPU OVERLAP step tail: conv1's reduce + update on 80 one-wave workgroups (1) or the
        # 20 conv1 parts of the 256-thread reduce launch (0); bitwise equal either way
        "c1_lanes": "conv1 reduce + update on one-wave workgroups (1) or the 256-thread parts (0)",
    }

    def apply_hooks(self, hooks: dict) -> None:
        """Engine variants by name (``HOOKS``); unknown names raise.  Process-wide ones
        (``dgrad_grid``) stay set until changed."""
        for k, v in hooks.items():
            if k == "fc_dw1_side":
                self.engine.fc_dw1_side = bool(int(v))
            elif k == "dgrad_grid":
                self.C.set_dgrad_grid(int(v))
            elif k == "w1t_pingpong":
                self.engine.w1t_pingpong = bool(int(v))
            elif k == "c1_lanes":
                self.engine.c1_lanes = bool(int(v))
            else:
                raise ValueError(f"unknown engine hook {k!r} (known: {sorted(self.HOOKS)})")

    # ------------------------------------------------------------------ schedule selection
    def _probe_streams(self) -> bool:
        """Both streams on distinct hardware queues (the device-counter hand-offs need it), on every rank."""
        from ..parallel.distributed import STARTUP_TIMEOUT_S, _all_ok
        with self.setup.phase("stream_probe"):
            ok = bool(self.engine.probe_stream_handoff(STARTUP_TIMEOUT_S))
            return _all_ok(ok, world=self.world)

    def _setup_single_gpu(self, overlap: bool) -> None:
        C = self.C
        # OVERLAP (default): the fc Adadelta step and conv2's reduce + update on the comm stream under
        # the conv backward (measured B = 200: 82.7 vs 85.2 us/step serial, then 70.8-71.2 with
        # conv2's part moved too); SERIAL when the streams share a hardware queue
        self.overlap = bool(overlap) and self._probe_streams()
        self.engine.set_schedule(C.SCHED_OVERLAP if self.overlap else C.SCHED_SERIAL)

    def _use_graph_set(self, name: str) -> None:
        self._graphs = self._graph_sets.setdefault(name, {})

    def _rccl_candidate(self, comm, pending):
        """The RCCL communicator: ``comm`` as given, else ``pending``'s (started now if it was deferred,
        then waited for).  Returns (comm or None, why-not): an init that fails or times out drops RCCL,
        it never ends the run by itself (the caller decides whether any transport is left)."""
        if comm is not None or pending is None:
            return comm, None
        with self.setup.phase("rccl_comm_wait"):
            try:
                comm = pending.result()
            except Exception as e:  # noqa: BLE001 - reported as the candidate's failure
                comm = None
                why = f"rank {self.rank}: RCCL communicator init failed ({type(e).__name__}: {e})"
            else:
                why = None
        self.setup.add_info("rccl_comm_init_thread_s", round(pending.seconds or 0.0, 4))
        # collective: a communicator is usable only when every rank has one
        from ..parallel.distributed import gather_strings
        msgs = [m for m in gather_strings(why or "", self.world) if m]
        if msgs and comm is not None:
            comm.abort()
            comm = None
        return comm, "; ".join(msgs) or None

    def _setup_ddp(self, comm, allreduce: str, two_buckets: bool, probe_world1: bool, train) -> None:
        """Build the candidate transports, validate + time their production schedules, keep one.

        * ``xgmi`` / ``rccl``: that transport only (an RCCL communicator that fails to initialise is
          the run's error).
        * ``auto`` (default): the direct xGMI kernels first (one node); once their production schedule
          has validated on every rank they are kept and RCCL is never waited for - a pending RCCL init
          is cancelled, a deferred one never starts - so RCCL's bootstrap and validation replays never
          sit inside the reference's timer.  Only when xGMI cannot be built or fails its validation is
          RCCL brought up and validated (its init error, timeout or stuck replay then fails the run).
        * ``fastest``: both validated and timed, the faster kept (an RCCL init that fails drops RCCL).
        """
        from ..parallel.distributed import create_xgmi_comm, release_xgmi_comm
        C = self.C
        self.overlap = False
        pending, self._rccl_pending = self._rccl_pending, None
        have_r = comm is not None or pending is not None
        want_x = allreduce == "xgmi" or (allreduce in ("auto", "fastest") and two_buckets
                                         and (self.world > 1 or probe_world1))
        x = None
        xpend, self._xgmi_pending = self._xgmi_pending, None
        if xpend is not None and not want_x:        # started by the caller, not a candidate after all
            with self.setup.phase("xgmi_comm"):
                x = xpend.result()
                if x is not None:
                    release_xgmi_comm(x, self.world)
                x = None
        if want_x:
            with self.setup.phase("xgmi_comm"):   # (with a pending setup: the wait for its helper thread)
                if xpend is not None:
                    x = xpend.result()
                    sub = dict(xpend.timings, helper_thread_s=round(xpend.seconds or 0.0, 4))
                else:
                    sub = {}
                    x = create_xgmi_comm(self.world, self.rank, self.device, self.ms.grad.numel(), timings=sub)
                self.setup.add_info("xgmi_comm_steps_s", sub)
        # compute / comm streams on distinct hardware queues: the device-counter hand-offs of the
        # XGMI schedule and of the RCCL schedule's fc update need it (one probe, every rank; after
        # the xGMI setup, whose self-test keeps three more streams busy - with few hardware queues per
        # process, as in the one-GPU rehearsals, the two would share queues)
        handoff = self._probe_streams() if (x is not None or (have_r and two_buckets)) else False
        self.engine.set_rccl_handoff(handoff)
        if want_x:
            if x is not None and not handoff:
                if self.rank == 0:
                    print("[engine] compute/comm streams share a hardware queue: no xGMI schedule", flush=True)
                release_xgmi_comm(x, self.world)
                x = None
            if x is None:
                self.transport_report["xgmi"] = {"ok": False, "validation": "setup, self-test or stream probe failed"}
        if x is None and allreduce != "xgmi":
            # no xGMI transport: RCCL is the only candidate left (its init is waited for only now)
            comm, why = self._rccl_candidate(comm, pending)
            pending = None
            if comm is None and have_r:
                self.transport_report["rccl"] = {"ok": False, "validation": why or "no communicator"}
            if comm is not None:
                self.comm = comm
                self.engine.attach_comm(comm)
        # DDP construction semantics: rank 0's parameters everywhere BEFORE the validations (they
        # compare the ranks' parameters after replaying the same steps)
        if x is not None or self.comm is not None or not self.transport_report:
            self.broadcast_params(x)
        if x is not None:
            self.engine.attach_xgmi(x)
            self.engine.set_schedule(C.SCHED_XGMI)
            self.xgmi = x
            self._use_graph_set("xgmi")
            both = allreduce == "fastest" and have_r   # two candidates: time each beyond its first replay
            ok, why, us = self._validate("xgmi", train, timed=both)
            if not ok and "differ" in why:
                # wrong sums, no timeout: retry with system-scope release / acquire fences around every
                # stage flag (the ordering rules R1-R4 of xgmi_allreduce.hip assume a memory model the
                # fences make explicit); graphs captured without them are dropped
                if self.rank == 0:
                    print(f"[xgmi] startup validation failed ({why}): retrying with fences", flush=True)
                x.set_fences(True)
                self._graph_sets["xgmi"] = {}
                self._use_graph_set("xgmi")
                ok, why2, us = self._validate("xgmi", train, timed=both)
                why = why2 if ok else f"{why}; fenced: {why2}"
            self.transport_report["xgmi"] = {"ok": ok, "validation": why, "us_per_step": us,
                                             "ordering": x.ordering}
            self.xgmi_validation = why
            if not ok and self.rank == 0:
                print(f"[xgmi] startup validation failed ({why})", flush=True)
            self.engine.attach_xgmi(None)           # detached while RCCL is evaluated (re-attached below)
            if not ok:
                release_xgmi_comm(x, self.world)
                x = self.xgmi = None
            if ok and allreduce == "auto":
                # validated on every rank (collective verdict): RCCL is not needed - every rank drops
                # its (pending or deferred) communicator, nobody's bootstrap waits for a peer
                if pending is not None:
                    pending.cancel()
                    self.transport_report["rccl"] = {"ok": None, "validation": "not needed: the xGMI "
                                                     f"transport validated first (RCCL init {pending.status})"}
                    pending = None
                elif comm is not None:
                    self.transport_report["rccl"] = {"ok": None, "validation": "not needed: the xGMI "
                                                     "transport validated first"}
                comm = None
            elif allreduce in ("auto", "fastest") and comm is None and pending is not None:
                comm, why = self._rccl_candidate(None, pending)   # xGMI failed (auto) / both timed
                pending = None
                if comm is None:
                    self.transport_report["rccl"] = {"ok": False, "validation": why or "no communicator"}
                else:
                    self.comm = comm
                    self.engine.attach_comm(comm)
        want_r = comm is not None and allreduce in ("rccl", "auto", "fastest") and \
            not (allreduce == "auto" and self.transport_report.get("xgmi", {}).get("ok"))
        if want_r:
            self.engine.set_schedule(C.SCHED_RCCL)
            self._use_graph_set("rccl")
            ok, why, us = self._validate("rccl", train, timed=x is not None)
            self.transport_report["rccl"] = {"ok": ok, "validation": why, "us_per_step": us}
        valid = {k: v["us_per_step"] for k, v in self.transport_report.items() if v.get("ok")}
        self.allreduce_timings = {k: round(v["us_per_step"], 2) for k, v in self.transport_report.items()
                                  if v.get("us_per_step") is not None}
        if not valid:
            msg = "; ".join(f"{k}: {v.get('validation')}" for k, v in self.transport_report.items())
            hint = "" if have_r else " (no RCCL communicator: rerun with --allreduce rccl or auto)"
            raise StartupValidationError(f"world size {self.world}: no gradient all-reduce passed its startup "
                                         f"validation ({msg or 'no candidate'}){hint}", self.transport_report,
                                         self.setup)
        pick = min(valid, key=valid.get)
        if pick == "xgmi":
            if self.comm is not None and allreduce != "fastest":
                self.engine.attach_comm(None)
                self.comm = None
            self.engine.attach_xgmi(x)
            self.engine.set_schedule(C.SCHED_XGMI)
        else:
            if x is not None:
                release_xgmi_comm(x, self.world)
                x = self.xgmi = None
            self.engine.set_schedule(C.SCHED_RCCL)
        self._use_graph_set(pick)
        self.allreduce = pick
        # the all-reduced gradients (xGMI: the communicator's output buffer; the inputs are written
        # to its input buffer instead of mstate.grad while it is attached)
        self.grad_out = self.xgmi.grad_out if self.xgmi is not None else None

    def broadcast_params(self, x=None) -> None:
        """DDP construction (reference mnist_ddp.py:173): rank 0's parameters to every rank, over the
        framework's transport - the xGMI peer mappings, else the RCCL communicator, else (gloo
        rehearsals) the process group - then the bf16 shadows are rebuilt."""
        if self.world == 1:
            return
        x = x if x is not None else self.xgmi
        from ..parallel.distributed import broadcast_, xgmi_broadcast_
        with torch.cuda.stream(self.compute), self.setup.phase("broadcast"):
            if x is not None:
                xgmi_broadcast_(x, self.ms.param, 0)
            elif self.comm is not None:
                self.engine.broadcast_params(0)
                self._wait_compute(rccl_watchdog_s(), "RCCL parameter broadcast")
            else:
                broadcast_(self.ms.param, 0)
            self.engine.refresh_shadows()
            torch.cuda.synchronize(self.device)

    def _drain(self, timeout_s: float) -> bool:
        """Both streams idle within ``timeout_s`` (events polled; never a blocking sync)."""
        evs = []
        for st in (self.compute, self.comm_stream):
            ev = torch.cuda.Event()
            ev.record(st)
            evs.append(ev)
        t0 = time.perf_counter()
        while not all(ev.query() for ev in evs):
            if time.perf_counter() - t0 > timeout_s:
                return False
            time.sleep(0.001)
        return True

    def _abort_rccl(self, hang: "TransportHang | None" = None) -> float:
        """Drop the RCCL candidate: ncclCommAbort (RCCL's device-side waits return), release an
        injected test stall, wait for the streams to drain.  Returns the seconds that took; re-raises
        ``hang`` (fatal) when the streams do not drain - then something is stuck for good."""
        t0 = time.perf_counter()
        if self.comm is not None:
            self.comm.abort()
        if self._fault_stall:
            self.engine.fault_release(int(self._fault_stream.cuda_stream))
            self._fault_stall = False
        if not self._drain(RCCL_DRAIN_S):
            if hang is not None:
                raise hang
            raise TransportHang(f"rank {self.rank}: the streams did not drain within {RCCL_DRAIN_S:.0f} s of "
                                "aborting the RCCL communicator")
        return time.perf_counter() - t0

    def _drop_rccl(self) -> None:
        """After a failed RCCL candidate: the engine no longer holds the (aborted) communicator and
        the graphs captured with its collectives are never replayed."""
        self.engine.attach_comm(None)
        self.comm = None
        self._graph_sets.pop("rccl", None)

    def _wait_compute(self, timeout_s: float, what: str) -> None:
        """Host watchdog on the compute stream (every chunk and step joins the comm stream into it)."""
        ev = torch.cuda.Event()
        ev.record(self.compute)
        t0 = time.perf_counter()
        while not ev.query():
            if time.perf_counter() - t0 > timeout_s:
                raise TransportHang(f"rank {self.rank}: {what} did not complete within {timeout_s:.0f} s "
                                    "(a collective is stuck on the device)")
            time.sleep(0.0002)

    # ------------------------------------------------------------------ startup validation
    def _validate(self, name: str, train: MNISTData, timed: bool = True) -> tuple[bool, str, float | None]:
        """Run the selected production schedule before training starts: the captured chunk graph of
        ``graph_steps`` steps that training replays (cached for training; eager steps when graphs are
        off), dropout off, on the live state, which is restored bit for bit afterwards.  Passes when
        no rank timed out (xGMI: STARTUP_TIMEOUT_S stage waits, read from device memory so the cached
        graph picks up the run timeout afterwards; RCCL: a host watchdog of ``rccl_watchdog_s()``)
        and every rank holds the same parameters afterwards.  A stuck RCCL replay is aborted
        (ncclCommAbort: RCCL's device-side waits return, the streams drain) and the candidate dropped
        on every rank - only streams that do not drain after that raise TransportHang (fatal).  Then
        (``timed``: two candidates) the chunk is replayed ``VALIDATE_TIMED`` more times and timed: the
        transport's µs per step (max over ranks) is the "auto" choice's measure; a single candidate is
        timed on its validation replay.  The verdict is collective and names every
        failing rank.  Fault injection for tests: ``MNIST_AMD_FAULT=validate_delay:R:S`` holds rank
        R's replay back S seconds; ``rccl_stall:R:S`` puts a device-side hold of up to S seconds in
        front of rank R's first RCCL replay."""
        from ..parallel.distributed import (RUN_TIMEOUT_S, STARTUP_TIMEOUT_S, _max_over_ranks, gather_strings,
                                            params_fingerprint_equal)
        _t0 = time.perf_counter()
        ms, eng = self.ms, self.engine
        n = self.graph_steps if self.use_graphs else 3
        n = max(1, min(n, self.steps_per_epoch))
        keys = ("param", "square_avg", "acc_delta", "state")
        torch.cuda.synchronize(self.device)
        snap = {k: getattr(ms, k).clone() for k in keys}
        idx = torch.arange(n * self.B, dtype=torch.int64) % max(1, len(train))
        delay = _fault_delay("validate_delay", self.rank)
        rccl = name == "rccl"
        # MNIST_AMD_FAULT=rccl_stall:R:S (tests): rank R's first RCCL replay sits behind a device-side
        # hold of up to S seconds - a collective that never completes, as seen by the host watchdog
        stall = _fault_delay("rccl_stall", self.rank) if rccl else 0.0
        if self.xgmi is not None and not rccl:
            self.xgmi.set_timeout_seconds(STARTUP_TIMEOUT_S)
        why, us, result = "", None, None

        def run_chunk():
            eng.begin_epoch(self.seed, 0, 0, FLAG_NO_DROPOUT)
            if stall and not self._fault_stall and not hung:
                self._fault_stall = True
                self._fault_stream = torch.cuda.Stream(device=self.device)
                eng.fault_hold(stall)
            if self.use_graphs:
                eng.replay(self._graph(n, self.B))
            else:
                eng.train_steps(n, self.B, self.B)

        def wait():
            if rccl:
                self._wait_compute(rccl_watchdog_s(), "RCCL schedule validation")
            eng.synchronize()                        # raises on a stage / hand-off timeout

        hung = False                                 # this rank's RCCL replay was stuck and aborted
        try:
            self.upload_indices(idx)
            if self.use_graphs:
                self._graph(n, self.B)               # captured (and cached) before the clock
            torch.cuda.synchronize(self.device)
            if delay:
                time.sleep(delay)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(self.compute)
            run_chunk()
            ev1.record(self.compute)
            wait()
            us = ev0.elapsed_time(ev1) * 1000.0 / n
            result = ms.param.cpu()                  # (host checks: no torch GPU kernel at startup)
            if not torch.isfinite(result).all():
                why = f"rank {self.rank}: non-finite parameters"
        except TransportHang as e:
            if not rccl:
                raise
            # a stuck RCCL replay is no longer fatal: abort the communicator, let the streams drain,
            # and report the candidate as failed (the xGMI candidate, validated first, stays usable)
            took = self._abort_rccl(e)
            hung = True
            why = (f"rank {self.rank}: replay stuck for {rccl_watchdog_s():.0f} s, communicator aborted "
                   f"after {rccl_watchdog_s() + took:.1f} s")
        except RuntimeError as e:
            why = f"rank {self.rank}: {e} (after {time.perf_counter() - _t0:.1f} s)"
        msgs = gather_strings(why, self.world)       # collective: every rank stops here together
        why = "; ".join(m for m in msgs if m)
        if why and rccl and not hung:                # a peer's replay failed: this communicator goes too
            self._abort_rccl()
            hung = True
        if not why and self.world > 1 and not params_fingerprint_equal(result, world=self.world):
            why = "parameters differ across ranks after the validation chunk"
        if not why and not timed:
            us = _max_over_ranks(us, world=self.world)
        elif not why:
            # timed replays of the same chunk (state need not be restored in between: the numbers do
            # not matter, the schedule's time does)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            try:
                torch.cuda.synchronize(self.device)
                ev0.record(self.compute)
                for _ in range(VALIDATE_TIMED):
                    run_chunk()
                ev1.record(self.compute)
                wait()
                us = ev0.elapsed_time(ev1) * 1000.0 / (VALIDATE_TIMED * n)
            except TransportHang as e:
                if not rccl:
                    raise
                took = self._abort_rccl(e)
                hung = True
                why = (f"rank {self.rank}: timed replay stuck for {rccl_watchdog_s():.0f} s, communicator aborted "
                       f"after {rccl_watchdog_s() + took:.1f} s")
            except RuntimeError as e:
                why = f"rank {self.rank}: timed replay: {e}"
            why = "; ".join(m for m in gather_strings(why, self.world) if m)
            if why and rccl and not hung:
                self._abort_rccl()
                hung = True
            if not why:
                us = _max_over_ranks(us, world=self.world)
        with torch.no_grad():
            for k in keys:
                getattr(ms, k).copy_(snap[k])
        torch.cuda.synchronize(self.device)
        eng.refresh_shadows()
        eng.reset_counters()                         # (an aborted chunk leaves the hand-offs unpaired)
        if self.xgmi is not None and not rccl:
            self.xgmi.set_timeout_seconds(RUN_TIMEOUT_S)
        torch.cuda.synchronize(self.device)
        self.setup.add(f"validate.{name}", time.perf_counter() - _t0)
        if hung:
            self._drop_rccl()
        if why:
            return False, why, None
        how = f"graph replay of the {n}-step training chunk" if self.use_graphs else f"{n} eager steps"
        clock = f"{VALIDATE_TIMED} timed replay(s)" if timed else "timed on the validation replay"
        return True, f"ok ({how}, ranks bitwise equal, {clock})", us

    def reset_model(self, module) -> None:
        """Start over from ``module``'s parameters with fresh optimizer state (zero Adadelta
        accumulators, dropout stream from the start) on this already-built trainer: engine, graphs,
        communicators, probe and validation are reused (bench.py's in-process 20-epoch run)."""
        self.synchronize()
        ms = self.ms
        with torch.no_grad():
            ms.square_avg.zero_()
            ms.acc_delta.zero_()
            ms.grad.zero_()
            self.loss_log.zero_()
        ms.bind(module)                      # copies the parameters into the flat buffer + shadows
        torch.cuda.synchronize(self.device)
        self.rng_base = 0

    def check_errors(self) -> None:
        """Raise if a device-side hand-off or xGMI stage wait timed out (the per-epoch check; a 4-byte
        D2H per flag after the epoch's work has completed)."""
        self.engine.check_errors()

    # ------------------------------------------------------------------ helpers
    def set_lr(self, lr: float) -> None:
        """StepLR's new rate for the kernels (device scalar): an asynchronous H2D copy on the compute
        stream from one of two pinned host scalars (stream-ordered with the epochs around it; no fill
        kernel).  A pageable source would make copy_ block until the stream is idle - at every epoch
        boundary of the pipelined driver.  Each pinned scalar is rewritten only after its previous
        copy has run (event), as the index upload does."""
        k = self._lr_k
        self._lr_k ^= 1
        if self._lr_ev[k] is not None:
            self._lr_ev[k].synchronize()
        self._lr_h[k][0] = float(lr)
        with torch.cuda.stream(self.compute):
            self.ms.lr.copy_(self._lr_h[k], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.compute)
        self._lr_ev[k] = ev

    def _graph(self, n: int, batch: int) -> int:
        key = (n, batch)
        gid = self._graphs.get(key)
        if gid is None:
            with self.setup.phase("graph_capture"):
                gid = self.engine.capture_train(n, batch, self.B)
            self._graphs[key] = gid
        return gid

    def _run(self, n: int, batch: int) -> None:
        if n <= 0:
            return
        if self.profile_left > 0:        # --profile window: eager steps, one roctx range per phase
            k = min(n, self.profile_left)
            self.engine.profile_steps(k, batch, self.B)
            self.profile_left -= k
            n -= k
            if n <= 0:
                return
        if self.use_graphs:
            self.engine.replay(self._graph(n, batch))
        else:
            self.engine.train_steps(n, batch, self.B)

    def upload_indices(self, idx: torch.Tensor, gather: bool = True) -> None:
        """Upload this epoch's sampler order; ``gather`` also pre-gathers the rows on the device."""
        n = idx.numel()
        if n > self.train_idx.numel():
            raise ValueError("epoch index vector larger than the device buffer")
        # the device gather and the step kernels read dataset rows by these indices unchecked: an
        # out-of-range index is a GPU memory fault, so it is refused here (one host pass, ~20 us)
        if n and (int(idx.min()) < 0 or int(idx.max()) >= self.train_u8.shape[0]):
            raise ValueError(f"epoch index out of range [0, {self.train_u8.shape[0]})")
        k = self._idx_k
        self._idx_k ^= 1
        if self._idx_ev[k] is not None:
            self._idx_ev[k].synchronize()           # that buffer's previous upload has been consumed
        host = self._idx_h[k][:n]
        host.copy_(idx)                              # (int64 -> int32)
        with torch.cuda.stream(self.compute):
            self.train_idx[:n].copy_(host, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.compute)
        self._idx_ev[k] = ev
        if gather:
            self.engine.gather_rows(0, n)

    # ------------------------------------------------------------------ training
    def train_epoch(self, epoch: int, idx: torch.Tensor, log_interval: int = 10, dry_run: bool = False,
                    log_fn=None, sync: bool = True, before_log=None) -> EpochStats:
        """Run one epoch over this rank's index vector ``idx``.

        ``log_fn(batch_idx, batch_len, loss)`` is called (in order) for every batch with
        ``batch_idx % log_interval == 0``; pass None to skip the per-chunk syncs entirely.
        ``sync=False`` returns as soon as the epoch is enqueued (``train_seconds`` is then the enqueue
        time): the caller overlaps host work - the next epoch's sampler order - with the GPU.
        ``before_log()`` runs once, before the first ``log_fn`` call (or at the end): the driver
        prints the previous epoch's test line there, after this epoch's first chunks are enqueued.
        """
        n = idx.numel()
        full, last = divmod(n, self.B)
        steps = full + (1 if last else 0)
        if dry_run:
            steps, full, last = 1, (1 if n >= self.B else 0), (0 if n >= self.B else n)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(self.compute)
        self.upload_indices(idx)
        self.engine.begin_epoch(self.seed, self.rng_base, 0, self.flags)
        self.rng_base += 2 * steps
        t0 = time.perf_counter()
        logged = {}
        # Logged losses are read one chunk late: the chunk after a logged step is enqueued before the
        # host waits for that step (an event, not the whole stream), so the GPU never idles while the
        # host reads the loss and prints.  Lines come out in the same order with the same values.
        pending = []
        hook = [before_log]

        def run_hook():
            if hook[0] is not None:
                h, hook[0] = hook[0], None
                h()

        def flush_one():
            run_hook()
            ev, b_idx, blen = pending.pop(0)
            ev.synchronize()
            loss = float(self.loss_log[b_idx].item())
            logged[b_idx] = loss
            log_fn(b_idx, blen, loss)

        def note(rows):
            """The logged steps (batch_idx, batch_len) of the chunk just enqueued: one event after
            it; the previous chunks' lines are printed first (their events), never this chunk's."""
            if not rows:
                return
            ev = torch.cuda.Event()
            ev.record(self.compute)
            while pending:
                flush_one()
            pending.extend((ev, b_idx, blen) for b_idx, blen in rows)

        # chunks of graph_steps regardless of the log interval: every logged step's loss stays in
        # loss_log, so a chunk holding several logged steps prints them all (in order) once it is
        # done - a chunk cut after every logged step (10 steps with the reference's log interval)
        # costs 1.4-2.2 us a step over 20-step chunks (profiles/r4/s2/ab/gs_sweep_*.txt)
        chunk = self.graph_steps if self.graph_steps > 0 else max(1, log_interval)
        done = 0
        while done < full:
            n_here = min(chunk, full - done)
            self._run(n_here, self.B)
            if log_fn is not None:
                first = -(-done // log_interval) * log_interval          # first logged index >= done
                note([(b, self.B) for b in range(first, done + n_here, log_interval)])
            done += n_here
        if last:
            self._run(1, last)
            if log_fn is not None and full % log_interval == 0:
                note([(full, last)])
        ev1.record(self.compute)
        while pending:
            flush_one()
        run_hook()
        dev_s = None
        if sync:
            self.compute.synchronize()
            if self.xgmi is not None or self.comm is not None or self.overlap:
                self.check_errors()        # fail at the first bad epoch, not after the last one
            dev_s = ev0.elapsed_time(ev1) / 1000.0
        return EpochStats(epoch, steps, min(n, steps * self.B), time.perf_counter() - t0, logged, dev_s, (ev0, ev1))

    # ------------------------------------------------------------------ raw step stream (bench)
    def start_stream(self, idx: torch.Tensor, gather: bool = True) -> None:
        """Upload a flat index stream (steps * B rows) and reset the device step counter.
        With ``gather=False`` the caller pre-gathers row ranges itself (``engine.gather_rows``)."""
        self.upload_indices(idx, gather=gather)
        self.engine.begin_epoch(self.seed, self.rng_base, 0, self.flags)
        self.rng_base += 2 * (idx.numel() // self.B)

    def _chunks(self, n: int) -> list[int]:
        """Graph sizes ``run_steps(n)`` replays: ``graph_steps`` each, the last one shorter."""
        c = self.graph_steps if self.graph_steps > 0 else max(1, n)
        return [min(c, n - k) for k in range(0, n, c)]

    def precapture(self, n: int) -> None:
        """Capture every graph ``run_steps(n)`` will replay (capture executes nothing)."""
        if self.use_graphs:
            for k in set(self._chunks(n)):
                self._graph(k, self.B)

    def warm_graphs(self, n: int, min_steps: int = 0) -> int:
        """Replay every graph ``run_steps(n)`` will use - once, or as many rounds as it takes to run
        ``min_steps`` steps (a step count, not a time, so every rank replays the same collectives) -
        then restore the model, optimizer and step state bit for bit: a later timed ``run_steps(n)``
        then starts on executables that have already run (code objects resident, packets uploaded)
        on a device that has been busy for a while (its clocks ramp over ~10 ms of load: a 20-step
        window measured from idle reads 67-68 us/step where 600 steps read 64.7), without counting
        extra steps.  Runs on every rank (the replays include the DDP collectives).  The rows the
        replays read must be gathered (``engine.gather_rows``) beforehand.  Returns the steps run."""
        if not self.use_graphs or n <= 0:
            return 0
        ms = self.ms
        torch.cuda.synchronize(self.device)
        snap = {k: getattr(ms, k).clone() for k in ("param", "square_avg", "acc_delta", "state")}
        torch.cuda.synchronize(self.device)
        sizes = sorted(set(self._chunks(n)))
        rounds = max(1, -(-int(min_steps) // sum(sizes)))
        for r in range(rounds):
            for k in sizes:
                self.engine.replay(self._graph(k, self.B))
            if r + 1 < rounds:
                # every round replays the same steps: the device step counter (which indexes the
                # gathered rows and the loss log) goes back to the snapshot, ordered after the round
                # on the compute stream (the chunk-end join has the comm stream's work behind it)
                with torch.cuda.stream(self.compute), torch.no_grad():
                    ms.state.copy_(snap["state"])
        self.synchronize()
        with torch.no_grad():
            for k, v in snap.items():
                getattr(ms, k).copy_(v)
        torch.cuda.synchronize(self.device)
        self.engine.refresh_shadows()
        torch.cuda.synchronize(self.device)
        return rounds * sum(sizes)

    def run_steps(self, n: int) -> None:
        """Enqueue ``n`` full-batch steps continuing from the device step counter (no host sync)."""
        for k in self._chunks(n):
            self._run(k, self.B)

    # ------------------------------------------------------------------ evaluation
    def evaluate(self) -> tuple[float, int, int]:
        """Return (sum of per-sample NLL, correct, N) over the whole test split."""
        return self.evaluate_async().result()

    def evaluate_async(self) -> "EvalHandle":
        """Enqueue the evaluation and its read-back; ``.result()`` waits for them (an event, not the
        stream) and reduces on the host, so work enqueued after this call keeps the GPU busy."""
        if self.n_test == 0:
            return EvalHandle(None, None, None, 0)
        # one batch = 3 launches: eager (a captured graph only pays when there are many batches)
        if self.use_graphs and self.n_test > self.eval_batch:
            if self._eval_graph is None:
                self._eval_graph = self.engine.capture_eval(self.n_test, self.eval_batch)
            self.engine.replay(self._eval_graph)
        else:
            self.engine.eval(self.n_test, self.eval_batch)
        # per-row results to the host (40 + 40 KB) and summed there in float64: no torch reduction
        # kernel (whose first use loads a code object inside the timed run) and a fixed order
        rows, hits = self._eval_rows_h, self._eval_hits_h
        with torch.cuda.stream(self.compute):
            rows.copy_(self.test_loss_rows, non_blocking=True)
            hits.copy_(self.test_correct, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.compute)
        return EvalHandle(ev, rows, hits, self.n_test)

    def synchronize(self) -> None:
        self.engine.synchronize()
