"""FusedTrainer: the reference train()/test() loops (mnist_ddp.py:65-105) on the native engine.

What changes versus the reference loop, and why (MI355X-first):

* the whole split lives in HBM as uint8 (47 MB); per epoch only the sampler's index vector is
  uploaded (one 240 KB H2D), the first kernel of each step gathers + normalises its rows -
  no DataLoader worker, no pinned-memory thread, no per-step H2D copy (reference :68);
* a training step is 8 kernels enqueued by C++ (``_C.Engine``) and chunks of ``graph_steps``
  steps are captured once into a hipGraph and replayed; the host only syncs where the reference
  prints (rank 0, every ``log_interval`` batches) and at eval;
* DDP: the fc gradient bucket (98.4 % of bytes) is all-reduced over RCCL on a second stream while
  the conv backward runs, then its Adadelta update runs on that stream too; the conv bucket
  follows.  Averaging (1/W) is folded into the gradient GEMM epilogues;
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


def _fault_delay(kind: str, rank: int) -> float:
    """Seconds to hold rank ``rank`` back at fault point ``kind`` (``MNIST_AMD_FAULT=kind:rank:seconds``,
    tests only); 0 when not injected."""
    spec = os.environ.get("MNIST_AMD_FAULT", "")
    parts = spec.split(":")
    if len(parts) == 3 and parts[0] == kind and int(parts[1]) == rank:
        return float(parts[2])
    return 0.0


@dataclass
class EpochStats:
    epoch: int
    steps: int
    samples: int
    train_seconds: float
    losses: dict = field(default_factory=dict)   # batch_idx -> loss for logged steps
    device_seconds: float | None = None          # HIP-event time of the epoch's training work


class FusedTrainer:
    def __init__(self, mstate: ModelState, train: MNISTData, test: MNISTData | None, batch_size: int,
                 test_batch_size: int, num_samples: int, world_size: int = 1, rank: int = 0,
                 comm=None, seed: int = 1, graph_steps: int = 10, dropout: bool = True,
                 two_buckets: bool = True, concurrent: bool | None = None, comm2=None,
                 fuse_fc_update: bool | None = None, allreduce: str | None = None):
        C = native.load()
        self.C, self.ms = C, mstate
        # host seconds per setup phase (engine, xgmi_comm, allreduce_probe, stream_probe, validation,
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
        self.compute = torch.cuda.Stream(device=dev)
        self.comm_stream = torch.cuda.Stream(device=dev, priority=-1)
        # ---- device-resident data
        self.train_u8 = train.images.reshape(len(train), -1).contiguous().to(dev)
        self.train_labels = train.targets.to(torch.int32).to(dev)
        self.train_idx = torch.zeros(self.steps_per_epoch * self.B, dtype=torch.int32, device=dev)
        # device-side DataLoader: each epoch's rows pre-gathered in sampler order (Engine::gather_rows)
        self.epoch_u8 = torch.empty(self.steps_per_epoch * self.B, 784, dtype=torch.uint8, device=dev)
        self.epoch_labels = torch.zeros(self.steps_per_epoch * self.B, dtype=torch.int32, device=dev)
        self.loss_log = torch.zeros(max(self.steps_per_epoch, 1), dtype=torch.float32, device=dev)
        self.n_test = len(test) if test is not None else 0
        if test is not None:
            self.test_u8 = test.images.reshape(self.n_test, -1).contiguous().to(dev)
            self.test_labels = test.targets.to(torch.int32).to(dev)
            self.test_idx = torch.arange(self.n_test, dtype=torch.int32, device=dev)
            self.test_loss_rows = torch.zeros(self.n_test, dtype=torch.float32, device=dev)
            self.test_correct = torch.zeros(self.n_test, dtype=torch.int32, device=dev)
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
        self.engine = C.Engine(bufs, self.B, max(self.eval_batch, self.TB, 1) if test is not None else 1,
                               int(self.compute.cuda_stream), int(self.comm_stream.cuda_stream),
                               world_size, mstate.rho, mstate.eps, mstate.weight_decay)
        self.engine.set_bucket_split(two_buckets)
        self._graphs: dict[tuple[int, int], int] = {}
        self._eval_graph: int | None = None
        # steps still to run in the profiling window (Engine.profile_steps; bitwise the graph path)
        self.profile_left = 0
        self.use_graphs = self.graph_steps > 0
        self.ramp = int(os.environ.get("MNIST_AMD_GRAPH_RAMP", "0"))   # see _chunks
        if concurrent is None:
            concurrent = os.environ.get("MNIST_AMD_CONCURRENT", "0") == "1"
        self.engine.set_concurrent(bool(concurrent))
        # single GPU, opt-in (MNIST_AMD_FUSE_FC=1): fc_bwd applies the fc Adadelta step in its
        # epilogue, bitwise equal to the step-tail update but ~1 us/step slower (the update is
        # HBM-bound either way and loses its overlap with the conv slab reduce; docs/PERF_NOTES.md)
        if fuse_fc_update is None:
            fuse_fc_update = os.environ.get("MNIST_AMD_FUSE_FC", "0") == "1"
        self.engine.set_fuse_fc_update(bool(fuse_fc_update))
        # single GPU: fc Adadelta step overlapped with the conv backward on the comm stream
        # (device-counter hand-offs, schedule-3 style; default on, MNIST_AMD_OVERLAP_FC=0 to disable:
        # measured 85.2 -> 82.7 us/step at B = 200)
        self.overlap_fc = (comm is None and world_size == 1 and not fuse_fc_update and not concurrent
                           and os.environ.get("MNIST_AMD_OVERLAP_FC", "1") == "1")
        self.engine.set_overlap_fc_update(self.overlap_fc)
        # single-GPU overlap schedule: conv2 reduce + update as extra workgroups of the dgrad launch
        # (opt-in MNIST_AMD_DGRAD_UPDATE=1, bitwise equal; measured 81.6-82.2 vs 80.9-81.8 us/step)
        self.engine.set_dgrad_update(os.environ.get("MNIST_AMD_DGRAD_UPDATE", "0") == "1")
        # captured chunks: side-stream nodes first, then the compute chain (MNIST_AMD_SIDE_FIRST=0: one
        # pass in step order; see Engine::capture_train)
        self.engine.set_side_first(os.environ.get("MNIST_AMD_SIDE_FIRST", "1") == "1")
        # single GPU: conv2's slab reduce + update on the comm stream under conv2_dgrad (default on,
        # MNIST_AMD_SIDE_CONV2=0 to compare; bitwise equal: 73.6 / 72.5 -> 70.8 / 71.2 us/step at B = 200)
        self.engine.set_side_conv2(os.environ.get("MNIST_AMD_SIDE_CONV2", "1") == "1")
        # DDP schedule: 3 (the fc bucket all-reduced + updated on the comm stream, overlapping the conv
        # backward and the step boundary, device-counter stream hand-offs; with one communicator the
        # conv all-reduce waits for the fc one on a counter) whenever a communicator is attached
        # (see csrc/runtime/engine.h; measured at world 1: 93.9 / 97.3 / 96.9 us for 3 / 2 / 1)
        sched = int(os.environ.get("MNIST_AMD_DIST_SCHED", "3"))
        self.engine.set_dist_schedule(sched)
        if comm is not None:
            self.engine.attach_comm(comm)
        if comm2 is not None:
            self.engine.attach_comm2(comm2)
        self.comm, self.comm2 = comm, comm2
        # gradient all-reduce: "rccl" (ncclAllReduce per bucket), "xgmi" (direct reduce-scatter +
        # all-gather over IPC-mapped peer buckets, csrc/runtime/xgmi_comm.h; self-tested at startup,
        # falls back to RCCL on every rank if any rank fails) or "auto" (default: with world > 1 and
        # RCCL comms attached, time both on this node's links and keep the faster).  Used on the DDP
        # path; RCCL stays attached for the parameter broadcast.
        if allreduce is None:
            allreduce = os.environ.get("MNIST_AMD_ALLREDUCE", "auto")
        if allreduce not in ("rccl", "xgmi", "auto"):
            raise ValueError(f"allreduce must be 'rccl', 'xgmi' or 'auto', got {allreduce!r}")
        self.xgmi, self.grad_out, self.allreduce_timings = None, None, {}
        self.conv_split, self.conv2_stream = False, None
        self.xgmi_validation = None
        if allreduce == "xgmi" and not two_buckets:
            raise ValueError("the xGMI all-reduce runs the engine's two-bucket schedule (two_buckets=True)")
        import torch.distributed as _dist
        want = allreduce == "xgmi" and (comm is not None or world_size > 1 or _dist.is_initialized())
        probe_always = os.environ.get("MNIST_AMD_PROBE_ALWAYS", "0") == "1"   # tests: probe at world 1
        want = want or (allreduce == "auto" and comm is not None and two_buckets and (world_size > 1 or probe_always))
        # Adadelta fused into the xGMI kernels (default; MNIST_AMD_XGMI_FUSE=0: separate launches).
        # Decided before the probe: only a fused schedule saves the RCCL side's separate conv update.
        self.xgmi_fuse = os.environ.get("MNIST_AMD_XGMI_FUSE", "1") != "0"
        if want:
            from ..parallel.distributed import choose_allreduce, create_xgmi_comm
            with self.setup.phase("xgmi_comm"):
                self.xgmi = create_xgmi_comm(world_size, rank, dev, mstate.grad.numel())
            if self.xgmi is not None and allreduce == "auto":
                split = mstate.bucket_split
                upd = []
                if self.xgmi_fuse:
                    # the RCCL schedule's separate conv update (fused away on the xGMI side) is timed
                    # on a scratch copy of the optimizer state, so the probe leaves the model untouched
                    scratch = {k: getattr(mstate, k).clone() for k in ("param", "square_avg", "acc_delta", "w2f", "w2d")}
                    p_ = native.ptr
                    upd = [lambda: C.adadelta(p_(scratch["param"]), p_(mstate.grad), p_(scratch["square_avg"]),
                                              p_(scratch["acc_delta"]), p_(mstate.lr), mstate.rho, mstate.eps,
                                              mstate.weight_decay, p_(scratch["w2f"]), p_(scratch["w2d"]),
                                              p_(mstate.w1), p_(mstate.w1t), 0, 2, True,
                                              int(torch.cuda.current_stream(dev).cuda_stream))]
                with torch.cuda.stream(self.compute), self.setup.phase("allreduce_probe"):
                    pick, self.allreduce_timings = choose_allreduce(
                        comm2 if comm2 is not None else comm, comm, self.xgmi, mstate.grad,
                        (0, split), (split, mstate.grad.numel() - split), dev, rccl_extra=upd)
                upd = None
                if pick != "xgmi":
                    self.xgmi = None
            if self.xgmi is not None:
                self.engine.set_dist_schedule(3)
                self.engine.attach_xgmi(self.xgmi)
                self.engine.set_xgmi_fuse_update(self.xgmi_fuse)
                # conv bucket split (fused schedule, opt-in MNIST_AMD_CONV_SPLIT=1): conv2's reduce +
                # exchange + update on a third stream under conv2_dgrad, only conv1's 320 values after
                # dgrad.  Bitwise equal; at world 1 it costs 1-2 us/step (88.0-89.1 vs 87.0-87.1: two
                # more hand-off kernels and a third graph branch) and what it saves at world > 1 (the
                # conv2 slab reduce off the critical path) is unmeasured on one GPU, so it is off.
                # MNIST_AMD_CONV_SPLIT=comm (default) queues the conv2 part on the comm stream after the
                # fc bucket instead (no third stream; part of every chunk's side graph): at world 1
                # neutral (78.9-80.3 vs 79.1-79.6 us/step), at world > 1 it takes conv2's slab reduce
                # + exchange + update (98 % of the conv bucket) off the critical path; bitwise equal
                split_mode = os.environ.get("MNIST_AMD_CONV_SPLIT", "comm")
                if self.xgmi_fuse and split_mode == "1":
                    self.conv2_stream = torch.cuda.Stream(device=dev)
                    self.engine.set_conv_split(True, int(self.conv2_stream.cuda_stream))
                    self.conv_split = True
                elif self.xgmi_fuse and split_mode == "comm":
                    self.engine.set_conv_split(True, int(self.comm_stream.cuda_stream))
                    self.conv_split = "comm"
        # schedule 3 spins on one stream for the other: make sure they sit on different hardware
        # queues on EVERY rank, else fall back everywhere to graph-edge joins (schedule 2 / 1, RCCL)
        uses_sched3 = self.xgmi is not None or (comm is not None and sched == 3) or self.overlap_fc
        if uses_sched3:
            from ..parallel.distributed import STARTUP_TIMEOUT_S, _all_ok
            _t_probe = time.perf_counter()
            ok = bool(self.engine.probe_stream_handoff(STARTUP_TIMEOUT_S))
            if world_size > 1:
                ok = _all_ok(ok, dev)
            if not ok and self.conv_split:               # the third stream shares a queue: no split
                self.conv_split = False
                self.engine.set_conv_split(False, 0)
                ok = bool(self.engine.probe_stream_handoff(STARTUP_TIMEOUT_S))
                if world_size > 1:
                    ok = _all_ok(ok, dev)
            if not ok and self.overlap_fc and self.xgmi is None and comm is None:
                self.overlap_fc = False                  # single GPU: plain serial schedule instead
                self.engine.set_overlap_fc_update(False)
                ok = True
            if not ok and comm is None:
                raise RuntimeError("DDP schedule 3 unusable (compute/comm streams share a hardware queue) "
                                   "and no RCCL communicator to fall back to")
            if not ok:
                if rank == 0:
                    print("[engine] compute/comm streams share a hardware queue: DDP schedule 3 disabled",
                          flush=True)
                self.engine.set_dist_schedule(2 if comm2 is not None else 1)   # graph-edge joins
                if self.xgmi is not None:
                    self.engine.attach_xgmi(None)
                    self.xgmi = None
            self.setup.add("stream_probe", time.perf_counter() - _t_probe)
        if self.xgmi is not None and os.environ.get("MNIST_AMD_XGMI_VALIDATE", "1") != "0":
            _t_val, _cap0 = time.perf_counter(), self.setup.s.get("graph_capture", 0.0)
            ok, self.xgmi_validation = self._validate_xgmi_schedule(train)
            # (the training graph it captures is booked under graph_capture)
            self.setup.add("validation", time.perf_counter() - _t_val - (self.setup.s.get("graph_capture", 0.0) - _cap0))
            if not ok:
                if comm is None:
                    raise RuntimeError(f"xGMI schedule failed its startup validation ({self.xgmi_validation}) "
                                       "and no RCCL communicator to fall back to")
                if rank == 0:
                    print(f"[xgmi] startup validation failed ({self.xgmi_validation}): using RCCL", flush=True)
                self.engine.attach_xgmi(None)
                self.xgmi = None
                self._graphs.clear()             # captured with the xGMI kernels: recapture on RCCL
                self.engine.set_dist_schedule(sched)
        if world_size > 1 and self.xgmi is None and comm is None:
            # no transport left (xGMI setup / self-test / validation failed and no RCCL communicator
            # was created, e.g. --allreduce xgmi): training on would let every rank drift apart
            # silently with a gradient 1/world too small - fail instead
            raise RuntimeError(f"world size {world_size}: the xGMI all-reduce is unavailable "
                               f"({self.xgmi_validation or 'setup or self-test failed'}) and no RCCL "
                               "communicator is attached; rerun with --allreduce rccl or auto")
        self.allreduce = "xgmi" if self.xgmi is not None else "rccl"
        # the all-reduced gradients (xGMI: the communicator's output buffer; the inputs are written
        # to its input buffer instead of mstate.grad while it is attached)
        self.grad_out = self.xgmi.grad_out if self.xgmi is not None else None
        self.setup.add("engine", time.perf_counter() - _t_init - self.setup.total())

    # ------------------------------------------------------------------ startup validation
    def _validate_xgmi_schedule(self, train: MNISTData) -> tuple[bool, str]:
        """Run the production xGMI DDP schedule before training starts: the captured chunk graph of
        ``graph_steps`` steps that training replays (cached and reused by training; eager steps only
        when graphs are off), dropout off, STARTUP_TIMEOUT_S stage timeouts (baked into that graph's
        kernel arguments), on the live state, which is restored bit for bit afterwards.  With the
        fused kernels the separate-launch schedule runs too (its own graph, not kept) and must give
        the same bits.  Passes when no rank timed out, fused == separate, and every rank holds the
        same parameters afterwards.  Every mode's verdict is collective (all ranks stop at the first
        failing mode, so no rank is left waiting in kernels its peers never launch) and the message
        names every failing rank.  Fault injection for tests: ``MNIST_AMD_FAULT=validate_delay:R:S``
        holds rank R's replay back S seconds (its peers' stage waits must time out)."""
        from ..parallel.distributed import STARTUP_TIMEOUT_S, gather_strings, params_fingerprint_equal
        ms, eng = self.ms, self.engine
        n = self.graph_steps if self.use_graphs else 3
        n = max(1, min(n, self.steps_per_epoch))
        keys = ("param", "square_avg", "acc_delta", "state")
        torch.cuda.synchronize(self.device)
        snap = {k: getattr(ms, k).clone() for k in keys}
        idx = torch.arange(n * self.B, dtype=torch.int64) % max(1, len(train))
        modes = [True, False] if self.xgmi_fuse else [False]
        delay = _fault_delay("validate_delay", self.rank)
        results, why = [], ""
        self.xgmi.set_timeout_seconds(STARTUP_TIMEOUT_S)
        for fuse in modes:
            mode = "fused" if fuse else "separate"
            t0 = time.perf_counter()
            try:
                with torch.no_grad():
                    for k in keys:
                        getattr(ms, k).copy_(snap[k])
                torch.cuda.synchronize(self.device)
                eng.refresh_shadows()
                eng.set_xgmi_fuse_update(fuse)
                self.upload_indices(idx)
                eng.begin_epoch(self.seed, 0, 0, FLAG_NO_DROPOUT)
                if self.use_graphs:
                    # the training graph itself for the trainer's mode; the other mode's is throwaway
                    gid = self._graph(n, self.B) if fuse == self.xgmi_fuse else eng.capture_train(n, self.B, self.B)
                    if delay:
                        eng.synchronize()
                        time.sleep(delay)
                    eng.replay(gid)
                else:
                    eng.train_steps(n, self.B, self.B)
                eng.synchronize()                       # raises on a stage / hand-off timeout
                results.append(ms.param.clone())
                if not torch.isfinite(results[-1]).all():
                    why = f"{mode}: non-finite parameters"
            except RuntimeError as e:
                why = f"{mode}: {e} (after {time.perf_counter() - t0:.1f} s)"
            msgs = gather_strings(why)                  # collective: every rank stops at the same mode
            if any(msgs):
                why = "; ".join(f"rank {r}: {m}" for r, m in enumerate(msgs) if m)
                break
        if not why and len(results) == 2 and not torch.equal(results[0], results[1]):
            why = f"rank {self.rank}: fused kernels differ from the separate launches"
        if self.world > 1:
            ok_fp = not why and params_fingerprint_equal(results[0], self.device)
            msgs = gather_strings(why or ("" if ok_fp else f"rank {self.rank}: parameters differ across ranks"))
            why = "; ".join(sorted(set(m for m in msgs if m)))
        with torch.no_grad():
            for k in keys:
                getattr(ms, k).copy_(snap[k])
        torch.cuda.synchronize(self.device)
        eng.refresh_shadows()
        eng.set_xgmi_fuse_update(self.xgmi_fuse)
        self.xgmi.set_timeout_seconds(60.0)
        torch.cuda.synchronize(self.device)
        if why:
            return False, why
        what = "fused == separate" if len(modes) == 2 else "separate"
        how = f"graph replay of the {n}-step training chunk" if self.use_graphs else f"{n} eager steps"
        return True, f"ok ({how}, {what})"

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
        with torch.cuda.stream(self.compute):
            self.ms.lr.fill_(float(lr))

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
        host = idx.to(torch.int32).pin_memory() if torch.cuda.is_available() else idx.to(torch.int32)
        with torch.cuda.stream(self.compute):
            self.train_idx[:n].copy_(host, non_blocking=True)
        if gather:
            self.engine.gather_rows(0, n)

    # ------------------------------------------------------------------ training
    def train_epoch(self, epoch: int, idx: torch.Tensor, log_interval: int = 10, dry_run: bool = False,
                    log_fn=None, sync: bool = True) -> EpochStats:
        """Run one epoch over this rank's index vector ``idx``.

        ``log_fn(batch_idx, batch_len, loss)`` is called (in order) for every batch with
        ``batch_idx % log_interval == 0``; pass None to skip the per-chunk syncs entirely.
        ``sync=False`` returns as soon as the epoch is enqueued (``train_seconds`` is then the enqueue
        time): the caller overlaps host work - the next epoch's sampler order - with the GPU.
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

        def flush_one():
            ev, b_idx, blen = pending.pop(0)
            ev.synchronize()
            loss = float(self.loss_log[b_idx].item())
            logged[b_idx] = loss
            log_fn(b_idx, blen, loss)

        def note(b_idx, blen):
            ev = torch.cuda.Event()
            ev.record(self.compute)
            while pending:
                flush_one()
            pending.append((ev, b_idx, blen))

        # chunk boundaries: when logging, end a chunk right after every logged step
        chunk = self.graph_steps if self.graph_steps > 0 else max(1, log_interval)
        done = 0
        while done < full:
            n_here = min(chunk, full - done)
            if log_fn is not None:
                # make the chunk end just after the next logged step (batch_idx % log_interval == 0)
                nxt = ((done + log_interval - 1) // log_interval) * log_interval
                if done % log_interval == 0:
                    nxt = done
                if nxt < done + n_here:
                    n_here = nxt - done + 1
            self._run(n_here, self.B)
            done += n_here
            if log_fn is not None and (done - 1) % log_interval == 0:
                note(done - 1, self.B)
        if last:
            self._run(1, last)
            if log_fn is not None and full % log_interval == 0:
                note(full, last)
        ev1.record(self.compute)
        while pending:
            flush_one()
        dev_s = None
        if sync:
            self.compute.synchronize()
            if self.xgmi is not None or self.comm is not None or self.overlap_fc:
                self.check_errors()        # fail at the first bad epoch, not after the last one
            dev_s = ev0.elapsed_time(ev1) / 1000.0
        return EpochStats(epoch, steps, min(n, steps * self.B), time.perf_counter() - t0, logged, dev_s)

    # ------------------------------------------------------------------ raw step stream (bench)
    def start_stream(self, idx: torch.Tensor, gather: bool = True) -> None:
        """Upload a flat index stream (steps * B rows) and reset the device step counter.
        With ``gather=False`` the caller pre-gathers row ranges itself (``engine.gather_rows``)."""
        self.upload_indices(idx, gather=gather)
        self.engine.begin_epoch(self.seed, self.rng_base, 0, self.flags)
        self.rng_base += 2 * (idx.numel() // self.B)

    def _chunks(self, n: int) -> list[int]:
        """Graph sizes ``run_steps(n)`` replays: ``graph_steps`` each, the last one shorter; with a
        launch ramp (``self.ramp`` = r > 0) the first graphs are r, 2r, 4r, .. steps, so after a host
        sync the GPU starts on a small graph while the host is still submitting the larger ones (a
        graph's host-side launch grows with its node count, ~2.4 us per node on ROCm 7)."""
        c = self.graph_steps if self.graph_steps > 0 else max(1, n)
        k = min(self.ramp, c) if self.ramp > 0 else c
        out = []
        while n > 0:
            take = min(k, n)
            out.append(take)
            n -= take
            k = min(2 * k, c)
        return out

    def precapture(self, n: int) -> None:
        """Capture every graph ``run_steps(n)`` will replay (capture executes nothing)."""
        if self.use_graphs:
            for k in set(self._chunks(n)):
                self._graph(k, self.B)

    def warm_graphs(self, n: int) -> None:
        """Replay once every graph ``run_steps(n)`` will use, then restore the model, optimizer and
        step state bit for bit: a later timed ``run_steps(n)`` then starts on executables that have
        already run (code objects resident, packets uploaded) without counting extra steps.  Runs
        on every rank (the replays include the DDP collectives).  The rows the replays read must be
        gathered (``engine.gather_rows``) beforehand."""
        if not self.use_graphs or n <= 0:
            return
        ms = self.ms
        torch.cuda.synchronize(self.device)
        snap = {k: getattr(ms, k).clone() for k in ("param", "square_avg", "acc_delta", "state")}
        torch.cuda.synchronize(self.device)
        for k in sorted(set(self._chunks(n))):
            self.engine.replay(self._graph(k, self.B))
        self.synchronize()
        with torch.no_grad():
            for k, v in snap.items():
                getattr(ms, k).copy_(v)
        torch.cuda.synchronize(self.device)
        self.engine.refresh_shadows()
        torch.cuda.synchronize(self.device)

    def run_steps(self, n: int) -> None:
        """Enqueue ``n`` full-batch steps continuing from the device step counter (no host sync)."""
        for k in self._chunks(n):
            self._run(k, self.B)

    # ------------------------------------------------------------------ evaluation
    def evaluate(self) -> tuple[float, int, int]:
        """Return (sum of per-sample NLL, correct, N) over the whole test split."""
        if self.n_test == 0:
            return 0.0, 0, 0
        # one batch = 3 launches: eager (a captured graph only pays when there are many batches)
        if self.use_graphs and self.n_test > self.eval_batch:
            if self._eval_graph is None:
                self._eval_graph = self.engine.capture_eval(self.n_test, self.eval_batch)
            self.engine.replay(self._eval_graph)
        else:
            self.engine.eval(self.n_test, self.eval_batch)
        # per-row results to the host (40 + 40 KB) and summed there in float64: no torch reduction
        # kernel (whose first use loads a code object inside the timed run) and a fixed order
        rows = torch.empty(self.n_test, dtype=torch.float32, pin_memory=True)
        hits = torch.empty(self.n_test, dtype=torch.int32, pin_memory=True)
        with torch.cuda.stream(self.compute):
            rows.copy_(self.test_loss_rows, non_blocking=True)
            hits.copy_(self.test_correct, non_blocking=True)
        self.compute.synchronize()
        loss_sum = float(rows.double().sum())
        correct = int(hits.sum())
        return loss_sum, correct, self.n_test

    def synchronize(self) -> None:
        self.engine.synchronize()
