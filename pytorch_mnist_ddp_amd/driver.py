"""Application drivers: the reference's ``main()`` of mnist.py (mnist.py:73-133) and mnist_ddp.py
(mnist_ddp.py:108-197) on the MI355X framework.

Two execution engines, same flags / log lines / checkpoints / RNG consumption:

* ``fused`` (default on GPU): the native step engine - HBM-resident data, 8 hand-written kernels
  per step captured in hipGraphs, DDP gradient buckets all-reduced over RCCL from C++.
* ``module``: the reference's literal loop (``model(data)``, ``F.nll_loss``, ``loss.backward()``,
  ``optimizer.step()``) over :class:`~pytorch_mnist_ddp_amd.models.Net` (fused kernels via autograd
  on GPU, torch ops on CPU), :class:`~pytorch_mnist_ddp_amd.parallel.DistributedDataParallel`
  hooks and :class:`~pytorch_mnist_ddp_amd.optim.Adadelta`.  Always used for ``--no-cuda``.
"""
from __future__ import annotations

import json
import os
import sys
import time

import torch
import torch.nn.functional as F

from . import cli
from .data import (DistributedIndexStream, HostLoader, RandomIndexStream, SequentialIndexStream,
                   consume_loader_base_seed, load_mnist, num_batches)
from .models.net import Net
from .optim import Adadelta, StepLR
from .utils.checkpoint import load_state_dict, save_state_dict
from .utils.logging import print_line, test_line, total_time_line, train_line
from .utils.profiling import PhaseTimes



# training steps per captured chunk (both graphs of a chunk are launched together; a chunk boundary
# costs a fork / join and a host hand-off): 600-step same-box sweep 25 / 50 / 100 -> 65.9 / 65.0-65.8 /
# 65.1-65.2 us a step, and chunks cut at every 10-step log interval 1.4-2.2 us a step more than
# 20-step chunks (profiles/r4/s2/ab/gs_sweep_*.txt); logged losses are read per chunk
DEFAULT_GRAPH_STEPS = 50

def _json_log(path, rec):
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


# ----------------------------------------------------------------------------- module engine
def _check_finite(loss: float, epoch: int, batch_idx: int) -> None:
    if loss != loss or loss in (float("inf"), float("-inf")):     # fail fast
        raise FloatingPointError(f"non-finite training loss {loss} at epoch {epoch} batch {batch_idx}")


def _train_module(args, model, device, loader, optimizer, epoch, distributed, world, rank):
    model.train()
    n_batches = len(loader)
    for batch_idx, (data, target) in enumerate(loader):
        data, target = data.to(device), target.to(device)
        optimizer.zero_grad()
        output = model(data)
        loss = F.nll_loss(output, target)
        loss.backward()
        optimizer.step()
        if batch_idx % args.log_interval == 0 and (not distributed or rank == 0):
            seen = (world if distributed else 1) * batch_idx * len(data)
            lv = loss.item()
            _check_finite(lv, epoch, batch_idx)
            print(train_line(epoch, seen, len(loader.dataset), batch_idx, n_batches, lv))
            if args.dry_run and not getattr(args, "_ddp_script", False):
                break
        if args.dry_run and getattr(args, "_ddp_script", False):
            break


def _test_module(model, device, loader):
    model.eval()
    test_loss, correct = 0.0, 0
    with torch.no_grad():
        for data, target in loader:
            data, target = data.to(device), target.to(device)
            output = model(data)
            test_loss += F.nll_loss(output, target, reduction='sum').item()
            pred = output.argmax(dim=1, keepdim=True)
            correct += pred.eq(target.view_as(pred)).sum().item()
    n = len(loader.dataset)
    test_loss /= n
    print(test_line(test_loss, correct, n))
    return test_loss, correct


# ----------------------------------------------------------------------------- main flows
def run(argv=None, ddp_script: bool = True, t_start: float | None = None, holder: dict | None = None) -> int:
    # startup phases inside the reference timer (--json-log "setup_s") + wall-clock marks since the
    # timer's start ("timeline_s": where the rest goes - epochs, evaluation, teardown)
    setup = PhaseTimes(origin=t_start)
    args = cli.parse_args(ddp=ddp_script, argv=argv)
    if holder is not None:
        holder["args"] = args
    args._ddp_script = ddp_script
    # is_available() brings the HIP runtime up (~60 ms) and device_count() initialises amdsmi
    # (~53 ms, measured under cProfile on the box), both on the main thread inside the timer; the
    # device nodes tell the same here, and the fused engine's HIP init runs on the prewarm thread
    # under the data build (a node without a usable GPU then fails there, loudly)
    use_cuda = not args.no_cuda and gpu_present()
    distributed, world, rank, gpu = False, 1, 0, 0
    args._setup = setup
    setup.mark("args")
    # the prewarm thread starts before the process-group init when this rank's device is already
    # known from the launcher's environment (torchrun: LOCAL_RANK; no launcher: GPU 0)
    fused = use_cuda and (getattr(args, "engine", None) or "fused") == "fused"
    early = _early_device(ddp_script) if fused else None
    args._prewarm = _start_prewarm(early) if early is not None else None
    if ddp_script:
        from .parallel.distributed import init_distributed_mode
        args._defer_set_device = use_cuda and (getattr(args, "engine", None) or "fused") == "fused"
        with setup.phase("pg_init"):
            init_distributed_mode(args)
        distributed = args.distributed
        if distributed:
            world, rank, gpu = args.world_size, args.rank, args.gpu
    if fused:
        # the CPU generator only (model init, samplers, loader seeds: the reference's draws); the
        # fused engine never uses torch's GPU RNG (dropout is in-kernel Philox), and a queued
        # torch.cuda.manual_seed_all would make torch's CUDA init count devices through amdsmi
        # (~53 ms on the prewarm thread, the startup's critical path)
        torch.default_generator.manual_seed(args.seed)
    else:
        torch.manual_seed(args.seed)
    device = torch.device(f"cuda:{gpu}" if use_cuda else "cpu") if ddp_script else \
        torch.device("cuda" if use_cuda else "cpu")
    engine = getattr(args, "engine", None) or ("fused" if use_cuda else "module")
    if not use_cuda:
        engine = "module"
    # the HIP context + the native extension's code objects come up on a helper thread while this
    # one builds the data set and the model's CPU init (joined in _run_fused: "hip_init")
    if args._prewarm is not None and (engine != "fused" or args._prewarm.device != device):
        args._prewarm.join()                 # (a device guess that did not hold: start over)
        args._prewarm = None
    if args._prewarm is None and engine == "fused":
        args._prewarm = _start_prewarm(device)
    # the fused engine's RCCL communicator (PendingRcclComm): with --allreduce rccl / fastest, and
    # under auto across nodes (no xGMI there), its non-blocking init starts now on a helper thread
    # while data, model and trainer are built; under auto on one node it is only created - started
    # by the trainer if the direct xGMI transport cannot be used, never waited for otherwise
    args._pending_comm = None
    allreduce = _allreduce_choice(args)
    if distributed and engine == "fused" and allreduce != "xgmi" and (world > 1 or allreduce != "auto"):
        from .parallel.distributed import start_rccl_comm
        eager = allreduce != "auto" or not _one_node_by_env(world)
        with setup.phase("rccl_comm_start"):
            args._pending_comm = start_rccl_comm(world, rank, gpu, start=eager)

    setup.mark("pg_init")
    with setup.phase("data"):
        train_data = load_mnist(args.data_root, True, args.synthetic, args.synthetic_train_size, verbose=rank == 0)
        test_data = load_mnist(args.data_root, False, args.synthetic, args.synthetic_test_size, verbose=rank == 0)
    setup.mark("data")
    if ddp_script:
        train_stream = (DistributedIndexStream(len(train_data), world, rank, shuffle=True) if distributed
                        else RandomIndexStream(len(train_data)))
        test_stream = SequentialIndexStream(len(test_data))
    else:  # mnist.py: shuffle=True for both loaders only on CUDA (mnist.py:103-110)
        train_stream = RandomIndexStream(len(train_data)) if use_cuda else SequentialIndexStream(len(train_data))
        test_stream = RandomIndexStream(len(test_data)) if use_cuda else SequentialIndexStream(len(test_data))

    model = Net()
    if getattr(args, "dtype", "bf16") == "fp32":     # module engine: stock torch fp32 ops; fused: f32_net.hip
        model.compute_dtype = torch.float32
    if args.resume:
        load_state_dict(model, args.resume, map_location="cpu")

    if engine == "fused":
        _run_fused(args, model, device, train_data, test_data, train_stream, test_stream, distributed, world,
                   rank, gpu, ddp_script)
    else:
        _run_module(args, model, device, train_data, test_data, train_stream, test_stream, distributed, world,
                    rank, gpu, ddp_script)
    return 0


def _run_module(args, model, device, train_data, test_data, train_stream, test_stream, distributed, world, rank,
                gpu, ddp_script):
    if distributed and device.type == "cuda" and getattr(args, "_defer_set_device", False):
        torch.cuda.set_device(gpu)
    model = model.to(device)
    model_without_ddp = model
    if distributed:
        from .parallel.ddp import DistributedDataParallel
        comm = None
        if device.type == "cuda":             # native C++ bucket reducer over the framework's RCCL comm
            from .parallel.distributed import create_rccl_comm
            comm = create_rccl_comm(world, rank, gpu)
        model = DistributedDataParallel(model, device_ids=[gpu] if device.type == "cuda" else None,
                                        bucket_cap_mb=args.bucket_cap_mb, first_bucket_cap_mb=args.first_bucket_mb,
                                        comm=comm)
        model_without_ddp = model.module
    optimizer = Adadelta(model.parameters(), lr=args.lr)
    scheduler = StepLR(optimizer, step_size=1, gamma=args.gamma)
    train_loader = HostLoader(train_data, train_stream, args.batch_size)
    test_loader = HostLoader(test_data, test_stream, args.test_batch_size)
    for epoch in range(1, args.epochs + 1):
        if distributed:
            train_stream.set_epoch(epoch)
        t0 = time.perf_counter()
        _train_module(args, model, device, train_loader, optimizer, epoch, distributed, world, rank)
        rec = {"epoch": epoch, "train_s": time.perf_counter() - t0}
        if not distributed or rank == 0:
            rec["test_loss"], rec["correct"] = _test_module(model_without_ddp, device, test_loader)
        if distributed and args.check_sync:
            from .parallel.ddp import assert_params_in_sync
            assert_params_in_sync(list(model_without_ddp.parameters()))
        _json_log(args.json_log, rec)
        scheduler.step()
    _save(args, model, distributed, rank, ddp_script)


def _stream_kind() -> str:
    from .engine.trainer import stream_kind
    return stream_kind()


def _schedule_name(trainer) -> str | None:
    eng = getattr(trainer, "engine", None)
    return ["serial", "overlap", "rccl", "xgmi"][eng.schedule] if eng is not None else None


def _allreduce_choice(args) -> str:
    return getattr(args, 'allreduce', None) or os.environ.get("MNIST_AMD_ALLREDUCE", "auto")


def _one_node_by_env(world: int) -> bool:
    """The launcher says every rank is on this node (torchrun / torch.distributed.launch export
    LOCAL_WORLD_SIZE); unknown (SLURM without a launcher) counts as "maybe not"."""
    try:
        return int(os.environ.get("LOCAL_WORLD_SIZE", "0")) == world
    except ValueError:
        return False


def close_pending_comm(args) -> None:
    """After the reference's timer: end a cancelled / unused RCCL init's helper thread (bounded) so
    the interpreter never tears down under it."""
    p = getattr(args, "_pending_comm", None)
    if p is not None:
        p.close(30.0)


def gpu_present() -> bool:
    """A GPU is usable by this process: torch is a ROCm build, the KFD + a DRM render node exist and
    are accessible, and HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES do not
    hide every device.  No runtime call (torch.cuda.is_available() brings HIP up: ~60 ms inside the
    reference timer); a node that passes this and still has no usable GPU fails loudly in the
    prewarm thread's runtime init."""
    import glob
    if not getattr(torch.version, "hip", None):       # CPU-only (or non-ROCm) torch build
        return False
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v.strip() in ("", "-1"):
            return False
    nodes = glob.glob("/dev/dri/renderD*")
    return os.access("/dev/kfd", os.R_OK | os.W_OK) and any(os.access(n, os.R_OK | os.W_OK) for n in nodes)


def _prewarm_body(device, steps: dict | None = None) -> None:
    """HIP runtime + context, code objects, torch's CUDA state, an allocator segment and the torch
    kernels the model state / trainer construction use - everything the main thread would otherwise
    pay on first touch inside the reference timer.  The native step runs with the GIL released."""
    steps = {} if steps is None else steps
    t = time.perf_counter()

    def lap(name):
        nonlocal t
        now = time.perf_counter()
        steps[name] = round(now - t, 4)
        t = now

    from .ops import native
    C = native.load()                        # the _C extension (dlopen; no device work)
    lap("native_load")
    # the engine's stream pair before any other stream of the process - the default stream included -
    # so that each has a hardware queue of its own (engine/trainer.py make_streams; brings the
    # runtime and the context up)
    from .engine.trainer import make_streams
    make_streams(device)
    lap("engine_streams")
    # GIL released: the HIP runtime + context, then every kernel TU's code object
    t_rt, t_co, t_cp, t_ms, t_h2d, t_d2h = C.hip_prewarm(device.index if device.index is not None else 0)
    steps["hip_runtime_context"], steps["code_objects"] = round(t_rt, 4), round(t_co, 4)
    steps["memset_copy_paths"] = round(t_cp, 4)
    steps["first_memset"], steps["first_h2d"], steps["first_d2h"] = round(t_ms, 4), round(t_h2d, 4), round(t_d2h, 4)
    lap("hip_prewarm_total")
    torch.cuda.init()
    lap("torch_cuda_init")
    if device.index is not None:
        torch.cuda.set_device(device)        # this thread's device
    torch.empty(1, device=device)
    lap("torch_first_alloc")
    # one 192 MB segment for the caching allocator: the model state, trainer buffers and datasets
    # are then carved from it instead of each paying a hipMalloc on the main thread.  (The setup
    # paths launch no torch kernels at all - native.zeros / H2D copies - so no torch code object
    # has to load inside the timer.)
    torch.empty(192 << 20, dtype=torch.uint8, device=device)
    lap("allocator_segment")


class _Prewarm:
    def __init__(self, device):
        import threading
        self.device, self.error, self.seconds, self.steps = device, None, None, {}
        self._t = threading.Thread(target=self._run, name="hip-prewarm", daemon=True)
        self._t.start()

    def _run(self):
        t0 = time.perf_counter()
        try:
            _prewarm_body(self.device, self.steps)
        except BaseException as e:  # noqa: BLE001 - re-raised by the joining thread
            self.error = e
        self.seconds = time.perf_counter() - t0

    def join(self):
        self._t.join()


def _start_prewarm(device):
    return _Prewarm(device)


def _early_device(ddp_script: bool):
    """This rank's device before init_distributed_mode, where the environment already fixes it:
    mnist.py -> cuda (current device); mnist_ddp.py under torchrun -> cuda:LOCAL_RANK (cuda:0 with
    MNIST_AMD_ONE_GPU=1); without a launcher -> cuda:0; SLURM (rank from the job) -> unknown."""
    if not ddp_script:
        return torch.device("cuda")
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        if os.environ.get("MNIST_AMD_ONE_GPU", "0") == "1":
            return torch.device("cuda:0")
        return torch.device(f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}")
    if "SLURM_PROCID" in os.environ:
        return None
    return torch.device("cuda:0")


def _run_fused(args, model, device, train_data, test_data, train_stream, test_stream, distributed, world, rank,
               gpu, ddp_script):
    from .engine.state import ModelState
    from .engine.trainer import FusedTrainer
    from .utils.profiling import roctx_range
    setup = args._setup
    with setup.phase("hip_init"):            # HIP context, first allocation, _C extension (prewarm thread)
        pw = args._prewarm
        if pw is not None:
            pw.join()
            setup.add_info("prewarm_thread_s", pw.seconds)
            setup.add_info("prewarm_steps_s", pw.steps)
            if pw.error is not None:
                raise pw.error
        else:
            _prewarm_body(device)
        if distributed:
            torch.cuda.set_device(gpu)       # (deferred by init_distributed_mode: runtime is up now)
    allreduce = _allreduce_choice(args)
    xgmi_pending = streams = None
    if distributed and world > 1 and allreduce in ("xgmi", "auto", "fastest"):
        # the trainer's two streams first: the setup thread's self-test streams must not take the
        # hardware queues they would otherwise get (few queues per process in one-GPU rehearsals)
        from .engine.trainer import make_streams
        streams = make_streams(device)
        # the xGMI communicator (IPC export / exchange / peer mapping / self-test) builds on a helper
        # thread while this one builds the model, wraps it and allocates the trainer's buffers
        from .ops import native
        from .parallel.distributed import PendingXgmiComm
        with setup.phase("xgmi_comm_start"):
            xgmi_pending = PendingXgmiComm(world, rank, device, int(native.load().PARAM_TOTAL))
    setup.mark("hip_native")
    t_model = time.perf_counter()
    ms = ModelState(model, device, lr=args.lr)
    model_for_save = model
    comm = None
    two_buckets = True
    setup.add("model", time.perf_counter() - t_model)
    if distributed:
        from .parallel.ddp import DistributedDataParallel, engine_bucket_layout
        with setup.phase("ddp_wrap"):
            ddp = DistributedDataParallel(model, device_ids=[gpu], engine_managed=True,
                                          bucket_cap_mb=args.bucket_cap_mb, first_bucket_cap_mb=args.first_bucket_mb)
        model_for_save = ddp
        two_buckets = engine_bucket_layout(ddp.bucket_indices)   # raises on a layout the engine cannot run
        if allreduce == "xgmi" and not two_buckets:
            raise ValueError("--allreduce xgmi needs the two-bucket layout (default --bucket-cap-mb/--first-bucket-mb)")
    # The optimizer here is the engine's fused Adadelta kernel (state in `ms`); StepLR(step_size=1)
    # (reference mnist_ddp.py:178, :189) reduces to lr <- lr * gamma after every epoch, computed in
    # the same double arithmetic as torch's scheduler and handed to the kernels as a device scalar.
    # (No torch.optim object: constructing one imports torch._dynamo, ~1.6 s inside the timed run.)
    lr = float(args.lr)
    graph_steps = DEFAULT_GRAPH_STEPS if args.graph_steps is None else args.graph_steps
    trainer = FusedTrainer(ms, train_data, test_data if (not distributed or rank == 0) else None,
                           args.batch_size, args.test_batch_size, num_samples=len(train_stream),
                           world_size=world, rank=rank, comm=comm, seed=args.seed, graph_steps=graph_steps,
                           allreduce=allreduce, two_buckets=two_buckets,
                           fp32=getattr(args, "dtype", "bf16") == "fp32", xgmi_pending=xgmi_pending,
                           streams=streams, rccl_pending=args._pending_comm)
    if xgmi_pending is not None:
        setup.add_info("xgmi_setup_thread_s", xgmi_pending.seconds)
    setup.mark("trainer")
    if distributed and rank == 0 and trainer.allreduce_timings:
        # stderr: stdout carries exactly the reference's line kinds
        print(f"| gradient all-reduce: {trainer.allreduce} (schedule us/step: {trainer.allreduce_timings})",
              file=sys.stderr, flush=True)
    if args.profile:
        trainer.profile_left = args.profile_steps
    n_train = len(train_data)
    n_batches = num_batches(len(train_stream), args.batch_size)
    log_rank = (not distributed) or rank == 0
    # Epoch pipelining: the evaluation after epoch e is enqueued behind its training and read back
    # while epoch e+1's first chunks run; its test line is printed (from train_epoch's before_log
    # hook) before any train line of e+1, and the next epoch's sampler order is drawn on the host
    # while the GPU works - the same lines, values and RNG draw order (train base seed, sampler
    # permutation, test base seed [, test permutation], next epoch's train base seed, ...) as the
    # reference's sequential loop, without a host sync and an idle GPU at every epoch boundary.
    # --check-sync compares parameters after each epoch, which needs the sequential form.
    pipelined = not (distributed and args.check_sync) and not args.profile

    def next_indices(epoch):
        if distributed:
            train_stream.set_epoch(epoch)
        consume_loader_base_seed()          # iter(train_loader)
        return train_stream.epoch_indices()

    def finish(p):
        """Epoch p["epoch"]'s test line, sync check and JSON record (its evaluation is complete or
        completes here)."""
        epoch, st, rec = p["epoch"], p["st"], p["rec"]
        if p["handle"] is not None:
            loss_sum, correct, n = p["handle"].result()
            print(test_line(loss_sum / n, correct, n))
            rec.update(test_loss=loss_sum / n, correct=correct)
            setup.mark(f"epoch{epoch}_eval")
        dev_s = st.device_time()
        if pipelined:
            # the epoch's work is complete (its end event): fail at the first bad epoch, as the
            # sequential form does in train_epoch - a stream hand-off or xGMI stage timeout would
            # otherwise surface only after the last epoch (two 4-byte reads)
            trainer.check_errors()
        rec["device_train_s"] = dev_s
        if dev_s:
            rec["device_img_per_s"] = st.samples / dev_s
            if pipelined:                     # host time is enqueue time here: report the device's
                rec["host_train_s"], rec["train_s"] = rec["train_s"], dev_s
        if distributed and args.check_sync:
            from .parallel.ddp import assert_params_in_sync
            trainer.synchronize()
            assert_params_in_sync([ms.param])
        _json_log(args.json_log, rec)

    idx = next_indices(1)
    pend = None
    for epoch in range(1, args.epochs + 1):
        trainer.set_lr(lr)

        def log_fn(batch_idx, blen, loss, epoch=epoch):
            _check_finite(loss, epoch, batch_idx)
            seen = (world if distributed else 1) * batch_idx * blen
            print(train_line(epoch, seen, n_train, batch_idx, n_batches, loss), flush=False)

        hook = (lambda p=pend: finish(p)) if pend is not None else None
        with roctx_range(f"train_epoch_{epoch}", args.profile):
            st = trainer.train_epoch(epoch, idx, args.log_interval, dry_run=args.dry_run,
                                     log_fn=log_fn if log_rank else None, sync=not pipelined, before_log=hook)
        pend = None
        setup.mark(f"epoch{epoch}_train")
        if epoch == 1:                     # the trainer's phases include epoch 1's graph captures
            setup.update(trainer.setup, prefix="trainer.")
            # (t_start_unix / trainer_ready_unix: the node's wall clock at the timer's start and when the
            # trainer was ready, so a multi-rank table can separate the launcher's start skew between
            # ranks - which the first collective absorbs - from the startup's own critical path)
            _json_log(args.json_log, {"setup_s": setup.rounded(), "setup_total_s": round(setup.total(), 4),
                                      "setup_info": setup.info, "allreduce": trainer.allreduce if distributed else None,
                                      "transport_report": trainer.transport_report or None,
                                      "schedule": _schedule_name(trainer), "streams": _stream_kind(),
                                      "t_start_unix": setup.origin,
                                      "trainer_ready_unix": setup.origin + setup.marks.get("trainer", 0.0)})
        rec = {"epoch": epoch, "train_s": st.train_seconds, "steps": st.steps,
               "img_per_s": st.samples / max(st.train_seconds, 1e-9)}
        handle = None
        if log_rank:
            consume_loader_base_seed()      # iter(test_loader)
            if isinstance(test_stream, RandomIndexStream):
                test_stream.epoch_indices()  # mnist.py CUDA path shuffles the test set: same RNG draw
            with roctx_range(f"eval_epoch_{epoch}", args.profile):
                handle = trainer.evaluate_async()
        if epoch < args.epochs:
            idx = next_indices(epoch + 1)   # host work under the evaluation / the epoch's tail
        pend = {"epoch": epoch, "st": st, "rec": rec, "handle": handle}
        if not pipelined:
            finish(pend)
            pend = None
        lr = lr * args.gamma                                   # scheduler.step()
    if pend is not None:
        finish(pend)
    trainer.synchronize()                 # (raises on a device hand-off / xGMI stage timeout)
    setup.mark("train_done")
    _save(args, model_for_save, distributed, rank, ddp_script)
    setup.mark("saved")
    _json_log(args.json_log, {"timeline_s": setup.marks})


def _save(args, model, distributed, rank, ddp_script):
    if not args.save_model:
        return
    if not ddp_script:
        save_state_dict(model, "mnist_cnn.pt")
    elif distributed:
        if rank == 0:
            save_state_dict(model, "mnist_cnn.pt")
    else:
        save_state_dict(model, "mnist_cnn_.pt")


def _fatal_exit(e: BaseException) -> None:
    """A collective stuck on the device (``TransportHang``: ``fatal``) cannot be cancelled, and the
    interpreter's teardown of the RCCL / HIP objects would wait for it: report, tell the other ranks
    through the store, and leave without the runtime's teardown (as bench.py does)."""
    print(f"FATAL: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
    try:
        from .parallel.hostcomm import get_hostcomm
        get_hostcomm().abort(f"{type(e).__name__}: {e}"[:300])
    except Exception:  # noqa: BLE001 - no process group / store: nothing to tell
        pass
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(3)


def main_mnist(argv=None) -> int:
    try:
        return run(argv, ddp_script=False)
    except BaseException as e:  # noqa: BLE001
        if getattr(e, "fatal", False):
            _fatal_exit(e)
        raise


def main_mnist_ddp(argv=None) -> int:
    start = time.time()
    holder = {}
    try:
        rc = run(argv, ddp_script=True, t_start=start, holder=holder)
    except BaseException as e:  # noqa: BLE001
        if getattr(e, "fatal", False):
            _fatal_exit(e)
        raise
    print_line(total_time_line(time.time() - start))
    sys.stdout.flush()
    if "args" in holder:
        close_pending_comm(holder["args"])
    return rc
