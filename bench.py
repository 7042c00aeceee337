#!/usr/bin/env python3
"""Headline benchmark: MNIST CNN DDP training throughput on N MI355X (one process per GPU).

Metric (BASELINE.json): "images/sec + 20-epoch wallclock, MNIST CNN DDP at 1/2/4/8 MI355X",
config = the reference README run (`mnist_ddp.py --batch-size 200 --epochs 20`, batch per GPU,
reference README.md:41-61): the reference `Net` (random init, seed 1), Adadelta(lr=1) + dropout,
DistributedSampler sharding of a 60,000-image synthetic 28x28 uint8 train split (no network),
bf16 MFMA compute with fp32 master weights / optimizer state / gradient all-reduce.

One "step" = everything the reference does per batch: gather+normalise the batch, forward,
NLL loss, backward, DDP gradient averaging over RCCL, Adadelta update.  W untimed warmup steps,
then exactly K steps bracketed by barrier + device synchronize on both sides; the reported
time is the max over ranks; ``value`` is the whole-job images/s (N * B * K / t).

With ``--full-run`` (default on) it then also measures the README's complete workload twice:

* ``total_cost_time_s`` - the reference's own metric, measured the reference's way: rank 0 launches
  ``mnist_ddp.py --batch-size B --epochs 20 --synthetic`` as a child job at the same N (plain
  ``python`` for N=1, ``torch.distributed.run`` for N>1, README.md:41-51) and reports the max over
  its ranks of the script's ``Total cost time`` line (mnist_ddp.py:200-203: PG init, data load, DDP
  construction, 20 x (train with the rank-0 loss prints every 10 batches + rank-0 eval));
* ``wallclock_20ep_s`` - the same 20 epochs timed in-process on already-built trainers (excludes
  PG init, data build, model init and communicator setup; no per-10-batch log syncs).

After the timed steps every rank's parameters are fingerprinted and compared (``params_in_sync``;
the run fails if they differ), and the JSON names the all-reduce actually used (``allreduce``,
``rccl_world``, probe timings, the xGMI startup validation and kernel grids).
``--cpu`` instead measures the reference's CPU config (``mnist.py --no-cuda``, batch 64) on this
host's CPU cores against BASELINE.md's 3,518 img/s anchor.

Launch: ``python bench.py`` (1 GPU), ``python bench.py --gpus N`` (bench.py starts its N ranks
itself: a ``torch.distributed.run --standalone`` child job, launched before this process touches a
GPU, whose rank 0 JSON line is re-printed), or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N``.

If any rank fails (transport setup, startup validation, a hang caught by a watchdog, a desync),
rank 0 still prints ONE JSON line - ``value`` null, ``error`` and every rank's failure record
(decoded error, transport, setup phases) - and the exit code is non-zero.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import re
import subprocess
import sys
import time
from datetime import timedelta

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from pytorch_mnist_ddp_amd.data.datasets import load_mnist  # noqa: E402
from pytorch_mnist_ddp_amd.data.samplers import DistributedIndexStream  # noqa: E402
from pytorch_mnist_ddp_amd.engine.state import ModelState  # noqa: E402
from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer, stream_kind  # noqa: E402
from pytorch_mnist_ddp_amd.models.net import Net  # noqa: E402
from pytorch_mnist_ddp_amd.parallel.distributed import (_max_over_ranks, barrier,  # noqa: E402
                                                        params_fingerprint_equal, start_rccl_comm)
from pytorch_mnist_ddp_amd.utils.profiling import PhaseTimes  # noqa: E402

METRIC = "images/sec + 20-epoch wallclock, MNIST CNN DDP at 1/2/4/8 MI355X"
CPU_ANCHOR_IMG_S = 3518.0      # torch fp32 CPU train step, B=64, 8 vCPU dev box
_LAUNCH_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
               "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")


def run_reference_script(world: int, batch: int, epochs: int, timeout: float = 900.0, extra=(),
                         with_setup: bool = True) -> dict:
    """The reference's README command at this N (mnist_ddp.py, README.md:41-51) as a child job;
    returns the max over ranks of its ``Total cost time`` print, the child's wall time, the last
    printed test accuracy and (``with_setup``: ``--json-log``) the per-phase startup seconds inside
    that timer (max over ranks per phase) plus the summed per-epoch train/eval time."""
    import tempfile
    script = os.path.join(ROOT, "mnist_ddp.py")
    jlog = tempfile.NamedTemporaryFile(prefix="mnist_amd_child_", suffix=".jsonl", delete=False).name
    sargs = ["--batch-size", str(batch), "--epochs", str(epochs), "--synthetic", *extra]
    if with_setup:
        sargs += ["--json-log", jlog]
    env = {k: v for k, v in os.environ.items() if k not in _LAUNCH_ENV and not k.startswith("TORCHELASTIC")}
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    if world == 1:
        cmd = [sys.executable, script] + sargs
    else:
        # --standalone: the launcher binds its own free port (no pick-then-bind race with other jobs)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
               "--nnodes", "1", "--nproc-per-node", str(world), script] + sargs
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    wall = time.perf_counter() - t0
    times = [float(x) for x in re.findall(r"Total cost time:([0-9.eE+-]+) ms", r.stdout)]
    accs = re.findall(r"Accuracy: (\d+)/(\d+)", r.stdout)
    out = {"cmd": " ".join(["python"] + cmd[1:]).replace(ROOT + "/", ""), "rc": r.returncode,
           "total_cost_time_s": round(max(times), 3) if times else None, "ranks_reporting": len(times),
           "child_wall_s": round(wall, 2),
           "test_acc": round(int(accs[-1][0]) / int(accs[-1][1]), 4) if accs else None}
    if r.returncode != 0 or len(times) != world:
        out["stderr_tail"] = r.stderr[-1500:]
    if with_setup:
        try:
            recs = [json.loads(ln) for ln in open(jlog) if ln.strip()]
            setups = [rc["setup_s"] for rc in recs if "setup_s" in rc]
            infos = [rc["setup_info"] for rc in recs if rc.get("setup_info")]
            if infos:                # helper-thread timings (prewarm steps, RCCL init) of the first rank logged
                out["setup_info"] = infos[0]
            if setups:
                keys = list(dict.fromkeys(k for st in setups for k in st))
                out["setup_phases_s"] = {k: round(max(st.get(k, 0.0) for st in setups), 3) for k in keys}
                out["setup_total_s"] = round(max(sum(st.values()) for st in setups), 3)
            ep = [rc for rc in recs if "epoch" in rc]
            if ep:
                out["epochs_train_s_rank_sum"] = round(sum(rc.get("train_s", 0.0) for rc in ep), 3)
            tls = [rc["timeline_s"] for rc in recs if "timeline_s" in rc]
            if tls:                  # wall-clock marks since the timer's start, max over ranks
                keys = list(dict.fromkeys(k for t in tls for k in t))
                tl = {k: max(t.get(k, 0.0) for t in tls) for k in keys}
                out["timeline_s"] = {k: tl[k] for k in keys if not k.startswith("epoch") or k.startswith(("epoch1_", f"epoch{epochs}_"))}
                out["timeline_epochs_s"] = round(tl.get(f"epoch{epochs}_eval", tl.get(f"epoch{epochs}_train", 0.0))
                                                 - tl.get("trainer", 0.0), 3)
        except (OSError, ValueError):
            pass
        finally:
            try:
                os.unlink(jlog)
            except OSError:
                pass
    return out


def cpu_bench(steps: int, warmup: int, batch: int = 64) -> int:
    """Reference config 1 (mnist.py --no-cuda, batch 64): the module engine's fp32 CPU train step."""
    import torch.nn.functional as F
    from pytorch_mnist_ddp_amd.optim import Adadelta
    torch.manual_seed(1)
    net = Net()
    opt = Adadelta(net.parameters(), lr=1.0)
    train = load_mnist(train=True, synthetic_data=True, verbose=False)
    x_all = ((train.images[: (warmup + steps) * batch].float() / 255.0 - 0.1307) / 0.3081).reshape(-1, 1, 28, 28)
    y_all = train.targets[: (warmup + steps) * batch].long()

    def step(i):
        x, y = x_all[i * batch:(i + 1) * batch], y_all[i * batch:(i + 1) * batch]
        opt.zero_grad()
        loss = F.nll_loss(net(x), y)
        loss.backward()
        opt.step()
        return loss
    def timed():
        net.train()
        for i in range(warmup):
            step(i)
        t0 = time.perf_counter()
        for i in range(warmup, warmup + steps):
            loss = step(i)
        return time.perf_counter() - t0, loss
    dt, loss = timed()
    img_s = batch * steps / dt
    # the same loop with stock torch.optim.Adadelta on this host (the anchor was measured elsewhere)
    torch.manual_seed(1)
    net = Net()
    opt = torch.optim.Adadelta(net.parameters(), lr=1.0)
    dt_stock, _ = timed()
    print(json.dumps({"metric": "images/sec, MNIST CNN train step on CPU (mnist.py --no-cuda config)",
                      "value": round(img_s, 1), "unit": "images/s", "n_gpus": 0, "steps": steps, "warmup": warmup,
                      "ms_per_step": round(1000 * dt / steps, 3), "higher_is_better": True, "scaling": "strong",
                      "vs_baseline": round(img_s / CPU_ANCHOR_IMG_S, 3), "dtype": "fp32",
                      "data": "synthetic 28x28 uint8 (normalised on the host); random-init weights",
                      "config": {"model": "mnist_cnn", "global_batch": batch, "seq_len": None, "parallelism": "none",
                                 "threads": torch.get_num_threads()},
                      "stock_torch_img_s": round(batch * steps / dt_stock, 1),
                      "vs_stock_torch_same_host": round(dt_stock / dt, 3),
                      "last_train_loss": round(float(loss.item()), 4)}), flush=True)
    return 0
# reference README.md:55-59 (20-epoch wallclock at B=200/GPU) -> images/s = 20*60000/t
BASELINE_WALLCLOCK = {1: 242.3, 2: 137.1, 4: 73.6}
TRAIN_N, TEST_N, EPOCHS = 60000, 10000, 20
_FAIL_KEY = "bench/fail"


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 600; --cpu: 200)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed warmup steps (default 50; --cpu: 10)")
    ap.add_argument("--batch-size", type=int, default=200, help="per-GPU batch (README config: 200)")
    ap.add_argument("--graph-steps", type=int, default=50, help="steps per captured hipGraph (0 = eager; 50 as the driver)")
    ap.add_argument("--single-bucket", action="store_true", help="one all-reduce per step (no overlap)")
    ap.add_argument("--no-full-run", dest="full_run", action="store_false")
    ap.add_argument("--epochs", type=int, default=EPOCHS, help="epochs for the full-run wallclock")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--force-comm", action="store_true",
                    help="attach the RCCL communicator even at world_size 1 (exercises the DDP schedule)")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16",
                    help="bf16: the bf16-MFMA step (default); fp32: the fp32 step (f32_net.hip; RCCL or xGMI at N > 1)")
    ap.add_argument("--allreduce", choices=["auto", "rccl", "xgmi", "fastest"],
                    default=os.environ.get("MNIST_AMD_ALLREDUCE", "auto"),
                    help="DDP gradient all-reduce: RCCL, the direct xGMI reduce-scatter/all-gather kernels, auto "
                         "(xGMI when its production schedule validates on one node; RCCL only as the fallback, "
                         "never waited for otherwise) or fastest (validate and time both, keep the faster)")
    ap.add_argument("--hook", action="append", default=[], metavar="NAME=VALUE",
                    help="engine variant for A/B runs (FusedTrainer.HOOKS: fc_dw1_side=0|1, dgrad_grid=N)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend (gloo + --allreduce xgmi: no RCCL, e.g. MNIST_AMD_ONE_GPU=1 rehearsals)")
    ap.add_argument("--cpu", action="store_true", help="reference CPU config (mnist.py --no-cuda, batch 64)")
    ap.add_argument("--no-script-run", dest="script_run", action="store_false",
                    help="skip the mnist_ddp.py child job (total_cost_time_s)")
    ap.add_argument("--script-last", dest="script_first", action="store_false",
                    help="run the mnist_ddp.py child job after this process's own run, beside its idle GPU "
                         "contexts (default: first, before any rank of this job touches a GPU - as a user "
                         "runs the command)")
    ap.add_argument("--no-warm-replay", dest="warm_replay", action="store_false",
                    help="do not replay the timed region's graphs (state restored) before the warmup")
    ap.add_argument("--warm-replay-steps", type=int, default=int(os.environ.get("MNIST_AMD_WARM_STEPS", "500")),
                    help="replay the timed region's graphs for at least this many steps before the warmup "
                         "(model / optimizer / step state restored bit for bit; 0 = one round).  The GPU's "
                         "clocks ramp over ~10 ms of load: a 20-step window opened on a device that ran "
                         "only the warmup reads 67.8-68.3 us/step of device time, after 500 warm steps "
                         "65.7-65.9 (600 steps: 64.7); profiles/r5/ab/warm_replay_steps.txt")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- self-launch
def self_launch(args, argv) -> int:
    """``--gpus N > 1`` without a launcher: start N ranks as a ``torch.distributed.run`` child job
    (this process never touches a GPU - no HIP context to inherit or exec away from), forward the
    child's output, and re-print rank 0's single JSON line (with ``launcher`` added)."""
    n = args.gpus
    one_gpu = os.environ.get("MNIST_AMD_ONE_GPU", "0") == "1"
    have = torch.cuda.device_count()          # (does not initialise HIP on this image)
    if not one_gpu and have < n:
        msg = (f"bench.py: --gpus {n} needs {n} visible GPUs, this node shows {have} "
               f"(HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES); one-GPU rehearsal: MNIST_AMD_ONE_GPU=1 "
               f"--dist-backend gloo --allreduce xgmi")
        print(msg, file=sys.stderr, flush=True)
        print(json.dumps({"metric": METRIC, "value": None, "unit": "images/s", "n_gpus": n, "steps": args.steps,
                          "warmup": args.warmup, "higher_is_better": True, "error": msg}), flush=True)
        return 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           "--nnodes", "1", "--nproc-per-node", str(n), os.path.abspath(__file__)] + list(argv)
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC")}
    t0 = time.perf_counter()
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, text=True, env=env, cwd=ROOT)
    lines = []
    for ln in proc.stdout:                       # forwarded as it arrives (progress for long runs)
        if ln.lstrip().startswith("{") and '"metric"' in ln:
            lines.append(ln.strip())
        else:
            sys.stdout.write(ln)
            sys.stdout.flush()
    rc = proc.wait()
    wall = time.perf_counter() - t0
    out = None
    for ln in lines:
        try:
            out = json.loads(ln)
        except ValueError:
            continue
    if out is None:
        out = {"metric": METRIC, "value": None, "unit": "images/s", "n_gpus": n, "steps": args.steps,
               "warmup": args.warmup, "higher_is_better": True,
               "error": f"the {n}-rank child job exited with {rc} without a result line"}
    out["launcher"] = {"kind": "bench.py self-launch (torch.distributed.run --standalone child)",
                       "child_rc": rc, "child_wall_s": round(wall, 2)}
    print(json.dumps(out), flush=True)
    return rc if rc != 0 else (0 if out.get("value") is not None else 1)


# ----------------------------------------------------------------------------- failure records
class Diag:
    """What a rank knows when it fails: the phase it was in, the transport, the setup seconds."""

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        self.phase = "start"
        self.phases = PhaseTimes()
        self.tr = None
        self.pending = None           # the PendingRcclComm, if any

    def record(self, exc: BaseException) -> dict:
        if getattr(exc, "setup", None) is not None:       # the trainer's phases up to the failure
            self.phases.update(exc.setup, prefix="trainer.")
        rec = {"rank": self.rank, "phase": self.phase, "error": f"{type(exc).__name__}: {exc}"[:4000],
               "setup_phases_s": self.phases.rounded(3)}
        if getattr(exc, "transport_report", None) is not None:
            rec["transport_report"] = exc.transport_report
        tr = self.tr
        if tr is not None:
            rec.update(allreduce=tr.allreduce, transport_report=tr.transport_report or None)
            try:
                e = tr.engine.errors()
                rec["device_errors"] = {"handoff_timeout": bool(e[0]),
                                        "xgmi": tr.C.Engine.describe_xgmi_error(e[1]) if e[1] else None}
            except Exception:  # noqa: BLE001 - the device may be unusable
                pass
        return rec


def _publish_failure(rec: dict, use_pg: bool) -> None:
    if not use_pg:
        return
    try:
        store = dist.distributed_c10d._get_default_store()
        store.set(f"{_FAIL_KEY}/{rec['rank']}", json.dumps(rec))
        from pytorch_mnist_ddp_amd.parallel.hostcomm import get_hostcomm
        get_hostcomm().abort(f"rank {rec['rank']} failed in {rec['phase']}: {rec['error'][:300]}")
    except Exception:  # noqa: BLE001
        pass


def _collect_failures(world: int, wait_s: float = 5.0) -> dict:
    """Rank 0: every rank's published failure record (waits briefly for the others')."""
    out = {}
    try:
        store = dist.distributed_c10d._get_default_store()
    except Exception:  # noqa: BLE001
        return out
    t0 = time.perf_counter()
    while True:
        for q in range(world):
            k = f"{_FAIL_KEY}/{q}"
            if q not in out and store.check([k]):
                out[q] = json.loads(store.get(k))
        if len(out) == world or time.perf_counter() - t0 > wait_s:
            return out
        time.sleep(0.1)


# ----------------------------------------------------------------------------- the rank's run
def run_rank(args, world: int, rank: int, local: int, diag: Diag) -> dict | None:
    phases = diag.phases             # host seconds per setup phase (JSON "setup_phases_s")
    t_setup = time.perf_counter()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    from pytorch_mnist_ddp_amd.engine.trainer import make_streams
    make_streams(dev)          # the engine's stream pair first: hardware queues of their own
    use_pg = world > 1 or (args.force_comm and "MASTER_ADDR" in os.environ)
    pending = None
    if use_pg:
        diag.phase = "pg_init"
        with phases.phase("pg_init"):
            # lazy (no device_id): ProcessGroupNCCL never builds a communicator - the engine's all-reduce
            # runs on its own RCCL communicator or the xGMI kernels, verdicts over the TCPStore
            if not dist.is_initialized():       # (the reference-first child job initialised it)
                dist.init_process_group(args.dist_backend, init_method="env://", world_size=world, rank=rank)
        if args.allreduce != "xgmi":
            # the RCCL communicator (as the driver): rccl / fastest start its non-blocking init now, while
            # data and model build; auto on one node defers it - the trainer starts it only if xGMI fails
            eager = args.allreduce != "auto" or int(os.environ.get("LOCAL_WORLD_SIZE", "0")) != world
            with phases.phase("rccl_comm_start"):
                pending = start_rccl_comm(world, rank, local, start=eager)
    diag.pending = pending
    xgmi_pending = streams = None
    probe_world1 = world == 1 and use_pg and args.allreduce in ("auto", "fastest")
    if (world > 1 or probe_world1) and args.allreduce != "rccl":   # the xGMI communicator (helper thread)
        from pytorch_mnist_ddp_amd.engine.trainer import make_streams
        from pytorch_mnist_ddp_amd.ops import native
        from pytorch_mnist_ddp_amd.parallel.distributed import PendingXgmiComm
        streams = make_streams(dev)              # (the trainer's streams before the thread's)
        with phases.phase("xgmi_comm_start"):
            xgmi_pending = PendingXgmiComm(world, rank, dev, int(native.load().PARAM_TOTAL))

    B = args.batch_size
    diag.phase = "data_model"
    with phases.phase("data_model"):
        torch.manual_seed(args.seed)
        net = Net()
        train = load_mnist(train=True, synthetic_data=True, verbose=False)
        test = load_mnist(train=False, synthetic_data=True, verbose=False) if rank == 0 else None
        sampler = DistributedIndexStream(len(train), world, rank, shuffle=True, seed=0)
        total = args.warmup + args.steps
        steps_per_epoch = math.ceil(len(sampler) / B)
        num_samples = max(total * B, steps_per_epoch * B)
        ms = ModelState(net, dev, lr=1.0)
    diag.phase = "trainer"
    t_tr = time.perf_counter()
    hooks = dict(h.split("=", 1) for h in args.hook)
    tr = FusedTrainer(ms, train, test, B, 1000, num_samples=num_samples, world_size=world, rank=rank,
                      seed=args.seed, graph_steps=args.graph_steps,
                      two_buckets=not args.single_bucket, allreduce=args.allreduce,
                      fp32=args.dtype == "fp32", xgmi_pending=xgmi_pending, streams=streams,
                      rccl_pending=pending, probe_world1=probe_world1, hooks=hooks)
    comm = tr.comm
    diag.tr = tr
    phases.add("trainer", time.perf_counter() - t_tr)

    # flat index stream = consecutive DistributedSampler epochs, full batches only
    diag.phase = "capture"
    parts, ep = [], 1
    while sum(p.numel() for p in parts) < total * B:
        sampler.set_epoch(ep)
        idx = sampler.epoch_indices()
        parts.append(idx[: (idx.numel() // B) * B])
        ep += 1
    stream = torch.cat(parts)[: total * B]
    tr.start_stream(stream, gather=False)
    cap0 = tr.setup.s.get("graph_capture", 0.0)
    tr.precapture(args.warmup)
    tr.precapture(args.steps)
    phases.add("graph_capture", tr.setup.s.get("graph_capture", 0.0) - cap0)
    warm_steps = 0
    if args.warm_replay and args.steps > 0:
        # every graph the timed region replays has run once before t0 (model, optimizer and step
        # state restored bit for bit): the first timed replay pays no first-launch cost, and exactly
        # --steps steps are timed after exactly --warmup warmup steps
        diag.phase = "warm_replay"
        with phases.phase("warm_replay"):
            first = sum(set(tr._chunks(args.steps))) if tr.use_graphs else 0   # rows the replays read
            tr.engine.gather_rows(0, min(total, max(first, args.warmup)) * B)
            warm_steps = tr.warm_graphs(args.steps, args.warm_replay_steps)
    diag.phase = "warmup"
    tr.engine.gather_rows(0, args.warmup * B)
    tr.run_steps(args.warmup)
    tr.synchronize()
    if use_pg:
        barrier()
    torch.cuda.synchronize()
    diag.phase = "timed"
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(tr.compute)                                   # device-side view of the same window (the
    t0 = time.perf_counter()                                 # streams are idle: it completes at once)
    tr.engine.gather_rows(args.warmup * B, args.steps * B)   # the device DataLoader work is timed too
    tr.run_steps(args.steps)
    ev1.record(tr.compute)                                   # (after the chunk's join: all streams)
    t_enq = time.perf_counter()                              # host: every timed chunk enqueued
    torch.cuda.synchronize()                                 # every stream of the device
    if use_pg:
        barrier()
    t1 = time.perf_counter()
    tr.check_errors()          # device hand-off / xGMI error flags of the timed steps (after the clock)
    elapsed = t1 - t0
    elapsed = _max_over_ranks(elapsed)
    final_loss = float(tr.loss_log[(total - 1) % tr.loss_log.numel()].item()) if tr.loss_log.numel() else float("nan")
    img_s = world * B * args.steps / elapsed
    # DDP correctness of the timed run: every rank must hold bitwise identical parameters
    diag.phase = "params_in_sync"
    in_sync = True
    if use_pg:
        in_sync = params_fingerprint_equal(ms.param)
    comm_info = {"allreduce": tr.allreduce,
                 "rccl_world": comm.world_size if comm is not None else None,
                 "rccl_comms": 1 if comm is not None else 0,
                 "rccl_aborted": bool(comm.aborted) if comm is not None else None,
                 "rccl_init": pending.status if pending is not None else None,
                 "hooks": hooks or None,
                 "allreduce_schedule_us": tr.allreduce_timings or None,
                 "transport_report": tr.transport_report or None,
                 "xgmi_validation": tr.xgmi_validation,
                 "xgmi_ordering": tr.xgmi.ordering if tr.xgmi is not None else None,
                 "xgmi_grids": ({k: v for k, v in tr.xgmi.grids.items() if not k.startswith("cap")}
                                if tr.xgmi is not None else None),
                 "schedule": ["serial", "overlap", "rccl", "xgmi"][tr.engine.schedule],
                 "streams": stream_kind()}
    phases.update(tr.setup, prefix="trainer.")
    # bimodal-slowdown guard (docs/DEBUGGING.md): the timed window against the same schedule's startup
    # validation replay (max over ranks, dropout off); > 1.25x flags a slow mode loudly
    sched_us = tr.allreduce_timings.get(tr.allreduce) if tr.allreduce else None
    slowdown = round(1e6 * elapsed / args.steps / sched_us, 3) if sched_us else None
    if slowdown is not None and slowdown > 1.25 and rank == 0:
        print(f"bench.py: SLOW MODE - {1e6 * elapsed / args.steps:.1f} us/step is {slowdown}x the {tr.allreduce} "
              f"schedule's validation replay ({sched_us} us/step)", file=sys.stderr, flush=True)
    comm_info.update(schedule_slowdown=slowdown, slow_mode=bool(slowdown is not None and slowdown > 1.25))

    # ---- the README workload end to end: 20 epochs train + rank-0 eval, fresh model, on the SAME
    # trainer (engine, graphs, communicators, transport choice and validation reused, state reset)
    wall = None
    acc = None
    desync_epoch = None
    if args.full_run and rank == 0:
        tr.evaluate()         # untimed, like the training kernels above: load the eval kernels' code
    if args.full_run:
        diag.phase = "full_run"
        from pytorch_mnist_ddp_amd.parallel.ddp import params_fingerprint
        torch.manual_seed(args.seed)
        tr.reset_model(Net())
        if use_pg:
            tr.broadcast_params()
        fps = []
        if use_pg:
            with torch.cuda.stream(tr.compute):
                params_fingerprint([ms.param])      # load its kernels' code outside the timed window
        tr.synchronize()
        if use_pg:
            barrier()
        torch.cuda.synchronize()
        w0 = time.perf_counter()
        sampler.set_epoch(1)
        idx = sampler.epoch_indices()
        pending = None
        for epoch in range(1, args.epochs + 1):
            tr.set_lr(1.0 * (0.7 ** (epoch - 1)))
            tr.train_epoch(epoch, idx, sync=False)       # enqueued; the GPU runs while the host
            if pending is not None:                      # reads the previous epoch's evaluation
                ls, correct, n = pending.result()
                acc = correct / max(1, n)
            if use_pg:                                   # per-epoch cross-rank fingerprint, on the
                with torch.cuda.stream(tr.compute):      # device (compared after the run: no sync)
                    fps.append(params_fingerprint([ms.param]))
            if rank == 0:
                pending = tr.evaluate_async()
            if epoch < args.epochs:                      # draws the next epoch's sampler order
                sampler.set_epoch(epoch + 1)
                idx = sampler.epoch_indices()
        if pending is not None:
            ls, correct, n = pending.result()
            acc = correct / max(1, n)
        tr.synchronize()
        if use_pg:
            barrier()
        w1 = time.perf_counter()
        wall = w1 - w0
        wall = _max_over_ranks(wall)
        if use_pg:                                       # which epoch (if any) first desynced
            from pytorch_mnist_ddp_amd.parallel.hostcomm import get_hostcomm
            mine = torch.stack(fps).cpu()
            allv = get_hostcomm().all_gather_bytes(mine.numpy().tobytes())
            per = [torch.frombuffer(bytearray(b), dtype=torch.int64).view(mine.shape) for b in allv]
            for e in range(len(fps)):
                if any(not torch.equal(v[e], per[0][e]) for v in per):
                    desync_epoch = e + 1
                    in_sync = False
                    break

    # ---- the reference's own metric, measured the reference's way (child job at the same N)
    script = getattr(args, "_script_first", None)
    if args.full_run and args.script_run and not args.script_first:
        diag.phase = "reference_script"
        torch.cuda.synchronize()
        if use_pg:
            barrier()
        if rank == 0:
            try:
                script = run_reference_script(world, B, args.epochs, extra=_script_extra(args))
            except Exception as e:  # noqa: BLE001 - reported in the JSON
                script = {"error": f"{type(e).__name__}: {e}"}
        if use_pg:   # the other ranks wait on the store (host-side), leaving their GPUs to the child job
            store = dist.distributed_c10d._get_default_store()
            if rank == 0:
                store.set("bench/script_done", "1")
            else:
                store.wait(["bench/script_done"], timedelta(seconds=1200))

    base = BASELINE_WALLCLOCK.get(world)
    base_img_s = (EPOCHS * TRAIN_N / base) if base else None
    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(img_s, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / base_img_s, 2) if base_img_s else None,
            "dtype": args.dtype,
            "data": "synthetic (60k/10k 28x28 uint8, deterministic); random-init weights",
            "config": {"model": "mnist_cnn (reference Net: conv32-conv64-maxpool-fc128-fc10, 1.2M params)",
                       "global_batch": B * world, "batch_per_gpu": B, "seq_len": None,
                       "parallelism": f"dp{world}", "optimizer": "Adadelta(lr=1.0)",
                       "graph_steps": args.graph_steps, "buckets": 1 if args.single_bucket else 2,
                       "warm_replay": bool(args.warm_replay), "warm_replay_steps": warm_steps, **comm_info},
            "params_in_sync": in_sync,
            "desync_epoch": desync_epoch,
            "total_cost_time_s": script.get("total_cost_time_s") if script else None,
            # the synthetic split is generated in-process by every run (native generator v3, no disk
            # cache), so the reference-timer run above IS the cold start; its data phase is reported
            "total_cost_time_cold_s": script.get("total_cost_time_s") if script else None,
            "synthetic_data": {"generator": "v3 native (csrc/data/synthetic_gen.cpp)", "disk_cache": None,
                               "child_data_phase_s": ((script or {}).get("setup_phases_s") or {}).get("data")},
            "reference_script": script,
            "wallclock_20ep_s": round(wall, 3) if wall is not None else None,
            "wallclock_20ep_note": "in-process 20 epochs on the built trainer (state reset): excludes PG init, "
                                   "data build, model/comm setup, log syncs (total_cost_time_s is the reference's timer)",
            "baseline_wallclock_20ep_s": base,
            "vs_baseline_wallclock": (round(base / script["total_cost_time_s"], 1)
                                      if (base and script and script.get("total_cost_time_s")) else None),
            "vs_baseline_wallclock_inprocess": round(base / wall, 1) if (wall and base) else None,
            "final_test_acc": round(acc, 4) if acc is not None else None,
            "last_train_loss": round(final_loss, 4),
            "setup_s": round(t0 - t_setup, 2),
            "timed_enqueue_ms": round(1000.0 * (t_enq - t0), 3),
            "timed_device_ms": round(ev0.elapsed_time(ev1), 3),
            "setup_phases_s": phases.rounded(3),
            "setup_info_s": phases.info or None,
        }
    diag.phase = "done"
    if not in_sync:
        where = f" (first differing epoch of the 20-epoch run: {desync_epoch})" if desync_epoch else ""
        raise RuntimeError(f"DDP desync - ranks hold different parameters{where}")
    return out


def _script_extra(args) -> list[str]:
    extra = []     # non-default transport choices carry over to the child job
    if args.dist_backend != "nccl":
        extra += ["--dist-backend", args.dist_backend]
    if args.allreduce != "auto":
        extra += ["--allreduce", args.allreduce]
    if args.dtype != "bf16":
        extra += ["--dtype", args.dtype]
    return extra


def reference_first(args, world: int, rank: int, use_pg: bool) -> dict | None:
    """The reference-timer child job before this job touches a GPU: the ranks meet on the process
    group's store (no device work: the nccl group is lazy), rank 0 runs ``mnist_ddp.py`` at this N, the
    others wait host-side.  Measured like a user's run on idle GPUs - run after the bench, beside its
    processes' idle HIP contexts, the child's runtime bring-up took 0.12 s instead of 0.06
    (``--script-last``)."""
    if use_pg and not dist.is_initialized():
        dist.init_process_group(args.dist_backend, init_method="env://", world_size=world, rank=rank)
    script = None
    if rank == 0:
        try:
            script = run_reference_script(world, args.batch_size, args.epochs, extra=_script_extra(args))
        except Exception as e:  # noqa: BLE001 - reported in the JSON
            script = {"error": f"{type(e).__name__}: {e}"}
        script["order"] = "first"
    if use_pg:
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            store.set("bench/script_first_done", "1")
        else:
            store.wait(["bench/script_first_done"], timedelta(seconds=1200))
    return script


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.cpu:
        return cpu_bench(200 if args.steps is None else args.steps, 10 if args.warmup is None else args.warmup)
    args.steps = 600 if args.steps is None else args.steps
    args.warmup = 50 if args.warmup is None else args.warmup
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args, argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks", file=sys.stderr)
        return 2
    if os.environ.get("MNIST_AMD_ONE_GPU", "0") == "1":
        local = 0                      # one-GPU multi-rank rehearsal (gloo + xgmi only)
    use_pg = world > 1 or (args.force_comm and "MASTER_ADDR" in os.environ)
    diag = Diag(rank, world)
    rc = 0
    try:
        if args.full_run and args.script_run and args.script_first:
            diag.phase = "reference_script"
            args._script_first = reference_first(args, world, rank, use_pg)
        out = run_rank(args, world, rank, local, diag)
        if out is not None:
            print(json.dumps(out), flush=True)
    except BaseException as e:  # noqa: BLE001 - every failure ends in one JSON line + non-zero rc
        rec = diag.record(e)
        print(f"bench.py rank {rank}: FAILED in {rec['phase']}: {rec['error']}", file=sys.stderr, flush=True)
        _publish_failure(rec, use_pg and dist.is_initialized())
        if rank == 0:
            recs = _collect_failures(world) if (use_pg and dist.is_initialized()) else {}
            recs[0] = rec
            print(json.dumps({"metric": METRIC, "value": None, "unit": "images/s", "n_gpus": world,
                              "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
                              "error": rec["error"], "failed_phase": rec["phase"],
                              "rank_failures": {str(q): recs[q] for q in sorted(recs)}}), flush=True)
        if getattr(e, "fatal", False):
            # a collective stuck on the device cannot be cancelled: leave without the runtime's
            # teardown (which would wait for it), the driver sees the exit code
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(3)
        rc = 1
    if getattr(diag, "pending", None) is not None:
        diag.pending.close(30.0)      # a cancelled / unused RCCL init's helper thread
    if use_pg and dist.is_initialized():
        try:
            if rc == 0:
                barrier()
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass
    return rc


if __name__ == "__main__":
    sys.exit(main())
