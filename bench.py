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

With ``--full-run`` (default on) it then also times the README's complete workload in-process:
20 epochs of train + per-epoch rank-0 test-set evaluation (10k images) - the reference's
"Total cost time" minus interpreter/import start-up - and reports it as ``wallclock_20ep_s``.

Launch: ``python bench.py`` (1 GPU) or
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N``.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from pytorch_mnist_ddp_amd.data.datasets import load_mnist  # noqa: E402
from pytorch_mnist_ddp_amd.data.samplers import DistributedIndexStream  # noqa: E402
from pytorch_mnist_ddp_amd.engine.state import ModelState  # noqa: E402
from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer  # noqa: E402
from pytorch_mnist_ddp_amd.models.net import Net  # noqa: E402
from pytorch_mnist_ddp_amd.parallel.distributed import create_rccl_comms  # noqa: E402

METRIC = "images/sec + 20-epoch wallclock, MNIST CNN DDP at 1/2/4/8 MI355X"
# reference README.md:55-59 (20-epoch wallclock at B=200/GPU) -> images/s = 20*60000/t
BASELINE_WALLCLOCK = {1: 242.3, 2: 137.1, 4: 73.6}
TRAIN_N, TEST_N, EPOCHS = 60000, 10000, 20


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=600)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--batch-size", type=int, default=200, help="per-GPU batch (README config: 200)")
    ap.add_argument("--graph-steps", type=int, default=25, help="steps per captured hipGraph (0 = eager)")
    ap.add_argument("--single-bucket", action="store_true", help="one all-reduce per step (no overlap)")
    ap.add_argument("--no-full-run", dest="full_run", action="store_false")
    ap.add_argument("--epochs", type=int, default=EPOCHS, help="epochs for the full-run wallclock")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--force-comm", action="store_true",
                    help="attach the RCCL communicator even at world_size 1 (exercises the DDP schedule)")
    ap.add_argument("--allreduce", choices=["auto", "rccl", "xgmi"], default=os.environ.get("MNIST_AMD_ALLREDUCE", "auto"),
                    help="DDP gradient all-reduce: RCCL, the direct xGMI reduce-scatter/all-gather kernel, or "
                         "auto (time both at startup, keep the faster)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        if world == 1 and args.gpus > 1:
            print(f"bench.py: --gpus {args.gpus} needs torch.distributed.run with {args.gpus} procs",
                  file=sys.stderr)
            return 2
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_pg = world > 1 or (args.force_comm and "MASTER_ADDR" in os.environ)
    if use_pg:
        dist.init_process_group("nccl", init_method="env://", world_size=world, rank=rank, device_id=dev)
    t_setup = time.perf_counter()

    B = args.batch_size
    torch.manual_seed(args.seed)
    net = Net()
    train = load_mnist(train=True, synthetic_data=True, verbose=False)
    test = load_mnist(train=False, synthetic_data=True, verbose=False) if rank == 0 else None
    sampler = DistributedIndexStream(len(train), world, rank, shuffle=True, seed=0)
    total = args.warmup + args.steps
    steps_per_epoch = math.ceil(len(sampler) / B)
    num_samples = max(total * B, steps_per_epoch * B)
    ms = ModelState(net, dev, lr=1.0)
    comm, comm2 = create_rccl_comms(world, rank, local) if use_pg else (None, None)
    tr = FusedTrainer(ms, train, test, B, 1000, num_samples=num_samples, world_size=world, rank=rank,
                      comm=comm, seed=args.seed, graph_steps=args.graph_steps,
                      two_buckets=not args.single_bucket, comm2=comm2, allreduce=args.allreduce)
    if comm is not None:
        tr.engine.broadcast_params(0)     # DDP construction semantics: rank-0 weights everywhere

    # flat index stream = consecutive DistributedSampler epochs, full batches only
    parts, ep = [], 1
    while sum(p.numel() for p in parts) < total * B:
        sampler.set_epoch(ep)
        idx = sampler.epoch_indices()
        parts.append(idx[: (idx.numel() // B) * B])
        ep += 1
    stream = torch.cat(parts)[: total * B]
    tr.start_stream(stream, gather=False)
    tr.precapture(args.warmup)
    tr.precapture(args.steps)
    if comm is not None:   # RCCL lazily sets up its channels on the first collective: do it untimed
        tr.synchronize()
    tr.engine.gather_rows(0, args.warmup * B)
    tr.run_steps(args.warmup)
    tr.synchronize()
    if use_pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.engine.gather_rows(args.warmup * B, args.steps * B)   # the device DataLoader work is timed too
    tr.run_steps(args.steps)
    tr.synchronize()
    torch.cuda.synchronize()
    if use_pg:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if use_pg:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(tr.loss_log[(total - 1) % tr.loss_log.numel()].item()) if tr.loss_log.numel() else float("nan")
    img_s = world * B * args.steps / elapsed

    # ---- the README workload end to end: 20 epochs train + rank-0 eval, fresh model
    wall = None
    acc = None
    if args.full_run and rank == 0:
        tr.evaluate()         # untimed, like the training kernels above: load the eval kernels' code
    if args.full_run:
        torch.manual_seed(args.seed)
        net2 = Net()
        ms2 = ModelState(net2, dev, lr=1.0)
        tr2 = FusedTrainer(ms2, train, test, B, 1000, num_samples=len(sampler), world_size=world, rank=rank,
                           comm=comm, seed=args.seed, graph_steps=args.graph_steps,
                           two_buckets=not args.single_bucket, comm2=comm2, allreduce=args.allreduce)
        if comm is not None:
            tr2.engine.broadcast_params(0)
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize()
        w0 = time.perf_counter()
        sampler.set_epoch(1)
        idx = sampler.epoch_indices()
        for epoch in range(1, args.epochs + 1):
            tr2.set_lr(1.0 * (0.7 ** (epoch - 1)))
            tr2.train_epoch(epoch, idx, sync=False)      # enqueued; the GPU runs while the host
            if epoch < args.epochs:                      # draws the next epoch's sampler order
                sampler.set_epoch(epoch + 1)
                idx = sampler.epoch_indices()
            if rank == 0:
                ls, correct, n = tr2.evaluate()
                acc = correct / max(1, n)
        tr2.synchronize()
        if use_pg:
            dist.barrier()
        w1 = time.perf_counter()
        wall = w1 - w0
        if use_pg:
            t = torch.tensor([wall], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            wall = float(t.item())

    base = BASELINE_WALLCLOCK.get(world)
    base_img_s = (EPOCHS * TRAIN_N / base) if base else None
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
            "dtype": "bf16",
            "data": "synthetic (60k/10k 28x28 uint8, deterministic); random-init weights",
            "config": {"model": "mnist_cnn (reference Net: conv32-conv64-maxpool-fc128-fc10, 1.2M params)",
                       "global_batch": B * world, "batch_per_gpu": B, "seq_len": None,
                       "parallelism": f"dp{world}", "optimizer": "Adadelta(lr=1.0)",
                       "graph_steps": args.graph_steps, "buckets": 1 if args.single_bucket else 2,
                       "allreduce": tr.allreduce if world > 1 or comm is not None else None,
                       "allreduce_probe_us": tr.allreduce_timings or None},
            "wallclock_20ep_s": round(wall, 3) if wall is not None else None,
            "baseline_wallclock_20ep_s": base,
            "vs_baseline_wallclock": round(base / wall, 1) if (wall and base) else None,
            "final_test_acc": round(acc, 4) if acc is not None else None,
            "last_train_loss": round(final_loss, 4),
            "setup_s": round(t0 - t_setup, 2),
        }
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
