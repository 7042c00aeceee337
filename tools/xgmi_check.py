"""Multi-process check + timing of the direct xGMI all-reduce (csrc/runtime/xgmi_comm.h).

    python tools/xgmi_check.py --world 4 [--same-device] [--engine-steps 30] [--iters 200]

Spawns ``--world`` ranks (gloo process group on 127.0.0.1 for the handle exchange and the verdicts).
Each rank uses GPU ``rank % device_count`` (``--same-device``: all on GPU 0 - on a one-GPU box
this exercises the IPC mappings, the flag protocol and the phase index sets; only the link is
not xGMI).  Checks, on every rank:
  1. the startup self-test of ``create_xgmi_comm`` passes;
  2. random fp32 buckets: every rank's output equals the rank-ordered fp32 sum, bitwise;
  3. the same through a captured hipGraph replayed with fresh inputs;
  4. (``--fault-test``) a rank that never arrives is detected by the others' stage timeouts
     (error flag set, no hang);
  5. (``--engine-steps``) the fused trainer with the xGMI all-reduce at this world size, dropout
     off: parameters stay bitwise identical across ranks and the loss decreases;
then prints per-call latency for the model's two bucket sizes.  Exit code 0 = all ranks passed.
"""
from __future__ import annotations

import argparse
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FC_N, CONV_N = 1181120, 18880          # the engine's two buckets (floats)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _inputs(torch, rank: int, n: int, it: int, dev):
    g = torch.Generator(device="cpu").manual_seed(1000 * it + rank)
    return torch.randn(n, generator=g, dtype=torch.float32).to(dev)


def _expect(torch, world: int, n: int, it: int, dev):
    s = _inputs(torch, 0, n, it, dev)
    for q in range(1, world):
        s = s + _inputs(torch, q, n, it, dev)     # rank order, one rounding per add (as the kernel)
    return s


def worker(rank: int, world: int, port: int, args, q) -> None:
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    ndev = torch.cuda.device_count()
    d = 0 if args.same_device else rank % ndev
    torch.cuda.set_device(d)
    dev = torch.device("cuda", d)
    dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank)
    from pytorch_mnist_ddp_amd.parallel.distributed import create_xgmi_comm
    msgs = []
    try:
        n = FC_N + CONV_N
        x = create_xgmi_comm(world, rank, dev, n)
        assert x is not None, "self-test failed"
        gin, gout = x.grad_in, x.grad_out            # the communicator's own (IPC-exported) buffers
        g = x.grids
        msgs.append(f"selftest ok (grids fc={g['fc_fused']} conv={g['conv_fused']} two={g['twoshot']} "
                    f"one={g['oneshot']}, load {g['load_fused']:.2f}/{g['load_separate']:.2f})")
        s = torch.cuda.current_stream()
        ranges = [(FC_N, CONV_N), (0, FC_N)]     # channel 0 = conv bucket, 1 = fc bucket
        for it in range(3):
            gin.copy_(_inputs(torch, rank, n, it, dev))
            for c, (off, cnt) in enumerate(ranges):
                x.allreduce(c, off, cnt, s.cuda_stream)
            torch.cuda.synchronize()
            assert x.error() == 0, "stage timeout"
            assert torch.equal(gout, _expect(torch, world, n, it, dev)), f"eager mismatch it={it}"
        msgs.append("eager ok")
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                for c, (off, cnt) in enumerate(ranges):
                    x.allreduce(c, off, cnt, side.cuda_stream)
        for it in range(3, 6):
            gin.copy_(_inputs(torch, rank, n, it, dev))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            assert x.error() == 0, "stage timeout (graph)"
            assert torch.equal(gout, _expect(torch, world, n, it, dev)), f"graph mismatch it={it}"
        msgs.append("graph ok")
        # latency per bucket (eager launches back to back; every call is a full two-phase all-reduce)
        for name, c, (off, cnt) in (("fc 4.72MB", 1, ranges[1]), ("conv 75KB", 0, ranges[0])):
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.iters):
                x.allreduce(c, off, cnt, s.cuda_stream)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / args.iters * 1e6
            msgs.append(f"{name}: {us:.1f} us/call")
        assert x.error() == 0
        if args.fault_test:
            msgs.append(_fault_check(torch, dist, world, rank, dev, x, s))
        if args.engine_steps:
            msgs.append(_engine_check(torch, dist, world, rank, dev, args.engine_steps))
        q.put((rank, True, "; ".join(msgs)))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, False, "; ".join(msgs + [f"{type(e).__name__}: {e}"])))
    finally:
        dist.destroy_process_group()


def _fault_check(torch, dist, world, rank, dev, x, s) -> str:
    """A peer that never arrives (rank world-1 skips one call): the others' stage waits must time
    out, set the error flag and return - no hang - and the flag must stay set (later calls return
    at once), which Engine::synchronize turns into an exception."""
    x.set_timeout_seconds(0.5)
    dist.barrier()
    t0 = time.perf_counter()
    if rank != world - 1:
        x.allreduce(0, FC_N, CONV_N, s.cuda_stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        code = x.error()
        assert code != 0, "missing peer was not detected"
        assert dt < 10.0, f"timeout took {dt:.1f} s"
        x.allreduce(0, FC_N, CONV_N, s.cuda_stream)      # poisoned: returns immediately
        torch.cuda.synchronize()
        from pytorch_mnist_ddp_amd.ops import native
        res = f"fault detected in {dt:.2f} s ({native.load().Engine.describe_xgmi_error(code)})"
    else:
        res = "skipped the call (the missing peer)"
    dist.barrier()
    return res


def _engine_check(torch, dist, world, rank, dev, steps) -> str:
    """Fused (all-reduce + update kernels) and separate-launch xGMI schedules must give the same bits."""
    res = []
    for fuse in (True, False):
        try:
            res.append(_engine_run(torch, dist, world, rank, dev, steps, fuse))
        except Exception as e:
            raise RuntimeError(f"engine run with xgmi_fuse={fuse}: {e}") from e
    assert torch.equal(res[0][0], res[1][0]), "fused updates differ from the separate launches"
    return res[0][1] + ", fused == separate launches"


def _engine_run(torch, dist, world, rank, dev, steps, fuse=True):
    from pytorch_mnist_ddp_amd.data.datasets import load_mnist
    from pytorch_mnist_ddp_amd.data.samplers import DistributedIndexStream
    from pytorch_mnist_ddp_amd.engine.state import ModelState
    from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
    from pytorch_mnist_ddp_amd.models.net import Net
    B = 200
    torch.manual_seed(1)
    ms = ModelState(Net(), dev, lr=1.0)
    train = load_mnist(train=True, synthetic_data=True, verbose=False)
    sampler = DistributedIndexStream(len(train), world, rank, shuffle=True, seed=0)
    tr = FusedTrainer(ms, train, None, B, 1000, num_samples=steps * B, world_size=world, rank=rank,
                      seed=1, graph_steps=10, dropout=False, allreduce="xgmi", xgmi_fuse=fuse)
    assert tr.allreduce == "xgmi", f"engine fell back to RCCL ({tr.xgmi_validation})"
    sampler.set_epoch(1)
    idx = sampler.epoch_indices()[: steps * B]
    tr.start_stream(idx, gather=True)
    tr.run_steps(steps)
    tr.synchronize()
    losses = tr.loss_log[:steps].cpu()
    p = ms.param.cpu()
    allp = [torch.zeros_like(p) for _ in range(world)]
    dist.all_gather(allp, p)
    same = all(torch.equal(allp[0], t) for t in allp)
    assert same, "parameters diverged across ranks"
    assert torch.isfinite(losses).all(), "non-finite loss"
    first, last = float(losses[:5].mean()), float(losses[-5:].mean())
    assert last < first, f"loss did not decrease ({first:.4f} -> {last:.4f})"
    return p, (f"engine ok ({steps} steps, loss {first:.3f} -> {last:.3f}, params identical; "
               f"startup validation {tr.xgmi_validation})")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--engine-steps", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=240.0)
    ap.add_argument("--fault-test", action="store_true",
                    help="last rank skips one call: the others must time out cleanly (run last; poisons the comm)")
    args = ap.parse_args()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if args.same_device and args.world > 1:
        # W processes on one GPU: 2 hardware queues each keeps the total under the GPU's hardware
        # queue slots; oversubscribed, the scheduler time-slices queues and the spinning all-reduce
        # kernels of one rank can wait seconds for a peer's (measured W=4: 70 -> 18 us per fc call)
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "2")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, args.world, port, args, q)) for r in range(args.world)]
    for p in procs:
        p.start()
    results = {}
    deadline = time.time() + args.timeout
    while len(results) < args.world and time.time() < deadline:
        try:
            r, ok, msg = q.get(timeout=1.0)
            results[r] = (ok, msg)
        except Exception:  # noqa: BLE001 - queue.Empty
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=max(1.0, deadline - time.time()))
        if p.is_alive():
            p.kill()
    good = len(results) == args.world and all(ok for ok, _ in results.values())
    for r in range(args.world):
        ok, msg = results.get(r, (False, f"no result (exit code {procs[r].exitcode})"))
        print(f"rank {r}: {'PASS' if ok else 'FAIL'}: {msg}", flush=True)
    print("XGMI_CHECK", "PASS" if good else "FAIL", flush=True)
    return 0 if good else 1


if __name__ == "__main__":
    sys.exit(main())
