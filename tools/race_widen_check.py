"""Race-window widening check: the overlapped schedules under the debug
build ``_C_rw`` - every kernel's workgroups sleep a random 0..20 us before their first global read,
every stream hand-off signal (start signals, signal launches, held completions) a random 0..20 us
before it is given (csrc/include/device_utils.h, RW_ENTRY / RW_SIGNAL) - must stay bitwise equal to
their one-stream references.  Each step of each chunk then runs under another interleaving of the
compute and comm streams, so a buffer a device-counter hand-off does not actually protect is read or
overwritten out of order somewhere in the run.

    MNIST_AMD_RACE_WIDEN=1 python tools/race_widen_check.py --case overlap   # prints RACE_WIDEN PASS

Cases (each: 2 epochs of dropout training, every parameter / optimizer state / logged loss compared):
  overlap, overlap_eager    bf16 OVERLAP (split graphs / eager) vs SERIAL, B = 200
  overlap_large             bf16 OVERLAP vs SERIAL, B = 1500 (split fc partials, side fc1 dW)
  fp32                      fp32 OVERLAP vs SERIAL
  xgmi, xgmi_fp32           world-1 XGMI schedule (fused all-reduce kernels) vs the single-GPU step
  rccl, rccl_fp32           world-1 RCCL schedule (one communicator, fc bucket on the comm stream) vs single
  broken_w1t                OVERLAP with the w1t ping-pong switched off (the race round 5 fixed): must
                            DIFFER from SERIAL - proof that the widening exposes that race class
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def trainer(dev, B=200, n=2000, graph_steps=3, **kw):
    import torch
    from pytorch_mnist_ddp_amd.data.datasets import load_mnist
    from pytorch_mnist_ddp_amd.engine.state import ModelState
    from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
    from pytorch_mnist_ddp_amd.models.net import Net
    torch.manual_seed(1)
    ms = ModelState(Net(), dev, lr=1.0)
    tr = load_mnist(train=True, synthetic_data=True, synthetic_size=n, verbose=False)
    t = FusedTrainer(ms, tr, None, B, 1000, num_samples=n, seed=1, graph_steps=graph_steps, **kw)
    return ms, t


def run(ms, t, n, epochs=2):
    """The trained state: fp32 master weights, optimizer state, logged losses, and (bf16 step) the
    bf16 weight shadows the next step reads (the fp32 step reads none: its xGMI update does not
    maintain the fc1 shadows at all, the single-GPU one does - not part of the comparison)."""
    import torch
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(5))
    for ep in range(1, epochs + 1):
        t.train_epoch(ep, idx)
    t.synchronize()
    keys = ("param", "square_avg", "acc_delta") + (() if t.fp32 else ("w1", "w1t", "w2f", "w2d"))
    return {k: getattr(ms, k).clone() for k in keys} | {"loss_log": t.loss_log.clone()}


def diff(a, b) -> list[str]:
    import torch
    return [k for k in a if not torch.equal(a[k], b[k])]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", required=True)
    args = ap.parse_args()
    import torch
    from pytorch_mnist_ddp_amd.ops import native
    C = native.load()
    widened = os.environ.get("MNIST_AMD_RACE_WIDEN") == "1"
    dev = torch.device("cuda", 0)
    case = args.case
    pg = None
    if case.startswith(("xgmi", "rccl")):
        from conftest import init_world1_pg
        import torch.distributed as dist
        init_world1_pg("nccl" if case.startswith("rccl") else "gloo", dev if case.startswith("rccl") else None)
        pg = dist
    fp32 = case.endswith("fp32")
    B, n, gs = (1500, 3000, 2) if case == "overlap_large" else (200, 2000, 0 if case == "overlap_eager" else 3)
    if case in ("overlap", "overlap_eager", "overlap_large", "fp32", "broken_w1t"):
        hooks = {"w1t_pingpong": 0} if case == "broken_w1t" else None
        ms_a, ta = trainer(dev, B, n, gs, overlap=True, fp32=fp32, hooks=hooks)
        assert ta.overlap, "streams share a hardware queue: no OVERLAP schedule"
        got = run(ms_a, ta, n)
        ms_b, tb = trainer(dev, B, n, gs, overlap=False, fp32=fp32)
        ref = run(ms_b, tb, n)
        what = "OVERLAP vs SERIAL"
    else:
        comm = None
        if case.startswith("rccl"):
            from pytorch_mnist_ddp_amd.parallel.distributed import create_rccl_comm
            comm = create_rccl_comm(1, 0, 0)
        ar = "rccl" if case.startswith("rccl") else "xgmi"
        ms_a, ta = trainer(dev, B, n, 4, comm=comm, allreduce=ar, fp32=fp32)
        assert ta.allreduce == ar, ta.transport_report
        got = run(ms_a, ta, n)
        ms_b, tb = trainer(dev, B, n, 4, fp32=fp32)
        ref = run(ms_b, tb, n)
        what = f"world-1 {ar.upper()} vs single GPU"
    bad = diff(got, ref)
    mode = "widened (_C_rw)" if widened else "product build"
    if case == "broken_w1t":
        ok = bool(bad)
        print(f"{case}: {what}, {mode}: {'DIFFERS in ' + ', '.join(bad) if bad else 'bitwise equal'} "
              f"(expected: differs)", flush=True)
    else:
        ok = not bad
        print(f"{case}: {what}, {mode}: {'bitwise equal' if ok else 'DIFFERS in ' + ', '.join(bad)}", flush=True)
    if pg is not None:
        pg.destroy_process_group()
    print("RACE_WIDEN PASS" if ok else "RACE_WIDEN FAIL", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
