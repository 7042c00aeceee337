"""Does the single-GPU step's speed depend on which hardware queues its two streams land on?

Builds K trainers one after another in one process (B = 200, one 300-step epoch each, device time per
step from HIP events) with the compute / comm streams taken from torch's stream pool (the default,
round 5's ``make_streams``), the product's ``make_streams`` (``product``), the SAME pool streams for every trainer (``reuse``), or raw streams created by the
native ``create_stream`` - CU-masked over every CU (``dedicated``: the runtime gives each a hardware
queue of its own) or plain non-blocking ``hipStreamCreateWithPriority`` (``raw``).

    python tools/queue_mapping.py --mode pool|reuse|dedicated|raw [--trainers 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="pool", choices=["pool", "reuse", "dedicated", "raw", "product"])
    ap.add_argument("--trainers", type=int, default=10)
    ap.add_argument("--steps", type=int, default=300)
    args = ap.parse_args()
    import torch
    from pytorch_mnist_ddp_amd.data.datasets import load_mnist
    from pytorch_mnist_ddp_amd.engine.state import ModelState
    from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer, make_streams
    from pytorch_mnist_ddp_amd.models.net import Net
    from pytorch_mnist_ddp_amd.ops import native
    C = native.load()
    dev = torch.device("cuda", 0)
    B = 200
    n = args.steps * B
    train = load_mnist(train=True, synthetic_data=True, synthetic_size=n, verbose=False)
    idx = torch.randperm(n, generator=torch.Generator().manual_seed(1))
    pool = lambda: (torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev, priority=-1))  # noqa: E731
    fixed = pool() if args.mode == "reuse" else None
    out = []
    for k in range(args.trainers):
        if args.mode == "pool":
            streams = pool()
        elif args.mode == "product":
            streams = make_streams(dev)              # (the trainer's own choice: the dedicated pair)
        elif args.mode == "reuse":
            streams = fixed
        else:
            hs = [C.create_stream(0, args.mode == "dedicated", p) for p in (0, -1)]
            streams = tuple(torch.cuda.ExternalStream(h, device=dev) for h in hs)
        torch.manual_seed(1)
        ms = ModelState(Net(), dev, lr=1.0)
        t = FusedTrainer(ms, train, None, B, 1000, num_samples=n, seed=1, graph_steps=50, streams=streams)
        t.train_epoch(1, idx)                       # capture + first replay
        t.synchronize()
        st = t.train_epoch(2, idx, sync=True)
        us = st.device_seconds * 1e6 / st.steps
        out.append(round(us, 2))
        print(json.dumps({"mode": args.mode, "trainer": k, "us_per_step": round(us, 2), "overlap": t.overlap,
                          "streams": [int(s.cuda_stream) for s in streams]}), flush=True)
        del t, ms
    print(json.dumps({"mode": args.mode, "us_per_step": out}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
