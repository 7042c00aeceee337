"""Per-epoch wallclock breakdown of the bench's 20-epoch run on one GPU (host-side timers):
    python tools/epoch_timing.py [--epochs 20] [--batch-size 200]
Prints, per epoch: enqueue time of train_epoch, time to the end of training (sync), eval time,
sampler time, so the non-training overhead of the wallclock metric is visible."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_mnist_ddp_amd.data.datasets import load_mnist  # noqa: E402
from pytorch_mnist_ddp_amd.data.samplers import DistributedIndexStream  # noqa: E402
from pytorch_mnist_ddp_amd.engine.state import ModelState  # noqa: E402
from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer  # noqa: E402
from pytorch_mnist_ddp_amd.models.net import Net  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--epochs", type=int, default=20)
ap.add_argument("--batch-size", type=int, default=200)
ap.add_argument("--graph-steps", type=int, default=25)
a = ap.parse_args()
dev = torch.device("cuda", 0)
train = load_mnist(train=True, synthetic_data=True, verbose=False)
test = load_mnist(train=False, synthetic_data=True, verbose=False)
sampler = DistributedIndexStream(len(train), 1, 0, shuffle=True, seed=0)
torch.manual_seed(1)
ms = ModelState(Net(), dev, lr=1.0)
tr = FusedTrainer(ms, train, test, a.batch_size, 1000, num_samples=len(sampler), graph_steps=a.graph_steps)
torch.cuda.synchronize()
T0 = time.perf_counter()
sampler.set_epoch(1)
idx = sampler.epoch_indices()
rows = []
for ep in range(1, a.epochs + 1):
    t0 = time.perf_counter()
    tr.set_lr(0.7 ** (ep - 1))
    tr.train_epoch(ep, idx, sync=False)
    t1 = time.perf_counter()
    if ep < a.epochs:
        sampler.set_epoch(ep + 1)
        idx = sampler.epoch_indices()
    t2 = time.perf_counter()
    tr.compute.synchronize()
    t3 = time.perf_counter()
    tr.evaluate()
    t4 = time.perf_counter()
    rows.append((ep, 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t0), 1e3 * (t4 - t3)))
T1 = time.perf_counter()
print("epoch  enqueue_ms  sampler_ms  train_done_ms  eval_ms")
for r in rows:
    print("%5d %11.2f %11.2f %14.2f %8.2f" % r)
print(f"total {T1 - T0:.3f} s")
