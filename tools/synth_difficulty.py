"""Calibrate the synthetic generator's difficulty (generator v3 knobs, synthetic.DEFAULT_PARAMS): for each
parameter set, the README workload (B = 200, 20 epochs, Adadelta lr 1 / StepLR 0.7, dropout) on the fused
engine, one GPU, and the final test accuracy.  Target: real MNIST's regime (~99 %), not a trivial 100 %.

    python tools/synth_difficulty.py [--epochs 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SETS = {
    "default": {},
    "ov0.7": {"overlay": 0.7},
    "ov0.75": {"overlay": 0.75},
    "ov0.8": {"overlay": 0.8},
    "ov0.85": {"overlay": 0.85},
    "ov0.9": {"overlay": 0.9},
    "ov0.7_warp": {"overlay": 0.7, "rot_deg": 16.0, "scale": 0.36, "shear": 0.36},
    "ov0.75_noise": {"overlay": 0.75, "nthr": 0.5, "namp": 0.3},
    "ov1.0_noise": {"overlay": 1.0, "nthr": 0.45, "namp": 0.35},
    "ov1.0_warp": {"overlay": 1.0, "rot_deg": 20.0, "scale": 0.4, "shear": 0.4},
    "ov1.1_jit": {"overlay": 1.1, "jitter": 2.5, "rot_deg": 18.0},
    "ov1.2_all": {"overlay": 1.2, "jitter": 3.0, "rot_deg": 20.0, "scale": 0.4, "shear": 0.4, "namp": 0.35},
    "ov1.4_all": {"overlay": 1.4, "jitter": 3.0, "rot_deg": 24.0, "scale": 0.45, "shear": 0.45, "namp": 0.4},
}


def run(name, params, epochs, dev):
    import torch
    from pytorch_mnist_ddp_amd.data import synthetic as S
    from pytorch_mnist_ddp_amd.data.datasets import MNISTData
    from pytorch_mnist_ddp_amd.data.samplers import DistributedIndexStream
    from pytorch_mnist_ddp_amd.engine.state import ModelState
    from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
    from pytorch_mnist_ddp_amd.models.net import Net
    tp = S.SynthPlan(S.TRAIN_SIZE, S.split_seed(True), S.LABEL_NOISE, params=params)
    ep = S.SynthPlan(S.TEST_SIZE, S.split_seed(False), 0.0, params=params)
    train = MNISTData(None, tp.labels, True, "synthetic", plan=tp)
    test = MNISTData(None, ep.labels, False, "synthetic", plan=ep)
    torch.manual_seed(1)
    ms = ModelState(Net(), dev, lr=1.0)
    sampler = DistributedIndexStream(len(train), 1, 0, shuffle=True, seed=0)
    t = FusedTrainer(ms, train, test, 200, 1000, num_samples=len(sampler), seed=1, graph_steps=50)
    accs = []
    t0 = time.perf_counter()
    for e in range(1, epochs + 1):
        t.set_lr(0.7 ** (e - 1))
        sampler.set_epoch(e)
        t.train_epoch(e, sampler.epoch_indices())
        ls, correct, n = t.evaluate()
        accs.append(round(correct / n, 4))
    return {"set": name, "params": params, "test_acc_per_epoch": accs, "final_test_acc": accs[-1],
            "final_test_loss": round(ls / n, 5), "seconds": round(time.perf_counter() - t0, 2)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--sets", nargs="*", default=list(SETS))
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    for name in args.sets:
        print(json.dumps(run(name, SETS[name], args.epochs, dev)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
