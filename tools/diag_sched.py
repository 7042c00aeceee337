"""Compare the single-GPU fused step tail with the DDP (comm-attached, world 1) schedule, per tensor."""
import sys

import torch

sys.path.insert(0, ".")
from pytorch_mnist_ddp_amd.data.datasets import load_mnist  # noqa: E402
from pytorch_mnist_ddp_amd.engine.state import ModelState  # noqa: E402
from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer  # noqa: E402
from pytorch_mnist_ddp_amd.models.net import Net  # noqa: E402
from pytorch_mnist_ddp_amd.ops import native  # noqa: E402

C = native.load()
dev = torch.device("cuda", 0)
tr = load_mnist(synthetic_data=True, train=True, synthetic_size=1024, verbose=False)
idx = torch.randperm(1024, generator=torch.Generator().manual_seed(0))
for nsteps in (1, 2):
    res = []
    for c in (None, C.RcclComm(C.RcclComm.unique_id(), 1, 0, 0)):
        torch.manual_seed(5)
        ms = ModelState(Net(), dev)
        t = FusedTrainer(ms, tr, None, 128, 1, num_samples=128 * nsteps, comm=c, graph_steps=0)
        t.train_epoch(1, idx[:128 * nsteps])
        t.synchronize()
        res.append({k: {n: v.clone() for n, v in ms.views(getattr(ms, k)).items()}
                    for k in ("param", "grad", "square_avg", "acc_delta")})
    for k in res[0]:
        print(nsteps, k, {n: f"{(res[0][k][n] - res[1][k][n]).abs().max().item():.2e}" for n in res[0][k]})
