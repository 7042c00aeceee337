"""a1 (bf16 ReLU(conv1)) of the fused trunk vs float64 conv1 of the normalised images: mismatch rate,
max error in bf16 ulps and the mismatch rate per a1 row (a strip / halo bug shows up as whole rows).
usage (GPU box): [MNIST_AMD_EXT_PATH=tools/so/X.so] python tools/a1_check.py B [B ...]"""
import sys

import torch
import torch.nn.functional as F

sys.path[:0] = [".", "tests"]
from test_gpu_numerics import _setup  # noqa: E402

from pytorch_mnist_ddp_amd.data.datasets import normalize_u8  # noqa: E402
from pytorch_mnist_ddp_amd.engine.state import FLAG_NO_DROPOUT  # noqa: E402
from pytorch_mnist_ddp_amd.ops import functional as Fk  # noqa: E402

dev = torch.device("cuda:0")
for B in [int(a) for a in sys.argv[1:]] or [200, 1500]:
    net, ref, ms, imgs, labels, u8, lab, idx, buf = _setup(B, dev)
    ms.set_state(0, seed=123, rng_base=0, flags=FLAG_NO_DROPOUT)
    Fk.train_step(ms, u8, lab, idx, buf, update=False)
    torch.cuda.synchronize()
    d = {n: v.detach().cpu().double() for n, v in ms.views(ms.param).items()}
    x = normalize_u8(imgs).double()
    z0 = F.conv2d(x, d["conv1.weight"], d["conv1.bias"])
    a_ref = F.relu(z0).float().to(torch.bfloat16).float()
    a1 = buf.a1[:B].cpu().float().permute(0, 3, 1, 2)
    mism = a1 != a_ref
    ulp = ((a1 - a_ref).abs() / (a_ref.abs() * 2.0 ** -8).clamp_min(1e-30)).max().item()
    rows = mism.float().mean((0, 1, 3))
    print(f"B={B}: a1 mismatch {mism.float().mean().item():.2e}, max rel {ulp:.2f} bf16 ulp, "
          f"max |z| err {((F.relu(z0) - a1.double()).abs().max().item()):.3e}")
    print(f"  kernel above / below the reference: {(a1 > a_ref).sum().item()} / {(a1 < a_ref).sum().item()}; "
          f"zero-sign flips (a1 > 0 != z0 > 0): {((a1 > 0) != (z0 > 0)).sum().item()}")
    print("  per-row mismatch:", " ".join(f"{v:.1e}" for v in rows.tolist()))
