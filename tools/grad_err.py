"""Per-parameter gradient error of the fused train step vs the bf16-emulating float64 oracle and vs
torch fp32 (test_gpu_numerics.test_train_step_grads_match_fp32_reference_without_dropout's numbers).
usage (GPU box): [MNIST_AMD_EXT_PATH=tools/so/X.so] python tools/grad_err.py B [B ...]"""
import sys

import torch

sys.path[:0] = [".", "tests"]
from refmodel import emulated_bf16_step, reference_step, rel_err  # noqa: E402
from test_gpu_numerics import _setup  # noqa: E402

from pytorch_mnist_ddp_amd.engine.state import FLAG_NO_DROPOUT  # noqa: E402
from pytorch_mnist_ddp_amd.ops import functional as Fk  # noqa: E402

dev = torch.device("cuda:0")
for B in [int(a) for a in sys.argv[1:]]:
    net, ref, ms, imgs, labels, u8, lab, idx, buf = _setup(B, dev)
    ms.set_state(0, seed=123, rng_base=0, flags=FLAG_NO_DROPOUT)
    Fk.train_step(ms, u8, lab, idx, buf, update=False)
    torch.cuda.synchronize()
    _, _, g_ref = reference_step(ref, imgs, labels)
    _, _, g_emu = emulated_bf16_step(ref, imgs, labels)
    grads = ms.views(ms.grad)
    print(f"B={B}: " + ", ".join(f"{n} {rel_err(grads[n], g_emu[n]):.2e}/{rel_err(grads[n], g_ref[n]):.2e}" for n in g_ref))
