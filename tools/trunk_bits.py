"""Fingerprint trunk_fwd's outputs (a1 copy, pooled + dropped activations, pmask) on fixed random
inputs, for bitwise A/B of trunk builds (run once per build, MNIST_AMD_EXT_PATH selecting it):

    python tools/trunk_bits.py                      # in-tree _C
    MNIST_AMD_EXT_PATH=tools/so/x.so python tools/trunk_bits.py

Prints one sha256 line per batch size (B <= 256: the whole-image form, larger: strips)."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_mnist_ddp_amd.ops import native  # noqa: E402


def main() -> int:
    C = native.load()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    n = 2048
    data = torch.randint(0, 256, (n, 784), generator=g, dtype=torch.uint8).to(dev)
    w1 = ((torch.rand(32, 9, generator=g) - 0.5) * 0.6).to(dev)
    b1 = ((torch.rand(32, generator=g) - 0.5) * 0.2).to(dev)
    w2 = ((torch.rand(64, 9, 32, generator=g) - 0.5) * 0.2).to(torch.bfloat16).to(dev)
    b2 = ((torch.rand(64, generator=g) - 0.5) * 0.2).to(dev)
    # StepState {int32 step, int32 flags, uint64 seed, uint64 rng_base}
    st = torch.tensor([0, 0, 0x1234, 0, 7, 0], dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for B in (200, 96, 1024):
        idx = torch.randperm(n, generator=g)[:B].to(torch.int32).to(dev)
        a1 = torch.zeros(B * 26 * 26 * 32, dtype=torch.int16, device=dev)
        p = torch.zeros(B * 9216, dtype=torch.int16, device=dev)
        pm = torch.zeros(B * 9216, dtype=torch.uint8, device=dev)
        C.trunk_fwd(data.data_ptr(), idx.data_ptr(), 0, st.data_ptr(), w1.data_ptr(), b1.data_ptr(),
                    w2.data_ptr(), b2.data_ptr(), a1.data_ptr(), p.data_ptr(), pm.data_ptr(), B, True, stream)
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for t in (a1, p, pm):
            h.update(t.cpu().numpy().tobytes())
        print(f"B={B} trunk outputs sha256 {h.hexdigest()[:32]} (p nonzero {int((p != 0).sum())})", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
