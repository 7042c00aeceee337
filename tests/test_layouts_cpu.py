"""Device-layout helpers that tests and tools use to read kernel buffers (CPU)."""
import torch

from pytorch_mnist_ddp_amd.ops.functional import pmask_flat


def test_pmask_flat_inverts_the_device_layout():
    """The trunk stores the pool/dropout flags as [b][pooled position / 4][channel][4]
    (mnist_common.h); pmask_flat returns torch flatten order c * 144 + s."""
    B = 3
    flat = torch.randint(0, 16, (B, 9216), dtype=torch.uint8)
    dev = torch.empty(B, 9216, dtype=torch.uint8)
    f = flat.view(B, 64, 144)
    for s in range(144):
        for c in range(64):
            dev[:, ((s // 4) * 64 + c) * 4 + s % 4] = f[:, c, s]
    assert torch.equal(pmask_flat(dev), flat)
