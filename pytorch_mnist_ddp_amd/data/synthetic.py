"""Deterministic synthetic MNIST-shaped data (uint8 1x28x28 images, 10 classes).

There is no network here, so ``torchvision.datasets.MNIST(download=True)``
(reference ``mnist_ddp.py:157``) cannot fetch the real files.  This generator
produces a *learnable* stand-in with MNIST's exact shapes, dtype and split sizes
(60,000 train / 10,000 test): each class is a fixed random "pen stroke"
template (a blurred polyline), and every sample is that template shifted by up
to +/-3 px, gain-scaled and noised.  The templates depend only on
``template_seed`` so train and test share classes; the per-split sample streams
use distinct seeds.  Generation is vectorised torch on the CPU (~0.3 s for
70k images) and never touches the global RNG (own ``torch.Generator``), so it
does not perturb the reference's seeded RNG consumption order.
"""
from __future__ import annotations

import torch

TRAIN_SIZE = 60000
TEST_SIZE = 10000
IMG = 28
_PAD = 3
TEMPLATE_SEED = 20250209


def make_templates(seed: int = TEMPLATE_SEED, num_classes: int = 10) -> torch.Tensor:
    """Return float32 [num_classes, 28+2*pad, 28+2*pad] stroke templates in [0,1]."""
    g = torch.Generator().manual_seed(seed)
    size = IMG + 2 * _PAD
    yy, xx = torch.meshgrid(torch.arange(size, dtype=torch.float32),
                            torch.arange(size, dtype=torch.float32), indexing="ij")
    grid = torch.stack([yy.reshape(-1), xx.reshape(-1)], dim=1)  # [S*S, 2]
    out = []
    for _ in range(num_classes):
        k = int(torch.randint(3, 6, (1,), generator=g))
        ctrl = _PAD + 4 + torch.rand(k, 2, generator=g) * (IMG - 8)
        t = torch.linspace(0, 1, 24).unsqueeze(1)
        pts = torch.cat([ctrl[i] * (1 - t) + ctrl[i + 1] * t for i in range(k - 1)], dim=0)
        d2 = torch.cdist(grid, pts).pow(2).min(dim=1).values
        sigma = 1.1 + 0.4 * float(torch.rand(1, generator=g))
        img = torch.exp(-d2 / (2 * sigma * sigma)).reshape(size, size)
        out.append(img / img.max())
    return torch.stack(out)


def generate(n: int, seed: int, templates: torch.Tensor | None = None,
             chunk: int = 8192) -> tuple[torch.Tensor, torch.Tensor]:
    """Generate ``n`` samples: (uint8 [n,28,28], int64 [n] labels)."""
    if templates is None:
        templates = make_templates()
    nc = templates.shape[0]
    g = torch.Generator().manual_seed(seed)
    labels = torch.randint(0, nc, (n,), generator=g)
    images = torch.empty(n, IMG, IMG, dtype=torch.uint8)
    ar = torch.arange(IMG)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        m = e - s
        lab = labels[s:e]
        dy = torch.randint(0, 2 * _PAD + 1, (m,), generator=g)
        dx = torch.randint(0, 2 * _PAD + 1, (m,), generator=g)
        rows = (dy[:, None] + ar[None, :])[:, :, None]
        cols = (dx[:, None] + ar[None, :])[:, None, :]
        img = templates[lab[:, None, None], rows, cols]
        # a faint second stroke from another class makes the task non-trivial
        other = (lab + torch.randint(1, nc, (m,), generator=g)) % nc
        img = img + 0.35 * torch.rand(m, 1, 1, generator=g) * templates[other[:, None, None], rows, cols]
        gain = 0.65 + 0.35 * torch.rand(m, 1, 1, generator=g)
        noise = torch.rand(m, IMG, IMG, generator=g)
        img = img * gain + 0.18 * noise * (noise > 0.6)
        images[s:e] = (img.clamp_(0, 1) * 255.0).round_().to(torch.uint8)
    return images, labels


def synthetic_mnist(train: bool, size: int | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    n = size if size is not None else (TRAIN_SIZE if train else TEST_SIZE)
    return generate(n, seed=(1 if train else 2) * 7919 + 17)
