"""MNIST dataset container (raw uint8 + labels) with torchvision-equivalent transforms.

Replaces ``datasets.MNIST(root, train, download, transform=Compose([ToTensor(),
Normalize((0.1307,), (0.3081,))]))`` from reference ``mnist_ddp.py:153-160``.
Images are kept as raw uint8 (47 MB for the train split) so the GPU path can
keep the whole split resident in HBM and gather+normalise inside the first
kernel; the CPU path applies exactly torchvision's float ops
(``u8.float().div(255)`` then ``sub_(mean).div_(std)``) for bit parity.
"""
from __future__ import annotations

import os
import sys

import torch

from . import idx, synthetic

MNIST_MEAN = 0.1307
MNIST_STD = 0.3081


class MNISTData:
    """uint8 images [N, 28, 28] + int64 targets [N].  A synthetic split holds its generator plan
    instead and renders the images on first use (``images``: on the host), or straight into device
    memory (``device_images``: the fused engine's HBM-resident copy, no host image tensor at all)."""

    def __init__(self, images: torch.Tensor | None, targets: torch.Tensor, train: bool, source: str, plan=None):
        self._images, self.targets, self.train, self.source, self.plan = images, targets, train, source, plan

    @property
    def images(self) -> torch.Tensor:
        if self._images is None:
            self._images = self.plan.render_cpu()
        return self._images

    def device_images(self, device) -> torch.Tensor:
        """uint8 [N, 784] on ``device`` (a synthetic split is rendered there by the generator kernel)."""
        if self._images is None and self.plan is not None:
            return self.plan.render_device(device)
        return self.images.reshape(len(self), -1).contiguous().to(device)

    def __len__(self) -> int:
        return int(self.targets.shape[0])

    def __getitem__(self, i):
        """(normalised float32 [1,28,28], int label) like torchvision + transform."""
        return normalize_u8(self.images[i:i + 1]), int(self.targets[i])


def normalize_u8(u8: torch.Tensor) -> torch.Tensor:
    """torchvision ToTensor()+Normalize((0.1307,),(0.3081,)) on a uint8 [..,28,28] batch.

    Returns float32 [..., 1, 28, 28] (channel dim inserted before H, W).
    """
    x = u8.to(torch.float32).div(255)
    x = x.sub_(MNIST_MEAN).div_(MNIST_STD)
    return x.unsqueeze(-3)


_warned = set()


def load_mnist(root: str = "./data", train: bool = True, synthetic_data: bool | None = None,
               synthetic_size: int | None = None, verbose: bool = True) -> MNISTData:
    """Load the MNIST split from IDX files under ``root`` or build synthetic data.

    ``synthetic_data``: True -> always synthetic; False -> IDX files required;
    None -> IDX if present, else synthetic (with one warning per split; the
    reference would try to download, which is impossible offline).
    """
    if synthetic_data is not True:
        loaded = idx.load_mnist_idx(root, train)
        if loaded is not None:
            images, labels = loaded
            return MNISTData(torch.from_numpy(images), torch.from_numpy(labels), train,
                             f"idx:{os.path.abspath(root)}")
        if synthetic_data is False:
            raise FileNotFoundError(
                f"MNIST IDX files not found under {root}/MNIST/raw and there is no network to "
                f"download them; pass --synthetic to use synthetic 28x28 data")
        if verbose and train not in _warned:
            _warned.add(train)
            print(f"[mnist-amd] MNIST {'train' if train else 'test'} IDX files not found under "
                  f"{root}; using deterministic synthetic 28x28 data", file=sys.stderr)
    plan = synthetic.synthetic_plan(train, synthetic_size)     # (native, in-process: no cache)
    return MNISTData(None, plan.labels, train, "synthetic", plan=plan)
