"""Host-side batch loader (CPU path) with torch DataLoader-identical ordering.

Used by the ``--no-cuda`` configuration (reference ``mnist.py --no-cuda``):
batches are ``(float32 [b,1,28,28], int64 [b])`` built by indexing the uint8
split and applying torchvision's normalisation.  Each ``iter()`` consumes the
global RNG exactly as ``torch.utils.data.DataLoader.__iter__`` does (base seed
first, then the sampler), and ``drop_last=False`` like the reference.

The GPU path does not use this: it keeps the split resident in HBM and its
first kernel gathers + normalises (see ``engine/device_data.py``).
"""
from __future__ import annotations

from .datasets import MNISTData, normalize_u8
from .samplers import consume_loader_base_seed, num_batches


class HostLoader:
    def __init__(self, data: MNISTData, index_stream, batch_size: int, drop_last: bool = False):
        self.dataset = data
        self.sampler = index_stream
        self.batch_size = batch_size
        self.drop_last = drop_last

    def __len__(self) -> int:
        return num_batches(len(self.sampler), self.batch_size, self.drop_last)

    def __iter__(self):
        consume_loader_base_seed()
        idx = self.sampler.epoch_indices()
        n = idx.numel()
        stop = n - n % self.batch_size if self.drop_last else n
        for s in range(0, stop, self.batch_size):
            b = idx[s:s + self.batch_size]
            yield normalize_u8(self.dataset.images[b]), self.dataset.targets[b]
