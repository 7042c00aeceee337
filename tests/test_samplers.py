"""T0: index streams are bit-identical to torch's samplers, including DataLoader RNG consumption."""
import pytest
import torch
from torch.utils.data import DataLoader, DistributedSampler, RandomSampler, SequentialSampler, TensorDataset

from pytorch_mnist_ddp_amd.data import (DistributedIndexStream, HostLoader, RandomIndexStream,
                                        SequentialIndexStream, consume_loader_base_seed)
from pytorch_mnist_ddp_amd.data.datasets import MNISTData


class _DS(torch.utils.data.Dataset):
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i


@pytest.mark.parametrize("n", [60000, 10000, 1001, 7])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_distributed_stream_equals_torch(n, world):
    for rank in range(world):
        ours = DistributedIndexStream(n, world, rank, shuffle=True, seed=0)
        ref = DistributedSampler(_DS(n), num_replicas=world, rank=rank, shuffle=True, seed=0)
        assert len(ours) == len(ref)
        for epoch in (1, 2, 3):
            ours.set_epoch(epoch)
            ref.set_epoch(epoch)
            assert ours.epoch_indices().tolist() == list(iter(ref))


def test_distributed_padding_wraps_like_torch():
    ours = DistributedIndexStream(5, 8, 7, shuffle=False)
    ref = DistributedSampler(_DS(5), num_replicas=8, rank=7, shuffle=False)
    assert ours.epoch_indices().tolist() == list(iter(ref))


def test_random_and_sequential_streams_equal_torch_samplers():
    torch.manual_seed(1)
    a = [RandomIndexStream(1000).epoch_indices().tolist() for _ in range(3)]
    torch.manual_seed(1)
    s = RandomSampler(_DS(1000))
    b = [list(iter(s)) for _ in range(3)]
    assert a == b
    assert SequentialIndexStream(9).epoch_indices().tolist() == list(iter(SequentialSampler(_DS(9))))


def test_host_loader_matches_dataloader_order_and_rng_consumption():
    """Epoch orders AND the global RNG state after each epoch match torch's DataLoader."""
    n, bs = 500, 64
    imgs = torch.randint(0, 256, (n, 28, 28), dtype=torch.uint8)
    labels = torch.arange(n) % 10
    data = MNISTData(imgs, labels, True, "test")
    torch.manual_seed(7)
    ours = HostLoader(data, RandomIndexStream(n), bs)
    test_ours = HostLoader(data, SequentialIndexStream(n), 100)
    got = []
    for _ in range(2):
        got.append(torch.cat([t for _, t in ours]).tolist())
        list(test_ours)
    after_ours = torch.rand(1).item()

    torch.manual_seed(7)
    ds = TensorDataset(torch.arange(n))
    dl = DataLoader(ds, batch_size=bs, sampler=RandomSampler(ds))
    tdl = DataLoader(ds, batch_size=100, sampler=SequentialSampler(ds))
    exp = []
    for _ in range(2):
        exp.append(torch.cat([b[0] for b in dl]).tolist())
        list(tdl)
    after_ref = torch.rand(1).item()
    assert [[labels[i].item() for i in e] for e in exp] == got
    assert after_ours == after_ref


def test_consume_base_seed_draws_one_int64():
    torch.manual_seed(3)
    consume_loader_base_seed()
    x = torch.rand(1).item()
    torch.manual_seed(3)
    torch.empty((), dtype=torch.int64).random_()
    assert torch.rand(1).item() == x
