from .datasets import MNIST_MEAN, MNIST_STD, MNISTData, load_mnist, normalize_u8
from .loader import HostLoader
from .samplers import (DistributedIndexStream, RandomIndexStream, SequentialIndexStream,
                       consume_loader_base_seed, num_batches)

__all__ = ["MNIST_MEAN", "MNIST_STD", "MNISTData", "load_mnist", "normalize_u8", "HostLoader",
           "DistributedIndexStream", "RandomIndexStream", "SequentialIndexStream",
           "consume_loader_base_seed", "num_batches"]
