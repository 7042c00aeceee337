#!/usr/bin/env python3
"""Data-parallel MNIST training - CLI-compatible with the reference mnist_ddp.py (mnist_ddp.py:108-203).

Launch exactly like the reference:
    python -m torch.distributed.launch --nproc_per_node=4 mnist_ddp.py --batch-size 200 --epochs 20
    torchrun --nproc-per-node 8 mnist_ddp.py --batch-size 200 --epochs 20
    python mnist_ddp.py --batch-size 200 --epochs 20            # single GPU
(``--local-rank`` and ``--local_rank`` are both accepted; env:// and SLURM rank discovery.)
Prints ``Total cost time:<seconds> ms`` on every rank, like the reference.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_mnist_ddp_amd.driver import main_mnist_ddp  # noqa: E402

if __name__ == '__main__':
    sys.exit(main_mnist_ddp())
