#!/usr/bin/env python3
"""Single-process MNIST training - CLI-compatible with the reference mnist.py (mnist.py:73-137).

Same flags, log lines and ``mnist_cnn.pt`` checkpoint; runs the MI355X-native engine on GPU and
the reference torch math on ``--no-cuda``.  See ``python mnist.py --help``.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_mnist_ddp_amd.driver import main_mnist  # noqa: E402

if __name__ == '__main__':
    sys.exit(main_mnist())
