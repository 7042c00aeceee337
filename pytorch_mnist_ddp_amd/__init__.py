"""pytorch_mnist_ddp_amd - MI355X-native (gfx950 / CDNA4) re-design of FlyingAnt2018/pytorch_mnist_ddp.

Layers: CLI (``cli``) -> drivers (``mnist.py`` / ``mnist_ddp.py``) ->
distributed runtime (``parallel``) -> data pipeline (``data``) -> model / optimizer
(``models``, ``optim``) -> native engine + hand-written HIP kernels (``engine``, ``ops``,
``csrc/``).
"""
import torch  # noqa: F401  (import before the native extension: shares torch's HIP runtime / RCCL)

__version__ = "0.1.0"
