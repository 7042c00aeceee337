"""Checkpoint save/load with the reference's file names and key layout.

* ``mnist.py``                      -> ``mnist_cnn.pt``,  bare keys            (reference mnist.py:133)
* ``mnist_ddp.py`` distributed      -> ``mnist_cnn.pt``,  ``module.``-prefixed (rank 0 only, :195)
* ``mnist_ddp.py`` non-distributed  -> ``mnist_cnn_.pt``, bare keys            (:197)

Tensors are fp32 and saved from the device they live on, each with its own storage (the
framework keeps parameters as views of one flat buffer; cloning keeps the file layout identical
to torch's ``state_dict`` of an ordinary module).  Loading uses ``weights_only=True``.
"""
from __future__ import annotations

from collections import OrderedDict

import torch


def save_state_dict(module, path: str) -> None:
    sd = OrderedDict((k, v.detach().clone()) for k, v in module.state_dict().items())
    torch.save(sd, path)


def load_state_dict(module, path: str, map_location=None, strict: bool = True):
    sd = torch.load(path, map_location=map_location, weights_only=True)
    has_prefix = all(k.startswith("module.") for k in sd)
    wants_prefix = all(k.startswith("module.") for k in module.state_dict())
    if has_prefix and not wants_prefix:
        sd = OrderedDict((k[len("module."):], v) for k, v in sd.items())
    elif wants_prefix and not has_prefix:
        sd = OrderedDict(("module." + k, v) for k, v in sd.items())
    return module.load_state_dict(sd, strict=strict)
