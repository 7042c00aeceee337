"""The reference CNN (``Net``, reference mnist.py:11-34 = mnist_ddp.py:39-62).

Parameter names, shapes, default initialisation and state_dict keys are identical to the
reference (``conv1``, ``conv2``, ``dropout1``, ``dropout2``, ``fc1``, ``fc2``), so checkpoints are
interchangeable in both directions and ``torch.manual_seed(s); Net()`` yields bit-identical
initial weights.  ``forward`` dispatches on the input device:

* CPU: the reference math with torch ops (the ``mnist.py --no-cuda`` configuration);
* GPU: the fused MI355X kernels (``ops.fused_net``) - gather/normalise-free conv trunk on
  MFMA, split-K fc1, fused head - with autograd support through ``TrunkFunction`` +
  ``HeadFunction`` (the fc gradients - and their DDP hooks - are final before the conv backward
  is enqueued; bf16 MFMA operands, fp32 accumulation / parameters).  ``compute_dtype = torch.float32``
  selects the stock-torch fp32 path on the GPU instead (the ``--dtype fp32`` parity mode).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

PARAM_NAMES = ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias",
               "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias")
PARAM_SHAPES = {"conv1.weight": (32, 1, 3, 3), "conv1.bias": (32,), "conv2.weight": (64, 32, 3, 3),
                "conv2.bias": (64,), "fc1.weight": (128, 9216), "fc1.bias": (128,),
                "fc2.weight": (10, 128), "fc2.bias": (10,)}
NUM_PARAMS = 1199882


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.compute_dtype = torch.bfloat16     # GPU: fused bf16-MFMA kernels; float32: torch ops
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.dropout1 = nn.Dropout(0.25)
        self.dropout2 = nn.Dropout(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)

    def forward_reference(self, x: torch.Tensor) -> torch.Tensor:
        """The reference forward with stock torch ops (any device)."""
        x = self.conv1(x)
        x = F.relu(x)
        x = self.conv2(x)
        x = F.relu(x)
        x = F.max_pool2d(x, 2)
        x = self.dropout1(x)
        x = torch.flatten(x, 1)
        x = self.fc1(x)
        x = F.relu(x)
        x = self.dropout2(x)
        x = self.fc2(x)
        return F.log_softmax(x, dim=1)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda and self.compute_dtype == torch.bfloat16:
            from ..ops.fused_net import fused_net_forward
            return fused_net_forward(self, x)
        return self.forward_reference(x)
