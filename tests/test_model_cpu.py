"""T0: model parity (names, shapes, init, forward math) and checkpoint formats."""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from pytorch_mnist_ddp_amd.models.net import NUM_PARAMS, PARAM_SHAPES, Net
from pytorch_mnist_ddp_amd.utils.checkpoint import load_state_dict, save_state_dict


class RefNet(nn.Module):
    """The reference Net (mnist_ddp.py:39-62), re-declared here as a test oracle."""

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.dropout1 = nn.Dropout(0.25)
        self.dropout2 = nn.Dropout(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = torch.flatten(self.dropout1(x), 1)
        x = self.dropout2(F.relu(self.fc1(x)))
        return F.log_softmax(self.fc2(x), dim=1)


def test_parameter_names_shapes_and_count():
    net = Net()
    shapes = {n: tuple(p.shape) for n, p in net.named_parameters()}
    assert shapes == PARAM_SHAPES
    assert sum(p.numel() for p in net.parameters()) == NUM_PARAMS == 1199882


def test_seeded_init_is_bit_identical_to_reference():
    torch.manual_seed(1)
    a = Net()
    torch.manual_seed(1)
    b = RefNet()
    for (n1, p1), (n2, p2) in zip(a.named_parameters(), b.named_parameters()):
        assert n1 == n2 and torch.equal(p1, p2)


def test_cpu_forward_equals_reference_in_train_and_eval():
    torch.manual_seed(0)
    a = Net()
    b = RefNet()
    b.load_state_dict(a.state_dict())
    x = torch.randn(4, 1, 28, 28)
    a.eval(), b.eval()
    assert torch.equal(a(x), b(x))
    a.train(), b.train()
    torch.manual_seed(5)
    ya = a(x)
    torch.manual_seed(5)
    yb = b(x)
    assert torch.equal(ya, yb)


def test_checkpoint_roundtrip_and_prefix_handling(tmp_path):
    torch.manual_seed(0)
    net = Net()
    p = os.path.join(tmp_path, "mnist_cnn_.pt")
    save_state_dict(net, p)
    sd = torch.load(p, weights_only=True)
    assert list(sd.keys()) == [f"{m}.{w}" for m in ("conv1", "conv2", "fc1", "fc2") for w in ("weight", "bias")]
    assert all(v.dtype == torch.float32 for v in sd.values())
    ref = RefNet()
    ref.load_state_dict(sd)                      # loads into the reference architecture
    # a module.-prefixed (DDP) checkpoint loads into a bare model and vice versa
    torch.save({"module." + k: v for k, v in sd.items()}, os.path.join(tmp_path, "ddp.pt"))
    other = Net()
    load_state_dict(other, os.path.join(tmp_path, "ddp.pt"))
    assert all(torch.equal(a, b) for a, b in zip(other.state_dict().values(), sd.values()))
