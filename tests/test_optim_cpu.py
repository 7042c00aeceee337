"""T0: Adadelta + StepLR parity on CPU."""
import torch

from pytorch_mnist_ddp_amd.models.net import Net
from pytorch_mnist_ddp_amd.optim import Adadelta, StepLR


def test_adadelta_cpu_equals_torch_and_steplr_schedule():
    torch.manual_seed(0)
    a, b = Net(), Net()
    b.load_state_dict(a.state_dict())
    oa, ob = Adadelta(a.parameters(), lr=1.0), torch.optim.Adadelta(b.parameters(), lr=1.0)
    sa, sb = StepLR(oa, step_size=1, gamma=0.7), torch.optim.lr_scheduler.StepLR(ob, step_size=1, gamma=0.7)
    lrs = []
    for _ in range(3):
        for pa, pb in zip(a.parameters(), b.parameters()):
            g = torch.randn_like(pa)
            pa.grad, pb.grad = g.clone(), g.clone()
        oa.step(), ob.step()
        lrs.append(oa.param_groups[0]["lr"])
        sa.step(), sb.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)
    assert [round(x, 6) for x in lrs] == [1.0, 0.7, 0.49]
    assert oa.state_dict()["param_groups"][0]["lr"] == ob.state_dict()["param_groups"][0]["lr"]
