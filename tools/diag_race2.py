import torch
from pytorch_mnist_ddp_amd.data.synthetic import generate
from pytorch_mnist_ddp_amd.engine.state import FLAG_NO_DROPOUT, ModelState
from pytorch_mnist_ddp_amd.models.net import Net
from pytorch_mnist_ddp_amd.ops import functional as Fk
dev = torch.device("cuda")
B = 200
torch.manual_seed(1); net = Net()
imgs, labels = generate(B, seed=5)
ms = ModelState(net, dev)
u8 = imgs.reshape(B, -1).contiguous().to(dev); lab = labels.int().to(dev)
idx = torch.arange(B, dtype=torch.int32, device=dev)
buf = Fk.StepBuffers.allocate(B, dev)
ms.set_state(0, 123, 0, FLAG_NO_DROPOUT)
Fk.trunk_fwd(ms, u8, idx, buf, True); Fk.fc1_fwd(ms, buf); Fk.head_train(ms, lab, idx, buf); Fk.fc_bwd(ms, buf)
outs = []
for rep in range(6):
    buf.c1part.fill_(7.0)
    Fk.conv_bwd(ms, u8, idx, buf); torch.cuda.synchronize()
    outs.append(buf.c1part.clone().view(4 * B, 32, 10))
for r in range(1, 6):
    d = (outs[0] - outs[r]).abs()
    nz = torch.nonzero(d)
    print("rep", r, "n diff", nz.shape[0], "by k:", torch.bincount(nz[:, 2], minlength=10).tolist(),
          "by strip:", torch.bincount(nz[:, 0] % 4, minlength=4).tolist(), "ci:", sorted(set(nz[:, 1].tolist()))[:10])
    for row in nz[:5].tolist():
        s, ci, k = row
        print("   slab", s, "ci", ci, "k", k, outs[0][s, ci, k].item(), outs[r][s, ci, k].item())
print("any 7.0 left:", (outs[0] == 7.0).sum().item())
