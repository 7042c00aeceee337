import copy, sys
import torch
from pytorch_mnist_ddp_amd.data.synthetic import generate
from pytorch_mnist_ddp_amd.engine.state import FLAG_NO_DROPOUT, ModelState
from pytorch_mnist_ddp_amd.models.net import Net
from pytorch_mnist_ddp_amd.ops import functional as Fk
dev = torch.device("cuda")
for B in (64, 128, 200, 256):
    torch.manual_seed(1); net = Net()
    imgs, labels = generate(B, seed=5)
    ms = ModelState(net, dev)
    u8 = imgs.reshape(B, -1).contiguous().to(dev); lab = labels.int().to(dev)
    idx = torch.arange(B, dtype=torch.int32, device=dev)
    buf = Fk.StepBuffers.allocate(B, dev)
    ms.set_state(0, 123, 0, FLAG_NO_DROPOUT)
    Fk.trunk_fwd(ms, u8, idx, buf, True); Fk.fc1_fwd(ms, buf); Fk.head_train(ms, lab, idx, buf)
    outs = []
    for rep in range(4):
        ms.grad.zero_(); buf.c1part.zero_(); buf.w2part.zero_(); buf.g.zero_()
        Fk.fc_bwd(ms, buf); torch.cuda.synchronize()
        fcg = ms.grad.clone(); g = buf.g.clone()
        Fk.conv_bwd(ms, u8, idx, buf); torch.cuda.synchronize()
        outs.append((fcg, g, buf.c1part.clone(), buf.w2part.clone(), ms.grad.clone()))
    names = ["fc_grads", "g", "c1part", "w2part", "all_grads"]
    for r in range(1, 4):
        diffs = {names[i]: (outs[0][i].float() - outs[r][i].float()).abs().max().item() for i in range(5)}
        print(f"B={B} rep{r}", diffs)
    # locate differing c1part slabs / w2part groups
    d = (outs[0][2] - outs[1][2]).abs().view(4 * B, 320).amax(1)
    bad = torch.nonzero(d).flatten().tolist()
    print("  c1part differing slabs (b*4+strip):", bad[:20], "count", len(bad))
    d2 = (outs[0][3] - outs[1][3]).abs().amax(1)
    print("  w2part differing groups:", torch.nonzero(d2).flatten().tolist()[:20])
    off = ms.offsets
    gd = (outs[0][4] - outs[1][4]).abs()
    for n in off:
        o = off[n]; sz = {"fc1.weight":1179648,"fc1.bias":128,"fc2.weight":1280,"fc2.bias":10,"conv1.weight":288,"conv1.bias":32,"conv2.weight":18432,"conv2.bias":64}[n]
        print(f"    {n}: max diff {gd[o:o+sz].max().item():.3e}")
