"""Diagnostics: kernel determinism (eager vs eager vs graph) and per-param grad errors."""
import copy, sys
sys.path.insert(0, "tests")
import torch
from pytorch_mnist_ddp_amd.data.datasets import load_mnist
from pytorch_mnist_ddp_amd.data.synthetic import generate
from pytorch_mnist_ddp_amd.engine.state import FLAG_NO_DROPOUT, ModelState
from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
from pytorch_mnist_ddp_amd.models.net import Net
from pytorch_mnist_ddp_amd.ops import functional as Fk
from refmodel import emulated_bf16_step, reference_step, rel_err

dev = torch.device("cuda")

def one_step_grads(B, seed=1):
    torch.manual_seed(seed); net = Net(); ref = copy.deepcopy(net)
    imgs, labels = generate(B, seed=5)
    ms = ModelState(net, dev)
    u8 = imgs.reshape(B, -1).contiguous().to(dev); lab = labels.int().to(dev)
    idx = torch.arange(B, dtype=torch.int32, device=dev)
    buf = Fk.StepBuffers.allocate(B, dev)
    ms.set_state(0, 123, 0, FLAG_NO_DROPOUT)
    Fk.train_step(ms, u8, lab, idx, buf, update=False); torch.cuda.synchronize()
    return ms, buf, ref, imgs, labels

for B in (7, 64, 200):
    ms, buf, ref, imgs, labels = one_step_grads(B)
    g1 = ms.grad.clone()
    ms2, buf2, *_ = one_step_grads(B)
    print(f"B={B} grad run-to-run identical: {torch.equal(g1, ms2.grad)}",
          {k: (buf.__dict__[k].float() - buf2.__dict__[k].float()).abs().max().item() for k in ("a1","p","pmask","z1part","dz1","g")})
    _, _, g_emu = emulated_bf16_step(ref, imgs, labels)
    _, _, g_ref = reference_step(ref, imgs, labels)
    v = ms.views(ms.grad)
    for n in g_ref:
        print(f"   {n:14s} emu {rel_err(v[n], g_emu[n]):.2e}  fp32 {rel_err(v[n], g_ref[n]):.2e}  emu-vs-fp32 {rel_err(g_emu[n], g_ref[n]):.2e}")

def trainer(gs):
    torch.manual_seed(1); net = Net()
    tr = load_mnist(synthetic_data=True, train=True, synthetic_size=2000, verbose=False)
    te = load_mnist(synthetic_data=True, train=False, synthetic_size=1000, verbose=False)
    ms = ModelState(net, dev, lr=1.0)
    return ms, FusedTrainer(ms, tr, te, 200, 1000, num_samples=2000, seed=1, graph_steps=gs)
idx = torch.randperm(2000, generator=torch.Generator().manual_seed(3))
res = []
for gs in (0, 0, 4, 4):
    ms, t = trainer(gs)
    t.train_epoch(1, idx); torch.cuda.synchronize()
    res.append((ms.param.clone(), t.loss_log.clone()))
    print("graph_steps", gs, "losses", [round(x, 5) for x in t.loss_log.tolist()])
for i in range(1, 4):
    print(i, "param equal to run0:", torch.equal(res[0][0], res[i][0]), (res[0][0]-res[i][0]).abs().max().item())
