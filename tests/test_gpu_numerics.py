"""T1: hand-written HIP kernels vs fp32 torch references (MI355X only)."""
import copy

import pytest
import torch

from pytorch_mnist_ddp_amd.data.datasets import normalize_u8
from pytorch_mnist_ddp_amd.data.synthetic import generate
from pytorch_mnist_ddp_amd.engine.state import FLAG_NO_DROPOUT, ModelState
from pytorch_mnist_ddp_amd.models.net import Net
from pytorch_mnist_ddp_amd.ops import functional as Fk

from refmodel import dropout_keep, emulated_bf16_step, reference_forward, reference_step, rel_err

pytestmark = pytest.mark.gpu


def _setup(B, dev, seed=1, data_seed=5):
    torch.manual_seed(seed)
    net = Net()
    ref = copy.deepcopy(net)
    imgs, labels = generate(B, seed=data_seed)
    ms = ModelState(net, dev)
    u8 = imgs.reshape(B, -1).contiguous().to(dev)
    lab = labels.to(torch.int32).to(dev)
    idx = torch.arange(B, dtype=torch.int32, device=dev)
    buf = Fk.StepBuffers.allocate(B, dev)
    return net, ref, ms, imgs, labels, u8, lab, idx, buf


@pytest.mark.parametrize("B", [1, 7, 100, 200, 1000, 8192])
def test_eval_forward_matches_fp32_reference(cuda_device, B):
    net, ref, ms, imgs, labels, u8, lab, idx, buf = _setup(B, cuda_device)
    Fk.eval_forward(ms, u8, lab, idx, buf)
    torch.cuda.synchronize()
    with torch.no_grad():
        lp_ref = reference_forward(ref, normalize_u8(imgs), train=False)
    lp = buf.logp.cpu()
    assert torch.isfinite(lp).all()
    assert (lp - lp_ref).abs().max().item() < 5e-2, (lp - lp_ref).abs().max()
    assert rel_err(lp, lp_ref) < 1e-2
    nll_ref = -lp_ref.gather(1, labels.view(-1, 1)).squeeze(1)
    assert (buf.loss_rows.cpu() - nll_ref).abs().max().item() < 5e-2
    agree = (buf.correct.cpu().bool() == (lp_ref.argmax(1) == labels)).float().mean().item()
    assert agree > 0.97


@pytest.mark.parametrize("B", [64, 200, 1500, 8192])
def test_train_step_grads_match_fp32_reference_without_dropout(cuda_device, B):
    net, ref, ms, imgs, labels, u8, lab, idx, buf = _setup(B, cuda_device)
    ms.set_state(0, seed=123, rng_base=0, flags=FLAG_NO_DROPOUT)
    ms.grad.fill_(float("nan"))          # every gradient element must be written
    Fk.train_step(ms, u8, lab, idx, buf, update=False)
    torch.cuda.synchronize()
    loss_ref, _, g_ref = reference_step(ref, imgs, labels)
    loss = buf.loss_rows.mean().item()
    assert abs(loss - loss_ref.item()) < 2e-2 * max(1.0, abs(loss_ref.item()))
    grads = ms.views(ms.grad)
    _, _, g_emu = emulated_bf16_step(ref, imgs, labels)
    errs = {n: (rel_err(grads[n], g_emu[n]), rel_err(grads[n], g_ref[n])) for n in g_ref}
    for name in g_ref:
        assert torch.isfinite(grads[name]).all(), name
    # kernels == bf16-emulated math up to accumulation order; bf16 vs fp32 stays small
    assert all(e < 2e-3 for e, _ in errs.values()), errs
    assert all(e < 0.1 for _, e in errs.values()), errs


def test_train_step_dropout_masks_consistent(cuda_device):
    B = 64
    net, ref, ms, imgs, labels, u8, lab, idx, buf = _setup(B, cuda_device)
    seed, base = 0x1234ABCD5678, 1000
    ms.set_state(3, seed=seed, rng_base=base)
    Fk.train_step(ms, u8, lab, idx, buf, update=False)
    torch.cuda.synchronize()
    pm = Fk.pmask_flat(buf.pmask).cpu()
    keep1 = ((pm >> 2) & 1).bool()
    rate = keep1.float().mean().item()
    assert abs(rate - 0.75) < 0.01, rate
    # exact Philox bits for a sample of elements (step 3 -> offset base + 6)
    off = base + 2 * 3
    for e in [0, 1, 2, 3, 4, 9215, 9216, 50000, B * 9216 - 1]:
        b, i = divmod(e, 9216)
        assert bool(keep1[b, i]) == dropout_keep(seed, off, e, 192), e
    # reconstruct the reference with the kernel's own masks: dropout-1 from pmask, dropout-2 from Philox
    mask2 = torch.zeros(B, 128)
    for b in range(B):
        for o in range(128):
            mask2[b, o] = float(dropout_keep(seed, off + 1, b * 128 + o, 128))
    loss_ref, _, g_ref = reference_step(ref, imgs, labels, mask1=keep1.float().view(B, 64, 12, 12), mask2=mask2)
    assert abs(buf.loss_rows.mean().item() - loss_ref.item()) < 3e-2
    grads = ms.views(ms.grad)
    m1 = keep1.float().view(B, 64, 12, 12)
    _, _, g_emu = emulated_bf16_step(ref, imgs, labels, mask1=m1, mask2=mask2)
    errs = {n: (rel_err(grads[n], g_emu[n]), rel_err(grads[n], g_ref[n])) for n in g_ref}
    assert all(e < 2e-3 for e, _ in errs.values()), errs
    assert all(e < 0.1 for _, e in errs.values()), errs
    # p is zero exactly where the mask drops
    p = buf.p[:B].float().cpu()
    assert (p[~keep1] == 0).all()


def test_adadelta_matches_torch(cuda_device):
    torch.manual_seed(0)
    net = Net()
    ref = copy.deepcopy(net)
    ms = ModelState(net, cuda_device, lr=0.7)
    opt = torch.optim.Adadelta(ref.parameters(), lr=0.7)
    for it in range(3):
        gs = {n: torch.randn_like(p) * (0.1 + it) for n, p in ref.named_parameters()}
        for n, p in ref.named_parameters():
            p.grad = gs[n].clone()
        opt.step()
        for n, v in ms.views(ms.grad).items():
            v.copy_(gs[n])
        Fk.adadelta_step(ms)
    torch.cuda.synchronize()
    for n, p in ref.named_parameters():
        ours = ms.views(ms.param)[n].cpu()
        assert torch.allclose(ours, p.detach(), rtol=1e-5, atol=1e-6), n
        st = opt.state[p]
        assert torch.allclose(ms.views(ms.square_avg)[n].cpu(), st["square_avg"], rtol=1e-5, atol=1e-9), n
        assert torch.allclose(ms.views(ms.acc_delta)[n].cpu(), st["acc_delta"], rtol=1e-4, atol=1e-9), n
    # bf16 shadows follow the fp32 masters in the kernel layouts
    w1 = ms.views(ms.param)["fc1.weight"].cpu()
    assert torch.equal(ms.w1.cpu().view(128, 9216), w1.to(torch.bfloat16))
    assert torch.equal(ms.w1t.cpu().view(9216, 128), w1.t().contiguous().to(torch.bfloat16))
    w2 = ms.views(ms.param)["conv2.weight"].cpu()          # [co, ci, ky, kx]
    w2f = w2.permute(0, 2, 3, 1).reshape(64, 9, 32).to(torch.bfloat16)
    w2d = w2.permute(2, 3, 1, 0).reshape(9, 32, 64).to(torch.bfloat16)
    assert torch.equal(ms.w2f.cpu().view(64, 9, 32), w2f)
    assert torch.equal(ms.w2d.cpu().view(9, 32, 64), w2d)


@pytest.mark.parametrize("B", [7, 200, 1500, 2100])
def test_backward_kernels_stagewise_exact(cuda_device, B):
    """Each backward kernel vs float64 math on the kernel's *own* bf16 inputs (no cascade)."""
    import torch.nn.functional as F
    import torch.nn.grad as G
    net, ref, ms, imgs, labels, u8, lab, idx, buf = _setup(B, cuda_device)
    ms.set_state(0, seed=9, rng_base=0)                     # dropout on
    Fk.train_step(ms, u8, lab, idx, buf, update=False)
    torch.cuda.synchronize()
    d = {n: v.detach().cpu().double() for n, v in ms.views(ms.param).items()}
    grads = {n: v.detach().cpu().double() for n, v in ms.views(ms.grad).items()}
    q = lambda t: t.float().to(torch.bfloat16).double()
    p = buf.p[:B].cpu().double()
    pm = Fk.pmask_flat(buf.pmask).cpu().long()
    dz1 = buf.dz1[:B].cpu().double()
    # fc1 weight/bias grads from the kernel's dz1 / p
    assert rel_err(grads["fc1.weight"], dz1.t() @ p) < 1e-5
    assert rel_err(grads["fc1.bias"], dz1.sum(0)) < 1e-5
    hq, dlq = buf.h_bf[:B].cpu().double(), buf.dl_bf[:B, :10].cpu().double()
    assert rel_err(grads["fc2.weight"], dlq.t() @ hq) < 1e-5
    assert rel_err(grads["fc2.bias"], dlq.sum(0)) < 1e-5
    # dgrad into the pooled map, masked by keep & (pooled > 0), scaled 4/3, routed to the argmax
    dp = dz1 @ q(d["fc1.weight"])
    keep_pos = ((pm & 12) == 12).double()
    g_ref = q(dp * keep_pos / 0.75).view(B, 64, 12, 12)
    arg = (pm & 3).view(B, 64, 12, 12)
    py = torch.arange(12).view(1, 1, 12, 1) * 2 + (arg >> 1)
    px = torch.arange(12).view(1, 1, 1, 12) * 2 + (arg & 1)
    dy_ref = torch.zeros(B, 64, 24, 24, dtype=torch.float64)
    bi = torch.arange(B).view(B, 1, 1, 1).expand(B, 64, 12, 12)
    ci = torch.arange(64).view(1, 64, 1, 1).expand(B, 64, 12, 12)
    dy_ref[bi, ci, py, px] = g_ref
    dy = Fk.dense_dy(buf).cpu().double().permute(0, 3, 1, 2)   # compact records -> dense NCHW
    mism = (dy != dy_ref).double().mean().item()
    assert mism < 1e-3 and rel_err(dy, dy_ref) < 1e-3, mism
    a1 = buf.a1.cpu().double().permute(0, 3, 1, 2)          # NHWC -> NCHW
    w2q = q(d["conv2.weight"])
    assert rel_err(grads["conv2.weight"], G.conv2d_weight(a1, w2q.shape, dy)) < 1e-4
    assert rel_err(grads["conv2.bias"], dy.sum((0, 2, 3))) < 1e-4
    from pytorch_mnist_ddp_amd.data.datasets import normalize_u8
    x = normalize_u8(imgs).double()
    z0 = F.conv2d(x, d["conv1.weight"], d["conv1.bias"])
    da1 = G.conv2d_input(a1.shape, w2q, dy) * (z0 > 0)
    # the dgrad kernel's da1 is fp32 in registers; its conv1 weight/bias GEMM takes bf16 operands
    assert rel_err(grads["conv1.weight"], G.conv2d_weight(q(x), d["conv1.weight"].shape, q(da1))) < 2e-3
    assert rel_err(grads["conv1.bias"], q(da1).sum((0, 2, 3))) < 2e-3
    # forward: a1 == bf16(relu(conv1)) exactly up to fp32 accumulation order
    a1_ref = q(F.relu(z0)).float()
    assert (a1.float() != a1_ref).float().mean().item() < 1e-3
