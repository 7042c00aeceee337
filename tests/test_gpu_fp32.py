"""The fp32 step (``--dtype fp32``, csrc/kernels/f32_net.hip) against the fp32 torch reference.

The reference trains in fp32 (mnist_ddp.py:49-73); this engine keeps every activation, gradient
operand and parameter in fp32 and runs the GEMM-shaped work on gfx950's f32-input MFMA
(v_mfma_f32_16x16x4_f32, exact fp32 products).  Against torch's fp32 CPU ops the only differences
are summation orders (and the max-pool routing of near ties), so the gradients are held to the float64
gradient within 3e-4 relative, or within 3x torch fp32's own error where cancellation makes that
larger (conv1.bias: 6.7e-4 against torch fp32 on the round-6 synthetic data) - two orders of magnitude tighter than the bf16 engine's tests (test_gpu_numerics.py).
"""
import copy
import os
import subprocess
import sys

import pytest
import torch

from pytorch_mnist_ddp_amd.data.datasets import load_mnist, normalize_u8
from pytorch_mnist_ddp_amd.engine.state import ModelState
from pytorch_mnist_ddp_amd.engine.trainer import FusedTrainer
from pytorch_mnist_ddp_amd.models.net import Net

from refmodel import philox4x32, reference_forward, reference_step, rel_err

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trainer(dev, B, n_train, dropout, graph_steps=0, seed=1, n_test=0, overlap=False):
    torch.manual_seed(seed)
    net = Net()
    ref = copy.deepcopy(net)
    tr = load_mnist(synthetic_data=True, train=True, synthetic_size=n_train, verbose=False)
    te = load_mnist(synthetic_data=True, train=False, synthetic_size=n_test, verbose=False) if n_test else None
    ms = ModelState(net, dev, lr=1.0)
    t = FusedTrainer(ms, tr, te, B, 1000, num_samples=n_train, seed=seed, graph_steps=graph_steps,
                     dropout=dropout, fp32=True, overlap=overlap)
    assert t.fp32 and t.engine.fp32
    assert t.engine.schedule == (t.C.SCHED_OVERLAP if overlap else t.C.SCHED_SERIAL)
    return ref, ms, t, tr, te


def _keep_mask(seed: int, offset: int, n: int, thr8: int) -> torch.Tensor:
    """Kernel dropout rule for elements [0, n): one Philox block per 16 elements, byte k of it."""
    out = torch.empty(n, dtype=torch.float32)
    for blk in range((n + 15) // 16):
        w = philox4x32((blk & 0xFFFFFFFF, blk >> 32, offset & 0xFFFFFFFF, offset >> 32),
                       (seed & 0xFFFFFFFF, seed >> 32))
        for k in range(min(16, n - 16 * blk)):
            out[16 * blk + k] = float(((w[k >> 2] >> (8 * (k & 3))) & 0xFF) < thr8)
    return out


@pytest.mark.parametrize("B,dropout", [(64, False), (200, False), (1100, False), (32, True)])
def test_fp32_step_gradients_match_torch_fp32(cuda_device, B, dropout):
    ref, ms, t, tr, _ = _trainer(cuda_device, B, B, dropout)
    idx = torch.randperm(B, generator=torch.Generator().manual_seed(7))
    for g in ms.views(ms.grad).values():             # every gradient element must be written
        g.fill_(float("nan"))
    t.train_epoch(1, idx)
    t.synchronize()
    imgs, labels = tr.images[idx], tr.targets[idx]
    m1 = m2 = None
    if dropout:                                      # step 0 of epoch 1: rng_base 0, offsets 0 / 1
        m1 = _keep_mask(t.seed, 0, B * 9216, 192).view(B, 64, 12, 12)
        m2 = _keep_mask(t.seed, 1, B * 128, 128).view(B, 128)
    loss_ref, _, g_ref = reference_step(ref, imgs, labels, m1, m2)
    _, _, g64 = reference_step(ref, imgs, labels, m1, m2, dtype=torch.float64)
    grads = ms.views(ms.grad)
    for n, g in g_ref.items():
        # against the float64 gradient: as accurate as torch's own fp32 CPU step (a gradient that
        # is a small sum of many cancelling terms - conv1.bias - has a large relative error in
        # either), and within 3e-4 of it otherwise
        e, e_torch = rel_err(grads[n], g64[n]), rel_err(g, g64[n])
        assert e < max(3e-4, 3.0 * e_torch), (n, e, e_torch)
    assert abs(t.loss_log[0].item() - loss_ref.item()) < 1e-5 * max(1.0, abs(loss_ref.item()))
    assert ms.get_step() == 1 and all(torch.isfinite(v).all() for v in ms.views(ms.param).values())


def test_fp32_adadelta_step_matches_torch(cuda_device):
    """One step: parameters after the engine's update == torch.optim.Adadelta applied to the
    reference gradients (lr = 1, the reference optimizer, mnist_ddp.py:176)."""
    B = 128
    ref, ms, t, tr, _ = _trainer(cuda_device, B, B, dropout=False)
    idx = torch.arange(B)
    t.train_epoch(1, idx)
    t.synchronize()
    net = copy.deepcopy(ref)
    opt = torch.optim.Adadelta(net.parameters(), lr=1.0)
    _, _, g_ref = reference_step(ref, tr.images[idx], tr.targets[idx])
    for n, p in net.named_parameters():
        p.grad = g_ref[n].clone()
    opt.step()
    got = ms.views(ms.param)
    for n, p in net.named_parameters():
        d_ref = p.detach() - dict(ref.named_parameters())[n].detach()
        d_got = got[n].cpu() - dict(ref.named_parameters())[n].detach()
        assert rel_err(d_got, d_ref) < 1e-3, n


def test_fp32_eval_matches_torch_fp32(cuda_device):
    ref, ms, t, tr, te = _trainer(cuda_device, 200, 400, dropout=True, n_test=3000)
    loss_sum, correct, n = t.evaluate()
    with torch.no_grad():
        lp = reference_forward(copy.deepcopy(ref).float(), normalize_u8(te.images), train=False)
    nll = -lp.gather(1, te.targets.view(-1, 1).long()).squeeze(1)
    assert n == 3000
    assert abs(loss_sum - float(nll.double().sum())) < 1e-4 * float(nll.double().sum())
    assert abs(correct - int((lp.argmax(1) == te.targets).sum())) <= 2    # near-tie argmaxes aside


def test_fp32_training_graphs_bitwise_equal_eager_and_converge(cuda_device):
    idx = torch.randperm(2000, generator=torch.Generator().manual_seed(3))
    _, ms_g, tg, _, _ = _trainer(cuda_device, 200, 2000, dropout=True, graph_steps=4, n_test=1000)
    _, ms_e, te, _, _ = _trainer(cuda_device, 200, 2000, dropout=True, graph_steps=0, n_test=1000)
    l0, _, n = tg.evaluate()
    for ep in (1, 2, 3):
        tg.train_epoch(ep, idx)
        te.train_epoch(ep, idx)
    torch.cuda.synchronize()
    assert torch.equal(ms_g.param, ms_e.param)
    assert torch.equal(tg.loss_log, te.loss_log)
    l1, c1, _ = tg.evaluate()
    assert l1 < 0.5 * l0 and c1 / n > 0.75, (l0 / n, l1 / n, c1 / n)   # 30 steps: 2.30 -> 0.50, 83.7 %


@pytest.mark.parametrize("graph_steps", [0, 4])
def test_fp32_overlap_schedule_bitwise_equals_serial(cuda_device, graph_steps):
    """The fp32 OVERLAP schedule (the fc update on the comm stream beside the conv backward, the next
    step's first kernel held by device counters; split-captured chunks) trains bitwise like SERIAL."""
    idx = torch.randperm(2000, generator=torch.Generator().manual_seed(5))
    _, ms_o, to, _, _ = _trainer(cuda_device, 200, 2000, dropout=True, graph_steps=graph_steps, overlap=True)
    _, ms_s, ts, _, _ = _trainer(cuda_device, 200, 2000, dropout=True, graph_steps=graph_steps)
    for ep in (1, 2):
        to.train_epoch(ep, idx)
        ts.train_epoch(ep, idx)
    to.synchronize()
    ts.synchronize()
    assert torch.equal(ms_o.param, ms_s.param)
    assert torch.equal(ms_o.square_avg, ms_s.square_avg) and torch.equal(ms_o.acc_delta, ms_s.acc_delta)
    assert torch.equal(to.loss_log, ts.loss_log)
    assert ms_o.get_step() == ms_s.get_step()


def test_mnist_ddp_dtype_fp32_runs_fused_fp32(cuda_device, tmp_path):
    """mnist_ddp.py --dtype fp32 trains through the fused engine's fp32 step (not torch ops)."""
    env = dict(os.environ, PYTHONPATH=ROOT, MNIST_AMD_NO_BUILD="1")
    cmd = [sys.executable, os.path.join(ROOT, "mnist_ddp.py"), "--epochs", "1", "--batch-size", "200",
           "--synthetic", "--synthetic-train-size", "2000", "--synthetic-test-size", "1000", "--dtype", "fp32",
           "--json-log", str(tmp_path / "log.jsonl")]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Test set: Average loss:" in r.stdout and "Total cost time" in r.stdout
    import json
    recs = [json.loads(ln) for ln in open(tmp_path / "log.jsonl")]
    assert any("epoch" in rec and rec.get("steps") == 10 for rec in recs)
