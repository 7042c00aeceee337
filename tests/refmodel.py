"""fp32 torch reference oracle for the numerics tests (never used by the product path).

``reference_step`` runs the reference forward/backward (mnist_ddp.py:49-72) with stock torch
ops in fp32 on the CPU, optionally with given dropout masks, and returns loss, log-probs and
per-parameter gradients.
"""
from __future__ import annotations

import copy

import torch
import torch.nn.functional as F

from pytorch_mnist_ddp_amd.data.datasets import normalize_u8


def reference_forward(net, x, mask1=None, mask2=None, train=True):
    x = F.relu(net.conv1(x))
    x = F.relu(net.conv2(x))
    x = F.max_pool2d(x, 2)
    if train and mask1 is not None:
        x = x * mask1.view_as(x) * (1.0 / 0.75)
    x = torch.flatten(x, 1)
    x = F.relu(net.fc1(x))
    if train and mask2 is not None:
        x = x * mask2.view_as(x) * 2.0
    x = net.fc2(x)
    return F.log_softmax(x, dim=1)


def reference_step(net, images_u8, labels, mask1=None, mask2=None, dtype=torch.float32):
    net = copy.deepcopy(net).cpu().to(dtype)
    net.zero_grad(set_to_none=True)
    x = normalize_u8(images_u8).to(dtype)
    mask1 = mask1.to(dtype) if mask1 is not None else None
    mask2 = mask2.to(dtype) if mask2 is not None else None
    out = reference_forward(net, x, mask1, mask2)
    loss = F.nll_loss(out, labels.long())
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
    return loss.detach(), out.detach(), grads


def rel_err(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


# ---------------------------------------------------------------- Philox-4x32-10 (numpy-free)
M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = (p0 >> 32) & MASK, p0 & MASK
        hi1, lo1 = (p1 >> 32) & MASK, p1 & MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0, k1 = (k0 + W0) & MASK, (k1 + W1) & MASK
    return c0, c1, c2, c3


def dropout_keep(seed: int, offset: int, elem: int, thr8: int) -> bool:
    """Kernel dropout rule: one Philox block per 16 elements, one byte per element, keep <=> byte < thr8."""
    blk = elem >> 4
    w = philox4x32((blk & MASK, blk >> 32, offset & MASK, offset >> 32), (seed & MASK, seed >> 32))
    k = elem & 15
    return ((w[k >> 2] >> (8 * (k & 3))) & 0xFF) < thr8


# ---------------------------------------------------------------- bf16-emulating reference
def emulated_bf16_step(net, images_u8, labels, mask1=None, mask2=None):
    """Manual fwd/bwd in float64 that rounds to bf16 exactly where the fused kernels do.

    Differences against the kernels are then only accumulation order (~1e-5 relative), so this
    oracle catches indexing/layout bugs that a bf16-vs-fp32 tolerance could hide.
    """
    import torch.nn.grad as G

    def q(t):
        return t.to(torch.float32).to(torch.bfloat16).to(torch.float64)

    d = {n: p.detach().cpu().double() for n, p in net.named_parameters()}
    B = images_u8.shape[0]
    x = normalize_u8(images_u8).double()
    z0 = F.conv2d(x, d["conv1.weight"], d["conv1.bias"])
    a1 = q(F.relu(z0))
    w2q = q(d["conv2.weight"])
    y2 = F.conv2d(a1, w2q, d["conv2.bias"])
    pooled, arg = F.max_pool2d(F.relu(y2), 2, return_indices=True)
    drop1 = mask1.double().view_as(pooled) * (1.0 / 0.75) if mask1 is not None else torch.ones_like(pooled)
    p = q(pooled * drop1).flatten(1)
    w1q = q(d["fc1.weight"])
    z1 = p @ w1q.t() + d["fc1.bias"]
    drop2 = mask2.double().view_as(z1) * 2.0 if mask2 is not None else torch.ones_like(z1)
    h = F.relu(z1) * drop2
    logits = h @ d["fc2.weight"].t() + d["fc2.bias"]
    lp = F.log_softmax(logits, 1)
    y = labels.long()
    loss = -lp.gather(1, y.view(-1, 1)).mean()
    dl = (lp.exp() - F.one_hot(y, 10).double()) / B
    dh = dl @ d["fc2.weight"]
    dz1 = dh * drop2 * (z1 > 0)
    dz1q, hq, dlq = q(dz1), q(h), q(dl)
    grads = {"fc2.weight": dlq.t() @ hq, "fc2.bias": dlq.sum(0),
             "fc1.weight": dz1q.t() @ p, "fc1.bias": dz1q.sum(0)}
    dp = dz1q @ w1q
    g = q(dp * drop1.flatten(1) * (pooled.flatten(1) > 0)).view_as(pooled)
    dy = F.max_unpool2d(g, arg, 2, output_size=y2.shape[-2:])
    grads["conv2.weight"] = G.conv2d_weight(a1, w2q.shape, dy)
    grads["conv2.bias"] = dy.sum((0, 2, 3))
    da1 = G.conv2d_input(a1.shape, w2q, dy) * (z0 > 0)
    # conv1 weight/bias gradient: bf16 MFMA operands (input image and masked da1), fp32 accumulation
    grads["conv1.weight"] = G.conv2d_weight(q(x), d["conv1.weight"].shape, q(da1))
    grads["conv1.bias"] = q(da1).sum((0, 2, 3))
    return loss, lp, grads
