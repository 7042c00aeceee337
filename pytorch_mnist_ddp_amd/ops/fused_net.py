"""Module-level GPU path: ``Net.forward(x)`` on a CUDA/ROCm tensor runs the fused MI355X kernels.

This is the reference's programming model (mnist_ddp.py:65-73: ``output = model(data);
loss = F.nll_loss(output, target); loss.backward(); optimizer.step()``) on the hand-written
kernels, with autograd.  One ``torch.autograd.Function`` covers the whole network:

forward  = TrunkFunction: trunk_fwd (conv1 -> conv2 MFMA -> ReLU -> max-pool -> dropout-1)
           HeadFunction:  fc1 split-K MFMA -> head_fwd (bias -> ReLU -> dropout-2 -> fc2 -> log_softmax)
backward = HeadFunction:  head_train (generic log_softmax backward from dlogp) -> fc_bwd
           [fc params' AccumulateGrad -> DDP hooks -> bucket 0 all-reduce launched]
           TrunkFunction: conv_bwd  [conv params' hooks -> bucket 1]
Two Functions (not one) so that autograd finalises the fc gradients - and DDP's hooks launch their
bucket's all-reduce on the comm stream - before conv_bwd is even enqueued (reference DDP overlap,
mnist_ddp.py:72).

Dropout masks come from the same counter-based Philox stream as the engine: the forward draws
a fresh (seed, offset) pair per call and the backward replays exactly that pair, so masks are
consistent without being stored (dropout-1's keep bits are in the saved pmask anyway).  Per-batch
activation sets are pooled per batch size (taken by the forward, returned after the backward's
last launch, or right after an eval forward): no per-step allocation or memset.

The module's parameters are re-pointed at a flat device buffer (``engine.state.ModelState``) on
the first GPU forward; the bf16 shadow copies the kernels read are refreshed lazily whenever any
parameter's version counter moved (an optimizer step, ``load_state_dict``, manual edits), so any
optimizer - ours or stock torch - can drive it.
"""
from __future__ import annotations

import torch

from . import native
from .functional import StepBuffers, round_up

_SEED_MIX = 0x9E3779B97F4A7C15


class _FusedState:
    def __init__(self, net, device):
        from ..engine.state import ModelState
        self.ms = ModelState(net, device)
        self.params = list(net.parameters())
        self.versions = self._snapshot()
        self.rng_offset = 0
        self.seed = (torch.initial_seed() * _SEED_MIX) & 0xFFFFFFFFFFFFFFFF
        self.pool: dict[tuple[int, int], list[StepBuffers]] = {}   # free sets per (batch, stream)
        self.last_pass = None             # TrunkFunction.forward -> the HeadFunction.forward after it

    def take(self, B: int, device) -> StepBuffers:
        """A per-batch activation set: reused when one is free (kernels are stream ordered on the
        current stream, so a set released after its last launch can be refilled by the next call)."""
        free = self.pool.get((B, native.stream_handle()))   # same stream only: ordering is the guard
        return free.pop() if free else StepBuffers.allocate(B, device)

    def give(self, buf: StepBuffers) -> None:
        self.pool.setdefault((buf.B, native.stream_handle()), []).append(buf)

    def _snapshot(self):
        return tuple((p._version, p.data_ptr()) for p in self.params)

    def sync(self):
        snap = self._snapshot()
        if snap != self.versions:
            ptrs = tuple(self.ms.views(self.ms.param)[n].data_ptr()
                         for n, _ in self.ms.module.named_parameters())
            if tuple(s[1] for s in snap) != ptrs:      # parameters were re-assigned: re-bind
                self.ms.bind(self.ms.module)
            else:
                self.ms.refresh_shadows()
            self.versions = self._snapshot()


def fused_state(net) -> _FusedState:
    st = getattr(net, "_amd_fused_state", None)
    dev = next(net.parameters()).device
    if st is None or st.ms.device != dev:
        st = _FusedState(net, dev)
        object.__setattr__(net, "_amd_fused_state", st)
    return st


def _dropout_flags(net) -> int:
    p1, p2 = net.dropout1.p, net.dropout2.p
    if (p1, p2) == (0.25, 0.5):
        return 0
    if (p1, p2) == (0.0, 0.0):
        return 1                                   # STEP_FLAG_NO_DROPOUT
    raise NotImplementedError(f"fused GPU Net supports dropout (0.25, 0.5) or (0, 0), got ({p1}, {p2})")


def _step_state(st: _FusedState, training: bool, device, flags: int = 0) -> torch.Tensor:
    t = torch.zeros(3, dtype=torch.int64)
    t[0] = (flags & 0xFFFFFFFF) << 32
    if training:
        t[1] = st.seed - (1 << 64) if st.seed >= (1 << 63) else st.seed
        t[2] = st.rng_offset
        st.rng_offset += 2
    return t.to(device, non_blocking=True)


class _Pass:
    """Per-call state the two Functions share: the activation set, the step state and (backward)
    the flat gradient buffer both halves write."""
    __slots__ = ("buf", "state", "grad", "x")

    def __init__(self, buf, state, x):
        self.buf, self.state, self.x, self.grad = buf, state, x, None


class TrunkFunction(torch.autograd.Function):
    """conv1 -> conv2 MFMA -> ReLU -> max-pool -> dropout-1 (trunk_fwd); backward = conv_bwd (conv2
    dgrad + wgrad, conv1 wgrad, fixed-order reduce).  Its output is the pooled bf16 feature map the
    head consumes; its "gradient" is the compact dy records fc_bwd left in the shared activation
    set, so the incoming tensor is a stride-0 placeholder."""

    @staticmethod
    def forward(ctx, x, st, training, flags, c1w, c1b, c2w, c2b):
        C = native.load()
        ms = st.ms
        p, o = native.ptr, ms.offsets
        x = x.reshape(x.shape[0], -1).to(torch.float32).contiguous()
        if x.shape[1] != 784:
            raise ValueError(f"Net expects [B,1,28,28] inputs, got {tuple(x.shape)}")
        B = x.shape[0]
        buf = st.take(B, x.device)
        state = _step_state(st, training, x.device, flags)
        P = p(ms.param)
        C.trunk_fwd(0, 0, 0, p(state), P + 4 * o["conv1.weight"], P + 4 * o["conv1.bias"], p(ms.w2f),
                    P + 4 * o["conv2.bias"], p(buf.a1) if training else 0, p(buf.p),
                    p(buf.pmask) if training else 0, B, bool(training), native.stream_handle(), xin=p(x))
        ctx.training = bool(training)
        ctx.st = st
        ctx.pas = _Pass(buf, state, x)
        st.last_pass = ctx.pas            # picked up by the HeadFunction.apply that follows
        return buf.p[:B]                  # differentiable: links the head's backward to ours

    @staticmethod
    def backward(ctx, dfeat):
        if not ctx.training:
            raise RuntimeError("fused Net backward requires model.train() mode during forward")
        C = native.load()
        st, pas = ctx.st, ctx.pas
        buf, ms = pas.buf, st.ms
        if pas.grad is None:
            raise RuntimeError("fused Net: the trunk backward ran without the head backward")
        p, o = native.ptr, ms.offsets
        P = p(ms.param)
        C.conv_bwd(p(buf.dyc), p(buf.a1), p(ms.w2d), P + 4 * o["conv1.weight"], P + 4 * o["conv1.bias"],
                   0, 0, 0, p(pas.state), p(buf.c1part), p(buf.w2part), p(pas.grad), 1.0, buf.B,
                   native.stream_handle(), xin=p(pas.x))
        st.give(buf)                      # last use enqueued: the next forward may refill it
        grad = pas.grad
        ctx.pas = None
        views = [grad[o[n]:o[n] + t.numel()].view(t.shape) for n, t in _named(ms, _CONV)]
        return (None, None, None, None, *views)


class HeadFunction(torch.autograd.Function):
    """fc1 split-K MFMA -> bias -> ReLU -> dropout-2 -> fc2 -> log_softmax (fc1_fwd + head_fwd);
    backward = head_train + fc_bwd: the fc gradients (DDP bucket 0, 98.4 % of the bytes) are final
    when this returns, so their hooks - and bucket 0's all-reduce - fire BEFORE the trunk's backward
    (conv_bwd) is enqueued, exactly torch DDP's overlap of the fc bucket with the conv backward."""

    @staticmethod
    def forward(ctx, feat, st, training, f1w, f1b, f2w, f2b):
        C = native.load()
        ms = st.ms
        pas, st.last_pass = st.last_pass, None
        p, o = native.ptr, ms.offsets
        buf = pas.buf
        B = buf.B
        s = native.stream_handle()
        P = p(ms.param)
        C.fc1_fwd(p(buf.p), p(ms.w1), p(buf.z1part), B, s)
        logp = torch.empty(B, 10, dtype=torch.float32, device=feat.device)
        C.head_fwd(p(buf.z1part), P + 4 * o["fc1.bias"], P + 4 * o["fc2.weight"], P + 4 * o["fc2.bias"],
                   p(pas.state), p(logp), B, bool(training), s)
        ctx.training = bool(training)
        ctx.st, ctx.pas = st, pas
        if not training:
            st.give(buf)                  # eval: nothing of the set is needed after the forward
        return logp

    @staticmethod
    def backward(ctx, dlogp):
        if not ctx.training:
            raise RuntimeError("fused Net backward requires model.train() mode during forward")
        C = native.load()
        st, pas = ctx.st, ctx.pas
        buf, ms = pas.buf, st.ms
        p, o = native.ptr, ms.offsets
        B = buf.B
        s = native.stream_handle()
        P = p(ms.param)
        dlogp = dlogp.to(torch.float32).contiguous()
        pas.grad = grad = torch.empty_like(ms.grad)
        C.head_train(p(buf.z1part), P + 4 * o["fc1.bias"], P + 4 * o["fc2.weight"], P + 4 * o["fc2.bias"],
                     0, 0, 0, p(pas.state), 1.0 / B, p(buf.loss_rows), p(buf.dz1), p(buf.h_bf), p(buf.dl_bf),
                     B, round_up(B, 32), s, dlogp=p(dlogp))
        C.fc_bwd(p(buf.dz1), p(buf.p), p(buf.pmask), p(ms.w1t), p(buf.h_bf), p(buf.dl_bf), p(buf.loss_rows),
                 p(pas.state), p(grad), p(buf.dyc), 0, 1.0, 1.0 / B, B, round_up(B, 32), s, part=p(buf.fcpart))
        ctx.pas = None
        views = [grad[o[n]:o[n] + t.numel()].view(t.shape) for n, t in _named(ms, _FC)]
        dfeat = _placeholder(buf.p.device, B)          # the real dy lives in buf.dyc
        return (dfeat, None, None, *views)


_CONV = ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias")
_FC = ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias")
_ZERO = {}


def _named(ms, names):
    params = dict(ms.module.named_parameters())
    return [(n, params[n]) for n in names]


def _placeholder(device, B: int) -> torch.Tensor:
    z = _ZERO.get(device)
    if z is None:
        z = _ZERO[device] = torch.zeros(1, 1, dtype=torch.bfloat16, device=device)
    return z.expand(B, 9216)


def fused_net_forward(net, x: torch.Tensor) -> torch.Tensor:
    st = fused_state(net)
    st.sync()
    flags = _dropout_flags(net) if net.training else 0
    named = dict(net.named_parameters())
    feat = TrunkFunction.apply(x, st, net.training, flags, *(named[n] for n in _CONV))
    return HeadFunction.apply(feat, st, net.training, *(named[n] for n in _FC))
