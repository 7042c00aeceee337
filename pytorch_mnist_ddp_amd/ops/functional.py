"""Kernel-level functional API over torch tensors.

Each function launches exactly one of the hand-written kernels on the current torch stream,
with torch-allocated inputs/outputs.  These are the units the numerics tests compare against
fp32 torch references (SURVEY §4 tier T1) and the building blocks of the module-level
``Net.forward`` on GPU.  ``StepBuffers`` allocates every per-batch activation at once.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import native

NFLAT, NH, NCLS = 9216, 128, 10
DYC_REC = 144                       # compact dy record bytes (csrc/include/kernels.h DYC_REC)


def _C():
    return native.load()


def _s() -> int:
    return native.stream_handle()


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class StepBuffers:
    B: int
    a1: torch.Tensor          # bf16 [B,26,26,32]
    p: torch.Tensor           # bf16 [Bp64, 9216]
    pmask: torch.Tensor       # u8 [B, 9216]
    z1part: torch.Tensor      # f32 [KSPLIT, B, 128]
    loss_rows: torch.Tensor   # f32 [B]
    dz1: torch.Tensor         # bf16 [Bp64, 128]
    h_bf: torch.Tensor        # bf16 [Bp64, 128]
    dl_bf: torch.Tensor       # bf16 [Bp64, 16]
    dyc: torch.Tensor         # uint8 [B, 144*144] compact grad wrt conv2 output (pooled grads + argmax planes)
    fcpart: torch.Tensor      # f32 fc-gradient split partials (B > 1024), else a 1-element placeholder
    c1part: torch.Tensor      # f32 [4B, 320]
    w2part: torch.Tensor      # f32 [G, 18496]
    correct: torch.Tensor     # i32 [B]
    logp: torch.Tensor        # f32 [B, 10]

    @staticmethod
    def allocate(B: int, device) -> "StepBuffers":
        C = _C()
        Bp = round_up(B, 64)
        G = C.conv_wgrad_groups(B)
        z = dict(device=device)
        bf = dict(dtype=torch.bfloat16, device=device)
        return StepBuffers(
            B=B,
            a1=torch.zeros(B, 26, 26, 32, **bf),
            p=torch.zeros(Bp, NFLAT, **bf),
            pmask=torch.zeros(B, NFLAT, dtype=torch.uint8, **z),
            z1part=torch.zeros(C.FC1_KSPLIT, B, NH, dtype=torch.float32, **z),
            loss_rows=torch.zeros(B, dtype=torch.float32, **z),
            dz1=torch.zeros(Bp, NH, **bf),
            h_bf=torch.zeros(Bp, NH, **bf),
            dl_bf=torch.zeros(Bp, 16, **bf),
            dyc=torch.zeros(B, 144 * DYC_REC, dtype=torch.uint8, device=device),
            fcpart=torch.zeros(max(1, (C.fc_bwd_splits(B) > 1) * C.fc_bwd_splits(B) * C.FCB_PART_STRIDE),
                               dtype=torch.float32, device=device),
            c1part=torch.zeros(4 * B, 320, dtype=torch.float32, **z),
            w2part=torch.zeros(G, 18432 + 64, dtype=torch.float32, **z),
            correct=torch.zeros(B, dtype=torch.int32, **z),
            logp=torch.zeros(B, NCLS, dtype=torch.float32, **z),
        )


def pmask_flat(pmask: torch.Tensor) -> torch.Tensor:
    """The trunk's pool/dropout flags in torch flatten order [B, 9216] (channel-major) from the device
    layout [B][36][64][4] (pooled position / 4, channel, position % 4; mnist_common.h)."""
    B = pmask.shape[0]
    return pmask.view(B, 36, 64, 4).permute(0, 2, 1, 3).reshape(B, 9216)


def trunk_fwd(ms, data_u8: torch.Tensor, idx: torch.Tensor, buf: StepBuffers, train: bool,
              idx_stride: int = 0, state: torch.Tensor | None = None) -> None:
    p, o = native.ptr, ms.offsets
    _C().trunk_fwd(p(data_u8), p(idx), idx_stride, p(state if state is not None else ms.state),
                   p(ms.param) + 4 * o["conv1.weight"], p(ms.param) + 4 * o["conv1.bias"], p(ms.w2f),
                   p(ms.param) + 4 * o["conv2.bias"], p(buf.a1) if train else 0, p(buf.p),
                   p(buf.pmask) if train else 0, buf.B, train, _s())


def fc1_fwd(ms, buf: StepBuffers) -> None:
    p = native.ptr
    _C().fc1_fwd(p(buf.p), p(ms.w1), p(buf.z1part), buf.B, _s())


def head_train(ms, labels: torch.Tensor, idx: torch.Tensor, buf: StepBuffers, idx_stride: int = 0) -> None:
    p, o = native.ptr, ms.offsets
    B = buf.B
    _C().head_train(p(buf.z1part), p(ms.param) + 4 * o["fc1.bias"], p(ms.param) + 4 * o["fc2.weight"],
                    p(ms.param) + 4 * o["fc2.bias"], p(labels), p(idx), idx_stride, p(ms.state), 1.0 / B,
                    p(buf.loss_rows), p(buf.dz1), p(buf.h_bf), p(buf.dl_bf), B, round_up(B, 32), _s())


def head_eval(ms, labels: torch.Tensor | None, idx: torch.Tensor | None, buf: StepBuffers) -> None:
    p, o = native.ptr, ms.offsets
    _C().head_eval(p(buf.z1part), p(ms.param) + 4 * o["fc1.bias"], p(ms.param) + 4 * o["fc2.weight"],
                   p(ms.param) + 4 * o["fc2.bias"], p(labels), p(idx), p(buf.loss_rows), p(buf.correct),
                   p(buf.logp), buf.B, _s())


def fc_bwd(ms, buf: StepBuffers, grad_scale: float = 1.0, loss_log: torch.Tensor | None = None) -> None:
    p = native.ptr
    B = buf.B
    _C().fc_bwd(p(buf.dz1), p(buf.p), p(buf.pmask), p(ms.w1t), p(buf.h_bf), p(buf.dl_bf), p(buf.loss_rows),
                p(ms.state), p(ms.grad), p(buf.dyc), p(loss_log), grad_scale, 1.0 / B, B, round_up(B, 32), _s(),
                part=p(buf.fcpart))


def conv_bwd(ms, data_u8: torch.Tensor, idx: torch.Tensor, buf: StepBuffers, grad_scale: float = 1.0,
             idx_stride: int = 0) -> None:
    p, o = native.ptr, ms.offsets
    _C().conv_bwd(p(buf.dyc), p(buf.a1), p(ms.w2d), p(ms.param) + 4 * o["conv1.weight"],
                  p(ms.param) + 4 * o["conv1.bias"], p(data_u8), p(idx), idx_stride, p(ms.state),
                  p(buf.c1part), p(buf.w2part), p(ms.grad), grad_scale, buf.B, _s())


def adadelta_step(ms, region: int = 0, advance_step: bool = False) -> None:
    p = native.ptr
    _C().adadelta(p(ms.param), p(ms.grad), p(ms.square_avg), p(ms.acc_delta), p(ms.lr), ms.rho, ms.eps,
                  ms.weight_decay, p(ms.w2f), p(ms.w2d), p(ms.w1), p(ms.w1t),
                  p(ms.state) if advance_step else 0, region, True, _s())


def train_step(ms, data_u8, labels, idx, buf: StepBuffers, idx_stride: int = 0, grad_scale: float = 1.0,
               loss_log: torch.Tensor | None = None, update: bool = True) -> None:
    """One full fused training step (no DDP): fwd, loss, bwd, optional Adadelta."""
    trunk_fwd(ms, data_u8, idx, buf, True, idx_stride)
    fc1_fwd(ms, buf)
    head_train(ms, labels, idx, buf, idx_stride)
    fc_bwd(ms, buf, grad_scale, loss_log)
    conv_bwd(ms, data_u8, idx, buf, grad_scale, idx_stride)
    if update:
        adadelta_step(ms, 0, advance_step=True)


def eval_forward(ms, data_u8, labels, idx, buf: StepBuffers) -> None:
    trunk_fwd(ms, data_u8, idx, buf, False)
    fc1_fwd(ms, buf)
    head_eval(ms, labels, idx, buf)


def route_codes(planes: torch.Tensor) -> torch.Tensor:
    """[..., 16] uint8 code bit planes of a record (byte 2 c8 + p: bit j = bit p of channel 8 c8 + j's
    argmax code) -> [..., 64] int64 codes 0..3."""
    pl = planes.long().view(*planes.shape[:-1], 8, 2)              # [..., chunk, plane]
    bits = (pl.unsqueeze(-1) >> torch.arange(8, device=planes.device)) & 1   # [..., chunk, plane, j]
    return (bits[..., 0, :] | (bits[..., 1, :] << 1)).reshape(*planes.shape[:-1], 64)


def dense_dy(buf: StepBuffers) -> torch.Tensor:
    """Expand the compact un-pooled gradient records to the dense NHWC bf16 [B,24,24,64] map
    (what the conv backward kernels stage in LDS); for tests and tools."""
    B = buf.B
    rec = buf.dyc.view(B, 12, 12, DYC_REC)
    g = rec[..., :128].contiguous().view(torch.bfloat16).view(B, 12, 12, 64)
    code = route_codes(rec[..., 128:])                              # [B,12,12,64] window position
    dense = torch.zeros(B, 12, 2, 12, 2, 64, dtype=torch.bfloat16, device=g.device)
    for q in range(4):
        sel = (code == q)
        dense[:, :, q >> 1, :, q & 1, :] = torch.where(sel, g, torch.zeros_like(g))
    return dense.view(B, 24, 24, 64)

