"""Device-resident model + optimizer state in the flat layouts the native kernels use.

* ``param`` / ``grad``: one fp32 buffer each (``PARAM_TOTAL`` = 1,200,000 elements; every tensor
  256-byte aligned).  The module's ``nn.Parameter``s are re-pointed at views of ``param`` and
  their ``.grad`` at views of ``grad`` - the gradient buffer *is* the DDP bucket storage
  (torch DDP's ``gradient_as_bucket_view=True`` taken to its conclusion: no copy-in/copy-out).
  Bucket 0 = fc params (98.4 % of bytes, ready first in backward), bucket 1 = conv params:
  the same rebuilt bucket layout torch DDP converges to for this model.
* ``square_avg`` / ``acc_delta``: Adadelta state, same flat layout.
* bf16 shadows ``w2f``, ``w2d``, ``w1``, ``w1t``: refreshed by the optimizer kernel.
* ``state``: the 24-byte device ``StepState`` (step counter, flags, Philox seed / base).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import native

FLAG_NO_DROPOUT = 1


class ModelState:
    def __init__(self, module: nn.Module, device: torch.device, lr: float = 1.0, rho: float = 0.9,
                 eps: float = 1e-6, weight_decay: float = 0.0):
        C = native.load()
        self.C = C
        self.device = torch.device(device)
        self.offsets = dict(C.PARAM_OFFSETS)
        total = int(C.PARAM_TOTAL)
        self.bucket_split = int(C.BUCKET_SPLIT)
        # device buffers zeroed by hipMemset / filled by H2D copies: no torch kernel launches
        # (their code objects would load on first use inside the reference timer)
        z = native.zeros
        f32, dev = torch.float32, self.device
        self.param = z(total, f32, dev)
        self.grad = z(total, f32, dev)
        self.square_avg = z(total, f32, dev)
        self.acc_delta = z(total, f32, dev)
        self.lr = native.host_to_device([float(lr)], f32, dev)
        self.rho, self.eps, self.weight_decay = rho, eps, weight_decay
        bf = torch.bfloat16
        self.w2f = z(64 * 9 * 32, bf, dev)
        self.w2d = z(9 * 32 * 64, bf, dev)
        self.w1 = z(128 * 9216, bf, dev)
        self.w1t = z(9216 * 128, bf, dev)
        self.state = z(3, torch.int64, dev)  # StepState (24 B)
        self.module = module
        self.bind(module)

    # ------------------------------------------------------------------ parameter binding
    def views(self, buf: torch.Tensor) -> dict[str, torch.Tensor]:
        out = {}
        for name, p in self.module.named_parameters():
            off = self.offsets[name]
            out[name] = buf[off:off + p.numel()].view(p.shape)
        return out

    def bind(self, module: nn.Module) -> None:
        """Copy the module's parameters into the flat buffer and alias them to it."""
        with torch.no_grad():
            for name, p in module.named_parameters():
                if name not in self.offsets:
                    raise KeyError(f"unexpected parameter {name}")
                off = self.offsets[name]
                view = self.param[off:off + p.numel()].view(p.shape)
                view.copy_(p.detach().to(self.device, torch.float32))
                p.data = view
                p.grad = self.grad[off:off + p.numel()].view(p.shape)
                p._amd_model_state = self     # lets the fused Adadelta find the flat buffers
        self.refresh_shadows()

    def refresh_shadows(self, stream: torch.cuda.Stream | None = None) -> None:
        C = self.C
        p = native.ptr
        C.adadelta(p(self.param), p(self.grad), p(self.square_avg), p(self.acc_delta), p(self.lr),
                   self.rho, self.eps, self.weight_decay, p(self.w2f), p(self.w2d), p(self.w1), p(self.w1t),
                   0, 0, False, native.stream_handle(stream))

    def buffers(self) -> dict[str, int]:
        p = native.ptr
        return {"param": p(self.param), "grad": p(self.grad), "square_avg": p(self.square_avg),
                "acc_delta": p(self.acc_delta), "lr": p(self.lr), "w2f": p(self.w2f), "w2d": p(self.w2d),
                "w1": p(self.w1), "w1t": p(self.w1t), "state": p(self.state)}

    def set_state(self, step: int, seed: int, rng_base: int, flags: int = 0) -> None:
        """Write the device StepState (step | flags<<32, seed, rng_base)."""
        packed = (int(step) & 0xFFFFFFFF) | ((int(flags) & 0xFFFFFFFF) << 32)
        vals = [packed, int(seed), int(rng_base)]
        vals = [v - (1 << 64) if v >= (1 << 63) else v for v in vals]
        self.state.copy_(torch.tensor(vals, dtype=torch.int64))

    def get_step(self) -> int:
        return int(self.state[0].item()) & 0xFFFFFFFF
