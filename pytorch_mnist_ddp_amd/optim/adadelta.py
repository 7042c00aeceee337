"""Adadelta (reference mnist_ddp.py:176: ``optim.Adadelta(model.parameters(), lr=args.lr)``).

A ``torch.optim.Adadelta`` subclass, so ``StepLR``, ``state_dict()``/``load_state_dict()`` and the
param-group API behave exactly like the reference's optimizer.  When the parameters belong to a
GPU :class:`~pytorch_mnist_ddp_amd.engine.state.ModelState` (the fused module path or the engine),
``step()`` is one launch of the fused multi-tensor HIP kernel over the flat buffer (update +
bf16 shadow refresh) instead of torch's ~11 foreach kernels; the per-parameter optimizer state
(``square_avg``, ``acc_delta``) is exposed as views of the flat state buffers so checkpoints have
torch's format.  On CPU it is stock torch Adadelta.
"""
from __future__ import annotations

import torch


class Adadelta(torch.optim.Adadelta):
    def __init__(self, params, lr: float = 1.0, rho: float = 0.9, eps: float = 1e-6, weight_decay: float = 0.0,
                 model_state=None):
        super().__init__(params, lr=lr, rho=rho, eps=eps, weight_decay=weight_decay)
        self._ms = model_state

    def _fused_state(self):
        if self._ms is not None:
            return self._ms
        params = [p for g in self.param_groups for p in g["params"]]
        for p in params:
            st = getattr(p, "_amd_model_state", None)
            if st is None:
                return None
        ms = getattr(params[0], "_amd_model_state", None)
        return ms if all(getattr(p, "_amd_model_state", None) is ms for p in params) else None

    @torch.no_grad()
    def step(self, closure=None):
        ms = self._fused_state()
        if ms is None or not ms.param.is_cuda or len(self.param_groups) != 1:
            return super().step(closure)
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        if g["rho"] != ms.rho or g["eps"] != ms.eps or g["weight_decay"] != ms.weight_decay:
            ms.rho, ms.eps, ms.weight_decay = g["rho"], g["eps"], g["weight_decay"]
        ms.lr.fill_(float(g["lr"]))
        sq_views, acc_views = ms.views(ms.square_avg), ms.views(ms.acc_delta)
        grad_views = ms.views(ms.grad)
        for name, p in ms.module.named_parameters():
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32)
                st["square_avg"] = sq_views[name]
                st["acc_delta"] = acc_views[name]
            st["step"] += 1
            gv = grad_views[name]
            if p.grad is None:
                gv.zero_()
            elif p.grad.data_ptr() != gv.data_ptr():
                gv.copy_(p.grad)
        from ..ops.functional import adadelta_step
        adadelta_step(ms)
        # the kernel wrote params in place: bump versions so lazily-refreshed consumers stay in sync
        fused = None
        for p in ms.module.parameters():
            fused = getattr(ms.module, "_amd_fused_state", None)
            break
        if fused is not None:
            fused.versions = fused._snapshot()
        return loss

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        ms = self._fused_state()
        if ms is not None:   # copy loaded tensors into the flat state and re-alias
            sq_views, acc_views = ms.views(ms.square_avg), ms.views(ms.acc_delta)
            for name, p in ms.module.named_parameters():
                st = self.state.get(p)
                if st and "square_avg" in st:
                    sq_views[name].copy_(st["square_avg"])
                    acc_views[name].copy_(st["acc_delta"])
                    st["square_avg"], st["acc_delta"] = sq_views[name], acc_views[name]
