"""torch.optim.SGD drop-in whose step runs on the HIP fused SGD-momentum kernel.

Semantics are torch.optim.SGD's (dampening 0, nesterov False), as configured by reference
src/train.py:154-158: d = g + wd*p; buf = d on the first step, else momentum*buf + d; p -= lr*buf.
It subclasses torch.optim.SGD so torch.optim.lr_scheduler.OneCycleLR (src/train.py:159-163,
cycle_momentum=True) drives its 'lr' / 'momentum' exactly as it drives the reference optimizer.

Fast path: when the optimizer holds exactly the parameters of one vitmi VisionTransformer in one
param group and their gradients are the engine's flat gradient buffer, one kernel launch updates
all parameters and refreshes the bf16 GEMM mirror in the same pass. Otherwise each parameter is
updated by the same kernel individually.
"""
from __future__ import annotations

import torch
from torch.autograd.graph import increment_version

from . import ops


class SGD(torch.optim.SGD):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, model=None):
        if dampening != 0.0 or nesterov:
            raise NotImplementedError("vitmi.optim.SGD implements dampening=0, nesterov=False (the reference config)")
        super().__init__(params, lr=lr, momentum=momentum, dampening=0.0, weight_decay=weight_decay,
                         nesterov=False)
        self._model = model
        self._flat_buf = None
        self._flat_first = True

    def _flat_engine(self):
        m = self._model
        if m is None or m._engine is None or len(self.param_groups) != 1 or not m._bound():
            return None
        eng = m._engine
        ps = self.param_groups[0]["params"]
        if len(ps) != len(m._flat_params) or set(map(id, ps)) != set(map(id, m._flat_params)):
            return None
        for n, p in zip(m._flat_names, m._flat_params):
            if p.grad is None or p.grad.data_ptr() != eng.layout.view(eng.grad, n).data_ptr():
                return None
        return eng

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        eng = self._flat_engine()
        if eng is not None:
            g = self.param_groups[0]
            if self._flat_buf is None:
                self._flat_buf = torch.zeros_like(eng.flat)
                for n, p in zip(self._model._flat_names, self._model._flat_params):
                    self.state[p]["momentum_buffer"] = eng.layout.view(self._flat_buf, n)
            ops.sgd_step(eng.flat, eng.grad, self._flat_buf, eng.mirror, eng.layout.numel, g["lr"], g["momentum"],
                         g["weight_decay"], self._flat_first)
            self._flat_first = False
            eng.refresh_mirror(full=False)           # repack q/k/v (+ padded conv) from updated masters
            eng.mark_mirror_fresh(self._model._version_sig())
            return loss
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.is_contiguous()):
                    raise TypeError("vitmi.optim.SGD expects contiguous fp32 GPU parameters and gradients")
                st = self.state[p]
                first = "momentum_buffer" not in st
                if first:
                    st["momentum_buffer"] = torch.empty_like(p)
                buf = st["momentum_buffer"]
                ops.sgd_step(p, p.grad, buf, None, p.numel(), group["lr"], group["momentum"], group["weight_decay"],
                             first)
                increment_version(p)  # raw-pointer update: let version-keyed bf16 mirrors see it
        return loss
