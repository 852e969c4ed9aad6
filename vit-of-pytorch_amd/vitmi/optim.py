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

import math

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


# ---- Res-ViT: AdamW + clip_grad_norm_ + the cosine schedules (res-vit/train.py:64-66, 272-291) ----------
class AdamW(torch.optim.AdamW):
    """torch.optim.AdamW drop-in (decoupled weight decay, bias correction; amsgrad / maximize not
    implemented) whose step is csrc/optim.hip over one flat buffer of the parameters
    (vitmi.flat.FlatParams, built here: the parameters become views of it).

    `max_grad_norm` folds res-vit/train.py:64-66's `clip_grad_norm_(params, max_norm, 2)` into the step:
    the norm is reduced on the device and the scale applied inside the update (the clipped gradient is
    also written back to .grad, as clip_grad_norm_ leaves it). Without it, call vitmi.optim.
    clip_grad_norm_ before step() exactly as the reference does. Parameters that received no gradient
    this step are skipped (their step count, moments and weights unchanged), as torch does for
    `.grad is None`. torch's LR schedulers drive param_groups[0]['lr'] as usual."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False, *,
                 maximize=False, max_grad_norm=None, flat=None):
        if amsgrad or maximize:
            raise NotImplementedError("vitmi.optim.AdamW implements amsgrad=False, maximize=False (the reference's)")
        params = [p for p in params if p.requires_grad] if flat is None else flat.params
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        if len(self.param_groups) != 1:
            raise NotImplementedError("vitmi.optim.AdamW: one parameter group")
        from .flat import FlatParams
        self.flat = flat if flat is not None else FlatParams(self.param_groups[0]["params"])
        f = self.flat
        self.max_grad_norm = max_grad_norm
        self.exp_avg = torch.zeros_like(f.data)
        self.exp_avg_sq = torch.zeros_like(f.data)
        self.steps = torch.zeros(f.nseg, device=f.device)
        self._table = torch.zeros(f.nseg, 4, device=f.device)
        self._parts = torch.zeros(f.sq_norm_parts(), device=f.device, dtype=torch.float64)
        self.last_norm = torch.zeros(2, device=f.device)  # {total grad norm, clip coefficient} of the last step
        for i, p in enumerate(f.params):
            self.state[p] = {"step": self.steps[i], "exp_avg": f.view(self.exp_avg, i),
                             "exp_avg_sq": f.view(self.exp_avg_sq, i)}

    def state_dict(self):
        """torch.optim.AdamW's format: state[i] = {step, exp_avg, exp_avg_sq} per parameter (copies of the
        flat moments), param_groups as torch's"""
        sd = super().state_dict()
        f = self.flat
        st = {}
        for k, p in enumerate(self.param_groups[0]["params"]):  # torch indexes state by group position
            i = f._index[id(p)]
            st[k] = {"step": self.steps[i].detach().clone(), "exp_avg": f.view(self.exp_avg, i).clone(),
                     "exp_avg_sq": f.view(self.exp_avg_sq, i).clone()}
        sd["state"] = st
        return sd

    def load_state_dict(self, state_dict):
        """copy a torch.optim.AdamW-format state into the flat moment / step buffers (the per-parameter
        state entries stay views of them, so step() keeps using what was loaded)"""
        f = self.flat
        groups = state_dict["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(f.params):
            raise ValueError("vitmi.optim.AdamW.load_state_dict: one group of %d parameters expected" % len(f.params))
        for k, v in groups[0].items():
            if k != "params":
                self.param_groups[0][k] = v
        for k, p in enumerate(self.param_groups[0]["params"]):
            i = f._index[id(p)]
            st = state_dict["state"].get(k, state_dict["state"].get(str(k)))
            if st is None:  # never stepped: zero moments
                f.view(self.exp_avg, i).zero_()
                f.view(self.exp_avg_sq, i).zero_()
                self.steps[i] = 0.0
                continue
            f.view(self.exp_avg, i).copy_(st["exp_avg"].reshape(f.params[i].shape))
            f.view(self.exp_avg_sq, i).copy_(st["exp_avg_sq"].reshape(f.params[i].shape))
            self.steps[i] = float(st["step"])

    def zero_grad(self, set_to_none: bool = True):
        """zero the flat gradient buffer (the .grad views stay in place; `set_to_none` semantics — a
        parameter without a gradient is skipped by step() — are kept by the used flags)"""
        self.flat.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        f = self.flat
        g = self.param_groups[0]
        beta1, beta2 = g["betas"]
        f.adopt_grads()
        used = f.upload_used()
        if self.max_grad_norm is not None:
            ops.sqnorm_partial(f.grad, f.numel, self._parts)
        ops.adamw_prep(self._parts if self.max_grad_norm is not None else None, used, self.steps, float(g["lr"]),
                       float(beta1), float(beta2), float(self.max_grad_norm or 0.0), self._table,
                       self.last_norm if self.max_grad_norm is not None else None)  # (else: clip_grad_norm_'s)
        ops.adamw_update(f.data, f.grad, self.exp_avg, self.exp_avg_sq, None, f.chunks, self._table, float(g["lr"]),
                         float(beta1), float(beta2), float(g["eps"]), float(g["weight_decay"]),
                         self.max_grad_norm is not None)
        for p in f.params:
            increment_version(p)
        return loss


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, flat=None):
    """torch.nn.utils.clip_grad_norm_ (res-vit/train.py:64-66) for parameters held by a
    vitmi.flat.FlatParams (pass it, or an AdamW owning it, as `flat`): the total 2-norm of every
    gradient reduced on the device (f64 partial sums, fixed order), then grads *= min(1, max_norm /
    (norm + 1e-6)). Returns the norm (a device scalar)."""
    if float(norm_type) != 2.0:
        raise NotImplementedError("clip_grad_norm_: norm_type 2 (the reference's)")
    f = getattr(flat, "flat", flat)
    if f is None:
        raise ValueError("clip_grad_norm_: pass the FlatParams (or vitmi AdamW) that holds the parameters")
    f.adopt_grads()
    parts = getattr(flat, "_parts", None)
    if parts is None:
        parts = torch.empty(f.sq_norm_parts(), device=f.device, dtype=torch.float64)
    out = getattr(flat, "last_norm", None)  # a vitmi AdamW keeps {norm, coef} of its last clip there
    if out is None:
        out = torch.empty(2, device=f.device)
    ops.sqnorm_partial(f.grad, f.numel, parts)
    ops.adamw_prep(parts, None, None, 0.0, 0.0, 0.0, float(max_norm), None, out)
    ops.scale_by_coef(f.grad, f.numel, out[1:])
    return out[0].clone()


def get_cosine_schedule_with_warmup(optimizer, num_warmup_steps, num_training_steps, num_cycles=0.5, last_epoch=-1):
    """transformers.get_cosine_schedule_with_warmup (res-vit/train.py:286-289; transformers' published
    schedule): linear warm-up from 0, then cosine decay to 0 over the remaining steps."""

    def lr_lambda(current_step):
        if current_step < num_warmup_steps:
            return float(current_step) / float(max(1, num_warmup_steps))
        progress = float(current_step - num_warmup_steps) / float(max(1, num_training_steps - num_warmup_steps))
        return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))

    return torch.optim.lr_scheduler.LambdaLR(optimizer, lr_lambda, last_epoch)
