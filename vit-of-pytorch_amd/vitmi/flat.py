"""One flat f32 buffer behind a set of nn.Parameters and one behind their gradients.

The Res-ViT training step (res-vit/train.py:51-68) clips and updates every trainable parameter
(`clip_grad_norm_(model.parameters(), 1.0)`, `AdamW.step()`); here those parameters are re-homed as
views of ONE flat buffer (64-element aligned segments, one per parameter, in reverse registration
order — roughly the order the backward finishes them), so the clip norm, the AdamW update and the
data-parallel gradient all-reduce are a handful of launches over contiguous memory
(csrc/optim.hip, vitmi.dist.FlatGradAllReducer) instead of per-tensor loops.

Gradients: each parameter's `.grad` is preset to its view of the flat gradient buffer; autograd
accumulates into an existing `.grad` in place, so the backward writes the flat buffer directly. A
post-accumulate hook marks which parameters received a gradient in this step — torch's AdamW skips a
parameter whose `.grad` is None (an approximator no token was routed to), and so does the HIP update
(`used` flags; vit_adamw_prep). The fused Res-ViT nodes (vitmi.resvit_fused) go one step further: their
weight-gradient reductions accumulate straight into a flat `.grad` view (`grad_sink`) and return None for
that parameter, so no AccumulateGrad add runs at all; they then run the same marking. A `.grad` replaced behind our back (module.zero_grad() setting it to
None, then a fresh tensor from autograd) is folded back into the flat buffer by `adopt_grads()`.
"""
from __future__ import annotations

import contextlib
import math
import weakref

import torch

from . import ops

ALIGN = 64

# parameter -> device bool scalar: this step's "did the parameter take part" for parameters whose
# forward runs on every row and selects (Res-ViT's approximators): the flat optimizer ANDs it into the
# used flags without a host synchronisation
_GATES = {}  # id(parameter) -> (weakref to it, flag)


def gate(params, flag):
    if len(_GATES) > 4096:  # (gated parameters no flat optimizer collects)
        _GATES.clear()
    for p in params:
        e = _GATES.get(id(p))
        if e is not None and e[0]() is p:  # a forward already ran this step (gradient accumulation, a shared
            flag = torch.logical_or(e[1], flag)  # module): the parameter took part if ANY call routed rows
        _GATES[id(p)] = (weakref.ref(p), flag)


def _take_gate(p):
    e = _GATES.get(id(p))
    if e is None or e[0]() is not p:
        return None
    del _GATES[id(p)]
    return e[1]


# A/B switch (bench.py VITMI_RESVIT_NO_SINK=1): False leaves every gradient to autograd's AccumulateGrad (one add
# into the flat view per parameter and step)
SINKS = True
# grad_sink answers only inside `sinks()`: the training steps (resvit_train.train_step, GraphedTrainStep) wrap their
# `total.backward()` in it. Elsewhere (torch.autograd.grad(loss, params), backward(inputs=[...]), any plain
# backward) every fused node returns its parameter gradients to autograd as usual. A module-level count, not a
# thread-local: autograd runs the CUDA nodes on its device threads while the caller waits in backward().
_SINK_DEPTH = 0


@contextlib.contextmanager
def sinks():
    """enable the in-place gradient sinks of the fused Res-ViT nodes for the backward run inside"""
    global _SINK_DEPTH
    _SINK_DEPTH += 1
    try:
        yield
    finally:
        _SINK_DEPTH -= 1


def grad_sink(p, need=True):
    """the gradient view a backward node may accumulate p's gradient into in place (returning None for p), or
    None: outside a `sinks()` block, p is not held by a live FlatParams, its .grad is no longer the flat view, or
    the backward records a graph (create_graph)"""
    if not (SINKS and need and _SINK_DEPTH > 0) or torch.is_grad_enabled():
        return None
    e = getattr(p, "_vitmi_flat", None)
    f = e[0]() if e is not None else None
    return f.sink(p) if f is not None else None


def sunk(p):
    """after a node accumulated p's gradient through grad_sink: p's used flag (what AccumulateGrad's post hook
    records). The gradient-exchange count (on_grad) is left to that hook, which autograd still runs for the None the
    node returns, once per parameter and after every node that sinks into it (a parameter two nodes sink into — an
    approximator applied at both layers of a block — then counts once, when its gradient is complete; counting here
    as well made the data-parallel reducer launch buckets before the last contribution landed). Were the hook not
    to run, the bucket would wait for the reducer's finish()."""
    f = p._vitmi_flat[0]()
    if f is not None:
        f.used_host[f._index[id(p)]] = True


def _rup(x, m):
    return (x + m - 1) // m * m


class FlatParams:
    def __init__(self, params, device=None):
        seen, ps = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                ps.append(p)
        if not ps:
            raise ValueError("FlatParams: no parameters")
        ps = ps[::-1]  # reverse registration order: the backward finishes the last modules first
        dev = torch.device(device) if device is not None else ps[0].device
        if dev.type != "cuda":
            raise RuntimeError("vitmi flat parameters live on the MI355X (no CPU path)")
        for p in ps:
            if p.dtype != torch.float32:
                raise TypeError("FlatParams: fp32 parameters expected (the reference trains in fp32)")
        self.params = ps
        self.device = dev
        self.offsets, off = [], 0
        for p in ps:
            self.offsets.append(off)
            off = _rup(off + p.numel(), ALIGN)
        self.numel = off
        self.data = torch.zeros(off, device=dev)
        self.grad = torch.zeros(off, device=dev)
        self._index = {}
        for i, (p, o) in enumerate(zip(ps, self.offsets)):
            n = p.numel()
            self.data[o:o + n].copy_(p.data.reshape(-1))
            p.data = self.data[o:o + n].view(p.shape)
            p.grad = self.grad[o:o + n].view(p.shape)
            self._index[id(p)] = i
        self.nseg = len(ps)
        self.used_host = [False] * self.nseg
        self.used = torch.zeros(self.nseg, device=dev)
        self.used_reduced = False  # set by vitmi.dist.FlatGradAllReducer: `used` already holds all ranks' flags
        # two pinned staging copies of the host flags, each reused only after its last upload completed
        self._used_pin = [torch.zeros(self.nseg, pin_memory=True) for _ in range(2)]
        self._used_ev = [None, None]
        self._gate_idx = {}
        self._used_k = 0
        self.on_grad = None  # callable(segment index) after each parameter's gradient accumulation
        me = weakref.ref(self)
        for i, p in enumerate(ps):
            p._vitmi_flat = (me, i)  # (grad_sink: fused backward nodes accumulate into the flat view in place)
        self._hooks = [p.register_post_accumulate_grad_hook(self._mark) for p in ps]
        # update chunks: (segment, start, length), <= vit_adamw_chunk_elems() elements, inside one segment
        ch = ops.adamw_chunk_elems()
        rows = []
        for i, (p, o) in enumerate(zip(ps, self.offsets)):
            n = p.numel()
            for s in range(0, n, ch):
                rows.append((i, o + s, min(ch, n - s)))
        self.chunks = torch.tensor(rows, dtype=torch.int64).reshape(-1).to(dev)

    def index(self, p):
        return self._index[id(p)]

    def view(self, buf, i):
        p, o = self.params[i], self.offsets[i]
        return buf[o:o + p.numel()].view(p.shape)

    def sink(self, p):
        """p's flat gradient view when p.grad still is that view (else None: autograd's own accumulation)"""
        i = self._index.get(id(p))
        if i is None or p.grad is None:
            return None
        o = self.offsets[i]
        return p.grad if p.grad.data_ptr() == self.grad[o:o + 1].data_ptr() else None

    def _mark(self, p):
        i = self._index[id(p)]
        self.used_host[i] = True
        if self.on_grad is not None:
            self.on_grad(i)

    def adopt_grads(self):
        """fold gradients that are not views of the flat buffer back into it (a .grad that was set to None
        and re-created by autograd); parameters whose .grad is None count as unused"""
        for i, (p, o) in enumerate(zip(self.params, self.offsets)):
            v = self.grad[o:o + p.numel()].view(p.shape)
            if p.grad is None:
                self.used_host[i] = False
                ops.zero_(v)
                p.grad = v
            elif p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v
                self.used_host[i] = True

    def zero_grad(self):
        """zero the flat gradient (one memset) and the used flags; .grad stays the flat view"""
        self.adopt_grads()
        ops.zero_(self.grad)
        self.used_host = [False] * self.nseg
        self.used_reduced = False
        # gate() ORs a forward's flag into an existing entry (several forwards before one step): entries left by a
        # forward that no step consumed (a skipped step, a metrics-only train-mode forward) must not leak into
        # the next zero_grad .. step window
        for p in self.params:
            e = _GATES.get(id(p))
            if e is not None and e[0]() is p:
                del _GATES[id(p)]

    def upload_used(self):
        """the host flags -> self.used (device f32), ordered on the current stream (unless a data-parallel
        reducer already left every rank's flags there)"""
        if self.used_reduced:
            self.used_reduced = False
            return self.used
        gated = [(i, g) for i, g in ((i, _take_gate(p)) for i, p in enumerate(self.params)) if g is not None]
        k = self._used_k = self._used_k ^ 1
        if self._used_ev[k] is not None:
            self._used_ev[k].synchronize()
        pin = self._used_pin[k]
        pin.copy_(torch.tensor(self.used_host, dtype=torch.float32))
        self.used.copy_(pin, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._used_ev[k] = ev
        if gated:
            key = tuple(i for i, _ in gated)
            idx = self._gate_idx.get(key)
            if idx is None:
                idx = self._gate_idx[key] = torch.tensor(key, dtype=torch.int64).to(self.device)
            flags = torch.stack([f.reshape(()) for _, f in gated]).to(self.used.dtype)
            self.used[idx] = self.used[idx] * flags
        return self.used

    def sq_norm_parts(self):
        return max(1, min(1024, math.ceil(self.numel / (256 * 4 * 16))))
