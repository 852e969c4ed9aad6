"""Data parallelism: one process per GPU, gradient all-reduce over RCCL (xGMI), overlapped with backward.

Replaces the reference's single-process torch.nn.DataParallel (src/train.py:128-129), whose
per-step parameter broadcast + reduce-to-GPU0 star is the wrong shape for point-to-point xGMI.
Every rank keeps a full persistent replica; the engine's flat gradient buffer is laid out in
backward-completion order, so each encoder layer's gradients form one contiguous bucket that is
all-reduced on a side stream as soon as the engine's backward releases it (grad_ready_hook),
while the backward of the layers below keeps running on the compute stream.

Gradient scaling: with average=True (default) the buckets are averaged over ranks (ReduceOp.AVG on
RCCL; SUM followed by a 1/world scale on backends without AVG, e.g. gloo), so a per-rank mean
cross entropy yields the global-batch mean gradient of the reference's DataParallel CE (computed on
the gathered batch). With average=False the buckets are summed (the caller pre-scales the loss by
1/(b*world), as bench.py does). Replicas stay bit-identical because every rank applies the same SGD
update to the same all-reduced gradient.

compress="bf16" halves the exchanged bytes (ViT-L/16: 1.22 GB of f32 gradients per step, ViT-H/14:
2.53 GB, at ~153 GB/s per xGMI link): each bucket is cast to bf16 on the exchange stream (HIP cast
kernel), all-reduced in bf16 and widened back into the f32 gradient buffer (HIP unpack kernel) before
the optimizer reads it. The sum is rounded to bf16 at every ring step (relative error ~2^-9 x ranks),
the trade the reference's DataParallel never offered; off by default.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

# Stream priority of the gradient exchange (torch: lower value = higher priority; -1 is the highest HIP
# exposes). The compute stream runs GEMMs of one 160 KiB-LDS workgroup per CU and a persistent attention
# backward sized to every CU, so an all-reduce queued at normal priority can find no free CU until the
# running kernel drains. At high priority the dispatcher hands the exchange's workgroups the first CUs that
# free up: the bucket of layer l goes out between the backward kernels of layer l-1 instead of behind them.
EXCHANGE_PRIORITY = -1


def init_process_group(backend=None, device=None):
    """torch.distributed.init_process_group for the training entry points (src/train.py:128-129's
    DataParallel replaced by one process per GPU). backend defaults to VITMI_DIST_BACKEND or "nccl"
    (= RCCL on ROCm); for RCCL its internal streams are created high-priority (EXCHANGE_PRIORITY) and the
    communicator is bound to `device` up front."""
    backend = backend or os.environ.get("VITMI_DIST_BACKEND", "nccl")
    kw = {}
    if backend == "nccl":
        if device is not None:
            kw["device_id"] = device
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        kw["pg_options"] = opts
    dist.init_process_group(backend, **kw)
    return backend


def exchange_stream(device):
    """the side stream the reducers issue their exchange work on (casts, widening, gloo / RCCL calls)"""
    return torch.cuda.Stream(device=device, priority=EXCHANGE_PRIORITY)


class GradAllReducer:
    def __init__(self, engine, group=None, min_bucket_elems=1 << 20, average=True, compress=None):
        if compress not in (None, "bf16"):
            raise ValueError(f"compress must be None or 'bf16', got {compress!r}")
        self.engine = engine
        self.compress = compress
        self._stage = None  # bf16 staging copy of the flat gradient buffer (compress="bf16")
        self._widen = []    # (f32 slice, bf16 slice) pairs still to be widened (CPU / async path)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.average = average
        backend = dist.get_backend(group) if dist.is_initialized() else None
        self.native_avg = average and backend == "nccl"
        self._to_scale = []
        self.cuda = engine.dev.type == "cuda"
        self.stream = exchange_stream(engine.dev) if self.cuda else None
        self.min_bucket = min_bucket_elems
        self._pending = None  # (buf, start) of a bucket being coalesced with the next one
        self._works = []
        # exchange accounting (bench.py's N > 1 dist_check): a list while enabled; per launched bucket
        # ("events", start, end, elems) — HIP events on the exchange stream around its all-reduce — or, on the CPU
        # (gloo async) path, ("host", ms waited in finish(), elems of the step)
        self.timing = None
        self._host_elems = 0

    def attach(self):
        self.engine.grad_ready_hook = self.hook
        self.engine.grad_ready_finish = self.finish
        return self

    def detach(self):
        self.engine.grad_ready_hook = None
        self.engine.grad_ready_finish = None

    def _staging(self, buf, start, end):
        if self._stage is None or self._stage.numel() < buf.numel():
            self._stage = torch.empty(buf.numel(), device=buf.device, dtype=torch.bfloat16)
        return self._stage[start:end]

    def _launch(self, buf, start, end, events=()):
        t = buf[start:end]
        op = dist.ReduceOp.AVG if self.native_avg else dist.ReduceOp.SUM
        if self.average and not self.native_avg:
            self._to_scale.append(t)
        if self.cuda:
            if not events:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.engine.dev))
                events = (ev,)
            for ev in events:  # the bucket's producers (main and side streams of the engine)
                self.stream.wait_event(ev)
            with torch.cuda.stream(self.stream):
                if self.timing is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e0.record(self.stream)
                if self.compress:
                    from . import ops
                    tb = self._staging(buf, start, end)
                    ops.cast_bf16(t, tb, end - start)
                    dist.all_reduce(tb, op=op, group=self.group)
                    ops.unpack_bf16_f32(tb, end - start, 1, end - start, t, end - start)
                else:
                    dist.all_reduce(t, op=op, group=self.group)
                if self.timing is not None:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record(self.stream)
                    self.timing.append(("events", e0, e1, end - start))
        else:
            if self.compress:
                tb = self._staging(buf, start, end)
                tb.copy_(t)
                self._widen.append((t, tb))
                t = tb
            self._works.append(dist.all_reduce(t, op=op, group=self.group, async_op=True))
            self._host_elems += end - start

    def timing_summary(self):
        """(all-reduce ms, buckets, elements) of the launches recorded since `timing` was set to []: the sum of the
        per-bucket HIP-event spans on the exchange stream (each all-reduce as the exchange stream sees it, from its
        launch after the bucket's producers to the collective's completion), or the CPU path's time waited"""
        if not self.timing:
            return 0.0, 0, 0
        ms = sum(a.elapsed_time(b) if kind == "events" else a for kind, a, b, _ in self.timing)
        n = sum(1 for kind, *_ in self.timing if kind == "events") or len(self.timing)
        return ms, n, sum(e for *_, e in self.timing)

    def hook(self, buf, name, start, end, events=()):
        if self.world == 1:
            return
        if self._pending is not None:
            start = self._pending
            self._pending = None
        if end - start < self.min_bucket and name != "embed":
            self._pending = start  # coalesce small buckets (head) with the next layer's
            return
        self._launch(buf, start, end, events)

    def finish(self):
        """Make the compute stream wait for every outstanding all-reduce."""
        if self.world == 1:
            return
        if self.cuda:
            torch.cuda.current_stream(self.engine.dev).wait_stream(self.stream)
        else:
            import time
            t0 = time.perf_counter()
            for w in self._works:
                w.wait()
            if self.timing is not None and self._works:
                self.timing.append(("host", (time.perf_counter() - t0) * 1e3, None, self._host_elems))
            self._works = []
            self._host_elems = 0
            for t, tb in self._widen:
                t.copy_(tb)
            self._widen = []
        for t in self._to_scale:
            t.mul_(1.0 / self.world)
        self._to_scale = []


class FlatGradAllReducer:
    """Data-parallel gradient exchange for parameters held by a vitmi.flat.FlatParams (the Res-ViT
    trainable set: LoRA, routers, approximators, head), overlapped with the autograd backward.

    The flat gradient buffer is cut into buckets of whole parameters (~bucket_elems each, in the
    buffer's order, which is the order the backward finishes them). Each parameter's post-accumulate
    hook counts it into its bucket; a complete bucket is all-reduced on the exchange stream while the
    backward continues. Buckets are launched strictly in index order — every rank issues the same
    sequence of collectives even when dynamic routing leaves a parameter without a gradient on one rank
    (its bucket then waits for finish(), which launches whatever is left, in order). The used flags
    (which parameters received a gradient anywhere) are summed across ranks in the last collective, so
    every replica's AdamW skips / updates the same parameters and the replicas stay bit-identical."""

    def __init__(self, flat, group=None, bucket_elems=4 << 20, average=True):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.average = average
        self.native_avg = average and dist.is_initialized() and dist.get_backend(group) == "nccl"
        self.cuda = flat.device.type == "cuda"
        self.stream = exchange_stream(flat.device) if self.cuda else None
        self.buckets, cur, start = [], [], 0
        self.bucket_of = [0] * flat.nseg
        for i, (p, o) in enumerate(zip(flat.params, flat.offsets)):
            cur.append(i)
            end = flat.offsets[i + 1] if i + 1 < flat.nseg else flat.numel
            if end - start >= bucket_elems or i + 1 == flat.nseg:
                self.buckets.append((start, end, len(cur)))
                for j in cur:
                    self.bucket_of[j] = len(self.buckets) - 1
                cur, start = [], end
        self._reset()

    def _reset(self):
        self.count = [0] * len(self.buckets)
        self.launched = 0

    def attach(self):
        self.flat.on_grad = self._on_grad
        return self

    def detach(self):
        self.flat.on_grad = None

    def _launch(self, k):
        s, e, _ = self.buckets[k]
        t = self.flat.grad[s:e]
        op = dist.ReduceOp.AVG if self.native_avg else dist.ReduceOp.SUM
        if self.cuda:
            self.stream.wait_stream(torch.cuda.current_stream(self.flat.device))
            with torch.cuda.stream(self.stream):
                dist.all_reduce(t, op=op, group=self.group)
        else:
            dist.all_reduce(t, op=op, group=self.group)

    def _on_grad(self, i):
        if self.world == 1:
            return
        k = self.bucket_of[i]
        self.count[k] += 1
        while self.launched < len(self.buckets) and self.count[self.launched] >= self.buckets[self.launched][2]:
            self._launch(self.launched)
            self.launched += 1

    def finish(self):
        """launch the buckets still pending (in order), OR the used flags over ranks, and make the current
        stream wait; call after backward, before clip / optimizer step"""
        if self.world == 1:
            self._reset()
            return
        for k in range(self.launched, len(self.buckets)):
            self._launch(k)
        f = self.flat
        used = f.upload_used()
        cur = torch.cuda.current_stream(f.device) if self.cuda else None
        if self.cuda:
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                dist.all_reduce(used, op=dist.ReduceOp.SUM, group=self.group)
            cur.wait_stream(self.stream)
        else:
            dist.all_reduce(used, op=dist.ReduceOp.SUM, group=self.group)
        f.used_reduced = True  # the device flags now hold the all-rank sums (> 0: received a gradient)
        if self.average and not self.native_avg:
            f.grad.mul_(1.0 / self.world)
        self._reset()
