"""ViT training-step engine: runs forward and backward of the whole network on libvit_hip.so.

This is the host-side orchestration of the hot path (reference src/model.py:196-211 forward,
autograd backward at src/train.py:23). Design:

* Parameters live in ONE flat fp32 buffer (`flat`) whose order is the order in which the
  backward finishes their gradients: classifier, final LayerNorm, encoder layers L-1 .. 0,
  embedding. The nn.Parameters of vitmi.model are views into it, the gradient buffer has the
  same layout, so data-parallel all-reduce buckets are contiguous slices released layer by layer.
* A bf16 mirror of `flat` (same offsets) feeds the MFMA GEMMs; q/k/v weights are additionally
  packed to one [D][3D] operand per layer so the QKV projection is a single GEMM.
* Activations are kept per layer (bf16 GEMM operands, fp32 residual stream and LN stats); rows
  are padded to a multiple of 64 with zeros so the weight-gradient GEMMs (K = tokens) need no
  tail handling.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict
from dataclasses import dataclass

import torch

from . import ops
from ._lib import (EPI_BF16, EPI_BIAS_BF16, EPI_BIAS_GELU_DGELU, EPI_BIAS_RESID_F32, EPI_MUL_BF16, EPI_PATCH,
                   EPI_SPLITK, K_CONTIG, MN_CONTIG)

ALIGN = 64  # elements; every parameter starts 256-B aligned in the flat buffers


def _rup(x, m):
    return (x + m - 1) // m * m


# partial-sum buffers per kind of bias-gradient reduction: one encoder layer queues at most two of a kind
# (LayerNorm 1 and 2) before its batch of reductions is issued (_BiasReducer)
_NBUF = 2

# workgroups a split-K weight gradient aims for (one per CU); VIT_WGRAD_TARGET for tuning sweeps
_WGRAD_TARGET = int(os.environ.get("VIT_WGRAD_TARGET", "256"))


@dataclass(frozen=True)
class ArchConfig:
    image_size: int = 224
    patch_size: int = 16
    emb_dim: int = 768
    mlp_dim: int = 3072
    num_heads: int = 12
    num_layers: int = 12
    num_classes: int = 1000

    @property
    def grid(self):
        return self.image_size // self.patch_size

    @property
    def tokens(self):
        return self.grid * self.grid + 1

    @property
    def head_dim(self):
        return self.emb_dim // self.num_heads

    @property
    def patch_k(self):
        return 3 * self.patch_size * self.patch_size


def layer_param_specs(cfg: ArchConfig, i: int):
    """(name, shape) of encoder layer i in reference state_dict order (src/model.py:104-130)."""
    D, M, H = cfg.emb_dim, cfg.mlp_dim, cfg.num_heads
    hd = D // H
    p = f"transformer.encoder_layers.{i}."
    out = [(p + "norm1.weight", (D,)), (p + "norm1.bias", (D,))]
    for w in ("query", "key", "value"):
        out += [(p + f"attn.{w}.weight", (D, H, hd)), (p + f"attn.{w}.bias", (H, hd))]
    out += [(p + "attn.out.weight", (H, hd, D)), (p + "attn.out.bias", (D,))]
    out += [(p + "norm2.weight", (D,)), (p + "norm2.bias", (D,))]
    out += [(p + "mlp.fc1.weight", (M, D)), (p + "mlp.fc1.bias", (M,))]
    out += [(p + "mlp.fc2.weight", (D, M)), (p + "mlp.fc2.bias", (D,))]
    return out


def flat_param_specs(cfg: ArchConfig):
    """All parameters in flat-buffer order (reverse of backward completion)."""
    D, P, C = cfg.emb_dim, cfg.patch_size, cfg.num_classes
    specs = [("classifier.weight", (C, D)), ("classifier.bias", (C,)),
             ("transformer.norm.weight", (D,)), ("transformer.norm.bias", (D,))]
    for i in reversed(range(cfg.num_layers)):
        specs += layer_param_specs(cfg, i)
    specs += [("embedding.weight", (D, 3, P, P)), ("embedding.bias", (D,)),
              ("transformer.pos_embedding.pos_embedding", (1, cfg.tokens, D)), ("cls_token", (1, 1, D))]
    return specs


class FlatLayout:
    def __init__(self, cfg: ArchConfig):
        self.cfg = cfg
        self.offsets = OrderedDict()
        self.shapes = OrderedDict()
        off = 0
        self.layer_ranges = {}
        for name, shape in flat_param_specs(cfg):
            n = math.prod(shape)
            self.offsets[name] = off
            self.shapes[name] = shape
            off = _rup(off + n, ALIGN)
        self.numel = off
        # contiguous [start, end) of every gradient bucket in backward-completion order
        L = cfg.num_layers
        self.buckets = []
        self.buckets.append(("head", 0, self.offsets[self._lname(L - 1, "norm1.weight")]))
        for i in reversed(range(L)):
            start = self.offsets[self._lname(i, "norm1.weight")]
            end = self.offsets[self._lname(i - 1, "norm1.weight")] if i > 0 else self.offsets["embedding.weight"]
            self.buckets.append((f"layer{i}", start, end))
        self.buckets.append(("embed", self.offsets["embedding.weight"], self.numel))

    @staticmethod
    def _lname(i, s):
        return f"transformer.encoder_layers.{i}.{s}"

    def view(self, buf, name):
        o = self.offsets[name]
        shape = self.shapes[name]
        return buf[o:o + math.prod(shape)].view(shape)


class _Acts:
    """Per-batch-size activation workspace (allocated once, rows padded to 64)."""

    def __init__(self, cfg: ArchConfig, b: int, dev):
        D, M, H, L, N = cfg.emb_dim, cfg.mlp_dim, cfg.num_heads, cfg.num_layers, cfg.tokens
        T = b * N
        Tp = _rup(T, 64)
        self.b, self.T, self.Tp = b, T, Tp
        z = lambda *s, dt=torch.bfloat16: torch.zeros(*s, device=dev, dtype=dt)
        f = torch.float32
        self.kpad = _rup(cfg.patch_k, 64)
        self.patches = z(Tp, self.kpad)
        self.h = [z(Tp, D, dt=f) for _ in range(L + 1)]        # layer inputs (fp32 residual stream)
        self.hm = [z(Tp, D, dt=f) for _ in range(L)]           # after attention
        self.ln1 = [z(Tp, D) for _ in range(L)]
        self.ln2 = [z(Tp, D) for _ in range(L)]
        self.mu1 = [z(T, dt=f) for _ in range(L)]
        self.rs1 = [z(T, dt=f) for _ in range(L)]
        self.mu2 = [z(T, dt=f) for _ in range(L)]
        self.rs2 = [z(T, dt=f) for _ in range(L)]
        self.qkv = [z(Tp, 3 * D) for _ in range(L)]
        self.o = [z(Tp, D) for _ in range(L)]
        self.lse = [z(b, H, N, dt=f) for _ in range(L)]
        self.gp = [z(Tp, M) for _ in range(L)]      # GELU'(fc1 pre-activation), for the backward
        self.g = [z(Tp, M) for _ in range(L)]
        self.lncls = z(b, D, dt=f)
        self.muf = z(b, dt=f)
        self.rsf = z(b, dt=f)
        self.logits = z(b, cfg.num_classes, dt=f)
        # backward scratch
        # (bf16 gradient operands are double-buffered: the weight-gradient GEMMs read them on a side
        #  stream while the main stream already produces the next layer's)
        self.dh = z(Tp, D, dt=f)
        self.dhb = [z(Tp, D), z(Tp, D)]
        self.dg = [z(Tp, M), z(Tp, M)]
        self.dyln = z(Tp, D)
        self.dO = z(Tp, D)
        self.dqkv = [z(Tp, 3 * D), z(Tp, 3 * D)]
        self.dlncls = z(b, D, dt=f)
        self.dlogits = z(b, cfg.num_classes, dt=f)
        self.row_stats = z(b, 3, dt=f)
        # bias-gradient partial sums, reduced a layer at a time (_BiasReducer: one vit_colsum_batch launch)
        self.lnparts = [z(ops.layernorm_bwd_blocks(T), 3 * D, dt=f) for _ in range(_NBUF)]
        self.gelu_parts = [z(-(-T // 128), M, dt=f) for _ in range(_NBUF)]  # per-M-tile column sums of dU (fc1 bias)
        # column sums of dq|dk|dv (q/k/v bias grads): per image (LDS-resident attention, N <= 320) or per
        # image and 64-row block (K/V-tiled attention, longer sequences)
        self.attn_bias_rows = ops.attention_bias_rows(N, D // H)
        self.qkv_bparts = [z(b * self.attn_bias_rows, 3 * D, dt=f) for _ in range(_NBUF)]
        nws = ops.attention_workspace_elems(b, N, H)
        self.attn_ws = z(nws, dt=f) if nws else None
        # last encoder layer on the cls rows only (ViTEngine.prune_last): compact operands, rows
        # padded to 64 with zeros that are never written (they are K rows of weight gradients)
        bp = _rup(b, 64)
        self.bp = bp
        self.c_o, self.c_ln2, self.c_dh, self.c_dh2, self.c_dyln = (z(bp, D) for _ in range(5))
        self.c_g, self.c_gp, self.c_dg = (z(bp, M) for _ in range(3))
        self.c_mu2, self.c_rs2 = z(b, dt=f), z(b, dt=f)


class _BiasReducer:
    """The bias-gradient column reductions of one backward, batched per encoder layer.

    Producers on the compute stream write per-block partial sums (LayerNorm backward: [nblk][dgamma |
    dbeta | dx]; the fc2-dgrad GEMM epilogue: per-tile dU column sums; the attention backward: per-image
    dq|dk|dv sums); reduce() queues a column reduction of one of them and flush() issues every queued
    reduction as ONE vit_colsum_batch launch on the compute stream, once per encoder layer (before its
    gradient bucket is released). No event and no second stream sit between the step's kernels: every
    event recorded on the compute stream idled it ~13 us, ~50 of them per B/16 step
    (profiles/r03/step_timeline_v1.txt), and the reductions on a second stream held CU slots the GEMMs
    wanted. The partial buffers rotate through rings of _NBUF (> the reductions queued between flushes),
    all in compute-stream order."""

    def __init__(self, eng, a):
        self.eng = eng
        self.a = a
        self.D = eng.cfg.emb_dim
        self.nxt = {}
        self.queued = {}  # kind -> partial buffers of that kind written since the last flush
        self.jobs = []

    def buf(self, kind, bufs):
        n = self.queued.get(kind, 0)
        if n == len(bufs):  # every buffer of the ring awaits its reduction
            self.flush()
            n = 0
        self.queued[kind] = n + 1
        i = self.nxt.get(kind, 0)
        self.nxt[kind] = (i + 1) % len(bufs)
        return bufs[i]

    def reduce(self, part, rows, cols, ld, outs, seg=0):
        """queue out_k[c - k*seg] = sum_r part[r*ld + c] (seg = 0: one output)"""
        self.jobs.append((part, rows, cols, ld, seg, outs, False))
        if len(self.jobs) == ops.COLSUM_BATCH_MAX:
            self.flush()

    def flush(self):
        if self.jobs:
            ops.colsum_batch(self.jobs)
            self.jobs = []
        self.queued.clear()

    def ln_bwd(self, dy, lddy, x, ldx, mean, rstd, gamma, dx, lddx, rows, dgamma_dbeta, dx_colsum, **kw):
        """LayerNorm backward on the compute stream; dgamma | dbeta (and the column sums of dx, the
        bias gradient of the layer feeding the residual stream) queued as one reduction."""
        part = self.buf("ln", self.a.lnparts)
        D = self.D
        ops.layernorm_bwd(dy, lddy, x, ldx, mean, rstd, gamma, dx, lddx, part, rows, D, **kw)
        self.reduce(part, ops.layernorm_bwd_blocks(rows), 3 * D, 3 * D, (dgamma_dbeta, dgamma_dbeta[D:], dx_colsum),
                    seg=D)


class ViTEngine:
    """Owns flat parameter/gradient buffers, the bf16 mirror and per-batch activations."""

    def __init__(self, cfg: ArchConfig, device="cuda", flat: torch.Tensor | None = None):
        if cfg.emb_dim % cfg.num_heads:
            raise ValueError("emb_dim must be divisible by num_heads")
        if cfg.head_dim % 16 or cfg.head_dim > 96:
            raise NotImplementedError(f"head_dim {cfg.head_dim} not supported by the HIP attention kernel "
                                      "(multiples of 16 up to 96)")
        if cfg.emb_dim % 64 or cfg.mlp_dim % 64:
            raise NotImplementedError("emb_dim and mlp_dim must be multiples of 64")
        self.cfg = cfg
        self.dev = torch.device(device)
        # attention forward kernel choice (ops.ATTN_AUTO; ops.ATTN_ONESHOT for same-box A/B of the persistent kernel)
        self.attn_fwd_path = ops.ATTN_AUTO
        self.layout = FlatLayout(cfg)
        n = self.layout.numel
        self.flat = flat if flat is not None else torch.zeros(n, device=self.dev)
        self.grad = torch.zeros(n, device=self.dev)
        self.mirror = torch.zeros(n, device=self.dev, dtype=torch.bfloat16)
        D, L = cfg.emb_dim, cfg.num_layers
        M = cfg.mlp_dim
        bf = torch.bfloat16
        # [in][q|k|v out]: the fused q|k|v GEMM's B operand, M/N-contiguous in the forward, K-contiguous in the
        # data gradient. Every other weight is read in place from the bf16 mirror in whichever layout its GEMM
        # sees it (the half-tile ping-pong runs an M/N-contiguous B as fast as a K-contiguous one since round 5:
        # no transposed copies)
        self.wqkv = torch.zeros(L, D, 3 * D, device=self.dev, dtype=bf)
        self.bqkv = torch.zeros(L, 3 * D, device=self.dev)
        kp = _rup(cfg.patch_k, 64)
        self.wconv = torch.zeros(D, kp, device=self.dev, dtype=torch.bfloat16) if kp != cfg.patch_k else None
        self._acts = {}
        self._mirror_sig = None
        # flat-buffer distance between consecutive encoder layers (constant: same specs, same alignment)
        o = [self.off(self.lname(i, "norm1.weight")) for i in range(L)]
        self.layer_stride = o[0] - o[1] if L > 1 else 0
        assert all(o[i] == o[0] - i * self.layer_stride for i in range(L))
        self._ws = None
        self.step_id = 0
        self.grad_ready_hook = None  # callable(grad_buf, bucket_name, start, end, events) during backward
        # callable() that completes every bucket the hook started (stream wait + any 1/world scaling); the
        # autograd node calls it before handing gradients to autograd, which may add them into existing
        # .grad tensors on the compute stream
        self.grad_ready_finish = None
        # weight-gradient GEMMs on a side stream, overlapped with the dgrad chain (VITMI_OVERLAP=1).
        # Off by default: the GEMMs of both streams share the CUs and each runs 30-40% slower than
        # alone, so the serial order is faster on one MI355X (B/16 bs256: 6778 vs 6588 img/s,
        # tools/sweep_env.sh). The DP all-reduce keeps its own stream either way (vitmi/dist.py).
        self.overlap_wgrad = os.environ.get("VITMI_OVERLAP", "0") == "1"
        # each layer's out-projection and q|k|v weight gradients in one split-K launch (ops.gemm_splitk_group);
        # VITMI_GROUP_WGRAD=0: two launches
        self.group_wgrad = os.environ.get("VITMI_GROUP_WGRAD", "1") != "0"
        # Only the cls token of the last layer's output reaches the classifier (src/model.py:210),
        # so that layer's out-projection, LayerNorm 2 and MLP (forward and backward) run on the b cls
        # rows and its attention on the first 32-query pair of each (image, head) (q_rows = 1); the
        # q|k|v projection stays full (every token is a key / value of the cls query). Same logits, loss and gradients (zero rows add exact zeros); VITMI_PRUNE_LAST=0
        # runs every token. Off while dropout is active.
        self.prune_last = os.environ.get("VITMI_PRUNE_LAST", "1") != "0"
        self._pruned = False
        self._side = None
        self._ev_pool, self._ev_next = [], 0
        self.probe = None  # list: (start, end) HIP events around every fc1 forward GEMM launch
        self.probe_wgrad = None  # list: (start, end, flop, K, grouped) around every split-K weight-gradient GEMM launch
        # dropout (nn.Dropout of PositionEmbs / EncoderBlock / MlpBlock, reference src/model.py:19-20,
        # 46-49, 124-125): counter-based Philox masks keyed by (seed, per-forward offset, site, row,
        # col), regenerated by the backward instead of stored. Seeded from torch's initial seed.
        self.drop_seed = (torch.initial_seed() * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & (2**64 - 1)
        self._drop_offset = 0
        self._drop = None  # (p, seed, offset) of the last forward, or None

    def _event(self):
        """the next event of the backward's pool (created once, re-recorded every step: a wait enqueued
        on an event binds to its record at that moment, so re-recording later is safe)"""
        if self._ev_next == len(self._ev_pool):
            self._ev_pool.append(torch.cuda.Event())
        ev = self._ev_pool[self._ev_next]
        self._ev_next += 1
        return ev

    # ---- parameters --------------------------------------------------------------------------
    def pv(self, name, buf=None):
        return self.layout.view(self.flat if buf is None else buf, name)

    def off(self, name):
        return self.layout.offsets[name]

    def lname(self, i, s):
        return f"transformer.encoder_layers.{i}.{s}"

    def load_params(self, params):
        for k, v in params.items():
            self.pv(k).copy_(v.to(self.dev, torch.float32).reshape(self.layout.shapes[k]))
        self.invalidate_mirror()

    def state(self):
        return OrderedDict((k, self.pv(k)) for k in self.layout.offsets)

    def invalidate_mirror(self):
        self._mirror_sig = None

    def refresh_mirror(self, full=True):
        """Re-derive the bf16 GEMM operands from the fp32 master weights."""
        cfg = self.cfg
        D = cfg.emb_dim
        if full:
            ops.cast_bf16(self.flat, self.mirror, self.layout.numel)
        # q|k|v packing, one launch over all layers (layers sit at a constant stride in the flat buffer, layer
        # L-1 first)
        M, L = cfg.mlp_dim, cfg.num_layers
        lst = self.layer_stride
        o0 = lambda s: self.off(self.lname(0, s))
        zs = self.off(self.lname(0, "attn.key.weight")) - o0("attn.query.weight")
        ops.pack_cols_batched(self.flat[o0("attn.query.weight"):], -lst, zs, D, D, D, 3, self.wqkv, D * 3 * D, 3 * D, L)
        ops.pack_cols_batched(self.flat[o0("attn.query.bias"):], -lst, zs, D, 1, D, 3, self.bqkv, 3 * D, 3 * D, L)
        if self.wconv is not None:
            w = self.off("embedding.weight")
            ops.cast_pad_rows(self.flat[w:], D, cfg.patch_k, self.wconv, self.wconv.shape[1])

    def mark_mirror_fresh(self, sig):
        self._mirror_sig = sig

    # ---- workspaces --------------------------------------------------------------------------
    def acts(self, b):
        a = self._acts.get(b)
        if a is None:
            if len(self._acts) >= 2:
                self._acts.pop(next(iter(self._acts)))
            a = _Acts(self.cfg, b, self.dev)
            self._acts[b] = a
        return a

    def _splitk(self, M, N, K, z=1):
        """split-K factor for a weight-gradient GEMM (K = tokens) on the 256x256 ping-pong tile (one
        workgroup per CU): ops.splitk_factor over _WGRAD_TARGET CUs (tools/gemm_bench.py: fc1/fc2 wgrad
        at split 7 = 36 x 7 = 252 workgroups)."""
        return ops.splitk_factor(M, N, K, z, _WGRAD_TARGET)

    def _workspace(self, numel):
        if self._ws is None or self._ws.numel() < numel:
            self._ws = torch.empty(numel, device=self.dev)
        return self._ws

    def _wgrad(self, A, lda, B, ldb, M, N, K, out, ldo, batch=1, b_bs=0, out_bs=0):
        """out[z] (f32, [M][N], ld ldo) = sum_t A[t][m] B[t][n]  (both operands K-major): split-K f32
        slabs, then their fixed-order reduction (vit_splitk_reduce), both on the calling stream."""
        s = self._splitk(M, N, K, batch)
        ws = self._workspace(batch * s * M * N)
        if self.probe_wgrad is not None:  # bench.py's roofline kernel: events on the stream it runs on
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        ops.gemm(A, B, ws, M, N, K, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=lda, ldb=ldb, ldc=N,
                 epilogue=EPI_SPLITK, batch=batch, b_bs=b_bs, split_k=s)
        if self.probe_wgrad is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self.probe_wgrad.append((ev0, ev1, 2.0 * M * N * K * batch, K, False))
        ops.splitk_reduce(ws, batch, s, M, N, out, ldo, out_bs)

    def _wgrad_group(self, specs):
        """Several _wgrad calls over the same K (token rows) as ONE split-K launch (ops.gemm_splitk_group) at a
        common split (ops.splitk_factor_group), then each member's fixed-order reduction. specs: [(A, lda, B, ldb,
        M, N, K, out, ldo, batch, b_bs, out_bs)]. Each output equals its _wgrad's up to the split (same slabs
        summed in the same order when the splits agree)."""
        K = specs[0][6]
        assert all(sp[6] == K for sp in specs)
        s = ops.splitk_factor_group([(sp[4], sp[5], sp[9]) for sp in specs], K, _WGRAD_TARGET)
        sizes = [sp[9] * s * sp[4] * sp[5] for sp in specs]
        ws = self._workspace(sum(sizes))
        members, views, o = [], [], 0
        for sp, n in zip(specs, sizes):
            A, lda, B, ldb, M, N, _, _, _, batch, b_bs, _ = sp
            w = ws[o:o + n]
            o += n
            views.append(w)
            members.append((A, B, w, M, N, K, dict(a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=lda, ldb=ldb, ldc=N,
                                                    epilogue=EPI_SPLITK, batch=batch, b_bs=b_bs, split_k=s)))
        if self.probe_wgrad is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        ops.gemm_splitk_group(members)
        if self.probe_wgrad is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self.probe_wgrad.append((ev0, ev1, sum(2.0 * sp[4] * sp[5] * K * sp[9] for sp in specs), K, True))
        ops.splitk_reduce_group([(w, sp[9], s, sp[4], sp[5], sp[7], sp[8], sp[11], False) for sp, w in zip(specs, views)])

    # ---- forward -------------------------------------------------------------------------------
    def _dd(self, site, row_stride=1):
        """dropout descriptor of `site` for the last forward (None when dropout is off)."""
        if self._drop is None:
            return None
        p, seed, off = self._drop
        return ops.dropout_desc(p, site, seed, off, row_stride)

    def forward(self, x: torch.Tensor, dropout_p: float = 0.0):
        """x: [b, 3, img, img] fp32 on the device. Returns logits [b, C] (fp32, engine-owned).
        dropout_p > 0: training-mode nn.Dropout(p) at the reference's four sites per model
        (position embedding; per layer the attention output, GELU output and fc2 output)."""
        cfg = self.cfg
        if x.dim() != 4 or x.shape[1] != 3 or x.shape[2] != cfg.image_size or x.shape[3] != cfg.image_size:
            raise ValueError(f"expected input [b, 3, {cfg.image_size}, {cfg.image_size}], got {tuple(x.shape)}")
        x = x.to(self.dev, torch.float32).contiguous()
        b = x.shape[0]
        a = self.acts(b)
        D, M, H, N, L = cfg.emb_dim, cfg.mlp_dim, cfg.num_heads, cfg.tokens, cfg.num_layers
        hd = D // H
        T = a.T
        mv = self.mirror
        f = self.flat
        if dropout_p and dropout_p > 0.0:
            if not dropout_p < 1.0:
                raise ValueError(f"dropout probability has to be in [0, 1), got {dropout_p}")
            self._drop_offset += 1
            self._drop = (float(dropout_p), self.drop_seed, self._drop_offset)
        else:
            self._drop = None
        dd = self._dd
        # patch embedding: im2col + GEMM with conv-bias / cls / pos-emb epilogue
        ops.im2col(x, a.patches, b, cfg.image_size, cfg.patch_size, a.kpad)
        wconv = self.wconv if self.wconv is not None else mv[self.off("embedding.weight"):]
        ops.gemm(a.patches, wconv, a.h[0], T, D, a.kpad, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=a.kpad,
                 ldb=a.kpad, ldc=D, epilogue=EPI_PATCH, bias=f[self.off("embedding.bias"):],
                 aux=f[self.off("transformer.pos_embedding.pos_embedding"):], ldaux=D,
                 aux2=f[self.off("cls_token"):], tokens=N, dropout=dd(0))
        scale = 1.0 / math.sqrt(hd)
        self._pruned = self.prune_last and self._drop is None
        for i in range(L):
            ln = lambda s: self.off(self.lname(i, s))
            ops.layernorm_fwd(a.h[i], D, f[ln("norm1.weight"):], f[ln("norm1.bias"):], a.ln1[i], D, a.mu1[i],
                              a.rs1[i], T, D)
            ops.gemm(a.ln1[i], self.wqkv[i], a.qkv[i], T, 3 * D, D, a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=D,
                     ldb=3 * D, ldc=3 * D, epilogue=EPI_BIAS_BF16, bias=self.bqkv[i])
            last = self._pruned and i == L - 1
            ops.attention_fwd(a.qkv[i], a.o[i], a.lse[i], b, N, H, hd, scale, q_rows=1 if last else None,
                              path=self.attn_fwd_path)
            if last:
                self._forward_last_cls(a, i, b)
                break
            ops.gemm(a.o[i], mv[ln("attn.out.weight"):], a.hm[i], T, D, D, a_layout=K_CONTIG, b_layout=MN_CONTIG,
                     lda=D, ldb=D, ldc=D, epilogue=EPI_BIAS_RESID_F32, bias=f[ln("attn.out.bias"):], aux=a.h[i],
                     ldaux=D, dropout=dd(1 + 3 * i))
            ops.layernorm_fwd(a.hm[i], D, f[ln("norm2.weight"):], f[ln("norm2.bias"):], a.ln2[i], D, a.mu2[i],
                              a.rs2[i], T, D)
            if self.probe is not None:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            ops.gemm(a.ln2[i], mv[ln("mlp.fc1.weight"):], a.gp[i], T, M, D, a_layout=K_CONTIG, b_layout=K_CONTIG,
                     lda=D, ldb=D, ldc=M, epilogue=EPI_BIAS_GELU_DGELU, bias=f[ln("mlp.fc1.bias"):], C2=a.g[i],
                     ldc2=M, dropout=dd(2 + 3 * i))
            if self.probe is not None:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record()
                self.probe.append((ev0, ev1))
            ops.gemm(a.g[i], mv[ln("mlp.fc2.weight"):], a.h[i + 1], T, D, M, a_layout=K_CONTIG, b_layout=K_CONTIG,
                     lda=M, ldb=M, ldc=D, epilogue=EPI_BIAS_RESID_F32, bias=f[ln("mlp.fc2.bias"):], aux=a.hm[i],
                     ldaux=D, dropout=dd(3 + 3 * i))
        # final LayerNorm on the cls rows only (only row 0 reaches the classifier, src/model.py:210)
        ops.layernorm_fwd(a.h[L], N * D, f[self.off("transformer.norm.weight"):], f[self.off("transformer.norm.bias"):],
                          a.lncls, D, a.muf, a.rsf, b, D)
        C = cfg.num_classes
        ops.gemm_f32(b, C, D, a.lncls, D, False, f[self.off("classifier.weight"):], D, True, a.logits, C,
                     bias=f[self.off("classifier.bias"):])
        self.step_id += 1
        self._last_b = b
        return a.logits

    def _forward_last_cls(self, a, i, b):
        """Out-projection + residual, LayerNorm 2 and MLP + residual of the last layer on the b cls
        rows (row stride N*D in the token-major buffers); compact copies for the backward."""
        cfg = self.cfg
        D, M, N = cfg.emb_dim, cfg.mlp_dim, cfg.tokens
        f, mv = self.flat, self.mirror
        ln = lambda s: self.off(self.lname(i, s))
        S = N * D
        ops.gemm(a.o[i], mv[ln("attn.out.weight"):], a.hm[i], b, D, D, a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=S,
                 ldb=D, ldc=S, epilogue=EPI_BIAS_RESID_F32, bias=f[ln("attn.out.bias"):], aux=a.h[i], ldaux=S)
        ops.copy2d(a.c_o, D * 2, a.o[i], S * 2, D * 2, b)    # cls rows: the out-proj weight-gradient operand
        ops.layernorm_fwd(a.hm[i], S, f[ln("norm2.weight"):], f[ln("norm2.bias"):], a.c_ln2, D, a.c_mu2, a.c_rs2,
                          b, D)
        ops.gemm(a.c_ln2, mv[ln("mlp.fc1.weight"):], a.c_gp, b, M, D, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=D,
                 ldb=D, ldc=M, epilogue=EPI_BIAS_GELU_DGELU, bias=f[ln("mlp.fc1.bias"):], C2=a.c_g, ldc2=M)
        ops.gemm(a.c_g, mv[ln("mlp.fc2.weight"):], a.h[i + 1], b, D, M, a_layout=K_CONTIG, b_layout=K_CONTIG,
                 lda=M, ldb=M, ldc=S, epilogue=EPI_BIAS_RESID_F32, bias=f[ln("mlp.fc2.bias"):], aux=a.hm[i], ldaux=S)

    def _backward_last_cls(self, a, i, b, g, on_side, bias):
        """Backward of _forward_last_cls: the gradient reaching the last layer's output is non-zero on
        the cls rows only (a.c_dh, from the final LayerNorm backward), so fc2 / fc1 (data and weight
        gradients), LayerNorm 2 and the out-projection run on those b rows (weight-gradient K = the
        compact rows, zero-padded to 64). Leaves dO (attention-output gradient) zero except on the
        cls rows, and dh = the gradient after the attention residual."""
        cfg = self.cfg
        D, M, N = cfg.emb_dim, cfg.mlp_dim, cfg.tokens
        S = N * D
        f, mv = self.flat, self.mirror
        gv = lambda name: g[self.off(self.lname(i, name)):]
        bp = a.bp
        on_side(lambda: self._wgrad(a.c_dh, D, a.c_g, M, D, M, bp, gv("mlp.fc2.weight"), M))
        gpart = bias.buf("gelu", a.gelu_parts)
        w2 = mv[self.off(self.lname(i, "mlp.fc2.weight")):]
        kw = dict(a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=D, ldb=M, ldc=M, epilogue=EPI_MUL_BF16, aux=a.c_gp,
                  ldaux=M, col_partial=gpart)
        ops.gemm(a.c_dh, w2, a.c_dg, b, M, D, **kw)
        tiles_m = ops.gemm_partial_rows(a.c_dh, w2, a.c_dg, b, M, D, **kw)
        bias.reduce(gpart, tiles_m, M, M, (gv("mlp.fc1.bias"),))
        on_side(lambda: self._wgrad(a.c_dg, M, a.c_ln2, D, M, D, bp, gv("mlp.fc1.weight"), D))
        ops.gemm(a.c_dg, mv[self.off(self.lname(i, "mlp.fc1.weight")):], a.c_dyln, b, D, M, a_layout=K_CONTIG,
                 b_layout=MN_CONTIG, lda=M, ldb=D, ldc=D, epilogue=EPI_BF16)
        bias.ln_bwd(a.c_dyln, D, a.hm[i], S, a.c_mu2, a.c_rs2, f[self.off(self.lname(i, "norm2.weight")):], a.dh, S, b,
                    gv("norm2.weight"), gv("attn.out.bias"), dres=a.dh, lddres=S, dx_bf16=a.c_dh2, lddxb=D)
        on_side(lambda: self._wgrad(a.c_o, D, a.c_dh2, D, D, D, bp, gv("attn.out.weight"), D))
        ops.zero_(a.dO)
        ops.gemm(a.c_dh2, mv[self.off(self.lname(i, "attn.out.weight")):], a.dO, b, D, D, a_layout=K_CONTIG,
                 b_layout=K_CONTIG, lda=D, ldb=D, ldc=S, epilogue=EPI_BF16)

    # ---- fp32 ("exact") forward -------------------------------------------------------------------
    def forward_exact(self, x: torch.Tensor):
        """The forward in the reference's own arithmetic: f32 operands and f32 accumulation in every
        projection (vit_gemm_f32), f32 attention and exact-erf GELU, f32 LayerNorm outputs; no bf16
        rounding anywhere. Forward only (logits-parity gate, fp32 evaluation); keeps no activations.
        x: [b, 3, img, img] -> logits [b, C] f32 (a fresh tensor)."""
        cfg = self.cfg
        if x.dim() != 4 or x.shape[1] != 3 or x.shape[2] != cfg.image_size or x.shape[3] != cfg.image_size:
            raise ValueError(f"expected input [b, 3, {cfg.image_size}, {cfg.image_size}], got {tuple(x.shape)}")
        x = x.to(self.dev, torch.float32).contiguous()
        b = x.shape[0]
        D, M, H, N, L, C = cfg.emb_dim, cfg.mlp_dim, cfg.num_heads, cfg.tokens, cfg.num_layers, cfg.num_classes
        hd = D // H
        T, kp = b * N, cfg.patch_k
        f = self.flat
        e = lambda *shape: torch.empty(*shape, device=self.dev)
        fv = lambda name: f[self.off(name):]
        patches = e(T, kp)
        ops.im2col_f32(x, patches, b, cfg.image_size, cfg.patch_size, kp)
        h = e(T, D)
        # Conv2d(k = s = P) as patches x W^T (W [D][3 P^2]), then cls row and position embedding
        ops.gemm_f32(T, D, kp, patches, kp, False, fv("embedding.weight"), kp, True, h, D, bias=fv("embedding.bias"))
        ops.embed_fwd_f32(h, b, N, D, fv("transformer.pos_embedding.pos_embedding"), fv("cls_token"))
        y, qkv, o, u = e(T, D), e(T, 3 * D), e(T, D), e(T, M)
        mu, rs = e(T), e(T)
        for i in range(L):
            ln = lambda s: fv(self.lname(i, s))
            ops.layernorm_fwd(h, D, ln("norm1.weight"), ln("norm1.bias"), y, D, mu, rs, T, D)
            for z, w in enumerate(("query", "key", "value")):   # LinearGeneral: W [D][H,hd] (in x out)
                ops.gemm_f32(T, D, D, y, D, False, ln(f"attn.{w}.weight"), D, False, qkv[:, z * D:], 3 * D,
                             bias=ln(f"attn.{w}.bias"))
            ops.attention_fwd_f32(qkv, o, b, N, H, hd, 1.0 / math.sqrt(hd))
            ops.gemm_f32(T, D, D, o, D, False, ln("attn.out.weight"), D, False, h, D, bias=ln("attn.out.bias"),
                         accumulate=True)                        # h += out(attn) (src/model.py:124)
            ops.layernorm_fwd(h, D, ln("norm2.weight"), ln("norm2.bias"), y, D, mu, rs, T, D)
            ops.gemm_f32(T, M, D, y, D, False, ln("mlp.fc1.weight"), D, True, u, M, bias=ln("mlp.fc1.bias"))
            ops.gelu_f32(u, u, T * M)
            ops.gemm_f32(T, D, M, u, M, False, ln("mlp.fc2.weight"), M, True, h, D, bias=ln("mlp.fc2.bias"),
                         accumulate=True)                        # h += mlp(ln2(h)) (src/model.py:129)
        lncls = e(b, D)
        ops.layernorm_fwd(h, N * D, fv("transformer.norm.weight"), fv("transformer.norm.bias"), lncls, D, mu, rs, b, D)
        logits = e(b, C)
        ops.gemm_f32(b, C, D, lncls, D, False, fv("classifier.weight"), D, True, logits, C, bias=fv("classifier.bias"))
        return logits

    # ---- loss ------------------------------------------------------------------------------------
    def cross_entropy(self, labels: torch.Tensor, grad_scale: float | None = None):
        """Fused CE on the last logits: fills dlogits (scaled by grad_scale, default 1/b) and
        per-row {loss, top1, top5}. Returns (dlogits, row_stats)."""
        a = self.acts(self._last_b)
        gs = 1.0 / a.b if grad_scale is None else grad_scale
        ops.cross_entropy(a.logits, labels.to(self.dev, torch.int64).contiguous(), a.dlogits, gs, a.row_stats)
        return a.dlogits, a.row_stats

    # ---- backward --------------------------------------------------------------------------------
    def backward(self, dlogits: torch.Tensor, grad: torch.Tensor | None = None):
        """Backward of the last forward given dL/dlogits [b, C]; writes every parameter gradient
        into `grad` (default self.grad, flat layout).

        Two streams: the main stream runs the data-gradient chain (dgrad GEMMs, LayerNorm and
        attention backward); the weight-gradient GEMMs, which nothing downstream waits for, run on
        a side stream as soon as their operands exist. bf16 gradient operands are double-buffered
        and each buffer is recycled only after the side stream has consumed it."""
        cfg = self.cfg
        b = self._last_b
        a = self.acts(b)
        g = self.grad if grad is None else grad
        D, M, H, N, L, C = cfg.emb_dim, cfg.mlp_dim, cfg.num_heads, cfg.tokens, cfg.num_layers, cfg.num_classes
        hd = D // H
        T = a.T
        f = self.flat
        mv = self.mirror
        gv = lambda name: g[self.off(name):]
        dl = dlogits.to(self.dev, torch.float32).contiguous()
        hook = self.grad_ready_hook
        dd = self._dd
        main = torch.cuda.current_stream(self.dev)
        overlap = self.overlap_wgrad
        if overlap and self._side is None:
            self._side = torch.cuda.Stream(device=self.dev)
        side = self._side if overlap else main
        free_ev = {}  # (buffer kind, index) -> event recorded on the side stream after its last read

        def on_side(fn):
            """run fn() on the side stream after everything issued so far on the main stream."""
            if not overlap:
                fn()
                return
            ev = self._event()
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                fn()

        def release(kind, idx):
            if overlap:
                ev = self._event()
                ev.record(side)
                free_ev[(kind, idx)] = ev

        def acquire(kind, idx):
            ev = free_ev.pop((kind, idx), None)
            if ev is not None:
                main.wait_event(ev)

        def fire(bucket):
            bias.flush()  # the layer's bias gradients (and, with DP, the bucket's)
            if not hook:
                return
            evs = []
            for st in ((main, side) if overlap else (main,)):
                ev = self._event()
                ev.record(st)
                evs.append(ev)
            hook(g, *bucket, evs)

        self._ev_next = 0  # the event pool is reused from the start by every backward
        group = self.group_wgrad and D >= 256  # (the grouped kernel takes M, N >= 256)
        out_wb = None  # dhb buffer of a deferred out-projection weight gradient (group)
        bias = _BiasReducer(self, a)
        # classifier head (f32): dWc = dl^T lncls, dbc = colsum(dl), dlncls = dl Wc
        ops.gemm_f32(C, D, b, dl, C, True, a.lncls, D, False, gv("classifier.weight"), D)
        bias.reduce(dl, b, C, C, (gv("classifier.bias"),))
        ops.gemm_f32(b, D, C, dl, C, False, f[self.off("classifier.weight"):], D, False, a.dlncls, D)
        # final LN backward on cls rows -> residual grad (zero elsewhere)
        # (its dx column sum is the last layer's fc2 bias gradient: only the cls rows are non-zero)
        wb = 0  # index of the dhb buffer holding the current residual-gradient copy
        pruned = self._pruned
        ops.zero_(a.dh)
        if not pruned:
            ops.zero_(a.dhb[wb])
        bias.ln_bwd(a.dlncls, D, a.h[L], N * D, a.muf, a.rsf, f[self.off("transformer.norm.weight"):], a.dh, N * D, b,
                    gv("transformer.norm.weight"), gv(self.lname(L - 1, "mlp.fc2.bias")),
                    dx_bf16=a.c_dh if pruned else a.dhb[wb], lddxb=D if pruned else N * D,
                    dx_dropout=dd(3 + 3 * (L - 1), N))
        fire(self.layout.buckets[0])
        scale = 1.0 / math.sqrt(hd)
        for i in reversed(range(L)):
            ln = lambda s: self.off(self.lname(i, s))
            li = i & 1
            if pruned and i == L - 1:
                # MLP, LayerNorm 2 and out-projection backward on the cls rows; dO = 0 elsewhere
                self._backward_last_cls(a, i, b, g, on_side, bias)
                wb ^= 1
            else:
                dhb = a.dhb[wb]
                # ---- MLP: h_{i+1} = hm + fc2(gelu(fc1(ln2(hm)))) ----
                # (fc2 bias grad = column sums of dh, already produced by the LayerNorm backward above)
                on_side(lambda: self._wgrad(dhb, D, a.g[i], M, D, M, a.Tp, gv(self.lname(i, "mlp.fc2.weight")), M))
                release("dhb", wb)
                dg = a.dg[li]
                acquire("dg", li)
                gpart = bias.buf("gelu", a.gelu_parts)
                w2 = mv[ln("mlp.fc2.weight"):]
                kw = dict(a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=D, ldb=M, ldc=M, epilogue=EPI_MUL_BF16, aux=a.gp[i],
                          ldaux=M, col_partial=gpart)
                ops.gemm(dhb, w2, dg, T, M, D, **kw)
                tiles_m = ops.gemm_partial_rows(dhb, w2, dg, T, M, D, **kw)
                bias.reduce(gpart, tiles_m, M, M, (gv(self.lname(i, "mlp.fc1.bias")),))
                on_side(lambda: self._wgrad(dg, M, a.ln2[i], D, M, D, a.Tp, gv(self.lname(i, "mlp.fc1.weight")), D))
                release("dg", li)
                ops.gemm(dg, mv[ln("mlp.fc1.weight"):], a.dyln, T, D, M, a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=M,
                         ldb=D, ldc=D, epilogue=EPI_BF16)
                wb ^= 1
                acquire("dhb", wb)
                dhb = a.dhb[wb]
                bias.ln_bwd(a.dyln, D, a.hm[i], D, a.mu2[i], a.rs2[i], f[ln("norm2.weight"):], a.dh, D, T,
                            gv(self.lname(i, "norm2.weight")), gv(self.lname(i, "attn.out.bias")),
                            dres=a.dh, lddres=D, dx_bf16=dhb, lddxb=D, dx_dropout=dd(1 + 3 * i))
                # ---- attention: hm = h + out(attn(ln1(h))) ----
                out_spec = (a.o[i], D, dhb, D, D, D, a.Tp, gv(self.lname(i, "attn.out.weight")), D, 1, 0, 0)
                if group:  # launched with the q|k|v weight gradient below (dhb stays intact until then)
                    out_wb = wb
                else:
                    on_side(lambda: self._wgrad(*out_spec[:9]))
                    release("dhb", wb)
                ops.gemm(dhb, mv[ln("attn.out.weight"):], a.dO, T, D, D, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=D,
                         ldb=D, ldc=D, epilogue=EPI_BF16)
            dqkv = a.dqkv[li]
            acquire("dqkv", li)
            qpart = bias.buf("qkv", a.qkv_bparts)
            ops.attention_bwd(a.qkv[i], a.o[i], a.dO, a.lse[i], dqkv, b, N, H, hd, scale, bias_partial=qpart,
                              q_rows=1 if pruned and i == L - 1 else None, workspace=a.attn_ws)
            qo = ln("attn.query.weight")
            zs = ln("attn.key.weight") - qo
            qb = ln("attn.query.bias")
            bias.reduce(qpart, b * a.attn_bias_rows, 3 * D, 3 * D, (g[qb:], g[qb + zs:], g[qb + 2 * zs:]), seg=D)
            qkv_spec = (a.ln1[i], D, dqkv, 3 * D, D, D, a.Tp, g[qo:], D, 3, D, zs)
            if out_wb is not None:
                # the out-projection (9 tiles at B/16) and q|k|v (27) weight gradients as one grid: one wave of
                # 252 workgroups at split 7 instead of 252 short ones (split 28) and 243 (split 9)
                on_side(lambda: self._wgrad_group([out_spec, qkv_spec]))
                release("dqkv", li)
                release("dhb", out_wb)
                out_wb = None
            else:
                on_side(lambda: self._wgrad(*qkv_spec[:9], batch=3, b_bs=D, out_bs=zs))
                release("dqkv", li)
            ops.gemm(dqkv, self.wqkv[i], a.dyln, T, D, 3 * D, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=3 * D,
                     ldb=3 * D, ldc=D, epilogue=EPI_BF16)
            wb ^= 1
            acquire("dhb", wb)
            bias.ln_bwd(a.dyln, D, a.h[i], D, a.mu1[i], a.rs1[i], f[ln("norm1.weight"):], a.dh, D, T,
                        gv(self.lname(i, "norm1.weight")), gv(self.lname(i - 1, "mlp.fc2.bias")) if i > 0 else None,
                        dres=a.dh, lddres=D, dx_bf16=a.dhb[wb], lddxb=D,
                        dx_dropout=dd(3 + 3 * (i - 1)) if i > 0 else dd(0))
            fire(self.layout.buckets[L - i])
        # ---- embedding: conv weight grad (wgrad over patches), bias / pos / cls ----
        dhb = a.dhb[wb]
        on_side(lambda: self._wgrad(dhb, D, a.patches, a.kpad, D, cfg.patch_k, a.Tp, gv("embedding.weight"),
                                    cfg.patch_k))
        ops.embed_grad(a.dh, b, N, D, gv("transformer.pos_embedding.pos_embedding"), gv("cls_token"),
                       gv("embedding.bias"), dropout=dd(0))
        fire(self.layout.buckets[-1])
        bias.flush()
        if overlap:
            main.wait_stream(side)
        return g
