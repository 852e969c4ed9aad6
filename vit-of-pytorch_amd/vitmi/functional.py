"""Autograd functions over libvit_hip.so for the standalone sub-module path.

`VisionTransformer.forward` runs the whole network as one fused engine node (vitmi.engine). A user
of the reference can also call its building blocks on their own (reference src/model.py:
`PositionEmbs` :16-22, `MlpBlock` :41-51, `LinearGeneral` :61-63, `SelfAttention` :83-101,
`EncoderBlock` :117-130, `Encoder` :148-156) and the torch.nn leaves inside them (nn.Linear,
nn.LayerNorm, nn.GELU, nn.Dropout). vitmi.model composes those forwards from the functions here, so
each standalone module runs — forward and backward — on the same hand-written gfx950 kernels as the
engine: the bf16 MFMA GEMM (f32 accumulation, f32 in / f32 out at this boundary), the attention
kernels (LDS-resident or K/V-tiled), LayerNorm, GELU, counter-based dropout.

There is no PyTorch compute fallback: every function raises on CPU tensors. Padding copies are
allocated per call (the standalone path favours generality over the engine's preallocated
workspaces); bf16 copies of weights that take no gradient (LoRA's frozen bases) are cached per
weight version.
"""
from __future__ import annotations

import math

import torch

from . import ops
from ._lib import EPI_BIAS_RESID_F32, EPI_F32, K_CONTIG, MN_CONTIG

F32, BF16 = torch.float32, torch.bfloat16


def _rup(x, m):
    return (x + m - 1) // m * m


def _gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("vitmi sub-modules run on the MI355X HIP path only; move the module and its inputs to "
                               "the GPU (no CPU fallback)")


def _f32(t):
    return t.contiguous() if t.dtype == F32 else t.to(F32).contiguous()


def _pad_bf16(x2, rows_p, cols_p):
    """bf16 copy of f32 [rows][cols] in a [rows_p][cols_p] buffer whose padding is zero (vit_cast_pad_rows
    zeroes the pad columns; only the pad rows are cleared separately)."""
    rows, cols = x2.shape
    out = torch.empty(rows_p, cols_p, device=x2.device, dtype=BF16)
    if rows:
        ops.cast_pad_rows(x2, rows, cols, out, cols_p)
    if rows_p > rows:
        ops.zero_(out[rows:])
    return out


_ZROW = {}


def _zero_row(n, dev):
    """a zero f32 row of >= n elements: the bias epilogue's residual operand at row stride 0 (bias only)"""
    z = _ZROW.get(dev)
    if z is None or z.numel() < n:
        z = torch.zeros(max(n, 4096), device=dev, dtype=F32)
        _ZROW[dev] = z
    return z


def _frozen_bf16(w, key, make):
    """bf16 operand copies of a weight that takes no gradient (LoRA's frozen bases, res-vit/model.py:573-584):
    made once per (weight, layout) and kept on the weight object itself, valid while its storage and
    version counter are unchanged, instead of per call"""
    if w.requires_grad:
        return make()
    cache = getattr(w, "_vitmi_bf16", None)
    if cache is None:
        cache = {}
        try:
            w._vitmi_bf16 = cache
        except AttributeError:
            return make()
    sig = (w.data_ptr(), w._version, tuple(w.shape))
    hit = cache.get(key)
    if hit is not None and hit[0] == sig:
        return hit[1]
    out = make()
    cache[key] = (sig, out)
    return out


# ---- Linear / LinearGeneral -------------------------------------------------------------------------
class HipLinear(torch.autograd.Function):
    """y [rows, n_out] = x [rows, k] @ W + b (bf16 MFMA operands, f32 accumulate and output).
    w_in_out: W stored [k][n_out] (LinearGeneral, JAX layout, src/model.py:58) instead of nn.Linear's
    [n_out][k]. Weight gradients: split-K over the rows (ops.wgrad)."""

    @staticmethod
    def forward(ctx, x2, w, b, w_in_out):
        rows, k = x2.shape
        n_out = w.shape[1] if w_in_out else w.shape[0]
        kp, rp, np8 = _rup(k, 64), _rup(max(rows, 1), 64), _rup(n_out, 8)
        x2 = _f32(x2)
        w2 = _f32(w).reshape(k, n_out) if w_in_out else _f32(w).reshape(n_out, k)
        xb = _pad_bf16(x2, rp, kp)
        if w_in_out:  # B(k, n) = W[k][n]: MN-contiguous rows of n_out (16-B padded), zero rows past k
            wb, bl, ldb = _frozen_bf16(w, "fwd", lambda: _pad_bf16(w2, kp, np8)), MN_CONTIG, np8
        else:         # B(k, n) = W[n][k]: K-contiguous
            wb, bl, ldb = _frozen_bf16(w, "fwd", lambda: _pad_bf16(w2, n_out, kp)), K_CONTIG, kp
        y = torch.empty(rows, n_out, device=x2.device, dtype=F32)
        if rows:
            if b is not None:
                ops.gemm(xb, wb, y, rows, n_out, kp, a_layout=K_CONTIG, b_layout=bl, lda=kp, ldb=ldb, ldc=n_out,
                         epilogue=EPI_BIAS_RESID_F32, bias=_f32(b).reshape(-1), aux=_zero_row(n_out, x2.device),
                         ldaux=0)
            else:
                ops.gemm(xb, wb, y, rows, n_out, kp, a_layout=K_CONTIG, b_layout=bl, lda=kp, ldb=ldb, ldc=n_out,
                         epilogue=EPI_F32)
        ctx.save_for_backward(xb, w2)
        ctx.w_obj = w  # the weight object (a Parameter): the frozen-weight cache lives on it
        ctx.dims = (rows, k, n_out, w_in_out, b is not None, tuple(w.shape))
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, w2 = ctx.saved_tensors
        rows, k, n_out, w_in_out, has_b, wshape = ctx.dims
        dy = _f32(dy)
        kp, rp, npd = _rup(k, 64), xb.shape[0], _rup(n_out, 64)
        dyb = _pad_bf16(dy, rp, npd)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(rows, k, device=dy.device, dtype=F32)
            if rows:
                w2r = w2.reshape(k, n_out) if w_in_out else w2.reshape(n_out, k)
                if w_in_out:  # B(kk = n, n' = k_in) = W[k_in][n]: K-contiguous [k][npd]
                    wt = _frozen_bf16(ctx.w_obj, "dgrad", lambda: _pad_bf16(_f32(w2r), k, npd))
                    bl, ldb = K_CONTIG, npd
                else:         # B(kk = n, n' = k_in) = W[n][k_in]: MN-contiguous [npd][k8]
                    k8 = _rup(k, 8)
                    wt = _frozen_bf16(ctx.w_obj, "dgrad", lambda: _pad_bf16(_f32(w2r), npd, k8))
                    bl, ldb = MN_CONTIG, k8
                ops.gemm(dyb, wt, dx, rows, k, npd, a_layout=K_CONTIG, b_layout=bl, lda=npd, ldb=ldb, ldc=k,
                         epilogue=EPI_F32)
        if ctx.needs_input_grad[1]:
            if w_in_out:  # dW [k][n_out] = x^T dy
                dw = torch.empty(k, n_out, device=dy.device, dtype=F32)
                ops.wgrad(xb, kp, dyb, npd, k, n_out, rp, dw, n_out)
            else:         # dW [n_out][k] = dy^T x
                dw = torch.empty(n_out, k, device=dy.device, dtype=F32)
                ops.wgrad(dyb, npd, xb, kp, n_out, k, rp, dw, k)
            dw = dw.reshape(wshape)
        if has_b and ctx.needs_input_grad[2]:
            db = torch.empty(n_out, device=dy.device, dtype=F32)
            part = torch.empty(ops.colsum_partial_rows(max(rows, 1)), n_out, device=dy.device, dtype=F32)
            ops.colsum(dy, rows, n_out, n_out, part, db)
        return dx, dw, db, None


def linear(x, weight, bias=None):
    """nn.Linear / F.linear (src/model.py:31-32,194) on the bf16 MFMA GEMM: weight [out][in]."""
    _gpu(x, weight, bias)
    lead = x.shape[:-1]
    y = HipLinear.apply(x.reshape(-1, x.shape[-1]), weight, bias, False)
    return y.reshape(*lead, weight.shape[0])


def linear_general(x, weight, bias, dims):
    """LinearGeneral.forward (src/model.py:61-63): torch.tensordot(x, weight, dims=dims) + bias, for the
    contraction the reference uses — x's trailing len(in) dims against weight's leading ones
    (dims=([2], [0]) for q/k/v, ([2, 3], [0, 1]) for out)."""
    _gpu(x, weight, bias)
    xd, wd = ([dims[0]], [dims[1]]) if isinstance(dims[0], int) else (list(dims[0]), list(dims[1]))
    n_in = len(xd)
    if wd != list(range(n_in)) or xd != list(range(x.dim() - n_in, x.dim())):
        raise NotImplementedError(f"LinearGeneral dims {dims}: the HIP path contracts x's trailing dims with the "
                                  "weight's leading dims (the reference's ([2],[0]) / ([2,3],[0,1]))")
    if tuple(x.shape[x.dim() - n_in:]) != tuple(weight.shape[:n_in]):
        raise ValueError(f"LinearGeneral: x {tuple(x.shape)} and weight {tuple(weight.shape)} do not contract")
    k = math.prod(weight.shape[:n_in])
    feat = tuple(weight.shape[n_in:])
    lead = tuple(x.shape[:x.dim() - n_in])
    y = HipLinear.apply(x.reshape(-1, k), weight.reshape(k, -1), bias.reshape(-1), True)
    return y.reshape(*lead, *feat)


# ---- LayerNorm ------------------------------------------------------------------------------------
class HipLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, gamma, beta, eps):
        rows, d = x2.shape
        x2 = _f32(x2)
        y = torch.empty_like(x2)
        mean = torch.empty(rows, device=x2.device, dtype=F32)
        rstd = torch.empty(rows, device=x2.device, dtype=F32)
        if rows:
            ops.layernorm_fwd(x2, d, _f32(gamma), _f32(beta), y, d, mean, rstd, rows, d, eps)
        ctx.save_for_backward(x2, gamma, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, gamma, mean, rstd = ctx.saved_tensors
        rows, d = x2.shape
        dy = _f32(dy)
        dx = torch.empty_like(x2)
        gb = torch.zeros(2 * d, device=dy.device, dtype=F32)
        if rows:
            part = torch.empty(ops.layernorm_bwd_partial_rows(rows), 3 * d, device=dy.device, dtype=F32)
            ops.layernorm_bwd(dy, d, x2, d, mean, rstd, _f32(gamma), dx, d, part, rows, d, dgamma_dbeta=gb)
        return dx, gb[:d].clone(), gb[d:].clone(), None


def layer_norm(x, weight, bias, eps=1e-5):
    """nn.LayerNorm over the last dim (src/model.py:108,114,146): biased variance, eps, affine."""
    _gpu(x, weight, bias)
    d = x.shape[-1]
    if weight is None or bias is None:
        raise NotImplementedError("vitmi LayerNorm needs elementwise_affine=True (the reference's)")
    return HipLayerNorm.apply(x.reshape(-1, d), weight, bias, float(eps)).reshape(x.shape)


# ---- elementwise -------------------------------------------------------------------------------
class HipGELU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u):
        u = _f32(u)
        g = torch.empty_like(u)
        ops.gelu_f32(u, g, u.numel())
        ctx.save_for_backward(u)
        return g

    @staticmethod
    def backward(ctx, dg):
        u, = ctx.saved_tensors
        du = torch.empty_like(u)
        ops.gelu_bwd_f32(u, _f32(dg), du, u.numel())
        return du


def gelu(x):
    """nn.GELU() (exact erf, src/model.py:33)"""
    _gpu(x)
    return HipGELU.apply(x)


_DROP_SEED = None
_DROP_OFFSET = [0]


def _drop_desc(p, cols):
    global _DROP_SEED
    if _DROP_SEED is None:
        _DROP_SEED = (torch.initial_seed() * 0x9E3779B97F4A7C15 + 0x2545F4914F6CDD1D) & (2**64 - 1)
    _DROP_OFFSET[0] += 1
    # site 0xFFFF: the standalone path's own stream, never one of the engine's sites
    return ops.dropout_desc(p, 0xFFFF, _DROP_SEED, _DROP_OFFSET[0])


class HipDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        x = _f32(x)
        cols = x.shape[-1] if x.dim() else 1
        rows = x.numel() // max(cols, 1)
        d = _drop_desc(p, cols)
        y = torch.empty_like(x)
        ops.dropout_apply_f32(d, x, y, rows, cols)
        ctx.desc, ctx.rc = d, (rows, cols)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = _f32(dy)
        dx = torch.empty_like(dy)
        ops.dropout_apply_f32(ctx.desc, dy, dx, *ctx.rc)
        return dx, None


def dropout(x, p, training):
    """nn.Dropout(p) (src/model.py:19-20,46-51,124-125): a counter-based Philox mask, regenerated by the
    backward; identity in eval mode or at p = 0."""
    if not training or p == 0.0:
        return x
    if not 0.0 <= p < 1.0:
        raise ValueError(f"dropout probability has to be in [0, 1), got {p}")
    _gpu(x)
    return HipDropout.apply(x, float(p))


class HipAdd(torch.autograd.Function):
    """out = x + y, y broadcast over x's leading dims (y.numel() divides x.numel())."""

    @staticmethod
    def forward(ctx, x, y):
        x, y = _f32(x), _f32(y)
        out = torch.empty_like(x)
        ops.add_bcast_f32(x, y, out, x.numel() // y.numel(), y.numel())
        ctx.shapes = (x.shape, y.shape, x.numel() // y.numel())
        return out

    @staticmethod
    def backward(ctx, dout):
        xs, ys, outer = ctx.shapes
        dout = _f32(dout)
        dy = None
        if ctx.needs_input_grad[1]:
            if outer == 1:
                dy = dout.reshape(ys)
            else:
                inner = dout.numel() // outer
                dy = torch.empty(inner, device=dout.device, dtype=F32)
                part = torch.empty(ops.colsum_partial_rows(outer), inner, device=dout.device, dtype=F32)
                ops.colsum(dout, outer, inner, inner, part, dy)
                dy = dy.reshape(ys)
        return dout, dy


def add(x, y):
    """x + y with y broadcast over x's leading dims (residual add `out += residual`,
    src/model.py:124,129; position embedding x + pos_embedding [1, N, D], :17)."""
    _gpu(x, y)
    ys = list(y.shape)
    while ys and ys[0] == 1 and len(ys) > 1:
        ys.pop(0)
    if len(ys) > x.dim() or list(x.shape[x.dim() - len(ys):]) != ys:
        raise ValueError(f"add: cannot broadcast {tuple(y.shape)} over {tuple(x.shape)}")
    return HipAdd.apply(x, y)


# ---- attention core -------------------------------------------------------------------------------
class HipAttention(torch.autograd.Function):
    """softmax((q k^T) / sqrt(hd)) v for q, k, v [b, n, H, hd] (src/model.py:90-97) on the fused
    attention kernels (bf16 operands, f32 softmax / accumulation)."""

    @staticmethod
    def forward(ctx, q, k, v):
        b, n, h, hd = q.shape
        d = h * hd
        t = b * n
        qkv = torch.empty(t, 3 * d, device=q.device, dtype=BF16)
        for z, x in enumerate((q, k, v)):
            ops.pack_cols(_f32(x).reshape(t, d), 0, d, t, d, 1, qkv[:, z * d:], 3 * d)
        o = torch.empty(t, d, device=q.device, dtype=BF16)
        lse = torch.empty(b, h, n, device=q.device, dtype=F32)
        ops.attention_fwd(qkv, o, lse, b, n, h, hd, 1.0 / math.sqrt(hd))
        out = torch.empty(t, d, device=q.device, dtype=F32)
        ops.unpack_bf16_f32(o, d, t, d, out, d)
        ctx.save_for_backward(qkv, o, lse)
        ctx.shape = (b, n, h, hd)
        return out.reshape(b, n, h, hd)

    @staticmethod
    def backward(ctx, dout):
        qkv, o, lse = ctx.saved_tensors
        b, n, h, hd = ctx.shape
        d, t = h * hd, b * n
        dob = torch.empty(t, d, device=qkv.device, dtype=BF16)
        ops.cast_bf16(_f32(dout), dob, t * d)
        dqkv = torch.empty(t, 3 * d, device=qkv.device, dtype=BF16)
        ops.attention_bwd(qkv, o, dob, lse, dqkv, b, n, h, hd, 1.0 / math.sqrt(hd))
        grads = []
        for z in range(3):
            g = torch.empty(b, n, h, hd, device=qkv.device, dtype=F32)
            ops.unpack_bf16_f32(dqkv[:, z * d:], 3 * d, t, d, g, d)
            grads.append(g)
        return tuple(grads)


def attention(q, k, v):
    _gpu(q, k, v)
    if q.dim() != 4 or q.shape != k.shape or q.shape != v.shape:
        raise ValueError(f"attention: q, k, v must share a [b, n, H, hd] shape, got {tuple(q.shape)}, "
                         f"{tuple(k.shape)}, {tuple(v.shape)}")
    return HipAttention.apply(q, k, v)


def attention_ragged(q, k, v, cu_q, max_q):
    """Ragged-query attention forward (Res-ViT inference, res-vit/model.py:494-529): q [total, H, hd]
    holds every sample's active query tokens back to back (sample b at rows cu_q[b] .. cu_q[b+1]), k / v
    [B, Nkv, H, hd] all of each sample's tokens; returns [total, H, hd] f32. One varlen kernel launch
    (vit_attention_fwd_varlen) for the batch. Forward only (the reference uses it under no_grad)."""
    _gpu(q, k, v, cu_q)
    if torch.is_grad_enabled() and any(t.requires_grad for t in (q, k, v)):
        raise NotImplementedError("ragged attention is the inference path (res-vit/model.py:494-529); it has no "
                                  "backward")
    total, h, hd = q.shape
    b, nkv = k.shape[0], k.shape[1]
    d = h * hd
    qb = torch.empty(max(total, 1), d, device=q.device, dtype=BF16)
    kb = torch.empty(b * nkv, d, device=q.device, dtype=BF16)
    vb = torch.empty(b * nkv, d, device=q.device, dtype=BF16)
    if total:
        ops.cast_bf16(_f32(q).reshape(-1), qb, total * d)
    ops.cast_bf16(_f32(k).reshape(-1), kb, b * nkv * d)
    ops.cast_bf16(_f32(v).reshape(-1), vb, b * nkv * d)
    ob = torch.empty(max(total, 1), d, device=q.device, dtype=BF16)
    ops.attention_fwd_varlen(qb, d, kb, d, vb, d, ob, d, cu_q.to(torch.int32).contiguous(), b, int(max_q), nkv, h, hd,
                             1.0 / math.sqrt(hd))
    out = torch.empty(total, h, hd, device=q.device, dtype=F32)
    if total:
        ops.unpack_bf16_f32(ob, d, total, d, out, d)
    return out


def patch_embed(x, weight, bias, patch):
    """nn.Conv2d(3, D, kernel = stride = patch) on images x [B, 3, H, W] as im2col (vit_im2col_f32) + the
    bf16 MFMA GEMM with bias, returned token-major [B, (H/P)(W/P), D] (the reference's
    rearrange(conv(x), 'b c h w -> b (h w) c'); res-vit/model.py:629-630, src/model.py:197-200).
    Gradients reach weight and bias (the images are inputs)."""
    _gpu(x, weight, bias)
    if x.requires_grad:
        raise NotImplementedError("patch_embed: no gradient with respect to the input images")
    b, c, hh, ww = x.shape
    if c != 3 or hh != ww:
        raise ValueError(f"patch_embed expects square 3-channel images, got {tuple(x.shape)}")
    g = hh // patch
    n = g * g
    k = 3 * patch * patch
    kpad = _rup(k, 64)
    cols = torch.empty(b * (n + 1), kpad, device=x.device, dtype=F32)
    ops.im2col_f32(_f32(x), cols, b, hh, patch, kpad)
    rows = cols.view(b, n + 1, kpad)[:, 1:, :k].reshape(b * n, k)  # drop the cls rows im2col leaves zero
    d = weight.shape[0]
    y = HipLinear.apply(rows, weight.reshape(d, k), bias, False)
    return y.view(b, n, d)
