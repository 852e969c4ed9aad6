"""Torch-tensor wrappers over the C ABI (include/vit_hip.h).

Every function launches hand-written gfx950 kernels from libvit_hip.so on the current torch
stream. Inputs must already live on the GPU with the documented dtype/layout; nothing here
falls back to a PyTorch implementation.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import COLSUM_BATCH_MAX, Dropout, GemmArgs, check

BF16 = torch.bfloat16
F32 = torch.float32


def lib():
    return _lib.load()


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _chk(t, dtype, name):
    if t is None:
        return
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")


# ---------------------------------------------------------------------------------------------
def _gemm_args(A, B, C, M, N, K, *, a_layout, b_layout, lda, ldb, ldc, epilogue, bias=None, aux=None, ldaux=0,
               C2=None, ldc2=0, aux2=None, batch=1, a_bs=0, b_bs=0, c_bs=0, bias_bs=0, split_k=1, tokens=0, tile=0,
               col_partial=None, dropout=None):
    a = GemmArgs()
    a.M, a.N, a.K = M, N, K
    a.A, a.lda, a.a_batch_stride, a.a_layout = A.data_ptr(), lda, a_bs, a_layout
    a.B, a.ldb, a.b_batch_stride, a.b_layout = B.data_ptr(), ldb, b_bs, b_layout
    a.C, a.ldc, a.c_batch_stride = C.data_ptr(), ldc, c_bs
    a.C2, a.ldc2 = (C2.data_ptr() if C2 is not None else None), ldc2
    a.bias, a.bias_batch_stride = (bias.data_ptr() if bias is not None else None), bias_bs
    a.aux, a.ldaux = (aux.data_ptr() if aux is not None else None), ldaux
    a.aux2 = aux2.data_ptr() if aux2 is not None else None
    a.batch, a.split_k, a.tokens = batch, split_k, tokens
    a.col_partial = col_partial.data_ptr() if col_partial is not None else None
    a.epilogue, a.tile = epilogue, tile
    a.dropout = ctypes.pointer(dropout) if dropout is not None else None
    return a


def dropout_desc(p, site, seed, offset, row_stride=1):
    """struct vit_dropout for nn.Dropout(p) at `site` (None when p == 0)."""
    if not p:
        return None
    return Dropout(float(p), int(site), int(seed) & (2**64 - 1), int(offset) & (2**64 - 1), int(row_stride))


def _dp(d):
    return ctypes.pointer(d) if d is not None else None


def dropout_mask(d, row0, rows, cols, out, ld):
    """out[r, c] = multiplier (0 or 1/(1-p)) of element (row0 + r, c) of dropout descriptor d."""
    _chk(out, F32, "out")
    check(lib().vit_dropout_mask(_dp(d), row0, rows, cols, _p(out), ld, _stream()), "vit_dropout_mask")


# bench.py's roofline_fwd_dgrad probe: when a list, every vit_gemm_bf16 call with M >= GEMM_PROBE_MIN_M
# that is not a split-K weight gradient appends (start event, end event, 2 M N K, epilogue), the events recorded
# on the stream the call runs on (one call = the 256x256 kernel and its wave-split remainder launch)
GEMM_PROBE = None
GEMM_PROBE_MIN_M = 0


def gemm(A, B, C, M, N, K, part=0, **kw):
    """bf16 MFMA GEMM, C[m,n] = sum_k A(m,k) B(k,n) + fused epilogue (see vit_gemm_args).
    part 1 / 2: only the whole-wave rows / the wave-split remainder rows (vit_gemm_bf16_part)."""
    _chk(A, BF16, "A")
    _chk(B, BF16, "B")
    a = _gemm_args(A, B, C, M, N, K, **kw)
    if part:
        check(lib().vit_gemm_bf16_part(ctypes.byref(a), int(part), _stream()), "vit_gemm_bf16_part")
        return
    probe = GEMM_PROBE is not None and M >= GEMM_PROBE_MIN_M and a.split_k == 1 and a.epilogue != _lib.EPI_SPLITK
    if probe:
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record()
    check(lib().vit_gemm_bf16(ctypes.byref(a), _stream()), "vit_gemm_bf16")
    if probe:
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        GEMM_PROBE.append((ev0, ev1, 2.0 * M * N * K * a.batch, int(a.epilogue)))


def gemm_tile_rows(A, B, C, M, N, K, **kw):
    return int(lib().vit_gemm_tile_rows(ctypes.byref(_gemm_args(A, B, C, M, N, K, **kw))))


def gemm_split_rows(A, B, C, M, N, K, **kw):
    """rows of the whole-wave part of a wave-split gemm(...) call (0: one launch)"""
    return int(lib().vit_gemm_split_rows(ctypes.byref(_gemm_args(A, B, C, M, N, K, **kw))))


def gemm_partial_rows(A, B, C, M, N, K, **kw):
    """rows of col_partial a gemm(...) call with these arguments writes (to be reduced)"""
    return int(lib().vit_gemm_partial_rows(ctypes.byref(_gemm_args(A, B, C, M, N, K, **kw))))


def splitk_reduce(ws, batch, split, M, N, out, ldo, out_bs=0, accumulate=False):
    _chk(ws, F32, "ws")
    _chk(out, F32, "out")
    check(lib().vit_splitk_reduce(_p(ws), batch, split, M, N, _p(out), ldo, out_bs, int(accumulate), _stream()),
          "vit_splitk_reduce")


def splitk_reduce_group(jobs):
    """several splitk_reduce calls in one launch (vit_splitk_reduce_group); jobs: [(ws, batch, split, M, N, out, ldo,
    out_bs, accumulate)], each output bit-identical to its own splitk_reduce"""
    for k in range(0, len(jobs), _lib.SPLITK_GROUP_MAX):
        part = jobs[k:k + _lib.SPLITK_GROUP_MAX]
        arr = (_lib.SplitkJob * len(part))()
        for i, (ws, batch, split, M, N, out, ldo, out_bs, acc) in enumerate(part):
            _chk(ws, F32, "ws")
            _chk(out, F32, "out")
            arr[i] = _lib.SplitkJob(_p(ws), batch, split, M, N, _p(out), ldo, out_bs, int(acc), 0)
        check(lib().vit_splitk_reduce_group(arr, len(part), _stream()), "vit_splitk_reduce_group")


def layernorm_fwd(x, ldx, gamma, beta, y, ldy, mean, rstd, rows, D, eps=1e-5):
    _chk(x, F32, "x")
    check(lib().vit_layernorm_fwd(_p(x), ldx, _p(gamma), _p(beta), _p(y), ldy, int(y.dtype == F32), _p(mean),
                                  _p(rstd), rows, D, eps, _stream()), "vit_layernorm_fwd")


def layernorm_bwd_partial_rows(rows):
    return int(lib().vit_layernorm_bwd_partial_rows(rows))


def layernorm_bwd_blocks(rows):
    """rows of block partials [nblk][3*D] a layernorm_bwd without dgamma/dx_colsum leaves to reduce."""
    return int(lib().vit_layernorm_bwd_blocks(rows))


def layernorm_bwd(dy, lddy, x, ldx, mean, rstd, gamma, dx, lddx, partial, rows, D, *, dres=None, lddres=0,
                  dx_bf16=None, lddxb=0, dgamma_dbeta=None, dx_colsum=None, accumulate=False, dx_dropout=None):
    check(lib().vit_layernorm_bwd(_p(dy), lddy, int(dy.dtype == F32), _p(x), ldx, _p(mean), _p(rstd), _p(gamma),
                                  _p(dres), lddres, _p(dx), lddx, _p(dx_bf16), lddxb, _p(partial), _p(dgamma_dbeta),
                                  _p(dx_colsum), int(accumulate), rows, D, _dp(dx_dropout), _stream()),
          "vit_layernorm_bwd")


# ATTN_ONESHOT: the LDS-resident kernels in their one-workgroup-per-(image, head) forms only (no persistent
# forward / backward); for A/B timing and the persistent kernels' parity tests
ATTN_AUTO, ATTN_RESIDENT, ATTN_TILED, ATTN_ONESHOT = 0, 1, 2, 3


def attention_bias_rows(N, hd, path=ATTN_AUTO):
    """rows of the backward's bias_partial per image (resident: 8 on the persistent kernel, else 1;
    tiled: ceil(N/64))."""
    return int(lib().vit_attention_bias_rows(N, hd, path))


def attention_workspace_elems(B, N, H, path=ATTN_AUTO):
    return int(lib().vit_attention_workspace_elems(B, N, H, path))


def attention_fwd(qkv, o, lse, B, N, H, hd, scale, q_rows=None, path=ATTN_AUTO):
    """q_rows: only queries [0, q_rows) are needed (None: all N). path: ATTN_AUTO picks the
    LDS-resident kernels for N <= 320 and the K/V-tiled ones above."""
    _chk(qkv, BF16, "qkv")
    _chk(o, BF16, "o")
    _chk(lse, F32, "lse")
    check(lib().vit_attention_fwd_ex(_p(qkv), _p(o), _p(lse), B, N, H, hd, scale, N if q_rows is None else q_rows,
                                     path, _stream()), "vit_attention_fwd")


def attention_bwd(qkv, o, dout, lse, dqkv, B, N, H, hd, scale, bias_partial=None, q_rows=None, path=ATTN_AUTO,
                  workspace=None):
    """q_rows: dout is zero outside queries [0, q_rows) (None: all N). bias_partial:
    [B * attention_bias_rows(N, hd, path)][3D] f32. workspace: >= attention_workspace_elems floats
    (allocated here when None and the path needs one)."""
    _chk(workspace, F32, "workspace")
    need = attention_workspace_elems(B, N, H, path)
    if need and (workspace is None or workspace.numel() < need):
        if workspace is not None:
            raise ValueError(f"attention workspace has {workspace.numel()} floats, needs {need}")
        workspace = torch.empty(need, device=qkv.device, dtype=F32)
    check(lib().vit_attention_bwd_ex(_p(qkv), _p(o), _p(dout), _p(lse), _p(dqkv), _p(bias_partial), B, N, H, hd,
                                     scale, N if q_rows is None else q_rows, path, _p(workspace if need else None),
                                     _stream()), "vit_attention_bwd")


def im2col(x, out, B, img, P, Kpad):
    _chk(x, F32, "x")
    _chk(out, BF16, "out")
    check(lib().vit_im2col(_p(x), _p(out), B, img, P, Kpad, _stream()), "vit_im2col")


def preprocess_u8(images, out, flips=None, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
    """images uint8 [B, H, W, 3] (device, image rows contiguous) -> out f32 [B, 3, h, w]:
    Pillow-exact bilinear resize, optional per-sample horizontal flip, ToTensor + Normalize."""
    _chk(images, torch.uint8, "images")
    _chk(out, F32, "out")
    _chk(flips, torch.uint8, "flips")
    if images.dim() != 4 or images.shape[3] != 3 or out.dim() != 4 or out.shape[1] != 3:
        raise ValueError(f"preprocess_u8: images [B,H,W,3] -> out [B,3,h,w], got {tuple(images.shape)} -> "
                         f"{tuple(out.shape)}")
    B, H, W, _ = images.shape
    if out.shape[0] != B or (flips is not None and flips.numel() != B):
        raise ValueError("preprocess_u8: batch mismatch")
    if images[0].stride() != (W * 3, 3, 1) or not out.is_contiguous():
        raise ValueError("preprocess_u8: images must have contiguous [H, W, 3] rows and out must be contiguous")
    ms = (ctypes.c_float * 6)(*[float(v) for v in mean], *[float(v) for v in std])
    check(lib().vit_preprocess_u8(_p(images), B, H, W, images.stride(0) if B > 1 else H * W * 3, _p(flips),
                                  out.shape[2], out.shape[3], ms, _p(out), _stream()), "vit_preprocess_u8")


def embed_grad(dh0, B, N, D, dpos, dcls, dconv_bias, dropout=None):
    check(lib().vit_embed_grad(_p(dh0), B, N, D, _p(dpos), _p(dcls), _p(dconv_bias), _dp(dropout), _stream()),
          "vit_embed_grad")


def colsum_partial_rows(rows):
    return int(lib().vit_colsum_partial_rows(rows))


def colsum(inp, rows, cols, ld, partial, out, accumulate=False):
    check(lib().vit_colsum(_p(inp), int(inp.dtype == BF16), rows, cols, ld, _p(partial), _p(out), int(accumulate),
                           _stream()), "vit_colsum")


def colsum_batch(jobs):
    """jobs: [(inp f32, rows, cols, ld, seg, (out0, out1, out2), accumulate)], at most COLSUM_BATCH_MAX:
    every column reduction in one launch (vit_colsum_batch)"""
    arr = (_lib.ColsumJob * len(jobs))()
    for k, (inp, rows, cols, ld, seg, outs, acc) in enumerate(jobs):
        if inp.dtype != F32:
            raise ValueError("colsum_batch: f32 inputs only")
        o = list(outs) + [None] * (3 - len(outs))
        arr[k] = _lib.ColsumJob(_p(inp), rows, cols, ld, seg, _p(o[0]), _p(o[1]), _p(o[2]), int(acc), 0)
    check(lib().vit_colsum_batch(arr, len(jobs), _stream()), "vit_colsum_batch")


def gemm_f32(M, N, K, A, lda, a_trans, B, ldb, b_trans, C, ldc, bias=None, accumulate=False):
    check(lib().vit_gemm_f32(M, N, K, _p(A), lda, int(a_trans), _p(B), ldb, int(b_trans), _p(C), ldc, _p(bias),
                             int(accumulate), _stream()), "vit_gemm_f32")


def cross_entropy(logits, labels, dlogits, grad_scale, row_stats):
    _chk(logits, F32, "logits")
    _chk(labels, torch.int64, "labels")
    B, C = logits.shape
    check(lib().vit_cross_entropy(_p(logits), _p(labels), B, C, _p(dlogits), grad_scale, _p(row_stats), _stream()),
          "vit_cross_entropy")


def sgd_step(p, g, buf, p_bf16, n, lr, momentum, wd, first):
    check(lib().vit_sgd_step(_p(p), _p(g), _p(buf), _p(p_bf16), n, lr, momentum, wd, int(first), _stream()),
          "vit_sgd_step")


def cast_bf16(inp, out, n):
    check(lib().vit_cast_f32_bf16(_p(inp), _p(out), n, _stream()), "vit_cast_f32_bf16")


def cast_pad_rows(inp, rows, cols, out, ldo):
    check(lib().vit_cast_pad_rows(_p(inp), rows, cols, _p(out), ldo, _stream()), "vit_cast_pad_rows")


def cast_pad_batch(jobs):
    """several f32 -> bf16 casts into zero-padded buffers in one launch per 8 (vit_cast_pad_batch); jobs: [(inp f32
    [rows][>= cols] row stride ldi, rows, cols, ldi, out bf16 (row stride ldo), ldo, rows_pad, cols_pad)]"""
    for k in range(0, len(jobs), _lib.CAST_BATCH_MAX):
        part = jobs[k:k + _lib.CAST_BATCH_MAX]
        arr = (_lib.CastJob * len(part))()
        for i, (inp, rows, cols, ldi, out, ldo, rows_pad, cols_pad) in enumerate(part):
            _chk(inp, F32, "inp")
            _chk(out, BF16, "out")
            arr[i] = _lib.CastJob(_p(inp), rows, cols, ldi, _p(out), ldo, rows_pad, cols_pad)
        check(lib().vit_cast_pad_batch(arr, len(part), _stream()), "vit_cast_pad_batch")


def axpby(x, y, n, a, b):
    check(lib().vit_axpby(_p(x), _p(y), n, a, b, _stream()), "vit_axpby")


def pack_cols(inp, zstride, ldi, rows, cols, Z, out, ldo):
    check(lib().vit_pack_cols(_p(inp), zstride, ldi, rows, cols, Z, _p(out), ldo, int(out.dtype == BF16), _stream()),
          "vit_pack_cols")


def pack_cols_batched(inp, in_bs, zstride, ldi, rows, cols, Z, out, out_bs, ldo, batch):
    """pack_cols for `batch` layers at strides in_bs (floats, may be negative) / out_bs (elements)."""
    check(lib().vit_pack_cols_batched(_p(inp), in_bs, zstride, ldi, rows, cols, Z, _p(out), out_bs, ldo,
                                      int(out.dtype == BF16), batch, _stream()), "vit_pack_cols_batched")


def transpose_bf16(inp, rows, cols, ldi, out, ldo, batch=1, in_bs=0, out_bs=0):
    """out[z][c*ldo + r] = bf16(inp[z][r*ldi + c]) (K-contiguous weight copies; z strides may be negative)."""
    _chk(out, BF16, "out")
    check(lib().vit_transpose_f32_bf16(_p(inp), rows, cols, ldi, _p(out), ldo, batch, in_bs, out_bs, _stream()),
          "vit_transpose_f32_bf16")


def colsum3(inp, rows, seg, ld, partial, out0, out1, out2, accumulate=False):
    """column sums of a [rows][3*seg] matrix, segment k -> out_k (q|k|v bias gradients)."""
    check(lib().vit_colsum3(_p(inp), int(inp.dtype == BF16), rows, seg, ld, _p(partial), _p(out0), _p(out1), _p(out2),
                            int(accumulate), _stream()), "vit_colsum3")


# ---- fp32 (exact) forward ---------------------------------------------------------------------
def im2col_f32(x, out, B, img, P, Kpad):
    _chk(x, F32, "x")
    _chk(out, F32, "out")
    check(lib().vit_im2col_f32(_p(x), _p(out), B, img, P, Kpad, _stream()), "vit_im2col_f32")


def embed_fwd_f32(h, B, N, D, pos, cls):
    check(lib().vit_embed_fwd_f32(_p(h), B, N, D, _p(pos), _p(cls), _stream()), "vit_embed_fwd_f32")


def gelu_f32(inp, out, n):
    check(lib().vit_gelu_f32(_p(inp), _p(out), n, _stream()), "vit_gelu_f32")


def attention_fwd_f32(qkv, o, B, N, H, hd, inv_sqrt_hd):
    _chk(qkv, F32, "qkv")
    _chk(o, F32, "o")
    check(lib().vit_attention_fwd_f32(_p(qkv), _p(o), B, N, H, hd, inv_sqrt_hd, _stream()), "vit_attention_fwd_f32")


# ---- standalone sub-module path -----------------------------------------------------------------
def gelu_bwd_f32(u, dy, dx, n):
    check(lib().vit_gelu_bwd_f32(_p(u), _p(dy), _p(dx), n, _stream()), "vit_gelu_bwd_f32")


def dropout_apply_f32(d, inp, out, rows, cols):
    check(lib().vit_dropout_apply_f32(_dp(d), _p(inp), _p(out), rows, cols, _stream()), "vit_dropout_apply_f32")


def add_bcast_f32(x, y, out, outer, inner):
    check(lib().vit_add_bcast_f32(_p(x), _p(y), _p(out), outer, inner, _stream()), "vit_add_bcast_f32")


def segment_colsum(inp, ld, segs, seg_rows, cols, out, ldo, seg_stride=None, row0=0, scale=1.0):
    """out[s][c] = scale * sum of rows [s*seg_stride + row0, + seg_rows) of inp's column c (f32 or bf16 inp, even ld;
    fixed order); seg_stride defaults to seg_rows"""
    _chk(out, F32, "out")
    st = seg_rows if seg_stride is None else seg_stride
    check(lib().vit_segment_colsum(_p(inp), int(inp.dtype == BF16), ld, segs, st, row0, seg_rows, cols, float(scale),
                                   _p(out), ldo, _stream()), "vit_segment_colsum")


def segment_colsum_bcast(inp, ld, segs, seg_rows, cols, out, ldo, bc, ldbc, bc_rows, seg_stride=None, row0=0,
                         scale=1.0):
    """segment_colsum, and each segment's result as bf16 into rows [s*seg_stride, + bc_rows) of bc (bf16, ld ldbc)"""
    _chk(out, F32, "out")
    _chk(bc, BF16, "bc")
    st = seg_rows if seg_stride is None else seg_stride
    check(lib().vit_segment_colsum_bcast(_p(inp), int(inp.dtype == BF16), ld, segs, st, row0, seg_rows, cols,
                                         float(scale), _p(out), ldo, _p(bc), ldbc, bc_rows, _stream()),
          "vit_segment_colsum_bcast")


def router_dx_gate_partial_rows(rows_pad):
    return int(lib().vit_router_dx_gate_partial_rows(rows_pad))


def router_dx_gate(dx, ldx, g, ldg, g_scale, gp, ldgp, T, N, reserve, cols, out, ldo, col_partial=None, ldp=0):
    """out (bf16 [rows_pad][cols_pad]) = bf16((dx + [t % N >= reserve] g_scale g[t // N]) * gp) on [T][cols], zeros
    in the padding; col_partial: per 64-row block column sums of the rounded values (vit_router_dx_gate)"""
    _chk(dx, F32, "dx")
    _chk(g, F32, "g")
    _chk(gp, BF16, "gp")
    _chk(out, BF16, "out")
    check(lib().vit_router_dx_gate(_p(dx), ldx, _p(g), ldg, float(g_scale), _p(gp), ldgp, T, N, reserve, cols, _p(out),
                                   ldo, out.shape[0], out.shape[1], _p(col_partial), ldp, _stream()),
          "vit_router_dx_gate")


def router_head_fwd(logits, noise, noise_mode, yhard, N, reserve, training, norm):
    """the Res-ViT router head on logits f32 [T][bs][2] (vit_router_head_fwd): returns (soft, y_soft or None, hard,
    indices [T], entropy [] ) as new f32 tensors; noise_mode 1: noise = Gumbel g, 2: noise = exponential draws"""
    _chk(logits, F32, "logits")
    T, bs = logits.shape[0], logits.shape[1]
    for t, n in ((noise, "noise"), (yhard, "yhard")):
        if t is not None:
            _chk(t, F32, n)
            if tuple(t.shape) != tuple(logits.shape):
                raise ValueError(f"router_head_fwd: {n} shape {tuple(t.shape)} != logits {tuple(logits.shape)}")
    dev = logits.device
    soft, hard = torch.empty_like(logits), torch.empty_like(logits)
    ysoft = torch.empty_like(logits) if training else None
    idx = torch.empty(T, device=dev, dtype=F32)
    part = torch.empty(max(int(lib().vit_router_head_partials(T)), 1), device=dev, dtype=F32)
    ent = torch.empty((), device=dev, dtype=F32)
    check(lib().vit_router_head_fwd(_p(logits), _p(noise), int(noise_mode), _p(yhard), T, N, bs, reserve, int(training),
                                    float(norm), _p(soft), _p(ysoft), _p(hard), _p(idx), _p(part), _p(ent), _stream()),
          "vit_router_head_fwd")
    return soft, ysoft, hard, idx, ent


def router_head_bwd(soft, ysoft, dsoft, dhard, dind, dent, N, reserve, training, norm):
    """dlogits f32 [T][bs][2] of router_head_fwd's outputs (vit_router_head_bwd); any gradient may be None"""
    _chk(soft, F32, "soft")
    for t, n in ((ysoft, "ysoft"), (dsoft, "dsoft"), (dhard, "dhard"), (dind, "dind"), (dent, "dent")):
        if t is not None:
            _chk(t, F32, n)
    T, bs = soft.shape[0], soft.shape[1]
    dl = torch.empty_like(soft)
    check(lib().vit_router_head_bwd(_p(soft), _p(ysoft), _p(dsoft), _p(dhard), _p(dind), _p(dent), float(norm), T, N,
                                    bs, reserve, int(training), _p(dl), _stream()), "vit_router_head_bwd")
    return dl


def cls_mse(x, ldx, t, ldt, B, D):
    """(loss [], e [B][D]) with e = x rows - t rows (row strides ldx / ldt floats) and loss = mean(e^2)
    (vit_cls_mse)"""
    _chk(x, F32, "x")
    _chk(t, F32, "t")
    e = torch.empty(B, D, device=x.device, dtype=F32)
    part = torch.empty(B, device=x.device, dtype=F32)
    loss = torch.empty((), device=x.device, dtype=F32)
    check(lib().vit_cls_mse(_p(x), ldx, _p(t), ldt, B, D, _p(e), _p(part), _p(loss), _stream()), "vit_cls_mse")
    return loss, e


def cls_mse_bwd(dx, lddx, e, g):
    """dx rows (stride lddx floats) += (2 / e.numel()) e g (vit_cls_mse_bwd; g a device scalar)"""
    _chk(dx, F32, "dx")
    _chk(e, F32, "e")
    _chk(g, F32, "g")
    check(lib().vit_cls_mse_bwd(_p(dx), lddx, _p(e), e.shape[0], e.shape[1], _p(g), _stream()), "vit_cls_mse_bwd")


def router_select(indices, active_sets, nkeys):
    """(active bool [npos][T], sel bool [nkeys][T], any bool [nkeys]) from the pattern index f32 [T]
    (vit_router_select): active[j] = isin(indices.long(), active_sets[j]) (values < 32), sel[k] = indices == k,
    any[k] = sel[k].any()"""
    _chk(indices, F32, "indices")
    if not indices.is_contiguous():
        raise ValueError("router_select: indices must be contiguous")
    T, dev = indices.numel(), indices.device
    masks = []
    for st in active_sets:
        m = 0
        for v in st:
            if not 0 <= int(v) < 32:
                raise ValueError(f"router_select: index value {v} outside [0, 32)")
            m |= 1 << int(v)
        masks.append(m)
    active = torch.empty(len(masks), T, device=dev, dtype=torch.bool)
    sel = torch.empty(nkeys, T, device=dev, dtype=torch.bool)
    anyf = torch.empty(nkeys, device=dev, dtype=torch.bool)
    arr = (ctypes.c_uint32 * max(len(masks), 1))(*masks)
    check(lib().vit_router_select(_p(indices), T, len(masks), arr, nkeys, _p(active), _p(sel), _p(anyf), _stream()),
          "vit_router_select")
    return active, sel, anyf


def cast_rows_masked(inp, ldi, rows, cols, mask, out, ldo):
    """out rows (bf16) = inp rows (f32) where mask (bool [rows], or None = all) is set, zeros elsewhere
    (vit_cast_rows_masked)"""
    _chk(inp, F32, "inp")
    _chk(out, BF16, "out")
    if mask is not None and (mask.dtype != torch.bool or not mask.is_contiguous() or mask.numel() != rows):
        raise ValueError("cast_rows_masked: mask must be a contiguous bool tensor of `rows` elements")
    check(lib().vit_cast_rows_masked(_p(inp), ldi, rows, cols, _p(mask), _p(out), ldo, _stream()),
          "vit_cast_rows_masked")


def unpack_bf16_f32(inp, ldi, rows, cols, out, ldo):
    """out[r*ldo + c] = f32(inp[r*ldi + c])"""
    _chk(inp, BF16, "inp")
    _chk(out, F32, "out")
    check(lib().vit_unpack_bf16_f32(_p(inp), ldi, rows, cols, _p(out), ldo, _stream()), "vit_unpack_bf16_f32")


def attention_fwd_varlen(q, ldq, k, ldk, v, ldv, o, ldo, cu_q, B, max_q, Nkv, H, hd, scale):
    """ragged-query attention forward (vit_attention_fwd_varlen): bf16 q / k / v / o row views, cu_q
    int32 [B + 1] on the device."""
    for t, n in ((q, "q"), (k, "k"), (v, "v"), (o, "o")):
        _chk(t, BF16, n)
    _chk(cu_q, torch.int32, "cu_q")
    check(lib().vit_attention_fwd_varlen(_p(q), ldq, _p(k), ldk, _p(v), ldv, _p(o), ldo, _p(cu_q), B, max_q, Nkv, H,
                                         hd, scale, _stream()), "vit_attention_fwd_varlen")


# ---- Res-ViT optimizer step: clip_grad_norm_ + AdamW over a flat buffer (csrc/optim.hip) ----------
def sqnorm_partial(g, n, partial):
    _chk(g, F32, "g")
    _chk(partial, torch.float64, "partial")
    check(lib().vit_sqnorm_partial(_p(g), n, _p(partial), partial.numel(), _stream()), "vit_sqnorm_partial")


def adamw_prep(partial, used, steps, lr, beta1, beta2, max_norm, table, norm_out):
    nseg = 0 if steps is None else steps.numel()
    check(lib().vit_adamw_prep(_p(partial), 0 if partial is None else partial.numel(), _p(used), _p(steps), nseg,
                               lr, beta1, beta2, max_norm, _p(table), _p(norm_out), _stream()), "vit_adamw_prep")


def adamw_update(p, g, m, v, p_bf16, chunks, table, lr, beta1, beta2, eps, wd, write_grad):
    # (1 - lr*wd) and (1 - beta) in double, then rounded: torch's Python-scalar arithmetic
    check(lib().vit_adamw_update(_p(p), _p(g), _p(m), _p(v), _p(p_bf16), _p(chunks), chunks.numel() // 3, _p(table),
                                 1.0 - lr * wd, beta1, beta2, 1.0 - beta1, 1.0 - beta2, eps, int(write_grad),
                                 _stream()), "vit_adamw_update")


def adamw_chunk_elems():
    return lib().vit_adamw_chunk_elems()


def scale_by_coef(g, n, coef):
    check(lib().vit_scale_by_coef(_p(g), n, _p(coef), _stream()), "vit_scale_by_coef")


def zero_(t):
    """t[...] = 0 with hipMemsetAsync on the current stream (contiguous tensors)"""
    if not t.is_contiguous():
        raise ValueError("zero_: contiguous tensor expected")
    check(lib().vit_zero(_p(t), t.numel() * t.element_size(), _stream()), "vit_zero")


def splitk_factor_group(shapes, K, cus=256):
    """common split-K factor of weight-gradient GEMMs [(M, N, batch), ...] over the same K launched as one grid
    (vit_gemm_splitk_group, 256 x 256 tiles): splitk_factor's model over their summed tiles and slabs"""
    tiles = sum(-(-M // 256) * -(-N // 256) * b for M, N, b in shapes)
    smax = max(1, min((K // 64) // 8, 32))
    t_tile = 2.0 * 256 * 256 * K / 4.0e12
    slab = sum(2.0 * M * N * 4 * b for M, N, b in shapes) / 5.0e12
    best, best_t = 1, None
    for s in range(1, smax + 1):
        t = -(-tiles * s // cus) * t_tile / s + s * slab
        if best_t is None or t < best_t * (1 - 1e-9):
            best, best_t = s, t
    return best


def gemm_splitk_group(members):
    """Up to 4 split-K weight-gradient GEMMs in one launch (vit_gemm_splitk_group). members: [(A, B, C, M, N, K,
    kwargs)], each exactly a gemm(A, B, C, M, N, K, **kwargs) call with epilogue EPI_SPLITK and both operands
    M/N-contiguous; the grid is the concatenation of theirs."""
    if not 1 <= len(members) <= 4:
        raise ValueError("gemm_splitk_group: 1 to 4 members")
    arr = (GemmArgs * len(members))()
    for i, (A, B, C, M, N, K, kw) in enumerate(members):
        _chk(A, BF16, "A")
        _chk(B, BF16, "B")
        arr[i] = _gemm_args(A, B, C, M, N, K, **kw)
    check(lib().vit_gemm_splitk_group(arr, len(members), _stream()), "vit_gemm_splitk_group")


def splitk_factor(M, N, K, batch=1, cus=256):
    """split-K factor of a weight-gradient GEMM (K = tokens) on `cus` compute units: the split with the
    least modelled time, ceil(tiles*s / slots) waves of 1/s of a tile's k-range each plus the f32 slab
    traffic (write + fixed-order reduce) of s slabs; at least 8 k-tiles per split, at most 32. One
    256 x 256 workgroup per CU (128 x 128 below 256 rows or columns: two). ViT-B/16 keeps its one-wave
    splits (fc1 / fc2 7, qkv 9, out-proj 28); ViT-H/14 at bs 128 (fc1 / fc2: 100 tiles) takes 5 (500
    workgroups, 1.95 waves) instead of 3 (300 workgroups: a second wave 17% full)."""
    tile = 256 if M >= 256 and N >= 256 else 128
    slots = cus if tile == 256 else 2 * cus
    tiles = -(-M // tile) * -(-N // tile) * batch
    smax = max(1, min((K // 64) // 8, 32))
    t_tile = 2.0 * tile * tile * K / 4.0e12        # one tile's k-range on one CU at ~0.4 of the MFMA peak
    slab = 2.0 * M * N * 4 * batch / 5.0e12        # one f32 slab written and read back
    best, best_t = 1, None
    for s in range(1, smax + 1):
        t = -(-tiles * s // slots) * t_tile / s + s * slab
        if best_t is None or t < best_t * (1 - 1e-9):
            best, best_t = s, t
    return best


def wgrad(A, lda, B, ldb, M, N, K, out, ldo, accumulate=False, batch=1, a_bs=0, b_bs=0, out_bs=0, target=256):
    """Weight gradient out[z] ([M][N] f32, row stride ldo) (+)= sum_t A[t][m] B[t][n] over K token rows
    (both operands token-major, i.e. M/N-contiguous; K a multiple of 64, rows past the data zero):
    split-K over the tokens into f32 slabs (splitk_factor over `target` CUs), then the fixed-order
    vit_splitk_reduce (deterministic; accumulate adds into `out`)."""
    from ._lib import EPI_SPLITK, MN_CONTIG
    s = splitk_factor(M, N, K, batch, target)
    ws = torch.empty(batch * s * M * N, device=out.device, dtype=F32)
    gemm(A, B, ws, M, N, K, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=lda, ldb=ldb, ldc=N, epilogue=EPI_SPLITK,
         batch=batch, a_bs=a_bs, b_bs=b_bs, split_k=s)
    splitk_reduce(ws, batch, s, M, N, out, ldo, out_bs, accumulate)


def rows_select(dst, mask, src=None):
    """rows r of the 2-D tensor dst with mask[r] False <- src's row r (zeros when src is None); mask: bool [rows]"""
    if mask.dtype != torch.bool or not mask.is_contiguous() or mask.numel() != dst.shape[0]:
        raise ValueError("rows_select: mask must be a contiguous bool tensor of dst.shape[0] elements")
    rb = dst.shape[1] * dst.element_size()
    if src is not None and (src.dtype != dst.dtype or src.shape[1] != dst.shape[1]):
        raise ValueError("rows_select: src must match dst's dtype and row width")
    check(lib().vit_rows_select(_p(dst), dst.stride(0) * dst.element_size(), _p(src),
                                0 if src is None else src.stride(0) * src.element_size(), _p(mask), dst.shape[0], rb,
                                _stream()), "vit_rows_select")


def copy2d(dst, dpitch, src, spitch, width, height):
    """height rows of `width` bytes, dst + r*dpitch <- src + r*spitch (byte pitches; hipMemcpy2DAsync)"""
    check(lib().vit_copy2d(_p(dst), dpitch, _p(src), spitch, width, height, _stream()), "vit_copy2d")


def sgd_step_dev(p, g, buf, p_bf16, n, hyper, wd):
    """vit_sgd_step with {lr, momentum, first} read from the device tensor `hyper` (graph-capturable)"""
    _chk(hyper, F32, "hyper")
    check(lib().vit_sgd_step_dev(_p(p), _p(g), _p(buf), _p(p_bf16), n, _p(hyper), wd, _stream()), "vit_sgd_step_dev")
