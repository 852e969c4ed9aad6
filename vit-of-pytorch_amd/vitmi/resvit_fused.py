"""One Res-ViT transformer layer (`TransformerBlock._full`, res-vit/model.py:213-317,471-492) as a single
autograd node on the engine's fused kernels, for the LoRA configuration of BASELINE config C5
(res-vit/config.py defaults: every base weight and LayerNorm frozen, res-vit/model.py:573-584; only
the rank-r LoRA factors on q / k / v take gradients here).

    h   = x + wo(attn(q, k, v)),  [q|k|v] = LN1(x) [Wq|Wk|Wv]^T + b + (LN1(x) A_z^T) B_z^T
    out = h + fc2(GELU(fc1(LN2(h))))

Forward (T = B*N token rows; bf16 GEMM operands, f32 accumulation / residual stream / LN statistics):
  LN1 writes its bf16 output into columns [0, D) of a [T][D + 64] operand; the LoRA down-projections
  u_z = LN1(x) A_z^T land in the next 3*r8 columns (one GEMM, N = 3 r8); the q|k|v GEMM then runs over
  K = D + 64 against [W_qkv | blockdiag(B_q, B_k, B_v)] — the LoRA up-projection folded into the same
  MFMA pass without rounding B A into the frozen weight (|BA| << |W| would vanish in bf16) — with the
  bias epilogue writing bf16 q|k|v for the attention kernel; attention (LDS-resident / tiled); out-proj
  + bias + f32 residual; LN2 (bf16); fc1 with the bias + GELU + GELU' epilogue; fc2 + bias + residual.
Backward: fc2 data gradient times GELU' (one epilogue), fc1 data gradient, LN2 backward with the
residual gradient added, out-proj data gradient, attention backward, LoRA: v_z = dq_z B_z (batched
GEMM), dB_z = dq_z^T u_z and dA_z = v_z^T LN1(x) (split-K over tokens), the q|k|v data gradient
dqkv W_qkv + v A (two GEMMs into f32), LN1 backward with the residual gradient. Frozen weights take no
gradient; their bf16 operand copies (forward and transposed for the data gradients) are cached per
weight version on the block.

The generic per-op path (vitmi.functional) remains for every other configuration (no LoRA: all
weights trainable; grouped-query attention; shapes the kernels do not cover).
"""
from __future__ import annotations

import math
import os

import torch

from . import flat as _flat
from . import ops
from ._lib import (EPI_BF16, EPI_BIAS_BF16, EPI_BIAS_GELU_DGELU, EPI_BIAS_RESID_F32, EPI_F32, EPI_MUL_BF16,
                   EPI_PATCH, EPI_SPLITK, K_CONTIG, MN_CONTIG)

BF16, F32 = torch.bfloat16, torch.float32
KX = 64  # extra K columns of the q|k|v operand (LoRA down-projections, zero padded)


def _rup(x, m):
    return (x + m - 1) // m * m


_ZROW = {}


def _alloc_pad(rows_p, cols_p, rows, cols, dev, dtype=BF16):
    """[rows_p][cols_p] buffer whose part outside [rows][cols] is zero; the caller writes the inside (instead of
    torch.zeros: no full-buffer fill — at Res-ViT-B/16 bs 128, T = 25 216 is a multiple of 64 and most operands
    have no padding at all)"""
    out = torch.empty(rows_p, cols_p, device=dev, dtype=dtype)
    if ZERO_FULL:
        out.zero_()
        return out
    if rows_p > rows:
        ops.zero_(out[rows:])
    if cols_p > cols and rows:
        out[:rows, cols:].zero_()
    return out


def _zero_row(n, dev):
    z = _ZROW.get(dev)
    if z is None or z.numel() < n:
        z = torch.zeros(max(n, 4096), device=dev, dtype=F32)
        _ZROW[dev] = z
    return z


def supported(block):
    """the fused layer covers: LoRA on, every base weight / norm frozen, n_kv_heads == n_heads, head dim a
    multiple of 16 up to 96, D and mlp_dim multiples of 64, rank <= 21"""
    a = block.attention
    if not block.use_lora or a.n_rep != 1:
        return False
    D = block.dim
    hd = a.head_dim
    M = block.feed_forward.fc1.weight.shape[0]
    r = a.lora_q.rank
    frozen = [a.wq, a.wk, a.wv, a.wo, block.feed_forward.fc1, block.feed_forward.fc2]
    if any(p.requires_grad for m in frozen for p in m.parameters()):
        return False
    if any(p.requires_grad for n in (block.attention_norm, block.ffn_norm) for p in n.parameters()):
        return False
    return D % 64 == 0 and M % 64 == 0 and hd % 16 == 0 and hd <= 96 and 3 * _rup(r, 8) <= KX


# A/B switch (bench.py VITMI_RESVIT_ZERO_FULL=1): every padded operand cleared whole, as before _alloc_pad
ZERO_FULL = False
# A/B switch (bench.py VITMI_RESVIT_PACK_EACH=1): False packs the LoRA factors and clears the q|k|v operand on
# every call, as before round 4's shared pack
SHARE_PACK = True
# the fused layer's LoRA gradients accumulated straight into their flat .grad views (vitmi.flat.grad_sink); False:
# returned to autograd (AccumulateGrad adds)
LORA_SINK = os.environ.get("VITMI_RESVIT_LORA_SINK", "1") != "0"


class _Frozen:
    """bf16 operand copies of a block's frozen weights, rebuilt when a weight's storage or version changes; the
    LoRA operand pack (A_all, the B columns of the q|k|v operand) and a persistent [Tp][D + 64] LN1 | u operand
    whose padding (columns past D + 3 r8, rows past T) is cleared once"""

    def __init__(self):
        self.sig = None
        self.a_all = None
        self.a1 = None
        self.a1_rows = 0
        # bumped on every rewrite of the shared a_all / a1 buffers (raw-pointer kernels: torch's version counter
        # does not see them); a backward checks that its forward's buffers were not rewritten since
        self.gen = 0

    def pack_lora(self, aq, bq, ak, bk, av, bv):
        """A_all [64][D] (row z*r8 + i = A_z[i], other rows zero) and B_z into columns D + z*r8 of wcat"""
        r, D = aq.shape
        r8 = _rup(r, 8)
        Kq = D + KX
        if self.a_all is None or self.a_all.shape != (KX, D) or self.a_all.device != aq.device:
            self.a_all = torch.zeros(KX, D, device=aq.device, dtype=BF16)
        # A_z into rows z*r8.. of A_all, B_z into columns D + z*r8.. of wcat: one launch
        jobs = [(A.detach().float().contiguous(), r, D, D, self.a_all[z * r8:], D, r, D)
                for z, A in enumerate((aq, ak, av))]
        jobs += [(Bz.detach().float().contiguous(), D, r, r, self.wcat[z * D:, D + z * r8:], Kq, D, r)
                 for z, Bz in enumerate((bq, bk, bv))]
        ops.cast_pad_batch(jobs)
        self.gen += 1
        return self.a_all

    def operand(self, T, Tp, Kq, dev):
        if self.a1 is None or self.a1.shape != (Tp, Kq) or self.a1.device != dev:
            self.a1 = torch.empty(Tp, Kq, device=dev, dtype=BF16)
            ops.zero_(self.a1)
        elif T != self.a1_rows and Tp > T:
            ops.zero_(self.a1[T:])  # rows past T (read by the split-K LoRA gradients) back to zero
        self.a1_rows = T
        self.gen += 1
        return self.a1

    def get(self, block):
        a, ff = block.attention, block.feed_forward
        ws = (a.wq.weight, a.wk.weight, a.wv.weight, a.wq.bias, a.wk.bias, a.wv.bias, a.wo.weight, ff.fc1.weight,
              ff.fc2.weight)
        sig = tuple((w.data_ptr(), w._version) for w in ws)
        if sig == self.sig:
            return self
        D, M = block.dim, ff.fc1.weight.shape[0]
        dev = a.wq.weight.device
        Kq = D + KX
        self.a_all = None  # a new wcat holds no LoRA columns yet: the next call packs
        # q|k|v forward operand [3D][D + 64] (K-contiguous); the LoRA columns are rewritten per call
        self.wcat = torch.zeros(3 * D, Kq, device=dev, dtype=BF16)
        for z, w in enumerate((a.wq.weight, a.wk.weight, a.wv.weight)):
            ops.pack_cols(w.detach(), 0, D, D, D, 1, self.wcat[z * D:], Kq)
        self.bqkv = torch.cat([a.wq.bias.detach(), a.wk.bias.detach(), a.wv.bias.detach()]).float().contiguous()
        # data-gradient operands: W^T, K-contiguous over the output features
        self.wqkv_t = torch.empty(D, 3 * D, device=dev, dtype=BF16)
        for z, w in enumerate((a.wq.weight, a.wk.weight, a.wv.weight)):
            ops.transpose_bf16(w.detach(), D, D, D, self.wqkv_t[:, z * D:], 3 * D)
        self.wo = torch.empty(D, D, device=dev, dtype=BF16)
        ops.cast_bf16(a.wo.weight.detach(), self.wo, D * D)
        self.wo_t = torch.empty(D, D, device=dev, dtype=BF16)
        ops.transpose_bf16(a.wo.weight.detach(), D, D, D, self.wo_t, D)
        self.w1 = torch.empty(M, D, device=dev, dtype=BF16)
        ops.cast_bf16(ff.fc1.weight.detach(), self.w1, M * D)
        self.w1_t = torch.empty(D, M, device=dev, dtype=BF16)
        ops.transpose_bf16(ff.fc1.weight.detach(), M, D, D, self.w1_t, M)
        self.w2 = torch.empty(D, M, device=dev, dtype=BF16)
        ops.cast_bf16(ff.fc2.weight.detach(), self.w2, D * M)
        self.w2_t = torch.empty(M, D, device=dev, dtype=BF16)
        ops.transpose_bf16(ff.fc2.weight.detach(), D, M, M, self.w2_t, D)
        self.sig = sig
        return self


class _FusedLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, aq, bq, ak, bk, av, bv, block, packed, active):
        a, ff = block.attention, block.feed_forward
        fz = block._vitmi_frozen.get(block)
        B, N, D = x.shape
        H, hd = a.n_local_heads, a.head_dim
        M = ff.fc1.weight.shape[0]
        r = aq.shape[0]
        r8 = _rup(r, 8)
        T = B * N
        Tp = _rup(T, 64)
        Kq = D + KX
        dev = x.device
        x = x.contiguous().float()
        xf = x.view(T, D)
        eps1, eps2 = block.attention_norm.layer_norm.eps, block.ffn_norm.layer_norm.eps
        n1, n2 = block.attention_norm.layer_norm, block.ffn_norm.layer_norm
        # LoRA factors as bf16 operands: A_all [64][D] (row z*r8 + i = A_z[i]); B columns of the q|k|v operand.
        # `packed`: this step's pack is already in place (the teacher pass of the same block packed it)
        a_all = fz.a_all if packed and SHARE_PACK and fz.a_all is not None else fz.pack_lora(aq, bq, ak, bk, av, bv)
        if SHARE_PACK:
            # one operand per block: the teacher pass writes it first, the student pass (saved for the
            # backward) last; LN1 and the u GEMM rewrite the same region every call, the padding stays zero
            a1 = fz.operand(T, Tp, Kq, dev)
        else:
            a1 = torch.empty(Tp, Kq, device=dev, dtype=BF16)
            ops.zero_(a1)
        mu1, rs1 = torch.empty(T, device=dev), torch.empty(T, device=dev)
        ops.layernorm_fwd(xf, D, n1.weight, n1.bias, a1, Kq, mu1, rs1, T, D, eps1)
        # u_z = LN1(x) A_z^T -> columns D + z*r8 .. of the same operand
        ops.gemm(a1, a_all, a1[:, D:], T, 3 * r8, D, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=Kq, ldb=D, ldc=Kq,
                 epilogue=EPI_BF16)
        qkv = torch.empty(Tp, 3 * D, device=dev, dtype=BF16)
        ops.gemm(a1, fz.wcat, qkv, T, 3 * D, Kq, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=Kq, ldb=Kq, ldc=3 * D,
                 epilogue=EPI_BIAS_BF16, bias=fz.bqkv)
        o = torch.empty(Tp, D, device=dev, dtype=BF16)
        lse = torch.empty(B, H, N, device=dev)
        scale = 1.0 / math.sqrt(hd)
        ops.attention_fwd(qkv, o, lse, B, N, H, hd, scale)
        h = torch.empty(T, D, device=dev)
        ops.gemm(o, fz.wo, h, T, D, D, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=D, ldb=D, ldc=D,
                 epilogue=EPI_BIAS_RESID_F32, bias=a.wo.bias.detach(), aux=xf, ldaux=D)
        a2 = torch.empty(Tp, D, device=dev, dtype=BF16)
        mu2, rs2 = torch.empty(T, device=dev), torch.empty(T, device=dev)
        ops.layernorm_fwd(h, D, n2.weight, n2.bias, a2, D, mu2, rs2, T, D, eps2)
        gp = torch.empty(Tp, M, device=dev, dtype=BF16)
        g = torch.empty(Tp, M, device=dev, dtype=BF16)
        ops.gemm(a2, fz.w1, gp, T, M, D, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=D, ldb=D, ldc=M,
                 epilogue=EPI_BIAS_GELU_DGELU, bias=ff.fc1.bias.detach(), C2=g, ldc2=M)
        out = torch.empty(T, D, device=dev)
        ops.gemm(g, fz.w2, out, T, D, M, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=M, ldb=M, ldc=D,
                 epilogue=EPI_BIAS_RESID_F32, bias=ff.fc2.bias.detach(), aux=h, ldaux=D)
        am = None
        if active is not None:  # where(active, layer(x), x): the inactive rows of the output take x's rows
            am = active.reshape(T)
            ops.rows_select(out, am, xf)
        ctx.active = am
        if torch.is_grad_enabled() or any(ctx.needs_input_grad):
            ctx.save_for_backward(xf, a1, mu1, rs1, qkv, o, lse, h, mu2, rs2, gp, a_all, bq, bk, bv)
            ctx.block = block
            ctx.lora = (aq, bq, ak, bk, av, bv)
            ctx.dims = (B, N, D, H, hd, M, r, r8, T, Tp, scale)
            ctx.gen = fz.gen if SHARE_PACK else None
        return out.view(B, N, D)

    @staticmethod
    def backward(ctx, dout):
        xf, a1, mu1, rs1, qkv, o, lse, h, mu2, rs2, gp, a_all, bq, bk, bv = ctx.saved_tensors
        block = ctx.block
        fz = block._vitmi_frozen.get(block)
        if ctx.gen is not None and fz.gen != ctx.gen:
            # a1 (LN1 | u) and a_all are per-block buffers shared by the block's forwards (SHARE_PACK); another
            # forward of this block rewrote them after the one this backward belongs to, so the LoRA gradients
            # would silently use its activations
            raise RuntimeError("Res-ViT fused layer: this block ran another forward after the one being "
                               "back-propagated (micro-batch accumulation / retain_graph reuse); its shared LN1 | u "
                               "operand was overwritten. Run backward before the next forward of the block, or set "
                               "vitmi.resvit_fused.SHARE_PACK = False")
        B, N, D, H, hd, M, r, r8, T, Tp, scale = ctx.dims
        Kq = D + KX
        dev = xf.device
        n1, n2 = block.attention_norm.layer_norm, block.ffn_norm.layer_norm
        dout = dout.contiguous().float().view(T, D)
        dob = torch.empty(T, D, device=dev, dtype=BF16)
        am = ctx.active
        # the layer's output gradient is dout on the active rows only: one pass, the inactive rows not read
        ops.cast_rows_masked(dout, D, T, D, am, dob, D)
        # fc2 data gradient x GELU'(fc1 pre-activation)
        dg = torch.empty(T, M, device=dev, dtype=BF16)
        ops.gemm(dob, fz.w2_t, dg, T, M, D, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=D, ldb=D, ldc=M,
                 epilogue=EPI_MUL_BF16, aux=gp, ldaux=M)
        dy2 = torch.empty(T, D, device=dev, dtype=BF16)
        ops.gemm(dg, fz.w1_t, dy2, T, D, M, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=M, ldb=M, ldc=D,
                 epilogue=EPI_BF16)
        del dg
        part = torch.empty(ops.layernorm_bwd_partial_rows(T), 3 * D, device=dev)
        dh = torch.empty(T, D, device=dev)
        dhb = torch.empty(T, D, device=dev, dtype=BF16)
        # with a row selection the residual path carries all of dout: on an inactive row the layer's branches
        # get no gradient (dy2 = 0 there) and dh = dout is exactly the where's gradient to x, carried on to the
        # LN1 backward's residual input; the attention branch's operand keeps the layer's own (masked) dh
        ops.layernorm_bwd(dy2, D, h, D, mu2, rs2, n2.weight, dh, D, part, T, D, dres=dout, lddres=D, dx_bf16=dhb,
                          lddxb=D)
        if am is not None:
            ops.rows_select(dhb, am)
        dO = torch.empty(T, D, device=dev, dtype=BF16)
        ops.gemm(dhb, fz.wo_t, dO, T, D, D, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=D, ldb=D, ldc=D,
                 epilogue=EPI_BF16)
        dqkv = torch.empty(Tp, 3 * D, device=dev, dtype=BF16)
        if Tp > T:
            ops.zero_(dqkv[T:])
        ops.attention_bwd(qkv, o, dO, lse, dqkv, B, N, H, hd, scale)
        # LoRA: v_z = dq_z B_z (batched), dB_z = dq_z^T u_z, dA_z = v_z^T LN1(x)
        b_all = torch.empty(3, D, r8, device=dev, dtype=BF16)  # rows written whole (zero-padded to r8) below
        ops.cast_pad_batch([(Bz.detach().float().contiguous(), D, r, r, b_all[z], r8, D, r8)
                            for z, Bz in enumerate((bq, bk, bv))])
        v_all = torch.empty(Tp, KX, device=dev, dtype=BF16)
        ops.zero_(v_all)
        ops.gemm(dqkv, b_all, v_all, T, r, D, a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=3 * D, ldb=r8, ldc=KX,
                 epilogue=EPI_BF16, batch=3, a_bs=D, b_bs=D * r8, c_bs=r8)
        need = ctx.needs_input_grad
        # dB_z and dA_z (batched over z): one grouped split-K launch and one grouped reduction, each at the split
        # ops.wgrad would give it alone (bit-identical sums)
        dB = torch.empty(3, D, r, device=dev)
        dA = torch.empty(3, r, D, device=dev)
        sB, sA = ops.splitk_factor(D, r, Tp, 3), ops.splitk_factor(r, D, Tp, 3)
        wsB = torch.empty(3 * sB * D * r, device=dev)
        wsA = torch.empty(3 * sA * r * D, device=dev)
        kw = dict(a_layout=MN_CONTIG, b_layout=MN_CONTIG, epilogue=EPI_SPLITK, batch=3)
        ops.gemm_splitk_group([(dqkv, a1[:, D:], wsB, D, r, Tp, dict(kw, lda=3 * D, ldb=Kq, ldc=r, a_bs=D, b_bs=r8,
                                                                      split_k=sB)),
                               (v_all, a1, wsA, r, D, Tp, dict(kw, lda=KX, ldb=Kq, ldc=D, a_bs=r8, split_k=sA))])
        # each factor's gradient straight into its flat .grad view where it has one (no AccumulateGrad add), else
        # into dA / dB
        marks, jobs, grads = [], [], []
        for z in range(3):
            for ws_, s_, M_, N_, full, p_, nd in ((wsA, sA, r, D, dA, ctx.lora[2 * z], need[1 + 2 * z]),
                                                   (wsB, sB, D, r, dB, ctx.lora[2 * z + 1], need[2 + 2 * z])):
                slab = ws_[z * s_ * M_ * N_:(z + 1) * s_ * M_ * N_]
                sk = _flat.grad_sink(p_, nd) if LORA_SINK else None
                if sk is not None:
                    jobs.append((slab, 1, s_, M_, N_, sk, N_, 0, True))
                    marks.append(p_)
                    grads.append(None)
                else:
                    jobs.append((slab, 1, s_, M_, N_, full[z], N_, 0, False))
                    grads.append(full[z] if nd else None)
        ops.splitk_reduce_group(jobs)
        # q|k|v data gradient: dqkv W_qkv + v A (f32), then LN1 backward with the residual gradient
        dy1 = torch.empty(T, D, device=dev)
        ops.gemm(v_all, a_all, dy1, T, D, KX, a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=KX, ldb=D, ldc=D,
                 epilogue=EPI_F32)
        ops.gemm(dqkv, fz.wqkv_t, dy1, T, D, 3 * D, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=3 * D, ldb=3 * D,
                 ldc=D, epilogue=EPI_BIAS_RESID_F32, bias=_zero_row(D, dev), aux=dy1, ldaux=D)
        dx = None
        if need[0]:
            dx = torch.empty(T, D, device=dev)
            ops.layernorm_bwd(dy1, D, xf, D, mu1, rs1, n1.weight, dx, D, part, T, D, dres=dh, lddres=D)
            dx = dx.view(B, N, D)
        _sunk(marks)
        return (dx, *grads, None, None, None)


def full_layer(block, x, packed=False, active=None):
    """TransformerBlock._full(x) (res-vit/model.py:471-492: attention + residual, FFN + residual) as one
    fused node; x [B, N, D] f32 -> [B, N, D] f32. packed: a call on the same block earlier in this forward
    (the teacher pass) packed the LoRA operands from the same weights. active (bool [B, N, 1]): the routed
    student's where(active, layer(x), x) (res-vit/model.py:507-512) folded into the node"""
    if not hasattr(block, "_vitmi_frozen"):
        block._vitmi_frozen = _Frozen()
    a = block.attention
    return _FusedLayer.apply(x, a.lora_q.lora_A.weight, a.lora_q.lora_B.weight, a.lora_k.lora_A.weight,
                             a.lora_k.lora_B.weight, a.lora_v.lora_A.weight, a.lora_v.lora_B.weight, block,
                             bool(packed and block._vitmi_frozen.a_all is not None),
                             None if active is None else active.contiguous())


class _RowsSelect(torch.autograd.Function):
    """where(active, full, x) for [B, N, D] f32 rows (active: bool [B, N, 1]) on vit_rows_select: forward a copy of
    full with x's rows where inactive, backward dout's active rows to full and its inactive rows to x"""

    @staticmethod
    def forward(ctx, full, x, active):
        B, N, D = full.shape
        m = active.reshape(B * N).contiguous()
        out = full.contiguous().clone()
        ops.rows_select(out.view(B * N, D), m, x.contiguous().view(B * N, D))
        ctx.save_for_backward(m)
        return out

    @staticmethod
    def backward(ctx, dout):
        (m,) = ctx.saved_tensors
        B, N, D = dout.shape
        d = dout.contiguous()
        dfull = d.clone()
        ops.rows_select(dfull.view(B * N, D), m)  # inactive rows: 0
        dx = d.clone()
        ops.rows_select(dx.view(B * N, D), torch.logical_not(m))  # active rows: 0
        return dfull, dx, None


class _ClsTap(torch.autograd.Function):
    """(x, x[:, 0, :]) with the cls rows' gradient added into x's incoming gradient: autograd's own slice backward
    materialises a zero [B, N, D] tensor, copies the rows in and adds it to the layer gradient (three passes over
    T x D f32 per routed layer, for the distillation loss on the cls token). With inplace=True the incoming gradient
    of the x output is updated in place, which is only safe when x's consumers hand no other input that same tensor:
    the caller (ResViT.forward) sets it only when x feeds the fused layer node (and the fused router), whose
    backwards return fresh gradients, or the final norm's slice; otherwise the gradient is copied first (an
    AddBackward-style consumer, as the per-op layer's residual add, gives both its inputs one gradient object)."""

    @staticmethod
    def forward(ctx, x, inplace=False):
        ctx.shape = x.shape
        ctx.inplace = bool(inplace)
        return x.view(x.shape), x[:, 0, :].clone()

    @staticmethod
    def backward(ctx, dx, dcls):
        if dx is None:
            dx = torch.zeros(ctx.shape, device=dcls.device, dtype=dcls.dtype)
        elif dcls is not None and not ctx.inplace:
            dx = dx.clone()
        if dcls is not None:
            dx = dx.contiguous()
            dx[:, 0, :] += dcls
        return dx, None


def cls_tap(x, inplace=False):
    """x, and its cls rows x[:, 0, :] for a loss, without the full-size zero gradient of a slice (_ClsTap)"""
    return _ClsTap.apply(x, inplace)


class _EmbedTokens(torch.autograd.Function):
    """patch embedding, cls token and position embeddings (res-vit/model.py:629-633: conv, cat(cls, ...), + pos) as
    one GEMM: the images' im2col in bf16 (the cls rows left zero) times the conv weight with the PATCH epilogue, which
    writes every token row in f32 — cls + pos[0] on the cls rows, conv + bias + pos[t] on the others — the engine's
    embedding (src/model.py:197-204). For the LoRA configuration (frozen conv weight / bias and position embeddings):
    the backward gives only the cls token its gradient, the column sum of the cls rows' gradient over the batch.
    Replaces the f32 im2col, the patch-row copy, the operand cast, the concatenation and the position add."""

    @staticmethod
    def forward(ctx, x, w, bias, cls, pos, patch):
        B, _, hh, _ = x.shape
        g = hh // patch
        N = g * g + 1
        K = 3 * patch * patch
        kpad = _rup(K, 64)
        D = w.shape[0]
        T = B * N
        dev = x.device
        cols = torch.empty(T, kpad, device=dev, dtype=BF16)
        ops.im2col(x.detach().float().contiguous(), cols, B, hh, patch, kpad)
        (wb,) = _pad_bf16_many([(w.detach().float().reshape(D, K).contiguous(), D, kpad)])
        out = torch.empty(B, N, D, device=dev, dtype=F32)
        ops.gemm(cols, wb, out, T, D, kpad, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=kpad, ldb=kpad, ldc=D,
                 epilogue=EPI_PATCH, bias=bias.detach().float().contiguous(),
                 aux=pos.detach().float().contiguous().view(N, D), ldaux=D,
                 aux2=cls.detach().float().contiguous().view(D), tokens=N)
        ctx.dims = (B, N, D)
        ctx.cls_shape = cls.shape
        return out

    @staticmethod
    def backward(ctx, dout):
        B, N, D = ctx.dims
        dcls = None
        if ctx.needs_input_grad[3]:
            dcls = torch.empty(D, device=dout.device, dtype=F32)
            d = dout.contiguous().float()
            ops.segment_colsum(d, N * D, 1, B, D, dcls.view(1, D), D)  # sum over the images of row 0
            dcls = dcls.view(ctx.cls_shape)
        return None, None, None, dcls, None, None


def embed_supported(model, x):
    """the LoRA configuration's embedding: conv weight / bias and position embeddings frozen, square images of a
    whole number of patches, as many tokens as position embeddings"""
    e, pe = model.embedding, model.pos_embedding.pos_embedding
    if not (x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and x.shape[2] == x.shape[3] and e.bias is not None):
        return False
    if e.weight.requires_grad or e.bias.requires_grad or pe.requires_grad or x.requires_grad:
        return False
    g = x.shape[2] // model.patch
    return x.shape[2] % model.patch == 0 and pe.shape[1] == g * g + 1 and pe.shape[2] == e.weight.shape[0]


def embed_tokens(model, x):
    """[B, N, D] f32 token rows (cls + patches, position embeddings added) as one node (_EmbedTokens)"""
    return _EmbedTokens.apply(x, model.embedding.weight, model.embedding.bias, model.cls_token,
                              model.pos_embedding.pos_embedding, int(model.patch))


class _ClsDistill(torch.autograd.Function):
    """(x, mse_loss(x[:, 0, :], t[:, 0, :])) for the distillation loss after a routed layer (res-vit/model.py:40-59,
    t the detached teacher output): forward one row-sum launch plus a fixed-order total (vit_cls_mse, which keeps
    e = x_cls - t_cls), backward ((2 / (B D)) e) g added in place into x's incoming gradient's cls rows
    (vit_cls_mse_bwd). Replaces the cls-row copy, the MSE forward (difference, square, mean) and its backward, and
    the slice gradient's add. With inplace=True the incoming gradient of the x output is updated in place, else a
    copy of it (the ownership rule of _ClsTap)"""

    @staticmethod
    def forward(ctx, x, t, inplace=False):
        ctx.set_materialize_grads(False)
        ctx.inplace = bool(inplace)
        B, N, D = x.shape
        xc, tc = x.detach().contiguous(), t.detach().contiguous()
        loss, e = ops.cls_mse(xc, N * D, tc, tc.shape[1] * tc.shape[2], B, D)
        ctx.save_for_backward(e)
        ctx.shape = x.shape
        return x.view(x.shape), loss

    @staticmethod
    def backward(ctx, dx, dloss):
        (e,) = ctx.saved_tensors
        B, N, D = ctx.shape
        if dloss is None:
            return dx, None, None
        if dx is None:
            dx = torch.zeros(ctx.shape, device=e.device, dtype=F32)
        elif not ctx.inplace:
            dx = dx.clone()
        dx = dx.contiguous()
        ops.cls_mse_bwd(dx, N * D, e, dloss.detach().float().contiguous())
        return dx, None, None


def cls_distill(x, t, inplace=False):
    """x and mse_loss(x[:, 0, :], t[:, 0, :].detach()) as one node (_ClsDistill)"""
    return _ClsDistill.apply(x, t, inplace)


class _RouterHead(torch.autograd.Function):
    """RouterModule.forward after out_conv (res-vit/model.py:191-211) as one node: softmax, the entropy, the Gumbel
    hard decision with its straight-through value, the reserved tokens' rows and the pattern index in one launch (plus
    the entropy's fixed-order sum), one launch backward (vit_router_head_fwd / _bwd). The ~25 ATen launches it replaces
    per routed layer (softmax, log, mul, sum, neg, div, log, neg, add, softmax, max, zeros, scatter, sub, add, clone,
    two fills, a cast and the index matmul) each move a few hundred KB. Same arithmetic per element as those ops (soft,
    y_soft, hard and the index bit-identical); the entropy is summed in a different order."""

    @staticmethod
    def forward(ctx, logits, noise, noise_mode, yhard, reserve, training, norm):
        ctx.set_materialize_grads(False)
        B, N, bs, _ = logits.shape
        l2 = logits.detach().contiguous().view(B * N, bs, 2)
        nz = noise.detach().float().contiguous().view(B * N, bs, 2) if noise is not None else None
        yh = yhard.detach().float().contiguous().view(B * N, bs, 2) if yhard is not None else None
        soft, ysoft, hard, idx, ent = ops.router_head_fwd(l2, nz, noise_mode, yh, N, reserve, training, norm)
        ctx.save_for_backward(soft, ysoft)
        ctx.dims = (B, N, bs, reserve, bool(training), float(norm))
        if not training:
            ctx.mark_non_differentiable(hard, idx)
        return hard.view(B, N, bs, 2), idx.view(B, N, 1), ent, soft.view(B, N, bs, 2)

    @staticmethod
    def backward(ctx, dhard, didx, dent, dsoft):
        soft, ysoft = ctx.saved_tensors
        B, N, bs, reserve, training, norm = ctx.dims
        f = lambda t, *shape: t.float().contiguous().reshape(shape) if t is not None else None
        dl = ops.router_head_bwd(soft, ysoft, f(dsoft, B * N, bs, 2), f(dhard, B * N, bs, 2), f(didx, B * N),
                                 f(dent), N, reserve, training, norm)
        return dl.view(B, N, bs, 2), None, None, None, None, None, None


def router_head_supported(logits, reserve):
    B, N, bs, two = logits.shape
    return logits.is_cuda and logits.dtype == F32 and two == 2 and 1 <= bs <= 8 and B * (N - reserve) * bs > 0


def router_head(logits, noise, noise_mode, yhard, reserve, training, norm):
    """(hard, indices, entropy, soft) of RouterModule.forward from its logits [B, N, bs, 2] as one node (_RouterHead);
    noise_mode 1: noise is the Gumbel noise, 2: exponential draws (g = -log), 0: none (evaluation)"""
    return _RouterHead.apply(logits, noise, int(noise_mode), yhard, int(reserve), bool(training), float(norm))


def teacher_and_student(block, x, active):
    """The first routed layer, whose teacher input is the student's (res-vit/model.py:496-512 with teacher_x = x):
    the full layer runs once with autograd, the teacher output is its detached value and the student output
    where(active, it, x) — the same values as a no-grad teacher pass plus a folded student pass, one layer forward
    fewer"""
    full = full_layer(block, x)
    return full.detach(), _RowsSelect.apply(full, x, active)


# ---- routed low-rank approximator step (res-vit/model.py:319-368) ------------------------------------
class _ApproxStep(torch.autograd.Function):
    """x_new = where(sel, x + up(down(x)), x) for one approximator of BlockPathApproximators (training path),
    as one node: x [T][D] f32, down_proj.weight Wd [r][D], up_proj.weight Wu [D][r] (nn.Linear layouts), sel
    [T] bool. Forward: h = bf16(x) Wd^T written as bf16 by the GEMM epilogue, its unselected rows zeroed
    (vit_rows_select), then x + h Wu^T by the bias + f32-residual epilogue — an unselected row gets x + 0 = x,
    so neither the per-op path's f32 add nor its `where` pass remains. Backward: dh = (dout Wu) masked to the selected rows, dx =
    dout + dh Wd (residual epilogue), dWu = dout^T h, dWd = dh^T bf16(x) (split-K over tokens). Same
    operands and roundings as the per-op path (vitmi.functional.HipLinear + add + where), so the results
    agree bit for bit (tests/test_resvit_train_gpu.py)."""

    @staticmethod
    def forward(ctx, x, wd, wu, sel):
        B, N, D = x.shape
        T = B * N
        r = wd.shape[0]
        kp, rp, rk = _rup(D, 64), _rup(max(T, 1), 64), _rup(r, 64)
        dev = x.device
        x2 = x.contiguous().float().view(T, D)
        # x, and Wd [r][D] and Wu [D][r], as bf16 with rows and columns padded to 64 with zeros, in one launch: the
        # forward's operands (Wd, Wu K-contiguous B) and, unchanged, the backward's M/N-contiguous ones
        xb, wdb, wub = _pad_bf16_many([(x2, rp, kp), (wd.detach().float().contiguous(), rk, kp),
                                       (wu.detach().float().contiguous(), kp, rk)])
        hb = _alloc_pad(rp, rk, T, r, dev)
        ops.gemm(xb, wdb, hb, T, r, kp, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=kp, ldb=kp, ldc=rk,
                 epilogue=EPI_BF16)
        selm = sel.reshape(T).to(torch.bool).contiguous()
        ops.rows_select(hb[:T], selm)  # unselected rows: h = 0 (only their bytes written)
        out = torch.empty(T, D, device=dev, dtype=F32)
        ops.gemm(hb, wub, out, T, D, rk, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=rk, ldb=rk, ldc=D,
                 epilogue=EPI_BIAS_RESID_F32, bias=_zero_row(D, dev), aux=x2, ldaux=D)
        ctx.save_for_backward(xb, hb, wdb, wub, selm)
        ctx.params = (wd, wu)
        ctx.dims = (B, N, D, T, r)
        return out.view(B, N, D)

    @staticmethod
    def backward(ctx, dout):
        xb, hb, wdb, wub, selm = ctx.saved_tensors
        B, N, D, T, r = ctx.dims
        kp, rp, rk = xb.shape[1], xb.shape[0], hb.shape[1]
        dev = dout.device
        d2 = dout.contiguous().float().view(T, D)
        (db,) = _pad_bf16_many([(d2, rp, kp)])
        # dh = dout Wu: B(kk = n, n' = j) = Wu[n][j], M/N-contiguous (the forward's padded [kp][rk] copy), rounded to
        # the bf16 operand by the GEMM's epilogue (the same RNE rounding as a cast of the f32 product)
        dhb = _alloc_pad(rp, rk, T, r, dev)
        ops.gemm(db, wub, dhb, T, r, kp, a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=kp, ldb=rk, ldc=rk,
                 epilogue=EPI_BF16)
        ops.rows_select(dhb[:T], selm)
        dx = None
        if ctx.needs_input_grad[0]:
            # dx = dout + dh Wd: B(kk = j, n' = k) = Wd[j][k], M/N-contiguous (the forward's padded [rk][kp] copy)
            dx = torch.empty(T, D, device=dev, dtype=F32)
            ops.gemm(dhb, wdb, dx, T, D, rk, a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=rk, ldb=kp, ldc=D,
                     epilogue=EPI_BIAS_RESID_F32, bias=_zero_row(D, dev), aux=d2, ldaux=D)
            dx = dx.view(B, N, D)
        # dWd [r][D] = dh^T x and dWu [D][r] = dout^T h: one grouped split-K launch (each alone is 3 tiles, under a
        # wave at any split)
        marks, need = [], (ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        wg = [m for m, nd in zip(((dhb, rk, xb, kp, r, D, 0), (db, kp, hb, rk, D, r, 1)), need) if nd]
        g = _finish_grads(rp, wg, [], ctx.params, (True, True), marks, dev, own_split=True)
        _sunk(marks)
        return dx, g.get(0), g.get(1), None


def approx_supported(m, x):
    """the fused approximator step covers the LowRankApproximator as built (no bias, f32 weights, CUDA)"""
    d, u = m.down_proj, m.up_proj
    return (x.is_cuda and x.dim() == 3 and d.bias is None and u.bias is None and d.weight.dtype == F32
            and u.weight.dtype == F32 and d.weight.shape[1] == x.shape[2] and u.weight.shape[0] == x.shape[2])


def approx_step(m, x, sel):
    """where(sel, x + m(x), x) (res-vit/model.py:349-368, training) as one fused node"""
    return _ApproxStep.apply(x, m.down_proj.weight, m.up_proj.weight, sel)


# ---- router MLP (RouterModule.out_conv, res-vit/model.py:150-156,190) ----------------------------------
def _pad_bf16_many(items):
    """[_pad_bf16(x2, rows_p, cols_p) for each item] in one launch (vit_cast_pad_batch per 8)"""
    outs, jobs = [], []
    for x2, rows_p, cols_p in items:
        rows, cols = x2.shape
        out = torch.empty(rows_p, cols_p, device=x2.device, dtype=BF16)
        outs.append(out)
        jobs.append((x2, rows, cols, x2.stride(0), out, cols_p, rows_p, cols_p))
    ops.cast_pad_batch(jobs)
    return outs


def _pad_bf16(x2, rows_p, cols_p):
    rows, cols = x2.shape
    out = torch.empty(rows_p, cols_p, device=x2.device, dtype=BF16)
    if rows:
        ops.cast_pad_rows(x2, rows, cols, out, cols_p)
    if rows_p > rows:
        ops.zero_(out[rows:])
    return out


def _colsum(x, rows, cols, ld, p=None, need=True, marks=None):
    """column sums of x (a bias gradient); with p: accumulated in place into p's flat .grad view when it has
    one (vitmi.flat.grad_sink: p appended to marks, None returned)"""
    part = torch.empty(ops.colsum_partial_rows(max(rows, 1)), cols, device=x.device, dtype=F32)
    sk = _flat.grad_sink(p, need) if p is not None else None
    if sk is not None:
        ops.colsum(x, rows, cols, ld, part, sk, accumulate=True)
        marks.append(p)
        return None
    out = torch.empty(cols, device=x.device, dtype=F32)
    ops.colsum(x, rows, cols, ld, part, out)
    return out


def _wgrad(A, lda, B, ldb, M, N, K, p=None, need=True, marks=None):
    """weight gradient [M][N] = A^T B (ops.wgrad), accumulated into p's flat .grad view in place when it has one
    (as _colsum); else a new f32 tensor. With the view, no AccumulateGrad add runs for p."""
    sk = _flat.grad_sink(p, need) if p is not None else None
    if sk is not None:
        ops.wgrad(A, lda, B, ldb, M, N, K, sk, N, accumulate=True)
        marks.append(p)
        return None
    out = torch.empty(M, N, device=A.device, dtype=F32)
    ops.wgrad(A, lda, B, ldb, M, N, K, out, N)
    return out


def _sunk(marks):
    for p in marks:
        _flat.sunk(p)


def _weight_pads(w1, w2, w3, kp, h1p, h2p):
    """bf16 [rows rounded to 64][cols] copies of the out_conv weights (zero padding): the forward GEMMs' K-contiguous
    B operands and, unchanged, the backward's M/N-contiguous B operands of the data gradients (K = the padded output
    rows)"""
    H1, H2, O = w1.shape[0], w2.shape[0], w3.shape[0]
    return _pad_bf16_many([(w.detach().float().contiguous(), _rup(n, 64), k)
                           for w, n, k in ((w1, H1, kp), (w2, H2, h1p), (w3, O, h2p))])


def _mlp_forward(xb, T, kp, w1, b1, w2, b2, w3, b3, ws=None):
    """the router's out_conv on a bf16 operand xb [rp][kp] (T valid rows): hidden layers as one GEMM each whose
    epilogue writes GELU(u) (the next operand) and GELU'(u) (kept for the backward); returns (logits f32 [T][O],
    saved activations, padded bf16 weights)"""
    rp, dev = xb.shape[0], xb.device
    H1, H2, O = w1.shape[0], w2.shape[0], w3.shape[0]
    h1p, h2p = _rup(H1, 64), _rup(H2, 64)
    if ws is None:
        ws = _weight_pads(w1, w2, w3, kp, h1p, h2p)
    acts = []
    a_in, k_in = xb, kp
    for (b, n, npad), wb in zip(((b1, H1, h1p), (b2, H2, h2p)), ws[:2]):
        g = _alloc_pad(rp, npad, T, n, dev)
        gp = _alloc_pad(rp, npad, T, n, dev)
        if T:
            ops.gemm(a_in, wb, gp, T, n, k_in, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=k_in, ldb=k_in, ldc=npad,
                     epilogue=EPI_BIAS_GELU_DGELU, bias=b.detach().float().contiguous(), C2=g, ldc2=npad)
        acts += [g, gp]
        a_in, k_in = g, npad
    out = torch.empty(T, O, device=dev, dtype=F32)
    if T:
        ops.gemm(a_in, ws[2], out, T, O, k_in, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=k_in, ldb=k_in, ldc=O,
                 epilogue=EPI_BIAS_RESID_F32, bias=b3.detach().float().contiguous(), aux=_zero_row(O, dev), ldaux=0)
    return out, acts, ws


def _dgrad_mul(dyb, wpad, ldw, n_in, T, gp, npad_out):
    """dU = (dY W) * GELU'(u) for W [n_out][n_in] given as its padded bf16 copy wpad ([>= dY width rows][ldw]: B(kk = j,
    n' = k) = W[j][k], M/N-contiguous); bf16 out [rp][npad_out] and its per-tile column partials (the bias gradient:
    (partials f32 [rows][n_in], rows))"""
    rp, dev = dyb.shape[0], dyb.device
    du = _alloc_pad(rp, npad_out, T, n_in, dev)
    kw = dict(a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=dyb.shape[1], ldb=ldw, ldc=npad_out, epilogue=EPI_MUL_BF16,
              aux=gp, ldaux=npad_out)
    rows = ops.gemm_partial_rows(dyb, wpad, du, T, n_in, dyb.shape[1], **kw) if T else 0
    part = torch.empty(max(rows, 1), n_in, device=dev, dtype=F32)
    if T:
        ops.gemm(dyb, wpad, du, T, n_in, dyb.shape[1], col_partial=part, **kw)
    return du, (part, rows)


def _dgrad_f32(dyb, wpad, ldw, n_in, T):
    """dX = dY W (f32 [T][n_in]) for W [n_out][n_in] given as its padded bf16 copy (as _dgrad_mul)"""
    dx = torch.empty(T, n_in, device=dyb.device, dtype=F32)
    if T:
        ops.gemm(dyb, wpad, dx, T, n_in, dyb.shape[1], a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=dyb.shape[1], ldb=ldw,
                 ldc=n_in, epilogue=EPI_F32)
    return dx


def _finish_grads(K, wgrads, biases, params, need, marks, dev, own_split=False):
    """The weight and bias gradients of a router backward, all at once: wgrads [(A, lda, B, ldb, M, N, i)] are
    [M][N] = A^T B over the same K (padded token) rows, as ONE split-K launch (ops.gemm_splitk_group) at a common
    split (own_split: each member at the split ops.wgrad would give it alone, so its sums are bit-identical to
    ops.wgrad's) and each member's fixed-order reduction; biases [(partials f32 [rows][cols], rows, cols, i)] are
    column sums of GEMM / gate partials, ONE vit_colsum_batch launch. i indexes params / need; a gradient goes to
    the parameter's flat .grad view in place when it has one (vitmi.flat.grad_sink: parameter appended to marks,
    None returned), else to a new f32 tensor. Returns {i: gradient or None}."""
    out = {}

    def dst(i, shape):
        p = params[i]
        sk = _flat.grad_sink(p, need[i]) if p is not None else None
        if sk is not None:
            marks.append(p)
            out[i] = None
            return sk, True
        t = torch.empty(*shape, device=dev, dtype=F32)
        out[i] = t
        return t, False

    if wgrads:
        if own_split:
            ss = [ops.splitk_factor(M, N, K) for (_, _, _, _, M, N, _) in wgrads]
        else:
            ss = [ops.splitk_factor_group([(M, N, 1) for (_, _, _, _, M, N, _) in wgrads], K)] * len(wgrads)
        ws = torch.empty(sum(s * M * N for s, (_, _, _, _, M, N, _) in zip(ss, wgrads)), device=dev, dtype=F32)
        members, views, o = [], [], 0
        for s, (A, lda, B, ldb, M, N, _) in zip(ss, wgrads):
            w = ws[o:o + s * M * N]
            o += s * M * N
            views.append(w)
            members.append((A, B, w, M, N, K, dict(a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=lda, ldb=ldb, ldc=N,
                                                    epilogue=EPI_SPLITK, split_k=s)))
        ops.gemm_splitk_group(members)
        jobs = []
        for s, (_, _, _, _, M, N, i), w in zip(ss, wgrads, views):
            d, acc = dst(i, (M, N))
            jobs.append((w, 1, s, M, N, d, N, 0, acc))
        ops.splitk_reduce_group(jobs)
    jobs = []
    for part, rows, cols, i in biases:
        d, acc = dst(i, (cols,))
        if rows:
            jobs.append((part, rows, cols, cols, 0, (d,), acc))
        elif not acc:
            d.zero_()
    for k in range(0, len(jobs), ops.COLSUM_BATCH_MAX):
        ops.colsum_batch(jobs[k:k + ops.COLSUM_BATCH_MAX])
    return out


def _mlp_backward(d2, T, xb, acts, ws, w1, w2, w3, need_dx, params, need, marks):
    """data gradients of _mlp_forward and the work list of its parameter gradients: returns (dX f32 [T][K1] or None,
    dU1 bf16 (the first layer's input-side gradient), wgrads, biases) in _finish_grads' form, indices 0..5 = (W1, b1,
    W2, b2, W3, b3); b3's gradient (column sums of the f32 dY) is taken here, through params / need / marks"""
    g1, gp1, g2, gp2 = acts
    rp, kp, h1p, h2p = xb.shape[0], xb.shape[1], g1.shape[1], g2.shape[1]
    H1, H2, O, K1 = w1.shape[0], w2.shape[0], w3.shape[0], w1.shape[1]
    (dlb,) = _pad_bf16_many([(d2, rp, _rup(O, 64))])
    du2, (p2, r2) = _dgrad_mul(dlb, ws[2], h2p, H2, T, gp2, h2p)
    du1, (p1, r1) = _dgrad_mul(du2, ws[1], h1p, H1, T, gp1, h1p)
    dx = _dgrad_f32(du1, ws[0], kp, K1, T) if need_dx else None
    wgrads = [(dlb, dlb.shape[1], g2, h2p, O, H2, 4), (du2, h2p, g1, h1p, H2, H1, 2), (du1, h1p, xb, kp, H1, K1, 0)]
    biases = [(p2, r2, H2, 3), (p1, r1, H1, 1)]
    if O % 2 == 0:
        # the output bias gradient (column sums of the f32 dY [T][O], O = 2): 64-row segment sums, summed with the
        # other bias partials in _finish_grads' one column-sum launch (the generic narrow-column reduction took
        # two launches and ~30 us at T = 25 216)
        nseg, tail = T // 64, T % 64
        p3 = torch.empty(nseg + (1 if tail else 0) or 1, O, device=d2.device, dtype=F32)
        if nseg:
            ops.segment_colsum(d2, O, nseg, 64, O, p3, O)
        if tail:
            ops.segment_colsum(d2[nseg * 64:], O, 1, tail, O, p3[nseg:], O)
        biases.append((p3, nseg + (1 if tail else 0), O, 5))
        db3 = None  # (in _finish_grads' result, index 5)
    else:
        db3 = _colsum(d2, T, O, O, params[5], need[5], marks)
    return dx, du1, wgrads, biases, db3


class _RouterMLP(torch.autograd.Function):
    """Linear -> GELU -> Linear -> GELU -> Linear (the router's out_conv) as one node: each hidden layer is one
    GEMM whose epilogue writes GELU(u) (the next GEMM's bf16 operand) and GELU'(u) (kept for the backward),
    the way the ViT engine runs fc1; the backward's data gradients multiply GELU' in their epilogue
    (EPI_MUL_BF16) and sum the hidden-bias gradients in it (column partials), and the three weight gradients run
    as one grouped split-K launch. Replaces, per hidden layer, the f32 GEMM output, the f32 GELU pass and the cast
    to the next operand (forward) and the f32 GELU backward and its cast (backward). Rounding differs from the
    per-op path only in GELU' being bf16 (as in the engine's MLP)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3):
        lead = x.shape[:-1]
        K1 = x.shape[-1]
        x2 = x.contiguous().float().reshape(-1, K1)
        T = x2.shape[0]
        xb = _pad_bf16(x2, _rup(max(T, 1), 64), _rup(K1, 64))
        out, acts, ws = _mlp_forward(xb, T, xb.shape[1], w1, b1, w2, b2, w3, b3)
        ctx.save_for_backward(xb, *acts, *ws, w1, w2, w3)
        ctx.params = (w1, b1, w2, b2, w3, b3)
        ctx.dims = (lead, T, K1)
        return out.reshape(*lead, w3.shape[0])

    @staticmethod
    def backward(ctx, dout):
        xb, g1, gp1, g2, gp2, wp1, wp2, wp3, w1, w2, w3 = ctx.saved_tensors
        lead, T, K1 = ctx.dims
        d2 = dout.contiguous().float().reshape(T, w3.shape[0])
        marks, need = [], ctx.needs_input_grad[1:7]
        dx, _, wgrads, biases, db3 = _mlp_backward(d2, T, xb, (g1, gp1, g2, gp2), (wp1, wp2, wp3), w1, w2, w3,
                                                   ctx.needs_input_grad[0], ctx.params, need, marks)
        g = _finish_grads(xb.shape[0], wgrads, biases, ctx.params, need, marks, d2.device)
        _sunk(marks)
        return (dx.reshape(*lead, K1) if dx is not None else None, g[0], g[1], g[2], g[3], g[4],
                g[5] if db3 is None else db3)


class _RouterNet(torch.autograd.Function):
    """the whole router network up to its logits (res-vit/model.py:186-190): x_embed = GELU(Linear(LN(x))),
    global = mean of x_embed over the non-reserved tokens, logits = out_conv(cat(x_embed, global)). One node:
    LN writes its bf16 output as the in_conv GEMM's operand, that GEMM's epilogue writes GELU(u) straight into
    the left half of the out_conv operand [T][2h] (and GELU'(u) aside), the per-image mean (of those bf16
    values) is broadcast into the right half, and out_conv runs as in _RouterMLP: no f32 x_embed, GELU pass,
    concatenation or cast. Backward: out_conv's input gradient splits into the x_embed part (one GEMM) and the
    per-image token sum of the global part, (sum_t dU1[t]) W1[:, h:] (vit_segment_colsum + a [B][h] f32 product),
    spread over the non-reserved tokens and times GELU' in one pass (vit_router_dx_gate, which also sums in_conv's
    bias gradient), then in_conv's data gradient and the LN backward; the four weight gradients are one grouped
    split-K launch and the three hidden-bias gradients one column-sum launch (_finish_grads)."""

    @staticmethod
    def forward(ctx, x, ln_w, ln_b, w0, b0, w1, b1, w2, b2, w3, b3, reserve, eps, through=False):
        B, N, D = x.shape
        ctx.through = through
        T = B * N
        Hh, K1 = w0.shape[0], w1.shape[1]
        dev = x.device
        rp, dp, h0p = _rup(max(T, 1), 64), _rup(D, 64), _rup(Hh, 64)
        kp = _rup(K1, 64)
        x2 = x.contiguous().float().view(T, D)
        lnb = _alloc_pad(rp, dp, T, D, dev)
        mean = torch.empty(T, device=dev, dtype=F32)
        rstd = torch.empty(T, device=dev, dtype=F32)
        if T:
            ops.layernorm_fwd(x2, D, ln_w.detach().float().contiguous(), ln_b.detach().float().contiguous(), lnb, dp,
                              mean, rstd, T, D, eps)
        # in_conv's and out_conv's padded bf16 weights: one launch
        H1, H2, O = w1.shape[0], w2.shape[0], w3.shape[0]
        h1p, h2p = _rup(H1, 64), _rup(H2, 64)
        w0b, *ws = _pad_bf16_many([(w0.detach().float().contiguous(), h0p, dp)] +
                                  [(w.detach().float().contiguous(), _rup(n, 64), k)
                                   for w, n, k in ((w1, H1, kp), (w2, H2, h1p), (w3, O, h2p))])
        xcat = _alloc_pad(rp, kp, T, K1, dev)  # [x_embed | global] operand of out_conv
        gp0 = _alloc_pad(rp, h0p, T, Hh, dev)
        if T:
            ops.gemm(lnb, w0b, gp0, T, Hh, dp, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=dp, ldb=dp, ldc=h0p,
                     epilogue=EPI_BIAS_GELU_DGELU, bias=b0.detach().float().contiguous(), C2=xcat, ldc2=kp)
        glob = torch.empty(B, Hh, device=dev, dtype=F32)  # [B][h]: mean of the bf16 x_embed values, reserved tokens out
        # the mean, and its bf16 broadcast into every token's global half, in one launch
        ops.segment_colsum_bcast(xcat, kp, B, N - reserve, Hh, glob, Hh, xcat[:, Hh:], kp, N, seg_stride=N,
                                 row0=reserve, scale=1.0 / (N - reserve))
        out, acts, ws = _mlp_forward(xcat, T, kp, w1, b1, w2, b2, w3, b3, ws=ws)
        ctx.save_for_backward(x2, mean, rstd, ln_w, lnb, gp0, xcat, *acts, w0b, *ws, w1)
        ctx.params = (w0, b0, w1, b1, w2, b2, w3, b3)
        ctx.dims = (B, N, D, T, Hh, K1, reserve)
        if through:  # x passed on for the layer: its gradient comes back here and joins the LN backward's dx
            return out.view(B, N, w3.shape[0]), x.view_as(x)
        return out.view(B, N, w3.shape[0])

    @staticmethod
    def backward(ctx, dout, dthrough=None):
        x2, mean, rstd, ln_w, lnb, gp0, xcat, g1, gp1, g2, gp2, w0b, wp1, wp2, wp3, w1 = ctx.saved_tensors
        B, N, D, T, Hh, K1, reserve = ctx.dims
        w0, w2, w3 = ctx.params[0], ctx.params[4], ctx.params[6]
        dev = dout.device
        rp, dp, h0p, kp = xcat.shape[0], lnb.shape[1], gp0.shape[1], xcat.shape[1]
        d2 = dout.contiguous().float().view(T, w3.shape[0])
        marks, need = [], ctx.needs_input_grad[3:11]  # w0, b0, w1, b1, w2, b2, w3, b3
        mp, mn = ctx.params[2:], need[2:]
        _, du1, wg, bs, db3 = _mlp_backward(d2, T, xcat, (g1, gp1, g2, gp2), (wp1, wp2, wp3), w1, w2, w3, False, mp, mn,
                                            marks)
        H1 = w1.shape[0]
        # out_conv's input gradient, by halves: the x_embed half as one GEMM (dU1 W1[:, :h], B = the padded W1's
        # first h columns); the global half only through its per-image token sum, which by linearity is
        # (sum_t dU1[t]) W1[:, h:] — a [B][h] product instead of a [T][h] GEMM, a copy and a token reduction of it
        dxe = _dgrad_f32(du1, wp1, kp, Hh, T)
        s1 = torch.empty(B, H1, device=dev, dtype=F32)
        ops.segment_colsum(du1, du1.shape[1], B, N, H1, s1, H1)
        gsum = torch.empty(B, Hh, device=dev, dtype=F32)
        w1f = w1.detach().float().contiguous()
        ops.gemm_f32(B, Hh, H1, s1, H1, False, w1f[:, Hh:], K1, False, gsum, Hh)
        # du0 = (dxe + [t non-reserved] gsum[image] / (N - reserve)) * GELU'(u0), bf16 [rp][h0p], and the column
        # partials of in_conv's bias gradient
        du0b = torch.empty(rp, h0p, device=dev, dtype=BF16)
        r0 = ops.router_dx_gate_partial_rows(rp)
        p0 = torch.empty(r0, Hh, device=dev, dtype=F32)
        ops.router_dx_gate(dxe, Hh, gsum, Hh, 1.0 / (N - reserve), gp0, h0p, T, N, reserve, Hh, du0b, h0p, p0, Hh)
        dln = _dgrad_f32(du0b, w0b, dp, D, T)
        # the mlp's members are indexed from 2 (w1 ..); in_conv's weight / bias are 0 / 1
        wg = [(a, la, b_, lb, m, n, i + 2) for a, la, b_, lb, m, n, i in wg] + [(du0b, h0p, lnb, dp, Hh, D, 0)]
        bs = [(p_, r_, c_, i + 2) for p_, r_, c_, i in bs] + [(p0, r0, Hh, 1)]
        g = _finish_grads(rp, wg, bs, ctx.params, need, marks, dev)
        dx = torch.empty(T, D, device=dev, dtype=F32)
        need_ln = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        gb = torch.zeros(2 * D, device=dev, dtype=F32) if need_ln else None
        if T:
            part = torch.empty(ops.layernorm_bwd_partial_rows(T), 3 * D, device=dev, dtype=F32)
            dres = dthrough.contiguous().view(T, D).float() if dthrough is not None else None
            ops.layernorm_bwd(dln, D, x2, D, mean, rstd, ln_w.detach().float().contiguous(), dx, D, part, T, D,
                              dgamma_dbeta=gb, dres=dres, lddres=D if dres is not None else 0)
        elif dthrough is not None:
            dx = dthrough.contiguous().view(T, D).float().clone()
        dg = gb[:D] if need_ln else None
        dbt = gb[D:] if need_ln else None
        _sunk(marks)
        return (dx.view(B, N, D), dg, dbt, g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7] if db3 is None else db3,
                None, None, None)


def router_mlp_supported(seq, x):
    """out_conv as built by RouterModule: Linear, GELU (exact), Linear, GELU, Linear, biases present; both hidden widths
    multiples of 8 (the data-gradient GEMMs of _dgrad_mul write the hidden-bias column partials, which the GEMM takes in
    8-column chunks only). Any other --dynamic_router_hdim runs the per-op path."""
    from .model import GELU as _GELU, Linear as _Linear
    if not x.is_cuda or len(seq) != 5:
        return False
    lins, gelus = (seq[0], seq[2], seq[4]), (seq[1], seq[3])
    if not all(type(l) is _Linear and l.bias is not None and l.weight.dtype == F32 for l in lins):
        return False
    if not all(type(g) is _GELU and g.approximate == "none" for g in gelus):
        return False
    if lins[0].weight.shape[0] % 8 or lins[1].weight.shape[0] % 8:
        return False
    return (lins[0].weight.shape[1] == x.shape[-1] and lins[1].weight.shape[1] == lins[0].weight.shape[0]
            and lins[2].weight.shape[1] == lins[1].weight.shape[0])


def router_mlp(seq, x):
    """seq(x) for RouterModule.out_conv (Linear, GELU, Linear, GELU, Linear) as one fused node"""
    l1, l2, l3 = seq[0], seq[2], seq[4]
    return _RouterMLP.apply(x, l1.weight, l1.bias, l2.weight, l2.bias, l3.weight, l3.bias)


def router_net_supported(router, x):
    """RouterModule as built: in_conv = (LayerNorm, Linear, GELU exact), out_conv as router_mlp_supported, at least
    one non-reserved token, an even in_conv width h (vit_router_dx_gate reads dX_embed in pairs, and the global half
    of the concatenated operand starts at column h: vit_segment_colsum_bcast needs it 4-byte aligned)"""
    from .model import GELU as _GELU, Linear as _Linear
    ic = router.in_conv
    if len(ic) != 3 or not (x.is_cuda and x.dim() == 3 and x.shape[1] > router.reserve_initials):
        return False
    ln = getattr(ic[0], "layer_norm", None)
    if ln is None or ln.weight is None or tuple(ln.normalized_shape) != (x.shape[-1],):
        return False
    if not (type(ic[1]) is _Linear and ic[1].bias is not None and type(ic[2]) is _GELU and ic[2].approximate == "none"):
        return False
    if ic[1].weight.shape[1] != x.shape[-1] or ic[1].weight.shape[0] % 2:
        return False
    probe = torch.empty(0, 0, 2 * ic[1].weight.shape[0], device=x.device)
    return router_mlp_supported(router.out_conv, probe)


def router_net(router, x, through=False):
    """RouterModule's logits (in_conv, mean, cat, out_conv) as one fused node; through: (logits, x passed on) — the
    caller feeds the passed-on x to the layer, so the layer's input gradient comes back through this node and is added
    inside its LayerNorm backward instead of by autograd (one [T][D] f32 add pass fewer per routed block)"""
    ln, l0 = router.in_conv[0].layer_norm, router.in_conv[1]
    l1, l2, l3 = router.out_conv[0], router.out_conv[2], router.out_conv[4]
    return _RouterNet.apply(x, ln.weight, ln.bias, l0.weight, l0.bias, l1.weight, l1.bias, l2.weight, l2.bias,
                            l3.weight, l3.bias, int(router.reserve_initials), float(ln.eps), bool(through))
