"""Drop-in ViT module surface (reference src/model.py) running on the MI355X HIP engine.

Class names, constructor signatures, parameter names/shapes/layouts and the constructor's RNG
consumption order match reference src/model.py:7-211, so `state_dict()` / `load_state_dict()`
interoperate with the reference's checkpoints (src/train.py:69-81, src/checkpoint.py:7-17) and a
seeded construction draws bit-identical initial weights.

`VisionTransformer.forward` runs the whole network (patch embedding, encoder, head) as one
autograd node whose forward and backward are the hand-written gfx950 kernels of libvit_hip.so
(vitmi.engine). The sub-modules (Encoder, EncoderBlock, SelfAttention, MlpBlock, LinearGeneral,
PositionEmbs) and the torch.nn leaves inside them (Linear, LayerNorm, GELU, Dropout: vitmi
subclasses with identical constructors and parameters) can also be called on their own, as in the
reference: their forwards are written like the reference's and run, forward and backward, on the
same kernels through vitmi.functional. There is no CPU or PyTorch-op fallback: the model must live
on a ROCm GPU.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import functional as HF
from .engine import ArchConfig, ViTEngine

__all__ = ["PositionEmbs", "MlpBlock", "MLPBlock", "LinearGeneral", "SelfAttention", "EncoderBlock", "Encoder",
           "VisionTransformer", "CrossEntropyLoss", "Linear", "LayerNorm", "GELU", "Dropout"]


# ---- torch.nn leaves on the HIP kernels (same constructors, parameters and RNG draws) --------------
class Linear(nn.Linear):
    """nn.Linear (src/model.py:31-32,194) with its forward on the bf16 MFMA GEMM."""

    def forward(self, x):
        return HF.linear(x, self.weight, self.bias)


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (src/model.py:108,114,146) with its forward on the HIP LayerNorm kernels."""

    def forward(self, x):
        if tuple(self.normalized_shape) != (x.shape[-1],):
            raise NotImplementedError("vitmi LayerNorm normalizes the last dim (the reference's use)")
        return HF.layer_norm(x, self.weight, self.bias, self.eps)


class GELU(nn.GELU):
    """nn.GELU() exact erf (src/model.py:33)."""

    def forward(self, x):
        if self.approximate != "none":
            raise NotImplementedError("vitmi GELU is the exact-erf form (the reference's default)")
        return HF.gelu(x)


class Dropout(nn.Dropout):
    """nn.Dropout (src/model.py:19-20,46-51,124-125) with a counter-based Philox mask on the device."""

    def forward(self, x):
        return HF.dropout(x, self.p, self.training)


class PositionEmbs(nn.Module):
    """reference src/model.py:7-22"""

    def __init__(self, num_patches, emb_dim, dropout_rate=0.1):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.randn(1, num_patches + 1, emb_dim))
        self.dropout = Dropout(dropout_rate) if dropout_rate > 0 else None

    def forward(self, x):
        out = HF.add(x, self.pos_embedding)
        if self.dropout:
            out = self.dropout(out)
        return out


class MlpBlock(nn.Module):
    """reference src/model.py:25-51 (fc1 -> exact GELU -> fc2)."""

    def __init__(self, in_dim, mlp_dim, out_dim, dropout_rate=0.1):
        super().__init__()
        self.fc1 = Linear(in_dim, mlp_dim)
        self.fc2 = Linear(mlp_dim, out_dim)
        self.act = GELU()
        if dropout_rate > 0.0:
            self.dropout1 = Dropout(dropout_rate)
            self.dropout2 = Dropout(dropout_rate)
        else:
            self.dropout1 = None
            self.dropout2 = None

    def forward(self, x):
        out = self.fc1(x)
        out = self.act(out)
        if self.dropout1:
            out = self.dropout1(out)
        out = self.fc2(out)
        if self.dropout2:
            out = self.dropout2(out)
        return out


MLPBlock = MlpBlock  # the reference README calls it MLPBlock (README.md:35)


class LinearGeneral(nn.Module):
    """reference src/model.py:54-63: weight [*in_dim, *feat_dim] (JAX layout), bias [*feat_dim]."""

    def __init__(self, in_dim=(768,), feat_dim=(12, 64)):
        super().__init__()
        self.weight = nn.Parameter(torch.randn(*in_dim, *feat_dim))
        self.bias = nn.Parameter(torch.zeros(*feat_dim))

    def forward(self, x, dims):
        return HF.linear_general(x, self.weight, self.bias, dims)


class SelfAttention(nn.Module):
    """reference src/model.py:66-101"""

    def __init__(self, in_dim, heads=8, dropout_rate=0.1):
        super().__init__()
        self.heads = heads
        self.head_dim = in_dim // heads
        self.scale = self.head_dim ** 0.5
        self.query = LinearGeneral((in_dim,), (self.heads, self.head_dim))
        self.key = LinearGeneral((in_dim,), (self.heads, self.head_dim))
        self.value = LinearGeneral((in_dim,), (self.heads, self.head_dim))
        self.out = LinearGeneral((self.heads, self.head_dim), (in_dim,))
        # built but never applied by the reference forward (src/model.py:78-81 vs :83-101)
        self.dropout = Dropout(dropout_rate) if dropout_rate > 0 else None

    def forward(self, x):
        q = self.query(x, dims=([2], [0]))
        k = self.key(x, dims=([2], [0]))
        v = self.value(x, dims=([2], [0]))
        out = HF.attention(q, k, v)  # (q k^T) / sqrt(hd), softmax, @ v (src/model.py:90-97)
        return self.out(out, dims=([2, 3], [0, 1]))


class EncoderBlock(nn.Module):
    """reference src/model.py:104-130 (pre-LN)."""

    def __init__(self, in_dim, mlp_dim, num_heads, dropout_rate=0.1, attn_dropout_rate=0.1):
        super().__init__()
        self.norm1 = LayerNorm(in_dim)
        self.attn = SelfAttention(in_dim, heads=num_heads, dropout_rate=attn_dropout_rate)
        self.dropout = Dropout(dropout_rate) if dropout_rate > 0 else None
        self.norm2 = LayerNorm(in_dim)
        self.mlp = MlpBlock(in_dim, mlp_dim, in_dim, dropout_rate)

    def forward(self, x):
        residual = x
        out = self.norm1(x)
        out = self.attn(out)
        if self.dropout:
            out = self.dropout(out)
        out = HF.add(out, residual)
        residual = out
        out = self.norm2(out)
        out = self.mlp(out)
        return HF.add(out, residual)


class Encoder(nn.Module):
    """reference src/model.py:133-156"""

    def __init__(self, num_patches, emb_dim, mlp_dim, num_layers=12, num_heads=12, dropout_rate=0.1,
                 attn_dropout_rate=0.0):
        super().__init__()
        self.pos_embedding = PositionEmbs(num_patches, emb_dim, dropout_rate)
        self.encoder_layers = nn.ModuleList()
        for _ in range(num_layers):
            self.encoder_layers.append(EncoderBlock(emb_dim, mlp_dim, num_heads, dropout_rate, attn_dropout_rate))
        self.norm = LayerNorm(emb_dim)

    def forward(self, x):
        out = self.pos_embedding(x)
        for layer in self.encoder_layers:
            out = layer(out)
        return self.norm(out)


class _ViTFunction(torch.autograd.Function):
    """Whole-network forward/backward on the HIP engine (one autograd node)."""

    @staticmethod
    def forward(ctx, model, x, *params):
        eng = model._engine
        logits = eng.forward(x, dropout_p=model.dropout_rate if model.training else 0.0)
        ctx.model = model
        ctx.step = eng.step_id
        return logits.clone()

    @staticmethod
    def backward(ctx, dlogits):
        model = ctx.model
        eng = model._engine
        if eng.step_id != ctx.step:
            raise RuntimeError("vitmi: backward of a stale forward (another forward ran on this model since); "
                               "the engine keeps one set of saved activations per batch size")
        params = model._flat_params
        accumulate = any(p.grad is not None for p in params)
        if accumulate:
            buf = model._scratch_grad()
        else:
            buf = eng.grad
        eng.backward(dlogits, buf)
        if eng.grad_ready_finish is not None:
            # data parallel: the buckets must be reduced (and averaged) before autograd adds them into
            # existing .grad tensors (zero_grad(set_to_none=False), gradient accumulation)
            eng.grad_ready_finish()
        grads = [eng.layout.view(buf, n) for n in model._flat_names]
        return (None, None, *grads)


class VisionTransformer(nn.Module):
    """reference src/model.py:159-211 — same ctor, state_dict and forward contract."""

    def __init__(self, image_size=(256, 256), patch_size=(16, 16), emb_dim=768, mlp_dim=3072, num_heads=12,
                 num_layers=12, num_classes=1000, attn_dropout_rate=0.0, dropout_rate=0.1, feat_dim=None):
        super().__init__()
        h, w = image_size
        fh, fw = patch_size
        if h != w or fh != fw:
            raise NotImplementedError("vitmi supports square images and patches")
        gh, gw = h // fh, w // fw
        num_patches = gh * gw
        self.embedding = nn.Conv2d(3, emb_dim, kernel_size=(fh, fw), stride=(fh, fw))
        self.cls_token = nn.Parameter(torch.zeros(1, 1, emb_dim))
        self.transformer = Encoder(num_patches=num_patches, emb_dim=emb_dim, mlp_dim=mlp_dim, num_layers=num_layers,
                                   num_heads=num_heads, dropout_rate=dropout_rate,
                                   attn_dropout_rate=attn_dropout_rate)
        self.classifier = Linear(emb_dim, num_classes)
        self.arch = ArchConfig(image_size=h, patch_size=fh, emb_dim=emb_dim, mlp_dim=mlp_dim, num_heads=num_heads,
                               num_layers=num_layers, num_classes=num_classes)
        self.dropout_rate = dropout_rate
        self.attn_dropout_rate = attn_dropout_rate
        # "bf16": the training path (bf16 MFMA operands, fp32 accumulation, autograd through the HIP
        # engine). "fp32": forward-only in the reference's own arithmetic (f32 operands everywhere),
        # for the logits-parity gate and fp32 evaluation; its output carries no autograd graph.
        self.precision = "bf16"
        self._engine = None
        self._flat_names = None
        self._flat_params = None
        self._scratch = None

    # ---- engine binding -----------------------------------------------------------------------
    def _bind_engine(self):
        """Move every parameter into the engine's flat buffer (Parameters become views of it)."""
        dev = self.embedding.weight.device
        if dev.type != "cuda":
            raise RuntimeError("vitmi.VisionTransformer runs on the MI355X HIP path only; move it to a GPU first "
                               "(model.to('cuda'))")
        named = dict(self.named_parameters())
        if self._engine is None or self._engine.dev != dev:
            eng = ViTEngine(self.arch, device=dev)
        else:
            eng = self._engine
        names = list(eng.layout.offsets.keys())
        with torch.no_grad():
            for n in names:
                p = named[n]
                v = eng.layout.view(eng.flat, n)
                if p.data.data_ptr() != v.data_ptr():
                    v.copy_(p.data)
                    p.data = v
        self._engine = eng
        self._flat_names = names
        self._flat_params = [named[n] for n in names]
        eng.invalidate_mirror()

    def _bound(self):
        if self._engine is None:
            return False
        return all(p.data_ptr() == self._engine.layout.view(self._engine.flat, n).data_ptr()
                   for n, p in zip(self._flat_names, self._flat_params))

    def _scratch_grad(self):
        if self._scratch is None or self._scratch.device != self._engine.dev:
            self._scratch = torch.zeros_like(self._engine.grad)
        return self._scratch

    def _version_sig(self):
        return sum(p._version for p in self._flat_params)

    def engine(self):
        if not self._bound():
            self._bind_engine()
        return self._engine

    def forward(self, x):
        # (attn_dropout_rate builds SelfAttention.dropout, which the reference never applies: src/model.py:78-99)
        eng = self.engine()
        if self.precision == "fp32":
            if self.training and self.dropout_rate > 0:
                raise NotImplementedError("precision='fp32' is the forward-only exact path; train-mode dropout runs on "
                                          "the bf16 path (use model.eval() for fp32 evaluation)")
            if torch.is_grad_enabled() and any(p.requires_grad for p in self._flat_params):
                raise RuntimeError("precision='fp32' is the forward-only exact path; run it under torch.no_grad() "
                                   "(training uses precision='bf16')")
            return eng.forward_exact(x)
        if self.precision != "bf16":
            raise ValueError(f"unknown precision {self.precision!r} (bf16 | fp32)")
        sig = self._version_sig()
        if eng._mirror_sig != sig:
            eng.refresh_mirror()
            eng.mark_mirror_fresh(sig)
        return _ViTFunction.apply(self, x, *self._flat_params)


class CrossEntropyLoss(nn.Module):
    """nn.CrossEntropyLoss() (mean) on the HIP cross-entropy kernel (reference src/train.py:151).
    The kernel also counts top-1 / top-5 hits per row (src/utils.py:28-41): `last_row_stats`
    holds {loss, top1, top5} [b, 3] of the latest call, which vitmi.train uses for accuracy."""

    def __init__(self):
        super().__init__()
        self.last_row_stats = None

    def forward(self, logits, target):
        st = torch.empty(logits.shape[0], 3, device=logits.device)
        loss = _CEFunction.apply(logits, target, st)
        self.last_row_stats = st
        return loss


class _CEFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, st):
        from . import ops
        logits = logits.float().contiguous()
        b, c = logits.shape
        dl = torch.empty_like(logits)
        ops.cross_entropy(logits, target.to(torch.int64).contiguous(), dl, 1.0 / b, st)
        ctx.save_for_backward(dl)
        return st[:, 0].mean()

    @staticmethod
    def backward(ctx, g):
        dl, = ctx.saved_tensors
        return dl * g, None, None
