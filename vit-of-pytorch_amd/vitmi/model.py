"""Drop-in ViT module surface (reference src/model.py) running on the MI355X HIP engine.

Class names, constructor signatures, parameter names/shapes/layouts and the constructor's RNG
consumption order match reference src/model.py:7-211, so `state_dict()` / `load_state_dict()`
interoperate with the reference's checkpoints (src/train.py:69-81, src/checkpoint.py:7-17) and a
seeded construction draws bit-identical initial weights.

`VisionTransformer.forward` runs the whole network (patch embedding, encoder, head) as one
autograd node whose forward and backward are the hand-written gfx950 kernels of
libvit_hip.so (vitmi.engine). There is no CPU or PyTorch-op fallback: the model must live on a
ROCm GPU. The sub-modules (Encoder, EncoderBlock, SelfAttention, MlpBlock, LinearGeneral,
PositionEmbs) exist for the parameter tree and state_dict; only the whole-model forward is
on the accelerated path.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .engine import ArchConfig, ViTEngine

__all__ = ["PositionEmbs", "MlpBlock", "MLPBlock", "LinearGeneral", "SelfAttention", "EncoderBlock", "Encoder",
           "VisionTransformer", "CrossEntropyLoss"]


def _submodule_forward(name):
    def forward(self, *args, **kwargs):
        raise NotImplementedError(
            f"{name}.forward on its own is not on the MI355X path; run the whole VisionTransformer "
            "(the encoder executes as one fused HIP engine)")
    return forward


class PositionEmbs(nn.Module):
    """reference src/model.py:7-22"""

    def __init__(self, num_patches, emb_dim, dropout_rate=0.1):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.randn(1, num_patches + 1, emb_dim))
        self.dropout = nn.Dropout(dropout_rate) if dropout_rate > 0 else None

    forward = _submodule_forward("PositionEmbs")


class MlpBlock(nn.Module):
    """reference src/model.py:25-51 (fc1 -> exact GELU -> fc2)."""

    def __init__(self, in_dim, mlp_dim, out_dim, dropout_rate=0.1):
        super().__init__()
        self.fc1 = nn.Linear(in_dim, mlp_dim)
        self.fc2 = nn.Linear(mlp_dim, out_dim)
        self.act = nn.GELU()
        if dropout_rate > 0.0:
            self.dropout1 = nn.Dropout(dropout_rate)
            self.dropout2 = nn.Dropout(dropout_rate)
        else:
            self.dropout1 = None
            self.dropout2 = None

    forward = _submodule_forward("MlpBlock")


MLPBlock = MlpBlock  # the reference README calls it MLPBlock (README.md:35)


class LinearGeneral(nn.Module):
    """reference src/model.py:54-63: weight [*in_dim, *feat_dim] (JAX layout), bias [*feat_dim]."""

    def __init__(self, in_dim=(768,), feat_dim=(12, 64)):
        super().__init__()
        self.weight = nn.Parameter(torch.randn(*in_dim, *feat_dim))
        self.bias = nn.Parameter(torch.zeros(*feat_dim))

    forward = _submodule_forward("LinearGeneral")


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
        self.dropout = nn.Dropout(dropout_rate) if dropout_rate > 0 else None

    forward = _submodule_forward("SelfAttention")


class EncoderBlock(nn.Module):
    """reference src/model.py:104-130 (pre-LN)."""

    def __init__(self, in_dim, mlp_dim, num_heads, dropout_rate=0.1, attn_dropout_rate=0.1):
        super().__init__()
        self.norm1 = nn.LayerNorm(in_dim)
        self.attn = SelfAttention(in_dim, heads=num_heads, dropout_rate=attn_dropout_rate)
        self.dropout = nn.Dropout(dropout_rate) if dropout_rate > 0 else None
        self.norm2 = nn.LayerNorm(in_dim)
        self.mlp = MlpBlock(in_dim, mlp_dim, in_dim, dropout_rate)

    forward = _submodule_forward("EncoderBlock")


class Encoder(nn.Module):
    """reference src/model.py:133-156"""

    def __init__(self, num_patches, emb_dim, mlp_dim, num_layers=12, num_heads=12, dropout_rate=0.1,
                 attn_dropout_rate=0.0):
        super().__init__()
        self.pos_embedding = PositionEmbs(num_patches, emb_dim, dropout_rate)
        self.encoder_layers = nn.ModuleList()
        for _ in range(num_layers):
            self.encoder_layers.append(EncoderBlock(emb_dim, mlp_dim, num_heads, dropout_rate, attn_dropout_rate))
        self.norm = nn.LayerNorm(emb_dim)

    forward = _submodule_forward("Encoder")


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
        self.classifier = nn.Linear(emb_dim, num_classes)
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
