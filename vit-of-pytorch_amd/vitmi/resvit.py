"""Res-ViT (reference res-vit/model.py, res-vit/model_utils.py) on the MI355X HIP kernels.

The reference's research variant: a ViT whose blocks from `dynamic_start_layer` on are grouped into
blocks of `block_size` layers; a DynamicViT-style router at each block head decides per token and per
layer whether the token runs the full transformer layer or a low-rank approximator (Gumbel hard routing
while training, argmax at inference), with LoRA on q / k / v over frozen base weights, a teacher
(all tokens) and a student (routed) path during training, and ragged attention at inference (queries =
the active tokens, keys = all tokens).

Same class names, constructor arguments, module / parameter names and constructor RNG order as the
reference (res-vit/model.py:13-702), so its state_dicts load. Compute runs on libvit_hip.so through
vitmi.functional: every Linear (q/k/v/o, LoRA, FFN, router MLP, approximators, classifier, the patch
embedding as im2col + GEMM), LayerNorm, GELU, residual adds, self-attention (fused kernels, forward and
backward) and the inference path's ragged attention (one vit_attention_fwd_varlen launch for the whole
batch instead of the reference's per-sample loop). The routing decisions themselves — a 2-way softmax,
Gumbel noise, argmax and the entropy / MSE scalars over [B, N, block_size] tensors — and the boolean-mask
row gathers / scatters are small device-side torch operations (data selection, no GEMM-shaped work).

Gumbel noise: `RouterModule.gumbel_noise` (default None = draw like torch.nn.functional.gumbel_softmax
on the device) may be set to a callable(logits) -> noise, which the parity tests use to replay the
reference's recorded draws.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import flat as _flat
from . import functional as HF
from . import ops as _ops
from . import resvit_fused as _fused
from .model import GELU, CrossEntropyLoss, LayerNorm as _HipLayerNorm, Linear

__all__ = ["ModelArgs", "DistillLoss", "ActiveLoss", "PositionEmbs", "LoRAModule", "LayerNorm", "RouterModule",
           "Attention", "FeedForward", "LowRankApproximator", "BlockPathApproximators", "TransformerBlock",
           "Transformer", "repeat_kv", "get_indices_from_LRA_mask"]


@dataclass
class ModelArgs:
    """reference res-vit/model.py:13-37"""
    dim: int = 768
    mlp_dim: int = 3072
    n_layers: int = 12
    n_heads: int = 12
    n_kv_heads: Optional[int] = 12
    norm_eps: float = 1e-5
    lora_rank: int = 8
    dynamic_active_target: float = 0.4
    dynamic_start_layer: int = 2
    dynamic_router_hdim: int = 512
    dynamic_reserve_initials: int = 1
    low_rank_dim: int = 256
    block_size: int = 2
    use_lora: bool = False
    use_reslr: bool = False
    image_size: Tuple[int, int] = (224, 224)
    patch_size: Tuple[int, int] = (16, 16)
    num_classes: int = 100
    dropout: float = 0.15
    num_patches: int = (224 // 16) * (224 // 16)
    device: str = "cuda"


_CONST = {}


def _const(values, device, dtype):
    """small constant tensors (routing tables, bit weights) made on the device once: torch.tensor(list,
    device=...) would copy from pageable host memory — a host-device synchronisation — every layer"""
    key = (values, str(device), dtype)
    t = _CONST.get(key)
    if t is None:
        t = torch.tensor(values, dtype=dtype).reshape(-1).to(device)
        _CONST[key] = t
    return t


# ---- model_utils (reference res-vit/model_utils.py) ---------------------------------------------
def repeat_kv(x: torch.Tensor, n_rep: int) -> torch.Tensor:
    """[b, s, n_kv, hd] -> [b, s, n_kv * n_rep, hd], each kv head repeated n_rep times (model_utils.py:3-12)."""
    if n_rep == 1:
        return x
    b, s, nkv, hd = x.shape
    return x.unsqueeze(3).expand(b, s, nkv, n_rep, hd).reshape(b, s, nkv * n_rep, hd)


# Router index tables (model_utils.py:25-66): entry [i][j] lists the router indices (the binary keep
# pattern of a token over the block's layers, most significant bit = first layer) whose tokens take,
# at block position j, the path with code i; stored as data.
_ROUTE_TABLES = {
    1: [[[0], []]],
    2: [[[1], [0]], [[], [2]]],
    4: [[[4, 5, 6, 7], [2, 3], [1], [0]],
        [[], [10, 11], [9], [8]],
        [[], [], [13, 5], [12, 4]],
        [[], [], [], [2, 6, 10, 14]]],
}


def _lra_coords(block_size: int):
    """(approximator, transformer, straight-through) table coordinates per block position j
    (model_utils.py:14-23)."""
    out = []
    for j in range(block_size):
        appr = [(i, j) for i in range(j + 1)]
        trans = [(i, jp) for jp in range(j) for i in range(jp + 1)]
        trans += [(i, jp) for jp in range(j + 1, block_size) for i in range(j + 1, jp + 1)]
        ste = [(i, jp) for jp in range(j + 1, block_size) for i in range(j + 1)]
        out.append((appr, trans, ste))
    return out


def get_indices_from_LRA_mask(block_size, mapping_table=None):
    """per block position: (approximator indices, transformer indices, straight-through indices), each sorted
    and de-duplicated; the all-ones pattern always runs the transformer (model_utils.py:69-107)."""
    table = mapping_table if mapping_table is not None else _ROUTE_TABLES.get(block_size)
    if table is None:
        raise ValueError(f"unsupported block_size: {block_size} (1, 2 or 4)")
    result = []
    for appr, trans, ste in _lra_coords(block_size):
        pick = lambda coords: sorted({v for i, jp in coords for v in table[i][jp]})
        t = sorted(set(pick(trans)) | {(1 << block_size) - 1})
        result.append((pick(appr), t, pick(ste)))
    return result


# ---- losses -------------------------------------------------------------------------------------------
class DistillLoss(nn.Module):
    """MSE between the student and (detached) teacher cls tokens (res-vit/model.py:40-59)."""

    def forward(self, student_cls: torch.Tensor, teacher_cls: torch.Tensor):
        return F.mse_loss(student_cls, teacher_cls.detach())


class ActiveLoss(nn.Module):
    """(mean keep ratio - target)^2 over the non-reserved tokens (res-vit/model.py:61-85)."""

    def __init__(self, target, reserve_initials):
        super().__init__()
        self.target = target
        self.reserve_initials = reserve_initials

    @torch.no_grad()
    def metric(self, activation: torch.Tensor):
        return {"non_low_rank_ratio": activation[:, self.reserve_initials:, :].mean(), "current_target": self.target}

    def forward(self, activation: torch.Tensor):
        ratio = activation[:, self.reserve_initials:, :].mean()
        return F.mse_loss(ratio, ratio.new_full((), self.target))  # (a device fill: no host copy)


# ---- modules --------------------------------------------------------------------------------------------
class PositionEmbs(nn.Module):
    """res-vit/model.py:87-100 (longer inputs keep their extra tokens unchanged)."""

    def __init__(self, num_patches, emb_dim):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.randn(1, num_patches + 1, emb_dim))

    def forward(self, x):
        n, npos = x.shape[1], self.pos_embedding.shape[1]
        if n == npos:
            return HF.add(x, self.pos_embedding)
        m = min(n, npos)
        out = HF.add(x[:, :m].contiguous(), self.pos_embedding[:, :m])
        return torch.cat([out, x[:, m:]], dim=1) if n > npos else out


class LoRAModule(nn.Module):
    """lora_B(lora_A(x)), both N(0, 0.01) (res-vit/model.py:103-115)."""

    def __init__(self, in_dim: int, rank: int, out_dim: int):
        super().__init__()
        self.in_dim, self.rank, self.out_dim = in_dim, rank, out_dim
        self.lora_A = Linear(in_dim, rank, bias=False)
        self.lora_B = Linear(rank, out_dim, bias=False)
        nn.init.normal_(self.lora_A.weight, mean=0.0, std=0.01)
        nn.init.normal_(self.lora_B.weight, mean=0.0, std=0.01)

    def forward(self, x):
        return self.lora_B(self.lora_A(x))


class LayerNorm(nn.Module):
    """res-vit/model.py:117-128: nn.LayerNorm wrapper, frozen under LoRA."""

    def __init__(self, dim: int, eps: float = 1e-6, use_lora: bool = False):
        super().__init__()
        self.layer_norm = _HipLayerNorm(dim, eps=eps)
        if use_lora:
            for p in self.layer_norm.parameters():
                p.requires_grad = False

    def forward(self, x):
        return self.layer_norm(x)


class RouterModule(nn.Module):
    """DynamicViT router (res-vit/model.py:133-211): per token, keep / approximate for each of the block's
    layers; reserved leading tokens (cls) always keep."""

    def __init__(self, in_dim: int, hidden_dim: int, reserve_initials: int, norm_eps: float, block_size: int = 1,
                 use_lora: bool = False):
        super().__init__()
        self.block_size = block_size
        self.reserve_initials = reserve_initials
        self.in_conv = nn.Sequential(LayerNorm(in_dim, norm_eps, use_lora=use_lora), Linear(in_dim, hidden_dim),
                                     GELU())
        self.out_conv = nn.Sequential(Linear(hidden_dim * 2, hidden_dim), GELU(), Linear(hidden_dim, hidden_dim // 2),
                                      GELU(), Linear(hidden_dim // 2, block_size * 2))
        nn.init.normal_(self.out_conv[-1].weight, mean=0, std=0.01)
        for i in range(block_size):
            self.out_conv[-1].bias.data[i * 2] = 0.0      # approximate
            self.out_conv[-1].bias.data[i * 2 + 1] = 5.0  # keep (full transformer layer)
        self.fused_mlp = True      # the router network as one fused node (vitmi.resvit_fused.router_net)
        self.gumbel_noise = None   # callable(logits) -> Gumbel noise (tests replay recorded draws)
        self.hard_override = None  # callable(logits) -> one-hot decisions (tests replay recorded decisions)

    @staticmethod
    def _router2indices(keep):
        """binary keep pattern over the block's layers -> index (first layer = most significant bit)."""
        n = keep.shape[-1]
        w = _const((tuple(2.0 ** (n - 1 - i) for i in range(n)),), keep.device, torch.float32).view(n, 1)
        return torch.matmul(keep.float(), w)

    def forward_through(self, x):
        """(x', forward(x)) where x' is x passed through the fused router node: feeding x' to the block's layer
        routes the layer's input gradient through the router's LayerNorm backward, which adds it (no separate
        autograd add of the two input gradients). Plain (x, forward(x)) where the fused router does not apply."""
        B, N, _ = x.shape
        if not (self.fused_mlp and _fused.router_net_supported(self, x)):
            return x, self.forward(x)
        logits, xt = _fused.router_net(self, x, through=True)
        return xt, self.head(logits.view(B, N, self.block_size, 2))

    def forward(self, x):
        B, N, _ = x.shape
        r = self.reserve_initials
        if self.fused_mlp and _fused.router_net_supported(self, x):
            # in_conv, the token mean, the concatenation and out_conv as one node (vitmi.resvit_fused)
            logits = _fused.router_net(self, x).view(B, N, self.block_size, 2)
        else:
            x_embed = self.in_conv(x)
            global_feat = (x_embed[:, r:, :] if r > 0 else x_embed).mean(dim=1, keepdim=True)
            fused = torch.cat([x_embed, global_feat.expand(B, N, -1)], dim=-1)
            if self.fused_mlp and _fused.router_mlp_supported(self.out_conv, fused):
                logits = _fused.router_mlp(self.out_conv, fused).view(B, N, self.block_size, 2)
            else:
                logits = self.out_conv(fused).view(B, N, self.block_size, 2)
        return self.head(logits)

    def head(self, logits):
        """(hard, indices, entropy, soft) from the router's logits [B, N, block_size, 2] (res-vit/model.py:191-211)"""
        B, N = logits.shape[:2]
        r = self.reserve_initials
        if FUSED_HEAD and self.fused_mlp and _fused.router_head_supported(logits, r):
            # softmax, entropy, Gumbel hard routing, reserved rows and the pattern index as one node
            noise, mode, yh = None, 0, None
            if self.training:
                if self.gumbel_noise is not None:
                    noise, mode = self.gumbel_noise(logits), 1
                else:  # the same draws as the per-op path; -log is taken inside the node
                    noise, mode = torch.empty_like(logits).exponential_(), 2
            if self.hard_override is not None:
                yh = self.hard_override(logits)
            return _fused.router_head(logits, noise, mode, yh, r, self.training, B * (N - r) * self.block_size)
        soft = F.softmax(logits, dim=-1)
        probs = soft[:, r:]
        entropy = -torch.sum(probs * torch.log(probs + 1e-8)) / (B * (N - r) * self.block_size)
        if self.training:  # gumbel_softmax(tau=1, hard=True): straight-through one-hot
            g = (self.gumbel_noise(logits) if self.gumbel_noise is not None
                 else -torch.empty_like(logits).exponential_().log())
            y_soft = (logits + g).softmax(-1)
            y_hard = (self.hard_override(logits) if self.hard_override is not None
                      else torch.zeros_like(logits).scatter_(-1, y_soft.max(-1, keepdim=True)[1], 1.0))
            hard = y_hard - y_soft.detach() + y_soft
        else:
            hard = (self.hard_override(logits) if self.hard_override is not None
                    else torch.zeros_like(soft).scatter_(-1, soft.argmax(dim=-1, keepdim=True), 1.0))
        if r > 0:
            hard = hard.clone()
            hard[:, :r, :, :] = 0
            hard[:, :r, :, 1] = 1
        return hard, self._router2indices(hard[:, :, :, 1]), entropy, soft


class Attention(nn.Module):
    """res-vit/model.py:213-299: nn.Linear q/k/v/o with bias, optional LoRA on q/k/v, GQA."""

    def __init__(self, args: ModelArgs):
        super().__init__()
        self.n_kv_heads = args.n_heads if args.n_kv_heads is None else args.n_kv_heads
        self.n_local_heads = args.n_heads
        self.n_local_kv_heads = self.n_kv_heads
        self.n_rep = self.n_local_heads // self.n_local_kv_heads
        self.head_dim = args.dim // args.n_heads
        self.use_lora = args.use_lora
        self.wq = Linear(args.dim, args.n_heads * self.head_dim, bias=True)
        self.wk = Linear(args.dim, self.n_kv_heads * self.head_dim, bias=True)
        self.wv = Linear(args.dim, self.n_kv_heads * self.head_dim, bias=True)
        self.wo = Linear(args.n_heads * self.head_dim, args.dim, bias=True)
        if self.use_lora:
            self.lora_q = LoRAModule(args.dim, args.lora_rank, self.head_dim * self.n_local_heads)
            self.lora_k = LoRAModule(args.dim, args.lora_rank, self.head_dim * self.n_local_kv_heads)
            self.lora_v = LoRAModule(args.dim, args.lora_rank, self.head_dim * self.n_local_kv_heads)

    def project(self, x, which):
        w = getattr(self, "w" + which)
        out = w(x)
        if self.use_lora:
            out = HF.add(out, getattr(self, "lora_" + which)(x))
        return out

    def forward(self, x: torch.Tensor, x_kv: Optional[torch.Tensor] = None):
        no_batch = x.dim() == 2
        if no_batch:
            x = x.unsqueeze(0)
            x_kv = x_kv.unsqueeze(0) if x_kv is not None else None
        bsz, sq, _ = x.shape
        kv_in = x if x_kv is None else x_kv
        skv = kv_in.shape[1]
        xq = self.project(x, "q").view(bsz, sq, self.n_local_heads, self.head_dim)
        keys = repeat_kv(self.project(kv_in, "k").view(bsz, skv, self.n_local_kv_heads, self.head_dim), self.n_rep)
        values = repeat_kv(self.project(kv_in, "v").view(bsz, skv, self.n_local_kv_heads, self.head_dim),
                           self.n_rep)
        if x_kv is None:
            out = HF.attention(xq.contiguous(), keys.contiguous(), values.contiguous())
        else:  # asymmetric (queries != keys): the ragged kernel with every sample's sq queries
            cu = torch.arange(0, (bsz + 1) * sq, sq, device=x.device, dtype=torch.int32)
            out = HF.attention_ragged(xq.reshape(bsz * sq, self.n_local_heads, self.head_dim), keys, values, cu, sq)
        out = self.wo(out.reshape(bsz, sq, -1))
        return out.squeeze(0) if no_batch else out

    def forward_ragged(self, xq_rows, x_kv, cu_q, max_q):
        """inference: active query rows of every sample back to back (cu_q offsets), keys / values from all
        of each sample's tokens; one varlen launch (res-vit/model.py:506-521 loops over samples)."""
        b, skv, _ = x_kv.shape
        total = xq_rows.shape[0]
        xq = self.project(xq_rows, "q").view(total, self.n_local_heads, self.head_dim)
        keys = repeat_kv(self.project(x_kv, "k").view(b, skv, self.n_local_kv_heads, self.head_dim), self.n_rep)
        values = repeat_kv(self.project(x_kv, "v").view(b, skv, self.n_local_kv_heads, self.head_dim), self.n_rep)
        out = HF.attention_ragged(xq, keys.contiguous(), values.contiguous(), cu_q, max_q)
        return self.wo(out.reshape(total, -1))


class FeedForward(nn.Module):
    """res-vit/model.py:302-317"""

    def __init__(self, dim: int, mlp_dim: int):
        super().__init__()
        self.fc1 = Linear(dim, mlp_dim, bias=True)
        self.fc2 = Linear(mlp_dim, dim, bias=True)
        self.act = GELU()

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


class LowRankApproximator(nn.Module):
    """up_proj(down_proj(x)), both N(0, 0.01), no bias (res-vit/model.py:319-333)."""

    def __init__(self, dim: int, rank: int):
        super().__init__()
        self.down_proj = Linear(dim, rank, bias=False)
        self.up_proj = Linear(rank, dim, bias=False)
        nn.init.normal_(self.down_proj.weight, mean=0.0, std=0.01)
        nn.init.normal_(self.up_proj.weight, mean=0.0, std=0.01)

    def forward(self, x):
        return self.up_proj(self.down_proj(x))


class BlockPathApproximators(nn.Module):
    """one approximator per non-all-ones router index (res-vit/model.py:336-368): rows of x whose index is
    in the mask get x + approximator(x)."""

    def __init__(self, dim: int, rank: int, block_size: int):
        super().__init__()
        self.block_size = block_size
        self.fused = True  # training: one fused node per approximator (vitmi.resvit_fused.approx_step)
        self.approximators = nn.ModuleDict()
        total = 2 ** block_size
        for key in range(total):
            if key != total - 1:
                self.approximators[str(key)] = LowRankApproximator(dim, rank)

    def forward(self, x, router_indices, LRA_mask, sel=None):
        """sel: (active, sel [nkeys][T], any [nkeys]) of vitmi.ops.router_select for router_indices, or None"""
        idx = router_indices.squeeze(-1)
        keys = [int(k) for k in (LRA_mask.tolist() if torch.is_tensor(LRA_mask) else LRA_mask)]
        if torch.is_grad_enabled():
            # training: every row through the approximator, the routed rows selected (the same values and
            # gradients as the reference's boolean gather / scatter, which needs the row count on the host:
            # a device sync per layer). Whether any row was routed to it — torch's AdamW skips an
            # approximator without a gradient — is handed to the flat optimizer as a device flag.
            for key in keys:
                if str(key) not in self.approximators:
                    continue
                if sel is not None and key < sel[1].shape[0]:
                    sk, anyk = sel[1][key].view(*idx.shape, 1), sel[2][key]
                else:
                    sk = (idx == key).unsqueeze(-1)
                    anyk = sk.any()
                m = self.approximators[str(key)]
                if self.fused and _fused.approx_supported(m, x):
                    x = _fused.approx_step(m, x, sk)  # same values, no f32 add / where passes
                else:
                    x = torch.where(sk, HF.add(m(x), x), x)
                _flat.gate(m.parameters(), anyk)
            return x
        for key in keys:
            if str(key) not in self.approximators:
                continue
            sub = idx == key
            if sub.any():
                rows = x[sub]
                x = x.clone()
                x[sub] = HF.add(self.approximators[str(key)](rows), rows)
        return x


# the routed student's where(active, layer(x), x) folded into the fused layer node (False: torch.where after it)
FOLD_SELECT = True
# where the teacher's input is the student's (the first routed layer), one grad-enabled layer forward gives both the
# teacher output (detached) and the student's (row selection after it) instead of a no-grad teacher pass plus a
# folded student pass (False: the two passes)
SHARE_TEACHER = True


def _active_dropout(module):
    """a dropout with p > 0 inside `module` in training mode: its forward is not deterministic, so a teacher output
    taken from the student's pass would differ from the reference's separate teacher pass (SHARE_TEACHER's premise)"""
    return module.training and any(isinstance(m, torch.nn.Dropout) and m.p > 0 for m in module.modules())


# the distillation loss's cls rows taken through vitmi.resvit_fused.cls_tap (their gradient added in place), and the
# final LayerNorm on the cls rows only (False: the slices and the all-row norm as written)
CLS_TAP = True
# the router's softmax / entropy / Gumbel hard routing / pattern index as one fused node (vitmi.resvit_fused.router_head;
# False: the per-op path as written)
FUSED_HEAD = True
# the distillation loss (MSE of the cls rows) as one node whose backward adds into the student's gradient in place
# (vitmi.resvit_fused.cls_distill; False: cls_tap + DistillLoss)
FUSED_DISTILL = True
# a routed block's per-position active masks and per-approximator selections (and their any-flags) from the pattern
# index in one launch (vitmi.ops.router_select; False: isin / == / any per layer and approximator)
FUSED_SELECT = True
# a routed block's input handed to its layer through the fused router node (RouterModule.forward_through), so the
# router's LayerNorm backward adds the layer's input gradient (False: autograd adds the two)
ROUTER_THROUGH = True
# the token embedding (patch conv, cls, position embeddings) as one GEMM with the engine's PATCH epilogue where the conv
# and the position embeddings are frozen (vitmi.resvit_fused.embed_tokens; False: conv, cat, add as written)
FUSED_EMBED = True


def _select_rows(mask, a, b):
    """mask [.., 1] bool: rows of a where set, of b elsewhere (the reference's mask * a + (~mask) * b)."""
    return torch.where(mask, a, b)


class TransformerBlock(nn.Module):
    """res-vit/model.py:371-529"""

    def __init__(self, layer_id: int, args: ModelArgs):
        super().__init__()
        self.n_heads = args.n_heads
        self.dim = args.dim
        self.head_dim = args.dim // args.n_heads
        self.layer_id = layer_id
        self.current_epoch = 0
        self.use_lora = args.use_lora
        self.use_reslr = args.use_reslr
        self.fused = True  # False: the per-op path (vitmi.functional) for every configuration
        self.attention = Attention(args)
        self.attention_norm = LayerNorm(args.dim, eps=args.norm_eps, use_lora=args.use_lora)
        self.feed_forward = FeedForward(dim=args.dim, mlp_dim=args.mlp_dim)
        self.ffn_norm = LayerNorm(args.dim, eps=args.norm_eps, use_lora=args.use_lora)
        self.dynamic_start_layer = args.dynamic_start_layer
        if self.use_reslr and layer_id >= args.dynamic_start_layer:
            self.block_size = args.block_size
            rel = layer_id - args.dynamic_start_layer
            self.is_block_head = rel % self.block_size == 0
            self.current_block_id = rel // self.block_size
            self.block_start_layer = args.dynamic_start_layer + self.current_block_id * self.block_size
            self.current_block_pos = layer_id - self.block_start_layer
            if self.is_block_head:
                self.router = RouterModule(args.dim, args.dynamic_router_hdim, args.dynamic_reserve_initials,
                                           args.norm_eps, block_size=self.block_size, use_lora=args.use_lora)
                self.block_path_approximators = BlockPathApproximators(args.dim, args.low_rank_dim, self.block_size)

    def takes_fused_path(self, x):
        """whether this layer consumes x only through fused nodes (the layer node and, on a block head, the fused
        router), whose backwards return gradients no other input shares"""
        if not (self.fused and x.dim() == 3 and x.is_cuda and _fused.supported(self)):
            return False
        if self.use_reslr and self.layer_id >= self.dynamic_start_layer and self.is_block_head:
            return bool(self.router.fused_mlp and _fused.router_net_supported(self.router, x))
        return True

    def _full(self, x, packed=False, active=None):
        """the full layer; with `active` (bool [B, N, 1]) where(active, layer(x), x), the routed student's rows"""
        if self.fused and x.dim() == 3 and x.is_cuda and _fused.supported(self):
            # one fused node (LoRA configuration, vitmi.resvit_fused), the row selection folded in
            return _fused.full_layer(self, x, packed, active)
        h = HF.add(self.attention(self.attention_norm(x)), x)
        out = HF.add(self.feed_forward(self.ffn_norm(h)), h)
        return out if active is None else _select_rows(active, out, x)

    def forward(self, x, teacher_x=None, block_info: Optional[Dict] = None, LRA_mask: Optional[List] = None):
        bsz, seqlen, _ = x.shape
        if block_info is None:
            block_info = {}
        if not self.use_reslr or self.layer_id < self.dynamic_start_layer:
            w = torch.ones((bsz, seqlen, 1), device=x.device)
            out = self._full(x)
            return (out, out, w, block_info) if self.training else (out, w, block_info)

        bid = self.current_block_id
        x_in = x  # (the caller's tensor: teacher_x is compared against it below)
        if self.is_block_head:
            if ROUTER_THROUGH and self.training and torch.is_grad_enabled():
                x, (routing, router_indices, router_entropy, soft_routing) = self.router.forward_through(x)
            else:
                routing, router_indices, router_entropy, soft_routing = self.router(x)
            block_info = {f"block_{bid}_approximators": self.block_path_approximators,
                          f"block_{bid}_routing": routing[:, :, :, 1],
                          f"block_{bid}_router_indices": router_indices,
                          f"block_{bid}_router_entropy": router_entropy,
                          f"block_{bid}_soft_routing": soft_routing[:, :, :, 1]}
            if (FUSED_SELECT and LRA_mask is not None and router_indices.is_cuda
                    and router_indices.dtype == torch.float32 and self.block_size <= 5):
                block_info[f"block_{bid}_select"] = _ops.router_select(
                    router_indices.reshape(-1).contiguous(), [LRA_mask[j][1] for j in range(self.block_size)],
                    2 ** self.block_size - 1)
        approximators = block_info[f"block_{bid}_approximators"]
        block_routing = block_info[f"block_{bid}_routing"]
        router_indices = block_info[f"block_{bid}_router_indices"]
        w = block_routing[:, :, self.current_block_pos:self.current_block_pos + 1]
        assert LRA_mask is not None, "LRA_mask must be provided"
        lra_lora = list(LRA_mask[self.current_block_pos][0])
        sel_info = block_info.get(f"block_{bid}_select")
        if sel_info is not None:
            active = sel_info[0][self.current_block_pos].view(bsz, seqlen, 1)
        else:
            active = torch.isin(router_indices.long(), _const(tuple(LRA_mask[self.current_block_pos][1]), x.device,
                                                              torch.int64))

        if self.training:
            if (SHARE_TEACHER and (teacher_x is None or teacher_x is x_in) and self.fused and x.dim() == 3 and x.is_cuda
                    and _fused.supported(self) and not _active_dropout(self)):
                # the teacher's input is the student's (the first routed layer): one layer forward serves both
                teacher_out, student_out = _fused.teacher_and_student(self, x, active)
                return teacher_out, approximators(student_out, router_indices, lra_lora, sel_info), w, block_info
            # teacher: every token, every layer. Its outputs reach the loss only through DistillLoss's
            # .detach() (res-vit/model.py:40-59), so no gradient flows through it: run without autograd
            with torch.no_grad():
                teacher_out = self._full(x if teacher_x is None else teacher_x)
            # same block, same LoRA weights: the teacher pass's operand pack serves the student pass
            if FOLD_SELECT:
                student_out = self._full(x, packed=True, active=active)
            else:  # A/B (bench.py VITMI_RESVIT_WHERE_OPS=1): the layer node, then torch.where
                student_out = _select_rows(active, self._full(x, packed=True), x)
            return teacher_out, approximators(student_out, router_indices, lra_lora, sel_info), w, block_info

        # inference: only the active tokens query (ragged), every token is a key / value
        x_normed = self.attention_norm(x)
        amask = active.squeeze(-1)
        counts = amask.sum(dim=1)
        cu = torch.zeros(bsz + 1, device=x.device, dtype=torch.int32)
        cu[1:] = torch.cumsum(counts, 0)
        max_q = int(counts.max()) if bsz else 0
        h = x.clone()
        if max_q > 0:
            attn_rows = self.attention.forward_ragged(x_normed[amask], x_normed, cu, max_q)
            h[amask] = HF.add(attn_rows, x[amask])
        output = HF.add(self.feed_forward(self.ffn_norm(h)), h)
        student_out = _select_rows(active, output, x)
        return approximators(student_out, router_indices, lra_lora), w, block_info


class Transformer(nn.Module):
    """res-vit/model.py:532-702: forward(x, labels) -> (c_loss, a_loss, d_loss, router_entropy, active_metric)."""

    def __init__(self, params: ModelArgs):
        super().__init__()
        self.device = params.device
        h, w = params.image_size
        fh, fw = params.patch_size
        if h != w or fh != fw:
            raise NotImplementedError("vitmi Res-ViT supports square images and patches")
        params.num_patches = (h // fh) * (w // fw)
        self.patch = fh
        self.embedding = nn.Conv2d(3, params.dim, kernel_size=(fh, fw), stride=(fh, fw))
        self.cls_token = nn.Parameter(torch.zeros(1, 1, params.dim))
        self.pos_embedding = PositionEmbs(params.num_patches, params.dim)
        self.criterion = CrossEntropyLoss()
        self.criterion_active = ActiveLoss(target=params.dynamic_active_target,
                                           reserve_initials=params.dynamic_reserve_initials)
        self.criterion_distill = DistillLoss()
        self.n_layers = params.n_layers
        self.layers = nn.ModuleList([TransformerBlock(i, params) for i in range(params.n_layers)])
        self.norm = LayerNorm(params.dim, eps=params.norm_eps, use_lora=params.use_lora)
        self.classifier = Linear(params.dim, params.num_classes)
        self.use_lora = params.use_lora
        self.use_reslr = params.use_reslr
        if self.use_lora:  # base weights frozen (res-vit/model.py:573-584)
            for name, param in self.named_parameters():
                if (name.startswith("embedding.") or name.startswith("pos_embedding.") or ".feed_forward." in name
                        or ".attention.wo." in name or ".attention.wq." in name or ".attention.wk." in name
                        or ".attention.wv." in name):
                    param.requires_grad = False
        if self.use_reslr:
            self.LRA_mask = get_indices_from_LRA_mask(params.block_size)

    def embed(self, x):
        """patch embedding Conv2d(k = s = P) as im2col + the bf16 MFMA GEMM, token-major [B, n, D]."""
        return HF.patch_embed(x, self.embedding.weight, self.embedding.bias, self.patch)

    def forward(self, x: torch.Tensor, labels: torch.Tensor):
        device = self.cls_token.device
        x, labels = x.to(device), labels.to(device)
        if FUSED_EMBED and _fused.embed_supported(self, x):
            x = _fused.embed_tokens(self, x)  # conv + cls + position embeddings: one GEMM (PATCH epilogue)
        else:
            x = self.embed(x)
            x = torch.cat([self.cls_token.expand(x.shape[0], 1, -1), x], dim=1)
            x = self.pos_embedding(x)
        self.acts = []
        self.soft_routing_probs = []
        self.routing_maps = {}
        d_loss = torch.zeros((), device=device)
        r_entropy = torch.zeros((), device=device)
        block_info = {}
        teacher_x, student_x = x, x
        for li, layer in enumerate(self.layers):
            if self.use_reslr and layer.layer_id >= layer.dynamic_start_layer:
                if self.training:
                    teacher_out, student_out, w, block_info = layer(student_x, teacher_x, block_info, self.LRA_mask)
                    # the cls nodes may add into the incoming gradient in place only when every consumer of their
                    # output returns a fresh gradient: the next layer's fused node (and router), or the final norm
                    nxt = self.layers[li + 1] if li + 1 < len(self.layers) else None
                    inplace = nxt is None or nxt.takes_fused_path(student_out)
                    if (FUSED_DISTILL and CLS_TAP and student_out.is_cuda and student_out.dtype == torch.float32
                            and teacher_out.dtype == torch.float32 and type(self.criterion_distill) is DistillLoss):
                        student_out, dl = _fused.cls_distill(student_out, teacher_out, inplace)
                        d_loss = d_loss + dl
                    else:
                        if CLS_TAP and student_out.is_cuda:
                            student_out, s_cls = _fused.cls_tap(student_out, inplace)
                        else:
                            s_cls = student_out[:, 0, :]
                        d_loss = d_loss + self.criterion_distill(s_cls, teacher_out[:, 0, :])
                    if layer.is_block_head:
                        bid = layer.current_block_id
                        r_entropy = r_entropy + block_info[f"block_{bid}_router_entropy"]
                        self.routing_maps[bid] = block_info[f"block_{bid}_routing"].detach()
                        self.soft_routing_probs.append(block_info[f"block_{bid}_soft_routing"])
                    teacher_x, student_x = teacher_out, student_out
                else:
                    student_x, w, block_info = layer(student_x, None, block_info, self.LRA_mask)
                    if layer.is_block_head:
                        bid = layer.current_block_id
                        r_entropy = r_entropy + block_info[f"block_{bid}_router_entropy"]
                        self.routing_maps[bid] = block_info[f"block_{bid}_routing"].detach()
            else:
                if self.training:
                    teacher_x, student_x, w, block_info = layer(student_x, teacher_x, block_info)
                else:
                    student_x, w, block_info = layer(student_x, None, block_info)
            self.acts.append(w)
        # the final LayerNorm is row-local and only the cls row reaches the classifier (res-vit/model.py:686-689):
        # normalise that row alone (same values; the other rows' zero gradient through the norm is exactly zero)
        if CLS_TAP:
            student_x = self.norm(student_x[:, 0:1])
        else:
            student_x = self.norm(student_x)
        activation = torch.cat(self.acts, dim=-1)
        output = self.classifier(student_x[:, 0])
        self.logits = output
        c_loss = self.criterion(output, labels)
        if self.use_reslr:
            a_loss = (self.criterion_active(torch.cat(self.soft_routing_probs, dim=-1)) if self.soft_routing_probs
                      else torch.zeros((), device=device))
            active_metric = self.criterion_active.metric(activation)
        else:
            a_loss, active_metric = None, None
            r_entropy = torch.zeros((), device=device)
        return c_loss, a_loss, d_loss, r_entropy, active_metric
