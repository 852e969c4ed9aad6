"""CPU oracle for the ViT training step — TEST INFRASTRUCTURE ONLY.

This module is the parity checker for the MI355X HIP path. It is a plain
PyTorch-CPU fp32 (or fp64) restatement, written independently, of the
reference's hot path:

  * VisionTransformer.__init__ RNG order      reference src/model.py:161-194
  * VisionTransformer.forward                 reference src/model.py:196-211
  * PositionEmbs / Encoder / EncoderBlock     reference src/model.py:7-22, 104-156
  * SelfAttention (LinearGeneral weights)     reference src/model.py:54-101
  * MlpBlock (exact-erf GELU)                 reference src/model.py:25-51
  * CrossEntropyLoss (mean)                   reference src/train.py:151,22
  * SGD(momentum, weight_decay) step          reference src/train.py:154-158 (torch SGD semantics)
  * OneCycleLR (cos anneal, cycle_momentum)   reference src/train.py:159-163 (torch OneCycleLR semantics)
  * top-k accuracy                            reference src/utils.py:28-41

Pinning: the restatement is checked against golden vectors produced by the
imported reference (tests/golden/make_golden.py -> tests/golden/*.npz/json):
constructor checksums (bit-exact), tiny-config logits/loss/grads/3-step
trajectory, ViT-B/16 tamed-init logits/loss/grad-norms, and a OneCycleLR
trace. See tests/test_oracle.py.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this file. The product path (vit-of-pytorch_amd/vitmi) never does.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from dataclasses import dataclass

import torch
import torch.nn.functional as F


@dataclass
class ViTConfig:
    image_size: int = 224
    patch_size: int = 16
    emb_dim: int = 768
    mlp_dim: int = 3072
    num_heads: int = 12
    num_layers: int = 12
    num_classes: int = 1000

    @property
    def grid(self) -> int:
        # Conv2d(k=s=P) floors non-divisible sizes (reference src/model.py:174-178)
        return self.image_size // self.patch_size

    @property
    def num_tokens(self) -> int:
        return self.grid * self.grid + 1

    @property
    def head_dim(self) -> int:
        return self.emb_dim // self.num_heads


# Arch presets: reference src/config.py:57-104
PRESETS = {
    "b16": dict(patch_size=16, emb_dim=768, mlp_dim=3072, num_heads=12, num_layers=12),
    "b32": dict(patch_size=32, emb_dim=768, mlp_dim=3072, num_heads=12, num_layers=12),
    "l16": dict(patch_size=16, emb_dim=1024, mlp_dim=4096, num_heads=16, num_layers=24),
    "l32": dict(patch_size=32, emb_dim=1024, mlp_dim=4096, num_heads=16, num_layers=24),
    "h14": dict(patch_size=14, emb_dim=1280, mlp_dim=5120, num_heads=16, num_layers=32),
}


def param_names(cfg: ViTConfig):
    """state_dict key order of the reference (reference src/model.py:161-194)."""
    names = ["cls_token", "embedding.weight", "embedding.bias", "transformer.pos_embedding.pos_embedding"]
    for i in range(cfg.num_layers):
        p = f"transformer.encoder_layers.{i}."
        names += [p + "norm1.weight", p + "norm1.bias"]
        for w in ("query", "key", "value", "out"):
            names += [p + f"attn.{w}.weight", p + f"attn.{w}.bias"]
        names += [p + "norm2.weight", p + "norm2.bias"]
        names += [p + "mlp.fc1.weight", p + "mlp.fc1.bias", p + "mlp.fc2.weight", p + "mlp.fc2.bias"]
    names += ["transformer.norm.weight", "transformer.norm.bias", "classifier.weight", "classifier.bias"]
    return names


def init_params(cfg: ViTConfig, seed: int | None = 42) -> "OrderedDict[str, torch.Tensor]":
    """Draw parameters from torch's CPU RNG in the reference constructor's order.

    Order (reference src/model.py:161-194, module construction order):
      1. embedding Conv2d(3, D, P, P): kaiming_uniform(a=sqrt(5)) weight, U(+-1/sqrt(fan_in)) bias
      2. cls_token zeros                                   (:181)
      3. PositionEmbs randn(1, N, D)                       (:10)
      4. per layer: LayerNorm (no draw), q/k/v randn(D,H,hd) + zero bias, out randn(H,hd,D) + zero bias
         (:58-59, 73-76), LayerNorm, fc1 Linear(D,M), fc2 Linear(M,D)  (:31-32)
      5. final LayerNorm (no draw)                          (:146)
      6. classifier Linear(D, C)                            (:194)
    The parameter draws go through torch.nn's own initialisers (not reference code).
    """
    if seed is not None:
        torch.manual_seed(seed)
    D, M, H, P = cfg.emb_dim, cfg.mlp_dim, cfg.num_heads, cfg.patch_size
    hd = D // H
    out = OrderedDict()
    conv = torch.nn.Conv2d(3, D, kernel_size=(P, P), stride=(P, P))
    cls = torch.zeros(1, 1, D)
    pos = torch.randn(1, cfg.num_tokens, D)
    out["cls_token"] = cls
    out["embedding.weight"] = conv.weight.detach().clone()
    out["embedding.bias"] = conv.bias.detach().clone()
    out["transformer.pos_embedding.pos_embedding"] = pos
    for i in range(cfg.num_layers):
        p = f"transformer.encoder_layers.{i}."
        out[p + "norm1.weight"] = torch.ones(D)
        out[p + "norm1.bias"] = torch.zeros(D)
        for w in ("query", "key", "value"):
            out[p + f"attn.{w}.weight"] = torch.randn(D, H, hd)
            out[p + f"attn.{w}.bias"] = torch.zeros(H, hd)
        out[p + "attn.out.weight"] = torch.randn(H, hd, D)
        out[p + "attn.out.bias"] = torch.zeros(D)
        out[p + "norm2.weight"] = torch.ones(D)
        out[p + "norm2.bias"] = torch.zeros(D)
        fc1 = torch.nn.Linear(D, M)
        fc2 = torch.nn.Linear(M, D)
        out[p + "mlp.fc1.weight"] = fc1.weight.detach().clone()
        out[p + "mlp.fc1.bias"] = fc1.bias.detach().clone()
        out[p + "mlp.fc2.weight"] = fc2.weight.detach().clone()
        out[p + "mlp.fc2.bias"] = fc2.bias.detach().clone()
    out["transformer.norm.weight"] = torch.ones(D)
    out["transformer.norm.bias"] = torch.zeros(D)
    head = torch.nn.Linear(D, cfg.num_classes)
    out["classifier.weight"] = head.weight.detach().clone()
    out["classifier.bias"] = head.bias.detach().clone()
    # reorder to the state_dict key order
    return OrderedDict((k, out[k]) for k in param_names(cfg))


def tame_params(params: "OrderedDict[str, torch.Tensor]", seed: int = 1) -> "OrderedDict[str, torch.Tensor]":
    """Deterministic well-conditioned rescale (SURVEY.md §8c parity protocol).

    Under the reference's std-1 init the forward is chaotic (fp32 vs fp64
    logits differ 85%), so parity is measured after this rescale:
    q/k/v/out weights <- randn(gen)/sqrt(D) and pos-emb, classifier.weight
    <- 0.02*randn(gen), in named-parameter order, gen = Generator(seed).
    """
    g = torch.Generator().manual_seed(seed)
    out = OrderedDict()
    for k, v in params.items():
        if ".attn." in k and k.endswith(".weight"):
            D = v.shape[0] if not k.endswith("out.weight") else v.shape[-1]
            out[k] = torch.randn(v.shape, generator=g) / math.sqrt(D)
        elif k == "transformer.pos_embedding.pos_embedding" or k == "classifier.weight":
            out[k] = 0.02 * torch.randn(v.shape, generator=g)
        else:
            out[k] = v.clone()
    return out


# ---- per-block restatements (the standalone sub-module forwards of reference src/model.py) ----------
def position_embs(x, pos):
    """PositionEmbs.forward without dropout (reference src/model.py:16-22): x + pos_embedding."""
    return x + pos


def linear_general(x, w, b, n_in):
    """LinearGeneral.forward (reference src/model.py:61-63) for dims = (trailing n_in dims of x,
    leading n_in dims of w): tensordot(x, w, dims) + b."""
    k = math.prod(w.shape[:n_in])
    out_shape = tuple(x.shape[:x.dim() - n_in]) + tuple(w.shape[n_in:])
    return (x.reshape(-1, k) @ w.reshape(k, -1) + b.reshape(-1)).reshape(out_shape)


def attention_core(q, k, v):
    """SelfAttention.forward's core (reference src/model.py:90-97): q, k, v [b, n, H, hd] ->
    softmax((q k^T) / sqrt(hd)) v, [b, n, H, hd]; the scores are divided AFTER the matmul (:94)."""
    hd = q.shape[-1]
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    s = (q @ k.transpose(-2, -1)) / (hd ** 0.5)
    return (torch.softmax(s, dim=-1) @ v).transpose(1, 2)


def self_attention(p, pre, x):
    """SelfAttention.forward (reference src/model.py:83-101); p[pre + 'query.weight'] etc."""
    q = linear_general(x, p[pre + "query.weight"], p[pre + "query.bias"], 1)
    k = linear_general(x, p[pre + "key.weight"], p[pre + "key.bias"], 1)
    v = linear_general(x, p[pre + "value.weight"], p[pre + "value.bias"], 1)
    return linear_general(attention_core(q, k, v), p[pre + "out.weight"], p[pre + "out.bias"], 2)


def mlp_block(p, pre, x, d1=None, d2=None):
    """MlpBlock.forward (reference src/model.py:41-51): fc1 -> exact-erf GELU -> [dropout1] -> fc2 ->
    [dropout2]; d1 / d2 optional dropout multipliers."""
    g = F.gelu(F.linear(x, p[pre + "fc1.weight"], p[pre + "fc1.bias"]))
    if d1 is not None:
        g = g * d1
    y = F.linear(g, p[pre + "fc2.weight"], p[pre + "fc2.bias"])
    return y * d2 if d2 is not None else y


def encoder_block(p, pre, h, da=None, d1=None, d2=None):
    """EncoderBlock.forward (reference src/model.py:117-130), pre-LN, eps 1e-5, in-place residuals."""
    D = h.shape[-1]
    y = F.layer_norm(h, (D,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], 1e-5)
    o = self_attention(p, pre + "attn.", y)
    h = h + (o * da if da is not None else o)
    y = F.layer_norm(h, (D,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], 1e-5)
    return h + mlp_block(p, pre + "mlp.", y, d1, d2)


def encoder(p, pre, x, num_layers, drop=None):
    """Encoder.forward (reference src/model.py:148-156): position embedding, blocks, final LayerNorm
    over every token. drop: as for forward()."""
    g = (lambda key: drop[key]) if drop else (lambda key: None)
    h = position_embs(x, p[pre + "pos_embedding.pos_embedding"])
    if drop:
        h = h * drop["pos"]
    for i in range(num_layers):
        q_ = f"{pre}encoder_layers.{i}."
        h = encoder_block(p, q_, h, g(("attn", i)), g(("d1", i)), g(("d2", i)))
    D = h.shape[-1]
    return F.layer_norm(h, (D,), p[pre + "norm.weight"], p[pre + "norm.bias"], 1e-5)


def forward(params, x: torch.Tensor, cfg: ViTConfig, drop=None) -> torch.Tensor:
    """Functional ViT forward (reference src/model.py:196-211 and the modules it calls).

    drop: optional train-mode dropout multipliers (0 or 1/(1-p)), applied where nn.Dropout sits in
    the reference: drop["pos"] [b, n, D] after the position embedding (:19-20); per layer i
    drop[("attn", i)] [b, n, D] on the attention output (:124-125), drop[("d1", i)] [b, n, M] after
    GELU (:46-47) and drop[("d2", i)] [b, n, D] after fc2 (:50-51)."""
    D = cfg.emb_dim
    p = params
    # patch embedding: Conv2d(k=s=P) (reference :179,197), token-major (:198-200)
    emb = F.conv2d(x, p["embedding.weight"], p["embedding.bias"], stride=cfg.patch_size)
    b = emb.shape[0]
    emb = emb.permute(0, 2, 3, 1).reshape(b, -1, D)
    # prepend cls (:203-204), then the encoder (:207; PositionEmbs, blocks, final LN)
    h = torch.cat([p["cls_token"].expand(b, 1, D), emb], dim=1)
    h = encoder(p, "transformer.", h, cfg.num_layers, drop)
    # classifier on the cls row (:210)
    return F.linear(h[:, 0], p["classifier.weight"], p["classifier.bias"])


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """mean over batch of -log_softmax[y] (nn.CrossEntropyLoss(), reference src/train.py:151)."""
    lse = torch.logsumexp(logits, dim=-1)
    return (lse - logits.gather(1, labels.view(-1, 1)).squeeze(1)).mean()


def loss_and_grads(params, x, labels, cfg: ViTConfig, dtype=torch.float32, drop=None):
    """Forward + CE + backward on CPU. Returns (logits, loss, grads OrderedDict)."""
    leaves = OrderedDict((k, v.detach().to(dtype).clone().requires_grad_(True)) for k, v in params.items())
    logits = forward(leaves, x.to(dtype), cfg, drop=drop)
    loss = cross_entropy(logits, labels)
    loss.backward()
    grads = OrderedDict((k, v.grad.detach().clone()) for k, v in leaves.items())
    return logits.detach(), loss.detach(), grads


class OneCycle:
    """OneCycleLR(max_lr, pct_start, total_steps), defaults anneal='cos', div_factor=25,
    final_div_factor=1e4, cycle_momentum=True (base 0.85, max 0.95), three_phase=False.
    Restates torch.optim.lr_scheduler.OneCycleLR as driven by reference src/train.py:159-163.
    """

    def __init__(self, max_lr, total_steps, pct_start, div_factor=25.0, final_div_factor=1e4,
                 base_momentum=0.85, max_momentum=0.95):
        self.initial_lr = max_lr / div_factor
        self.max_lr = max_lr
        self.min_lr = self.initial_lr / final_div_factor
        self.total_steps = total_steps
        self.phase_end = [float(pct_start * total_steps) - 1, float(total_steps - 1)]
        self.base_m, self.max_m = base_momentum, max_momentum

    @staticmethod
    def _cos(start, end, pct):
        return end + (start - end) / 2.0 * (math.cos(math.pi * pct) + 1)

    def at(self, step: int):
        """(lr, momentum) used by the optimizer step number `step` (0-based)."""
        start = 0.0
        phases = [(self.initial_lr, self.max_lr, self.max_m, self.base_m),
                  (self.max_lr, self.min_lr, self.base_m, self.max_m)]
        for i, (lr0, lr1, m0, m1) in enumerate(phases):
            end = self.phase_end[i]
            if step <= end or i == len(phases) - 1:
                pct = (step - start) / (end - start)
                return self._cos(lr0, lr1, pct), self._cos(m0, m1, pct)
            start = end
        raise AssertionError


def sgd_step(params, grads, bufs, lr, momentum, weight_decay, first: bool):
    """torch.optim.SGD (dampening 0, nesterov False) as used by reference src/train.py:154-158:
    d = g + wd*p; buf = d (first step) else momentum*buf + d; p -= lr*buf."""
    for k in params:
        d = grads[k] + weight_decay * params[k] if weight_decay != 0 else grads[k]
        if first:
            bufs[k] = d.clone()
        else:
            bufs[k].mul_(momentum).add_(d)
        params[k] = params[k] - lr * bufs[k]
    return params, bufs


def accuracy(logits: torch.Tensor, target: torch.Tensor, topk=(1,)):
    """top-k accuracy in percent (reference src/utils.py:28-41)."""
    maxk = max(topk)
    _, pred = logits.topk(maxk, 1, True, True)
    correct = pred.t().eq(target.view(1, -1).expand(maxk, -1))
    return [correct[:k].reshape(-1).float().sum(0) / target.size(0) * 100.0 for k in topk]


def train_flops_per_image(cfg: ViTConfig) -> float:
    """Algorithmic train FLOPs per image = 3*fwd - patch-embed fwd (matmul/conv MACs x2)."""
    D, M, C, P = cfg.emb_dim, cfg.mlp_dim, cfg.num_classes, cfg.patch_size
    n = cfg.grid * cfg.grid
    N = n + 1
    patch = 2 * n * 3 * P * P * D
    fwd = patch + cfg.num_layers * 2 * (3 * N * D * D + 2 * N * N * D + N * D * D + 2 * N * D * M) + 2 * D * C
    return 3 * fwd - patch
