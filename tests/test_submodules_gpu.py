"""Standalone sub-module forwards/backwards (reference src/model.py:7-156) on the HIP kernels vs the
oracle's per-block restatements (oracle/vit_oracle.py position_embs / linear_general / self_attention /
mlp_block / encoder_block / encoder), fp32 CPU autograd. GPU only.

Tolerances (bf16 operands, f32 accumulation): outputs relative Frobenius error
<= 1e-2, every gradient <= 3e-2 (attn key bias: true gradient 0 by softmax shift invariance, compared
with an absolute bound against the largest gradient).
"""
import math

import pytest
import torch

from oracle import vit_oracle as O

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _tame(module, seed=0):
    """well-conditioned weights (the tamed-init protocol): LinearGeneral weights randn/sqrt(fan-in),
    everything else its constructor draw, LayerNorm affine perturbed so it is exercised."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in module.named_parameters():
            if "query" in n or "key" in n or "value" in n or n.endswith("out.weight") or n.endswith("out.bias"):
                if n.endswith("weight"):
                    fan = p.shape[0] if "out" not in n else p.shape[0] * p.shape[1]
                    p.copy_(torch.randn(p.shape, generator=g) / math.sqrt(fan))
                else:
                    p.copy_(0.1 * torch.randn(p.shape, generator=g))
            elif "norm" in n:
                p.copy_((1.0 if n.endswith("weight") else 0.0) + 0.1 * torch.randn(p.shape, generator=g))
            elif "pos_embedding" in n:
                p.copy_(0.02 * torch.randn(p.shape, generator=g))
    return module


def _compare(mod, ref_fn, x, key_bias_names=()):
    """run mod(x) on the GPU and ref_fn(params, x) on the CPU; compare output, dx and every param grad."""
    torch.manual_seed(1)
    gy = None
    params = {n: p.detach().clone().requires_grad_(True) for n, p in mod.named_parameters()}
    xr = x.detach().clone().requires_grad_(True)
    yr = ref_fn(params, xr)
    gy = torch.randn(yr.shape)
    (yr * gy).sum().backward()
    md = mod.cuda()
    xg = x.detach().cuda().requires_grad_(True)
    y = md(xg)
    (y * gy.cuda()).sum().backward()
    assert y.shape == yr.shape
    assert rel(y, yr) < 1e-2, rel(y, yr)
    assert rel(xg.grad, xr.grad) < 3e-2, rel(xg.grad, xr.grad)
    gmax = max(float(p.grad.abs().max()) for p in params.values())
    for n, p in md.named_parameters():
        assert p.grad is not None, n
        if any(n.endswith(k) for k in key_bias_names):
            assert float((p.grad.cpu() - params[n].grad).abs().max()) <= 1e-2 * gmax, n
        else:
            assert rel(p.grad, params[n].grad) < 3e-2, (n, rel(p.grad, params[n].grad))


@pytest.mark.parametrize("n_in", [1, 2])
def test_linear_general(n_in):
    from vitmi.model import LinearGeneral
    torch.manual_seed(3)
    if n_in == 1:   # q/k/v: x [b, n, D] . W [D, H, hd] over dims ([2], [0])
        m, x, dims = LinearGeneral((64,), (2, 32)), torch.randn(2, 17, 64), ([2], [0])
    else:           # out: x [b, n, H, hd] . W [H, hd, D] over dims ([2, 3], [0, 1])
        m, x, dims = LinearGeneral((2, 32), (96,)), torch.randn(2, 17, 2, 32), ([2, 3], [0, 1])
    with torch.no_grad():
        m.weight.mul_(1.0 / 8.0)
        m.bias.normal_()
    fan = m.weight.shape[:n_in]

    class Wrap(torch.nn.Module):
        def __init__(self, lg):
            super().__init__()
            self.lg = lg

        def forward(self, x):
            return self.lg(x, dims=dims)
    _compare(Wrap(m), lambda p, x: O.linear_general(x, p["lg.weight"], p["lg.bias"], len(fan)), x)


def test_nn_leaves_linear_layernorm_gelu():
    from vitmi.model import GELU, LayerNorm, Linear
    torch.manual_seed(4)
    seq = torch.nn.Sequential(LayerNorm(96), Linear(96, 200), GELU(), Linear(200, 72))
    with torch.no_grad():
        seq[0].weight.normal_(1.0, 0.1)
        seq[0].bias.normal_(0.0, 0.1)
    ref = lambda p, x: torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(
        torch.nn.functional.layer_norm(x, (96,), p["0.weight"], p["0.bias"], 1e-5), p["1.weight"], p["1.bias"])),
        p["3.weight"], p["3.bias"])
    _compare(seq, ref, torch.randn(5, 7, 96) * 3 + 1)


def test_position_embs():
    from vitmi.model import PositionEmbs
    torch.manual_seed(5)
    m = _tame(PositionEmbs(16, 64, dropout_rate=0.0))
    _compare(m, lambda p, x: O.position_embs(x, p["pos_embedding"]), torch.randn(3, 17, 64))


def test_mlp_block():
    from vitmi.model import MlpBlock
    torch.manual_seed(6)
    m = MlpBlock(128, 256, 128, dropout_rate=0.0)
    _compare(m, lambda p, x: O.mlp_block(p, "", x), torch.randn(2, 17, 128))


@pytest.mark.parametrize("n", [17, 197, 325])  # 325 tokens > 320: the K/V-tiled attention kernels
def test_self_attention(n):
    from vitmi.model import SelfAttention
    torch.manual_seed(7)
    m = _tame(SelfAttention(128, heads=2, dropout_rate=0.0))
    _compare(m, lambda p, x: O.self_attention(p, "", x), torch.randn(2, n, 128), key_bias_names=("key.bias",))


def test_encoder_block():
    from vitmi.model import EncoderBlock
    torch.manual_seed(8)
    m = _tame(EncoderBlock(128, 256, 2, dropout_rate=0.0, attn_dropout_rate=0.0))
    _compare(m, lambda p, x: O.encoder_block(p, "", x), torch.randn(2, 33, 128), key_bias_names=("key.bias",))


def test_encoder():
    from vitmi.model import Encoder
    torch.manual_seed(9)
    m = _tame(Encoder(16, 128, 256, num_layers=2, num_heads=2, dropout_rate=0.0, attn_dropout_rate=0.0))
    _compare(m, lambda p, x: O.encoder(p, "", x, 2), torch.randn(2, 17, 128), key_bias_names=("key.bias",))


def test_encoder_matches_whole_model_engine():
    """model.transformer(...) standalone equals the fused engine's encoder inside VisionTransformer.forward:
    the classifier applied to the standalone encoder's cls row reproduces the fused logits."""
    from vitmi.model import VisionTransformer
    torch.manual_seed(42)
    m = VisionTransformer(image_size=(32, 32), patch_size=(8, 8), emb_dim=128, mlp_dim=256, num_heads=2,
                          num_layers=2, num_classes=10, dropout_rate=0.0)
    cfg = O.ViTConfig(image_size=32, patch_size=8, emb_dim=128, mlp_dim=256, num_heads=2, num_layers=2,
                      num_classes=10)
    m.load_state_dict(O.tame_params(O.init_params(cfg, seed=42)))
    m = m.cuda()
    x = torch.randn(3, 3, 32, 32, generator=torch.Generator().manual_seed(2)).cuda()
    with torch.no_grad():
        fused = m(x)
        emb = m.embedding(x).permute(0, 2, 3, 1).reshape(3, -1, 128)
        h = torch.cat([m.cls_token.expand(3, 1, 128), emb], dim=1)
        feat = m.transformer(h)
        logits = m.classifier(feat[:, 0])
    assert rel(logits, fused) < 1e-2


def test_dropout_train_mode_mask_and_backward():
    from vitmi.model import Dropout
    d = Dropout(0.25).cuda().train()
    x = (torch.rand(64, 256) + 0.5).cuda().requires_grad_(True)
    y = d(x)
    mult = (y / x).detach()
    kept = mult != 0
    assert abs(float(kept.float().mean()) - 0.75) < 0.02
    assert torch.allclose(mult[kept], torch.full_like(mult[kept], 1 / 0.75))
    g = torch.randn_like(x)
    y.backward(g)
    assert torch.allclose(x.grad, g * mult)
    d.eval()
    assert torch.equal(d(x), x)
