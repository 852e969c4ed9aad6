"""Train-mode dropout on the HIP path (GPU only).

nn.Dropout's own RNG stream cannot be reproduced (see oracle/dropout.py), so parity is checked in
two layers: (1) every kernel that applies or back-propagates a mask uses exactly the masks of the
oracle's Philox restatement (bit-exact masks, per-kernel numerics against PyTorch fp32 with those
masks); (2) a whole training step with dropout_rate 0.1 matches the oracle forward/backward run
with the same masks, at the bf16-step tolerances of tests/test_parity_gpu.py."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle.dropout import dropout_mult
from oracle.vit_oracle import ViTConfig, init_params, loss_and_grads, tame_params
from vitmi import ops
from vitmi._lib import EPI_BIAS_GELU_DGELU, EPI_BIAS_RESID_F32, EPI_PATCH, K_CONTIG

DEV = "cuda"
SEED, OFF = 0x1234_5678_9ABC_DEF1, 0x2_0000_0007


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def mult(site, rows, cols, row0=0, row_stride=1, p=0.1):
    return torch.from_numpy(dropout_mult(p, site, SEED, OFF, rows, cols, row0, row_stride)).to(DEV)


def test_mask_kernel_matches_oracle():
    d = ops.dropout_desc(0.1, 5, SEED, OFF)
    out = torch.empty(300, 136, device=DEV)
    ops.dropout_mask(d, 1000, 300, 130, out, 136)
    assert torch.equal(out[:, :130], mult(5, 300, 130, row0=1000))
    d = ops.dropout_desc(0.25, 2, SEED, OFF, row_stride=197)
    out = torch.empty(8, 64, device=DEV)
    ops.dropout_mask(d, 0, 8, 64, out, 64)
    assert torch.equal(out, mult(2, 8, 64, row_stride=197, p=0.25))


@pytest.mark.parametrize("M,N,K", [(700, 512, 256), (50432, 768, 64)])
def test_gemm_epilogue_dropout(M, N, K):
    """BIAS_RESID_F32 (incl. the wave-split launch at M = 50432) and BIAS_GELU_DGELU with masks."""
    A = torch.randn(M, K, device=DEV).bfloat16()
    B = torch.randn(N, K, device=DEV).bfloat16()
    acc = A.float() @ B.float().t()
    bias = torch.randn(N, device=DEV)
    d = ops.dropout_desc(0.1, 4, SEED, OFF)
    mk = mult(4, M, N)
    R = torch.randn(M, N, device=DEV)
    C = R.clone()
    ops.gemm(A, B, C, M, N, K, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=K, ldb=K, ldc=N, epilogue=EPI_BIAS_RESID_F32,
             bias=bias, aux=C, ldaux=N, dropout=d)
    assert rel(C, (acc + bias) * mk + R) < 1e-5
    if M > 10000:
        return
    gp = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    g = torch.empty_like(gp)
    ops.gemm(A, B, gp, M, N, K, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=K, ldb=K, ldc=N,
             epilogue=EPI_BIAS_GELU_DGELU, bias=bias, C2=g, ldc2=N, dropout=d)
    u = (acc + bias).requires_grad_(True)
    ge = torch.nn.functional.gelu(u)
    gd, = torch.autograd.grad(ge.sum(), u)
    assert rel(g.float(), ge.detach() * mk) < 5e-3
    assert rel(gp.float(), gd * mk) < 5e-3


def test_patch_epilogue_dropout():
    tokens, D, Kp = 5, 128, 64
    M = 3 * tokens
    A = torch.randn(M, Kp, device=DEV).bfloat16()
    A[::tokens] = 0
    W = torch.randn(D, Kp, device=DEV).bfloat16()
    bias, pos, cls = torch.randn(D, device=DEV), torch.randn(tokens, D, device=DEV), torch.randn(D, device=DEV)
    C = torch.empty(M, D, device=DEV)
    ops.gemm(A, W, C, M, D, Kp, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=Kp, ldb=Kp, ldc=D, epilogue=EPI_PATCH,
             bias=bias, aux=pos, ldaux=D, aux2=cls, tokens=tokens, dropout=ops.dropout_desc(0.1, 0, SEED, OFF))
    ref = A.float() @ W.float().t() + bias + pos.repeat(3, 1)
    ref[::tokens] = cls + pos[0]
    assert rel(C, ref * mult(0, M, D)) < 1e-5


@pytest.mark.parametrize("stride", [1, 7])
def test_layernorm_bwd_dropout(stride):
    rows, D = 333, 768
    x = torch.randn(rows, D, device=DEV) * 2 + 1
    gam = torch.randn(D, device=DEV)
    mean = x.mean(1)
    rstd = 1.0 / torch.sqrt(x.var(1, unbiased=False) + 1e-5)
    dy = torch.randn(rows, D, device=DEV).bfloat16()
    dx = torch.empty(rows, D, device=DEV)
    dxb = torch.empty(rows, D, device=DEV, dtype=torch.bfloat16)
    part = torch.empty(ops.layernorm_bwd_partial_rows(rows), 3 * D, device=DEV)
    dgb = torch.empty(2 * D, device=DEV)
    dsum = torch.empty(D, device=DEV)
    d = ops.dropout_desc(0.1, 9, SEED, OFF, row_stride=stride)
    ops.layernorm_bwd(dy, D, x, D, mean, rstd, gam, dx, D, part, rows, D, dx_bf16=dxb, lddxb=D, dgamma_dbeta=dgb,
                      dx_colsum=dsum, dx_dropout=d)
    xr = x.clone().requires_grad_(True)
    ref, = torch.autograd.grad(torch.nn.functional.layer_norm(xr, (D,), gam, None, 1e-5), xr, dy.float())
    mk = mult(9, rows, D, row_stride=stride)
    assert rel(dx, ref) < 1e-4                       # the residual gradient itself is not masked
    assert rel(dxb.float(), ref * mk) < 5e-3         # the branch operand is
    assert rel(dsum, (ref * mk).sum(0)) < 1e-4


def test_embed_grad_dropout():
    B, N, D = 3, 17, 64
    dh = torch.randn(B * N, D, device=DEV)
    dpos, dcls, dcb = torch.empty(N, D, device=DEV), torch.empty(D, device=DEV), torch.empty(D, device=DEV)
    ops.embed_grad(dh, B, N, D, dpos, dcls, dcb, dropout=ops.dropout_desc(0.1, 0, SEED, OFF))
    r = (dh * mult(0, B * N, D)).view(B, N, D).sum(0)
    assert rel(dpos, r) < 1e-6 and rel(dcls, r[0]) < 1e-6 and rel(dcb, r[1:].sum(0)) < 1e-6


def test_train_step_with_dropout_matches_oracle():
    """dropout_rate 0.1, train mode: loss / logits / every gradient vs the oracle run with the engine's masks."""
    from vitmi.model import CrossEntropyLoss, VisionTransformer
    cfg = ViTConfig(image_size=32, patch_size=8, emb_dim=64, mlp_dim=128, num_heads=2, num_layers=2, num_classes=10)
    params = tame_params(init_params(cfg, seed=42))
    g = torch.Generator().manual_seed(5)
    bs = 6
    x = torch.randn(bs, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (bs,), generator=g)
    torch.manual_seed(42)
    m = VisionTransformer(image_size=(32, 32), patch_size=(8, 8), emb_dim=64, mlp_dim=128, num_heads=2, num_layers=2,
                          num_classes=10, attn_dropout_rate=0.1, dropout_rate=0.1)
    m.load_state_dict(params)
    m = m.cuda().train()
    logits = m(x.cuda())
    loss = CrossEntropyLoss()(logits, y.cuda())
    loss.backward()
    p, seed, off = m.engine()._drop
    N, D, M = cfg.num_tokens, cfg.emb_dim, cfg.mlp_dim
    T = bs * N
    mk = lambda site, cols: torch.from_numpy(dropout_mult(p, site, seed, off, T, cols)).view(bs, N, cols)
    drop = {"pos": mk(0, D)}
    for i in range(cfg.num_layers):
        drop[("attn", i)] = mk(1 + 3 * i, D)
        drop[("d1", i)] = mk(2 + 3 * i, M)
        drop[("d2", i)] = mk(3 + 3 * i, D)
    kept = float(torch.cat([v.flatten() for v in drop.values()]).gt(0).double().mean())
    assert abs(kept - 0.9) < 0.01
    ref_logits, ref_loss, ref_grads = loss_and_grads(params, x, y, cfg, drop=drop)
    assert rel(logits, ref_logits) < 1e-2
    assert abs(float(loss.detach()) - float(ref_loss)) <= 1e-3 * abs(float(ref_loss))
    tot = math.sqrt(sum(float(v.double().norm()) ** 2 for v in ref_grads.values()))
    named = dict(m.named_parameters())
    for k, gr in ref_grads.items():
        mine = named[k].grad
        if k.endswith("attn.key.bias") or float(gr.double().norm()) < 1e-4 * tot:
            assert float((mine.double().cpu() - gr.double()).norm()) <= 1e-3 * tot, k
        else:
            assert rel(mine, gr) < 3e-2, (k, rel(mine, gr))
    # eval mode: no dropout (deterministic, equals the dropout-free oracle)
    m.eval()
    with torch.no_grad():
        ev = m(x.cuda())
    ref_eval, _, _ = loss_and_grads(params, x, y, cfg)
    assert rel(ev, ref_eval) < 1e-2
