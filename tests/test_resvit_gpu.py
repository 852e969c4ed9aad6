"""Res-ViT (vitmi.resvit) on the MI355X vs the reference res-vit/model.py, through the fixture
tests/golden/resvit_tiny.npz written from the imported reference (tests/golden/make_resvit_golden.py).
GPU only.

Routing decisions are discrete: a token whose router logit margin is below bf16 noise could flip and
send the whole comparison down another path. So the router is checked on its own (its logits from the
reference's recorded router input, and every decision whose margin exceeds that noise), and the
end-to-end checks replay the reference's recorded decisions (and, in training, its Gumbel draws).
Tolerances (bf16 operands, f32 accumulation): logits relative 1e-2, losses 1e-3
relative (router entropy / ratio loss 1e-2: small differences of nearly-saturated probabilities),
every trainable gradient 3e-2 relative or 1e-3 of the global gradient norm when tiny.
"""
import math
import os

import numpy as np
import pytest
import torch

from test_resvit_cpu import TINY

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "resvit_tiny.npz"))


def build(golden):
    from vitmi import resvit
    torch.manual_seed(42)
    m = resvit.Transformer(resvit.ModelArgs(**dict(TINY, device="cuda")))
    m.load_state_dict({k[2:]: torch.from_numpy(golden[k]) for k in golden.files if k.startswith("p/")})
    return m.cuda()


def routers(m):
    return [l.router for l in m.layers if hasattr(l, "router")]


def replay(m, golden, tag):
    """feed the reference's recorded decisions (and Gumbel draws) to the routers, in call order"""
    for j, r in enumerate(routers(m)):
        hard = torch.from_numpy(golden[f"{tag}/router{j}_hard"]).cuda()
        r.hard_override = lambda logits, h=hard: h
        if tag == "train":
            g = torch.from_numpy(golden[f"train/gumbel{j}"]).cuda()
            r.gumbel_noise = lambda logits, g=g: g


@pytest.mark.parametrize("tag,fused", [("eval", False), ("train", False), ("eval", True), ("train", True)])
def test_router_matches_reference(golden, tag, fused):
    """each router on the reference's recorded input: logits within bf16 tolerance, and the same keep
    decision for every token / layer whose reference logit margin exceeds 5% of the logit scale. fused:
    out_conv as one node (vitmi.resvit_fused.router_mlp), its logits read back from the soft routing
    probabilities against the reference's softmax."""
    m = build(golden)
    m.train(tag == "train")
    for j, r in enumerate(routers(m)):
        r.fused_mlp = fused
        x = torch.from_numpy(golden[f"{tag}/router{j}_x"]).cuda()
        ref_logits = torch.from_numpy(golden[f"{tag}/router{j}_logits"])
        if tag == "train":
            g = torch.from_numpy(golden[f"train/gumbel{j}"]).cuda()
            r.gumbel_noise = lambda logits, g=g: g
        seen = {}
        h = r.out_conv.register_forward_hook(lambda mod, i, o: seen.setdefault("logits", o.detach()))
        with torch.no_grad():
            hard, idx, ent, soft = r(x)
        h.remove()
        if fused:
            assert "logits" not in seen  # out_conv's modules did not run
            ref_soft = torch.softmax(ref_logits.view(soft.shape).double(), -1)
            assert rel(soft, ref_soft) < 1e-2
        else:
            assert rel(seen["logits"], ref_logits) < 1e-2
        ref_hard = torch.from_numpy(golden[f"{tag}/router{j}_hard"])
        z = ref_logits.view(*ref_logits.shape[:2], -1, 2).double()
        if tag == "train":
            z = z + torch.from_numpy(golden[f"train/gumbel{j}"]).double()
        margin = (z[..., 1] - z[..., 0]).abs()
        sure = margin > 0.05 * float(z.abs().max())
        sure[:, :1] = True  # the reserved cls token is forced to keep
        assert int(sure.sum()) > 0.8 * sure.numel()
        assert torch.equal(hard.cpu()[..., 1][sure], ref_hard[..., 1][sure]), (tag, j)


def test_eval_ragged_forward_matches_reference(golden):
    """inference: router argmax, ragged attention (active queries, all keys; one varlen launch), FFN,
    approximators on the inactive tokens (res-vit/model.py:494-529)."""
    m = build(golden).eval()
    replay(m, golden, "eval")
    x = torch.from_numpy(golden["x"]).cuda()
    y = torch.from_numpy(golden["y"]).cuda()
    with torch.no_grad():
        c, a, d, ent, metric = m(x, y)
    for k, v in m.routing_maps.items():
        assert torch.equal(v.cpu(), torch.from_numpy(golden[f"eval/routing{k}"])), k
    assert rel(m.logits, golden["eval/logits"]) < 1e-2
    assert abs(float(c) - float(golden["eval/c_loss"])) <= 1e-3 * float(golden["eval/c_loss"])
    assert abs(float(ent) - float(golden["eval/r_entropy"])) <= 1e-2 * abs(float(golden["eval/r_entropy"])) + 1e-6
    assert abs(float(metric["non_low_rank_ratio"]) - float(golden["eval/active_ratio"])) < 1e-6


def test_train_step_matches_reference(golden):
    """training: teacher (every token) and student (routed) paths, Gumbel straight-through routing, LoRA
    over frozen base weights; 10 c_loss + 10 a_loss + 1 d_loss (res-vit/train.py:56) and the gradient of
    every trainable parameter."""
    m = build(golden).train()
    replay(m, golden, "train")
    x = torch.from_numpy(golden["x"]).cuda()
    y = torch.from_numpy(golden["y"]).cuda()
    c, a, d, ent, metric = m(x, y)
    (10.0 * c + 10.0 * a + 1.0 * d).backward()
    assert rel(m.logits, golden["train/logits"]) < 1e-2
    assert abs(float(c.detach()) - float(golden["train/c_loss"])) <= 1e-3 * float(golden["train/c_loss"])
    assert abs(float(d) - float(golden["train/d_loss"])) <= 1e-2 * float(golden["train/d_loss"])
    assert abs(float(a) - float(golden["train/a_loss"])) <= 1e-2 * float(golden["train/a_loss"]) + 1e-6
    assert abs(float(ent) - float(golden["train/r_entropy"])) <= 1e-2 * abs(float(golden["train/r_entropy"])) + 1e-6
    named = dict(m.named_parameters())
    trainable = [str(t) for t in golden["trainable"]]
    assert [n for n, p in m.named_parameters() if p.requires_grad] == trainable
    tot = math.sqrt(sum(float(np.square(golden["grad/" + n].astype(np.float64)).sum()) for n in trainable))
    bad = []
    for n in trainable:
        ref = torch.from_numpy(golden["grad/" + n])
        mine = named[n].grad
        mine = torch.zeros_like(ref) if mine is None else mine.detach().cpu()
        gn = float(ref.double().norm())
        if gn < 1e-3 * tot:
            if float((mine.double() - ref.double()).norm()) > 1e-3 * tot:
                bad.append((n, "abs"))
        elif rel(mine, ref) > 3e-2:
            bad.append((n, rel(mine, ref)))
    assert not bad, bad
    # frozen base weights receive no gradient (res-vit/model.py:573-584)
    assert all(p.grad is None for n, p in m.named_parameters() if not p.requires_grad)


# ---- Res-ViT-B/16 @224 (BASELINE config C5's model, res-vit/config.py defaults), batch 2 ----
@pytest.fixture(scope="module")
def golden_b16(golden_dir):
    return np.load(os.path.join(golden_dir, "resvit_b16.npz"))


def build_b16(golden_b16):
    """seed-42 constructor + the fixture's deterministic rescale, checked against the reference's
    per-tensor fingerprints (f64 sum and sum of squares) before use"""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_resvit_golden import B16, b16_inputs, tame  # our generator script: data only, no reference code
    from vitmi import resvit
    torch.manual_seed(42)
    m = resvit.Transformer(resvit.ModelArgs(**B16))
    tame(m)
    for k, v in m.state_dict().items():
        t = v.detach().double()
        ref = golden_b16["fp/" + k]
        assert abs(float(t.sum()) - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])) ** 0.5 + 1e-12 * abs(ref[0]), k
        assert abs(float((t * t).sum()) - ref[1]) <= 1e-9 * abs(ref[1]) + 1e-12, k
    x, y = b16_inputs()
    return m.cuda(), x.cuda(), y.cuda()


def test_b16_eval_ragged_forward_matches_reference(golden_b16):
    """Res-ViT-B/16 inference: 10 routers, ragged attention over the kept tokens of each image."""
    m, x, y = build_b16(golden_b16)
    m.eval()
    replay(m, golden_b16, "eval")
    with torch.no_grad():
        c, a, d, ent, metric = m(x, y)
    for k, v in m.routing_maps.items():
        assert torch.equal(v.cpu(), torch.from_numpy(golden_b16[f"eval/routing{k}"])), k
    assert rel(m.logits, golden_b16["eval/logits"]) < 1e-2
    assert abs(float(c) - float(golden_b16["eval/c_loss"])) <= 1e-3 * float(golden_b16["eval/c_loss"])
    assert abs(float(metric["non_low_rank_ratio"]) - float(golden_b16["eval/active_ratio"])) < 1e-6


def test_b16_train_step_matches_reference(golden_b16):
    """Res-ViT-B/16 training step (teacher + routed student, LoRA over frozen bases): losses and the
    norm of every trainable parameter's gradient."""
    m, x, y = build_b16(golden_b16)
    m.train()
    replay(m, golden_b16, "train")
    c, a, d, ent, metric = m(x, y)
    (10.0 * c + 10.0 * a + 1.0 * d).backward()
    assert rel(m.logits, golden_b16["train/logits"]) < 1e-2
    assert abs(float(c) - float(golden_b16["train/c_loss"])) <= 1e-3 * float(golden_b16["train/c_loss"])
    assert abs(float(d) - float(golden_b16["train/d_loss"])) <= 1e-2 * float(golden_b16["train/d_loss"])
    assert abs(float(a) - float(golden_b16["train/a_loss"])) <= 1e-2 * float(golden_b16["train/a_loss"]) + 1e-6
    named = dict(m.named_parameters())
    trainable = [str(t) for t in golden_b16["trainable"]]
    assert [n for n, p in m.named_parameters() if p.requires_grad] == trainable
    tot = math.sqrt(sum(float(golden_b16["gnorm/" + n]) ** 2 for n in trainable))
    bad = []
    for n in trainable:
        ref = float(golden_b16["gnorm/" + n])
        g = named[n].grad
        mine = 0.0 if g is None else float(g.double().norm())
        if ref < 1e-3 * tot:
            if abs(mine - ref) > 1e-3 * tot:
                bad.append((n, "abs", mine, ref))
        elif abs(mine - ref) > 3e-2 * ref:
            bad.append((n, mine, ref))
    assert not bad, bad
    assert all(p.grad is None for n, p in m.named_parameters() if not p.requires_grad)


@pytest.mark.parametrize("bs,reserve,training", [(1, 1, True), (2, 1, True), (4, 0, True), (1, 1, False),
                                                 (2, 2, False)])
@pytest.mark.parametrize("mode", ["gumbel", "expo", "override"])
def test_router_head_matches_per_op(bs, reserve, training, mode):
    """the fused router head (vitmi.resvit_fused.router_head: softmax, entropy, Gumbel straight-through decision,
    reserved rows, pattern index in one node) against RouterModule's per-op head on the same logits and draws: soft,
    hard and indices bit-identical, the entropy to f32 summation order; the logits' gradient from the soft
    probabilities, the entropy and (training) the straight-through outputs within 1e-5"""
    from vitmi import resvit
    torch.manual_seed(5)
    B, N = 3, 37
    r = resvit.RouterModule(64, 32, reserve, 1e-5, block_size=bs).cuda().train(training)
    base = torch.randn(B, N, bs, 2, device="cuda") * 3
    base[0, 5] = 0.0  # tied logits: argmax takes the first index
    g = -torch.empty_like(base).exponential_().log()
    yh = torch.zeros_like(base).scatter_(-1, torch.randint(0, 2, (B, N, bs, 1), device="cuda"), 1.0)
    w_soft, w_hard, w_idx = (torch.randn(B, N, bs, 2, device="cuda"), torch.randn(B, N, bs, 2, device="cuda"),
                             torch.randn(B, N, 1, device="cuda"))
    outs = {}
    for fused in (False, True):
        resvit.FUSED_HEAD = fused
        try:
            r.gumbel_noise = (lambda lg: g) if mode == "gumbel" else None
            r.hard_override = (lambda lg: yh) if mode == "override" else None
            logits = base.clone().requires_grad_(True)
            torch.cuda.manual_seed(11)  # the same exponential draws for both paths (mode "expo")
            hard, idx, ent, soft = r.head(logits)
            loss = (soft * w_soft).sum() + 0.7 * ent
            if training:
                loss = loss + (hard * w_hard).sum() + (idx * w_idx).sum()
            loss.backward()
            outs[fused] = [t.detach() for t in (hard, idx, ent, soft)] + [logits.grad]
        finally:
            resvit.FUSED_HEAD = True
    (h0, i0, e0, s0, d0), (h1, i1, e1, s1, d1) = outs[False], outs[True]
    assert h1.shape == h0.shape and i1.shape == i0.shape and e1.shape == e0.shape and s1.shape == s0.shape
    assert torch.equal(s1, s0)
    assert torch.equal(h1, h0)
    assert torch.equal(i1, i0)
    assert abs(float(e1) - float(e0)) <= 1e-6 * abs(float(e0)) + 1e-7
    assert rel(d1, d0) < 1e-5


def test_cls_distill_matches_per_op():
    """the fused distillation loss (vitmi.resvit_fused.cls_distill: MSE of the cls rows, its gradient added in place
    into the student's) against cls_tap + torch's mse_loss: loss to f32 summation order, x's gradient within 1e-6,
    also when only the loss reaches x"""
    import torch.nn.functional as F
    from vitmi import resvit_fused as rf
    torch.manual_seed(3)
    B, N, D = 5, 17, 300
    x0, t, w = (torch.randn(B, N, D, device="cuda") for _ in range(3))
    for with_out in (True, False):
        res = []
        for fused in (False, True):
            x = x0.clone().requires_grad_(True)
            if fused:
                y, loss = rf.cls_distill(x, t)
            else:
                y, s = rf.cls_tap(x)
                loss = F.mse_loss(s, t[:, 0, :])
            total = 3.0 * loss + ((y * w).sum() if with_out else 0.0)
            total.backward()
            res.append((float(loss), x.grad.clone()))
        (l0, g0), (l1, g1) = res
        assert abs(l1 - l0) <= 1e-6 * l0
        assert rel(g1, g0) < 1e-6
        assert torch.equal(g1[:, 1:], g0[:, 1:])


class _AliasAdd(torch.autograd.Function):
    """a + b whose backward hands both inputs ONE gradient object (as an AddBackward of the per-op layer path can)"""

    @staticmethod
    def forward(ctx, a, b):
        return a + b

    @staticmethod
    def backward(ctx, g):
        return g, g


@pytest.mark.parametrize("node", ["distill", "tap"])
def test_cls_nodes_copy_a_shared_gradient(node):
    """The cls nodes' in-place gradient add (advisor, round 5): by default (inplace=False, what ResViT.forward passes
    when the next consumer is not the fused layer node) the incoming gradient is copied before the cls rows are added,
    so a consumer that gave the same gradient object to another input still sees its own values. The other input's
    node is created first, so autograd runs the cls node's backward before it."""
    import torch.nn.functional as F
    from vitmi import resvit_fused as rf
    torch.manual_seed(5)
    B, N, D = 3, 9, 64
    x0, t, w = (torch.randn(B, N, D, device="cuda") for _ in range(3))
    v = torch.randn(B, N, D, device="cuda", requires_grad=True)
    u = v * 3.0  # created before the cls node: its backward runs after it
    x = x0.clone().requires_grad_(True)
    if node == "distill":
        y, loss = rf.cls_distill(x, t)
    else:
        y, s = rf.cls_tap(x)
        loss = F.mse_loss(s, t[:, 0, :])
    z = _AliasAdd.apply(y, u)
    (2.0 * loss + (z * w).sum()).backward()
    assert torch.equal(v.grad, 3.0 * w)  # not touched by the cls rows' loss gradient
    dcls = 2.0 * 2.0 * (x0[:, 0, :] - t[:, 0, :]) / (B * D)
    ref = w.clone()
    ref[:, 0, :] += dcls
    assert rel(x.grad, ref) < 1e-6


@pytest.mark.parametrize("T", [3 * 197, 4 * 197])
@pytest.mark.parametrize("bs", [1, 2, 4])
def test_router_select_matches_torch(bs, T):
    """vitmi.ops.router_select (one launch per routed block) against the per-layer torch ops it replaces:
    isin(indices.long(), the position's transformer set), indices == key and its any(), on pattern indices that
    include values just below an integer (the straight-through sum (1 - y) + y can land there: .long() truncates,
    == does not match)"""
    from vitmi import ops, resvit
    torch.manual_seed(7)
    n = 2 ** bs
    idx = torch.randint(0, n, (T,), device="cuda").float()
    idx[::7] -= 6e-8  # 0.99999994-style values (and -6e-8 for 0)
    idx[5] = float(n - 1)
    lra = resvit.get_indices_from_LRA_mask(bs)
    act, sel, anyf = ops.router_select(idx, [lra[j][1] for j in range(bs)], n - 1)
    for j in range(bs):
        ref = torch.isin(idx.long(), torch.tensor(lra[j][1], device="cuda"))
        assert torch.equal(act[j], ref), j
    for k in range(n - 1):
        assert torch.equal(sel[k], idx == k), k
        assert bool(anyf[k]) == bool((idx == k).any()), k
    # a key no token takes
    idx2 = torch.zeros(T, device="cuda")
    _, sel2, any2 = ops.router_select(idx2, [], n - 1)
    assert bool(any2[0]) and not any(bool(any2[k]) for k in range(1, n - 1))


@pytest.mark.parametrize("img,patch", [(224, 16), (32, 8), (56, 14)])
def test_embed_tokens_matches_per_op(img, patch):
    """the fused token embedding (vitmi.resvit_fused.embed_tokens: im2col + one GEMM with the PATCH epilogue writing
    cls + pos and conv + bias + pos) against Transformer.embed + cat + PositionEmbs (frozen conv and position
    embeddings, the LoRA configuration): token rows within 1e-5 (the same bf16 GEMM operands; the cls rows exact)
    and the cls token's gradient within 1e-6"""
    from vitmi import resvit
    from vitmi import resvit_fused as rf
    torch.manual_seed(11)
    args = resvit.ModelArgs(dim=128, mlp_dim=256, n_layers=1, n_heads=2, n_kv_heads=2, lora_rank=4, use_lora=True,
                            use_reslr=False, image_size=(img, img), patch_size=(patch, patch), num_classes=10)
    m = resvit.Transformer(args).cuda()
    assert not m.embedding.weight.requires_grad and m.cls_token.requires_grad
    x = torch.randn(3, 3, img, img, device="cuda")
    assert rf.embed_supported(m, x)
    w = torch.randn(3, (img // patch) ** 2 + 1, 128, device="cuda")
    outs = []
    for fused in (False, True):
        m.cls_token.grad = None
        if fused:
            t = rf.embed_tokens(m, x)
        else:
            t = m.embed(x)
            t = torch.cat([m.cls_token.expand(t.shape[0], 1, -1), t], dim=1)
            t = m.pos_embedding(t)
        (t * w).sum().backward()
        outs.append((t.detach(), m.cls_token.grad.clone()))
    (t0, g0), (t1, g1) = outs
    assert t1.shape == t0.shape
    assert torch.equal(t1[:, 0], t0[:, 0])
    assert rel(t1, t0) < 1e-5  # (the same bf16 operands and k order; the adds of bias and pos in the same order)
    assert rel(g1, g0) < 1e-6
