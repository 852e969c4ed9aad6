"""The Res-ViT training step (BASELINE config C5; res-vit/train.py:23-68) on the MI355X against three
steps of the reference itself: tests/golden/resvit_train3.npz, written by
tests/golden/make_resvit_train_golden.py from the imported res-vit/model.py driven by torch.optim.AdamW,
torch.nn.utils.clip_grad_norm_(params, 1.0) and transformers.get_cosine_schedule_with_warmup. GPU only.

* optimizer alone: the reference's recorded gradients fed to vitmi's clip_grad_norm_ + AdamW
  (csrc/optim.hip, flat buffer): the clip norm, the clipped gradients, and after three steps every
  parameter and its AdamW moments / step count to f32 rounding (1e-5 relative), including the
  parameters some steps leave without a gradient (skipped, as torch skips `.grad is None`);
* end to end: the three steps through vitmi.resvit_train.train_step with the reference's Gumbel draws
  and routing decisions replayed: every step's losses (1e-3 relative; bf16 operands), clip norm
  (2e-2) and the parameter trajectory (the accumulated update p3 - p0 of every tensor with a
  meaningful update within 0.10 relative: Adam's first steps are ~lr * sign(g), so bf16-level gradient
  noise flips the sign of near-zero gradient elements; measured round 4: at most 6.5e-2, layer 1's
  lora_k and approximator up-projection, both paths).
"""
import os

import numpy as np
import pytest
import torch

from test_resvit_cpu import TINY

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gold(golden_dir):
    return np.load(os.path.join(golden_dir, "resvit_train3.npz"))


def rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def hp(gold):
    lr, wd, b1, b2, eps, warm, total, lc, la, ld = gold["hparams"].tolist()
    return dict(lr=lr, wd=wd, betas=(b1, b2), eps=eps, warmup=int(warm), total=int(total), lc=lc, la=la, ld=ld)


def build(gold):
    from vitmi import resvit
    torch.manual_seed(42)
    m = resvit.Transformer(resvit.ModelArgs(**dict(TINY, device="cuda")))
    m.load_state_dict({k[3:]: torch.from_numpy(gold[k]) for k in gold.files if k.startswith("p0/")})
    return m.cuda()


@pytest.mark.parametrize("fused", [False, True])
def test_adamw_and_clip_match_reference_on_recorded_grads(gold, fused):
    from vitmi.optim import AdamW, clip_grad_norm_, get_cosine_schedule_with_warmup
    h = hp(gold)
    m = build(gold)
    trainable = [str(t) for t in gold["trainable"]]
    named = dict(m.named_parameters())
    opt = AdamW(m.parameters(), lr=h["lr"], weight_decay=h["wd"], betas=h["betas"], eps=h["eps"],
                max_grad_norm=1.0 if fused else None)
    sched = get_cosine_schedule_with_warmup(opt, h["warmup"], h["total"])
    f = opt.flat
    assert sorted(map(id, f.params)) == sorted(id(named[n]) for n in trainable)
    for s in range(3):
        assert opt.param_groups[0]["lr"] == pytest.approx(float(gold[f"s{s}/lr"]), rel=1e-12)
        opt.zero_grad()
        for n in trainable:  # the reference's gradients, as the backward would leave them
            if bool(gold[f"s{s}/has_grad/{n}"]):
                named[n].grad.copy_(torch.from_numpy(gold[f"s{s}/grad/{n}"]))
                f.used_host[f.index(named[n])] = True
        if not fused:
            norm = clip_grad_norm_(None, 1.0, flat=opt)
            assert float(norm) == pytest.approx(float(gold[f"s{s}/norm"]), rel=1e-6)
        opt.step()
        sched.step()
        if fused:
            assert float(opt.last_norm[0]) == pytest.approx(float(gold[f"s{s}/norm"]), rel=1e-6)
        for n in trainable:  # .grad holds the clipped gradient afterwards (clip_grad_norm_ is in place)
            if bool(gold[f"s{s}/has_grad/{n}"]):
                assert rel(named[n].grad, gold[f"s{s}/cgrad/{n}"]) < 1e-6, (s, n)
    bad = []
    for n in trainable:
        i = f.index(named[n])
        if rel(named[n], gold["p3/" + n]) > 1e-5:
            bad.append((n, "p", rel(named[n], gold["p3/" + n])))
        d_ref = gold["p3/" + n].astype(np.float64) - gold["p0/" + n].astype(np.float64)
        d_me = named[n].detach().double().cpu() - torch.from_numpy(gold["p0/" + n]).double()
        if np.abs(d_ref).max() > 0 and rel(d_me, d_ref) > 1e-4:
            bad.append((n, "update", rel(d_me, d_ref)))
        if ("m3/" + n) in gold.files:
            assert float(opt.steps[i]) == float(gold["t3/" + n]), n
            rm, rv = rel(f.view(opt.exp_avg, i), gold["m3/" + n]), rel(f.view(opt.exp_avg_sq, i), gold["v3/" + n])
            if rm > 1e-5 or rv > 1e-5:
                bad.append((n, "moments", rm, rv))
        else:
            assert float(opt.steps[i]) == 0.0, n
    assert not bad, bad
    # a parameter with no gradient in some step kept its step count behind the others (torch's skip)
    assert len({float(v) for v in opt.steps.cpu()}) > 1


def _replay(m, gold, s):
    routers = [l.router for l in m.layers if hasattr(l, "router")]
    for j, r in enumerate(routers):
        hard = torch.from_numpy(gold[f"s{s}/router{j}_hard"]).cuda()
        g = torch.from_numpy(gold[f"s{s}/gumbel{j}"]).cuda()
        r.hard_override = lambda logits, hh=hard: hh
        r.gumbel_noise = lambda logits, gg=g: gg


@pytest.mark.parametrize("fused", [False, True])
def test_three_training_steps_match_reference(gold, fused):
    from vitmi.optim import AdamW, get_cosine_schedule_with_warmup
    from vitmi.resvit_train import train_step
    h = hp(gold)
    m = build(gold).train()
    opt = AdamW(m.parameters(), lr=h["lr"], weight_decay=h["wd"], betas=h["betas"], eps=h["eps"],
                max_grad_norm=1.0 if fused else None)
    sched = get_cosine_schedule_with_warmup(opt, h["warmup"], h["total"])
    trainable = [str(t) for t in gold["trainable"]]
    named = dict(m.named_parameters())
    for s in range(3):
        _replay(m, gold, s)
        x = torch.from_numpy(gold[f"s{s}/x"]).cuda()
        y = torch.from_numpy(gold[f"s{s}/y"]).cuda()
        total, c, a, d, ent, _ = train_step(m, x, y, opt, sched, h["la"], h["ld"], h["lc"], clip_grad_norm=True)
        assert abs(float(c) - float(gold[f"s{s}/c_loss"])) <= 1e-3 * float(gold[f"s{s}/c_loss"]), s
        assert abs(float(total) - float(gold[f"s{s}/total"])) <= 1e-3 * float(gold[f"s{s}/total"]), s
        assert abs(float(d) - float(gold[f"s{s}/d_loss"])) <= 2e-2 * float(gold[f"s{s}/d_loss"]), s
        # (after the first update the parameter trajectory itself carries bf16-level differences)
        assert rel(m.logits, gold[f"s{s}/logits"]) < (1e-2 if s == 0 else 2e-2), s
        # which parameters the update treated as having a gradient is the reference's (routing replayed;
        # an approximator no token was routed to runs on every row but is gated off on the device)
        used = opt.flat.used.cpu()
        for n in trainable:
            assert bool(used[opt.flat.index(named[n])] > 0) == bool(gold[f"s{s}/has_grad/{n}"]), (s, n)
        # the clip's input norm (vitmi AdamW keeps {norm, coef} of its last clip, fused or not)
        assert float(opt.last_norm[0]) == pytest.approx(float(gold[f"s{s}/norm"]), rel=2e-2), s
    tot_upd = sum(float(np.square(gold["p3/" + n].astype(np.float64) - gold["p0/" + n]).sum()) for n in trainable)
    bad = []
    for n in trainable:
        d_ref = gold["p3/" + n].astype(np.float64) - gold["p0/" + n].astype(np.float64)
        if float(np.square(d_ref).sum()) < 1e-4 * tot_upd:
            continue
        d_me = named[n].detach().double().cpu() - torch.from_numpy(gold["p0/" + n]).double()
        e = rel(d_me, d_ref)
        print(f"update rel {n}: {e:.3e}")
        if e > 0.10:
            bad.append((n, e))
    assert not bad, bad


@pytest.mark.parametrize("fused,warmup", [(False, 0), (True, 0), (True, 1)])
def test_graphed_step_matches_eager_and_reference(gold, fused, warmup):
    """GraphedTrainStep (forward + backward replayed from one HIP graph, optimizer eager) computes what
    train_step computes: the reference's three recorded steps (Gumbel draws / routing replayed through
    static buffers the graph reads) give bit-identical losses and parameters to the eager steps, and the
    eager steps are pinned to the reference by test_three_training_steps_match_reference."""
    from vitmi.optim import AdamW, get_cosine_schedule_with_warmup
    from vitmi.resvit_train import GraphedTrainStep, train_step
    h = hp(gold)
    runs = []
    for graphed in (False, True):
        m = build(gold).train()
        opt = AdamW(m.parameters(), lr=h["lr"], weight_decay=h["wd"], betas=h["betas"], eps=h["eps"],
                    max_grad_norm=1.0 if fused else None)
        sched = get_cosine_schedule_with_warmup(opt, h["warmup"], h["total"])
        routers = [l.router for l in m.layers if hasattr(l, "router")]
        hard = [torch.from_numpy(gold[f"s0/router{j}_hard"]).cuda() for j in range(len(routers))]
        gum = [torch.from_numpy(gold[f"s0/gumbel{j}"]).cuda() for j in range(len(routers))]
        for r, hh, gg in zip(routers, hard, gum):  # the graph reads these buffers: refilled every step
            r.hard_override = lambda logits, hh=hh: hh
            r.gumbel_noise = lambda logits, gg=gg: gg
        x = torch.from_numpy(gold["s0/x"]).cuda()
        y = torch.from_numpy(gold["s0/y"]).cuda()
        # warmup=0: the eager run before it created the device constants (no pageable copy under capture);
        # warmup=1: one forward + backward on batch 0 inside the constructor, which leaves the parameters, the
        # optimizer and the schedule untouched (the eager run takes no extra step)
        g = GraphedTrainStep(m, x, y, opt, sched, h["la"], h["ld"], h["lc"], True, warmup=warmup) if graphed else None
        losses = []
        for s in range(3):
            for j in range(len(routers)):
                hard[j].copy_(torch.from_numpy(gold[f"s{s}/router{j}_hard"]))
                gum[j].copy_(torch.from_numpy(gold[f"s{s}/gumbel{j}"]))
            x = torch.from_numpy(gold[f"s{s}/x"]).cuda()
            y = torch.from_numpy(gold[f"s{s}/y"]).cuda()
            out = (g.step(x, y) if graphed else
                   train_step(m, x, y, opt, sched, h["la"], h["ld"], h["lc"], clip_grad_norm=True))
            losses.append(torch.stack([out[0], out[1], out[3]]).detach().clone())
            assert abs(float(out[1]) - float(gold[f"s{s}/c_loss"])) <= 1e-3 * float(gold[f"s{s}/c_loss"]), s
        runs.append((torch.stack(losses), [p.detach().clone() for p in opt.flat.params], opt.flat.used.clone()))
    (le, pe, ue), (lg, pg, ug) = runs
    assert torch.isfinite(le).all() and le[0, 0] != le[2, 0]  # the graph's gradients reach the parameters
    assert torch.equal(le, lg)
    assert torch.equal(ue, ug)
    assert all(torch.equal(a, b) for a, b in zip(pe, pg))


def test_grad_sinks_match_autograd_accumulation(gold, monkeypatch):
    """vitmi.flat.grad_sink: the fused router-MLP / approximator nodes accumulate their weight gradients in place
    into the flat .grad views (no AccumulateGrad add) — three reference steps (routing replayed) end with
    bit-identical losses, parameters and used flags to the same steps through autograd's accumulation, and
    the sinks were taken."""
    from vitmi import flat as vflat
    from vitmi.optim import AdamW, get_cosine_schedule_with_warmup
    from vitmi.resvit_train import train_step
    h = hp(gold)
    taken = []
    real_sunk = vflat.sunk
    monkeypatch.setattr(vflat, "sunk", lambda p: (taken.append(id(p)), real_sunk(p)))
    runs = []
    for sinks in (False, True):
        monkeypatch.setattr(vflat, "SINKS", sinks)
        m = build(gold).train()
        opt = AdamW(m.parameters(), lr=h["lr"], weight_decay=h["wd"], betas=h["betas"], eps=h["eps"],
                    max_grad_norm=1.0)
        sched = get_cosine_schedule_with_warmup(opt, h["warmup"], h["total"])
        routers = [l.router for l in m.layers if hasattr(l, "router")]
        losses = []
        for s in range(3):
            for j, r in enumerate(routers):
                hh = torch.from_numpy(gold[f"s{s}/router{j}_hard"]).cuda()
                gg = torch.from_numpy(gold[f"s{s}/gumbel{j}"]).cuda()
                r.hard_override = lambda logits, hh=hh: hh
                r.gumbel_noise = lambda logits, gg=gg: gg
            x = torch.from_numpy(gold[f"s{s}/x"]).cuda()
            y = torch.from_numpy(gold[f"s{s}/y"]).cuda()
            out = train_step(m, x, y, opt, sched, h["la"], h["ld"], h["lc"], clip_grad_norm=True)
            losses.append(torch.stack([out[0], out[1], out[3]]).detach().clone())
        runs.append((torch.stack(losses), [p.detach().clone() for p in opt.flat.params], opt.flat.used.clone(),
                     len(taken)))
    (l0, p0, u0, n0), (l1, p1, u1, n1) = runs
    assert n0 == 0 and n1 > 0, (n0, n1)
    assert torch.equal(l0, l1)
    assert torch.equal(u0, u1)
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))


def test_flat_params_keep_grad_views_and_skip_unused():
    """FlatParams: parameters become views of one buffer, autograd accumulates into the preset .grad
    views in place, a parameter outside the graph is marked unused, module.zero_grad() (set_to_none)
    is recovered by adopt_grads()."""
    from vitmi.flat import FlatParams
    a = torch.nn.Parameter(torch.randn(5, 7, device="cuda"))
    b = torch.nn.Parameter(torch.randn(3, device="cuda"))
    c = torch.nn.Parameter(torch.randn(130, device="cuda"))
    a0, b0 = a.detach().clone(), b.detach().clone()
    f = FlatParams([a, b, c])
    assert torch.equal(a.detach(), a0) and torch.equal(b.detach(), b0)
    assert all(o % 64 == 0 for o in f.offsets)
    f.zero_grad()
    (a.sum() * 2 + (b * b).sum()).backward()
    assert a.grad.data_ptr() == f.view(f.grad, f.index(a)).data_ptr()
    assert torch.allclose(a.grad, torch.full_like(a, 2.0)) and torch.allclose(b.grad, 2 * b0)
    assert f.used_host[f.index(a)] and f.used_host[f.index(b)] and not f.used_host[f.index(c)]
    f.zero_grad()
    assert float(f.grad.abs().sum()) == 0.0 and not any(f.used_host)
    a.grad = None  # e.g. nn.Module.zero_grad()
    (a * 3).sum().backward()
    f.adopt_grads()
    assert a.grad.data_ptr() == f.view(f.grad, f.index(a)).data_ptr()
    assert torch.allclose(a.grad, torch.full_like(a, 3.0))


def test_adamw_state_dict_round_trip_and_gate_or():
    """AdamW.state_dict() is torch.optim.AdamW's format (so it loads into torch's AdamW and back), and
    load_state_dict() lands in the flat moment buffers that step() uses: a resumed optimizer continues the
    trajectory of the original bit for bit. flat.gate ORs the flags of repeated forwards before a step."""
    from vitmi.flat import _take_gate, gate
    from vitmi.optim import AdamW
    g = torch.Generator(device="cuda").manual_seed(3)
    shapes = [(5, 7), (3,), (130,)]
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda", generator=g)) for s in shapes]
    grads = [[torch.randn(s, device="cuda", generator=g) for s in shapes] for _ in range(4)]
    opt = AdamW(ps, lr=1e-2, weight_decay=0.05)
    for k in range(2):
        opt.zero_grad()
        for p, gr in zip(ps, grads[k]):
            (p * gr).sum().backward()
        opt.step()
    sd = opt.state_dict()
    ref = torch.optim.AdamW([torch.nn.Parameter(p.detach().clone()) for p in ps], lr=1e-2, weight_decay=0.05)
    ref.load_state_dict(sd)  # torch accepts the format
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt2 = AdamW(qs, lr=1e-2, weight_decay=0.05)
    opt2.load_state_dict(sd)
    for k in (2, 3):
        for o, params in ((opt, ps), (opt2, qs)):
            o.zero_grad()
            for p, gr in zip(params, grads[k]):
                (p * gr).sum().backward()
            o.step()
    for p, q in zip(ps, qs):
        assert torch.equal(p.detach(), q.detach())
    assert float(opt2.state_dict()["state"][0]["step"]) == 4.0
    x = torch.nn.Parameter(torch.zeros(2, device="cuda"))
    gate([x], torch.tensor(True, device="cuda"))
    gate([x], torch.tensor(False, device="cuda"))
    assert bool(_take_gate(x))


def test_resvit_data_parallel_two_ranks(tmp_path):
    """Res-ViT DP (new: the reference is single-device): 2 ranks on one GPU over gloo, 4 images each,
    FlatGradAllReducer on the LoRA / router / approximator / head gradients, vitmi AdamW with the clip
    folded in. Both replicas end bit-identical, the graphed step (GraphedTrainStep with the reducer: the
    exchange after each replay) equals the eager one bit for bit, and (lambda_active = 0: the ratio loss is a non-linear
    function of the per-rank mean) equal to one 8-image step of a single process within 2e-2 of the
    update."""
    script = tmp_path / "dp_resvit.py"
    script.write_text(r'''
import os, sys, torch, numpy as np, torch.distributed as dist
sys.path.insert(0, os.path.join(os.environ["REPO"], "vit-of-pytorch_amd")); sys.path.insert(0, os.environ["REPO"])
sys.path.insert(0, os.path.join(os.environ["REPO"], "tests"))
from test_resvit_cpu import TINY
from vitmi import resvit
from vitmi.optim import AdamW
from vitmi.dist import FlatGradAllReducer
from vitmi.resvit_train import train_step
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
g = torch.Generator().manual_seed(5)
X = torch.randn(8, 3, 32, 32, generator=g); Y = torch.randint(0, 10, (8,), generator=g)

def make():
    torch.manual_seed(42)
    m = resvit.Transformer(resvit.ModelArgs(**dict(TINY, device="cuda"))).cuda().train()
    gn = torch.Generator().manual_seed(9)
    for j, l in enumerate([l for l in m.layers if hasattr(l, "router")]):
        noise = -torch.empty(8, 17, 2, 2).exponential_(generator=gn).log()  # [B, tokens, block_size, 2]
        l.router.gumbel_noise = (lambda nz: lambda logits: nz[:logits.shape[0]] if logits.shape[0] == 8 else
                                 nz[rank * 4:(rank + 1) * 4])(noise.cuda())
    return m

def run(m, x, y, reducer=None, graphed=False):
    opt = AdamW(m.parameters(), lr=1e-2, weight_decay=0.05, max_grad_norm=1.0)
    if reducer:
        red = FlatGradAllReducer(opt.flat, bucket_elems=2000).attach()
    if graphed:  # forward + backward replayed from a HIP graph, the exchange after each replay
        from vitmi.resvit_train import GraphedTrainStep
        gs = GraphedTrainStep(m, x, y, opt, None, 0.0, 1e-2, 1.0, True, reducer=red)
        for _ in range(2):
            gs.step()
    else:
        for _ in range(2):
            train_step(m, x, y, opt, None, 0.0, 1e-2, 1.0, True, red if reducer else None)
    torch.cuda.synchronize()
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu()

m = make()
flat = run(m, X[rank * 4:(rank + 1) * 4].cuda(), Y[rank * 4:(rank + 1) * 4].cuda(), reducer=True)
out = [torch.zeros_like(flat) for _ in range(world)]
dist.all_gather(out, flat)
# the graphed data-parallel step (bench.py's default at N > 1): the same two steps, bit-identical to the eager one
flat_g = run(make(), X[rank * 4:(rank + 1) * 4].cuda(), Y[rank * 4:(rank + 1) * 4].cuda(), reducer=True, graphed=True)
assert torch.equal(flat_g, flat), float((flat_g - flat).abs().max())
if rank == 0:
    assert torch.equal(out[0], out[1]), "replicas diverged"
    torch.manual_seed(42)
    p0 = torch.cat([p.detach().reshape(-1) for p in resvit.Transformer(resvit.ModelArgs(**dict(TINY, device="cuda"))).parameters()])
    ref = run(make(), X.cuda(), Y.cuda())
    r = float((flat - ref).norm() / (ref - p0).norm())
    print("rel", r)
    assert r < 2e-2, r
dist.barrier()
dist.destroy_process_group()
open(os.path.join(os.environ["OUTDIR"], f"rank{rank}.ok"), "w").write("ok")
''')
    import subprocess
    import sys
    env = dict(os.environ, REPO=REPO, OUTDIR=str(tmp_path), MASTER_ADDR="127.0.0.1", MASTER_PORT="29541")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", "29541", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert (tmp_path / "rank0.ok").exists() and (tmp_path / "rank1.ok").exists()


@pytest.mark.parametrize("dims", [dict(dim=64, mlp_dim=128, n_heads=2, n_kv_heads=2, lora_rank=4),
                                  dict(dim=768, mlp_dim=3072, n_heads=12, n_kv_heads=12, lora_rank=8)],
                         ids=["tiny", "b16"])
def test_fused_layer_matches_per_op_path(dims):
    """vitmi.resvit_fused (one autograd node per TransformerBlock._full, LoRA folded into the q|k|v GEMM as
    extra K columns) against the per-op path on the same kernels (vitmi.functional): output, input
    gradient and the six LoRA factor gradients of one layer; N = 197 tokens, 3 images."""
    from vitmi import resvit, resvit_fused
    torch.manual_seed(3)
    args = resvit.ModelArgs(**dict(TINY, **dims, device="cuda"))
    m = resvit.Transformer(args).cuda()
    blk = m.layers[0]
    with torch.no_grad():  # LoRA factors at a scale where their contribution is visible
        for p in blk.attention.parameters():
            if p.requires_grad:
                p.normal_(0.0, 0.05)
    assert resvit_fused.supported(blk)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(3, 197, args.dim, device="cuda", generator=g)
    w = torch.randn(3, 197, args.dim, device="cuda", generator=g)
    lora = [p for p in blk.attention.parameters() if p.requires_grad]
    assert len(lora) == 6
    res = {}
    for fused in (True, False):
        blk.fused = fused
        xi = x.clone().requires_grad_(True)
        for p in lora:
            p.grad = None
        out = blk._full(xi)
        (out * w).sum().backward()
        res[fused] = (out.detach(), xi.grad.detach(), [p.grad.detach().clone() for p in lora])
    (o1, dx1, g1), (o0, dx0, g0) = res[True], res[False]
    assert rel(o1, o0) < 2e-3
    assert rel(dx1, dx0) < 1e-2
    for a, b in zip(g1, g0):
        assert rel(a, b) < 2e-2


def test_fused_layer_row_selection_matches_where():
    """The routed student's where(active, layer(x), x) (res-vit/model.py:507-512) folded into the fused layer node
    (vit_rows_select on the output, the output gradient masked in the backward, the where's x-gradient carried on
    the LN1 backward's residual input) against the same node followed by torch.where: output and the six LoRA
    gradients bit for bit, the input gradient to one f32 rounding; T = 3 x 197 rows, about half active."""
    from vitmi import resvit
    torch.manual_seed(3)
    args = resvit.ModelArgs(**dict(TINY, dim=128, n_heads=2, n_kv_heads=2, mlp_dim=256, device="cuda"))
    m = resvit.Transformer(args).cuda()
    blk = m.layers[0]
    with torch.no_grad():
        for p in blk.attention.parameters():
            if p.requires_grad:
                p.normal_(0.0, 0.05)
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(3, 197, args.dim, device="cuda", generator=g)
    w = torch.randn(3, 197, args.dim, device="cuda", generator=g)
    active = torch.rand(3, 197, 1, device="cuda", generator=g) < 0.5
    lora = [p for p in blk.attention.parameters() if p.requires_grad]
    res = []
    for folded in (True, False):
        xi = x.clone().requires_grad_(True)
        for p in lora:
            p.grad = None
        out = blk._full(xi, active=active) if folded else torch.where(active, blk._full(xi), xi)
        (out * w).sum().backward()
        res.append((out.detach(), xi.grad.detach(), [p.grad.detach().clone() for p in lora]))
    (o1, dx1, g1), (o0, dx0, g0) = res
    assert torch.equal(o1, o0)
    for a, b in zip(g1, g0):
        assert torch.equal(a, b)
    # dx: on the inactive rows the LN1 backward now adds dout inside its fused multiply-add instead of autograd
    # adding it after the kernel's own rounding: equal up to that one rounding
    assert bool(((dx1 - dx0).abs() <= 2.0 ** -22 * dx0.abs() + 1e-30).all()) or rel(dx1, dx0) < 1e-6


@pytest.mark.parametrize("B,N,r", [(3, 197, 16), (2, 17, 256), (1, 65, 32)])
def test_fused_approximator_matches_per_op_path(B, N, r):
    """vitmi.resvit_fused.approx_step (one node: down GEMM with a bf16 epilogue, unselected rows zeroed, up GEMM
    with the f32 residual epilogue) against the per-op path it replaces (HipLinear x2 + add + where,
    res-vit/model.py:349-368): output, input gradient and both weight gradients bit for bit, routed rows mixed
    with unrouted ones; T = B*N not a multiple of 64."""
    from vitmi import resvit
    torch.manual_seed(7)
    D = 64
    bpa = resvit.BlockPathApproximators(D, r, 1).cuda()
    m = bpa.approximators["0"]
    with torch.no_grad():  # a visible low-rank update
        m.down_proj.weight.normal_(0.0, 0.2)
        m.up_proj.weight.normal_(0.0, 0.2)
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(B, N, D, device="cuda", generator=g)
    w = torch.randn(B, N, D, device="cuda", generator=g)
    idx = torch.randint(0, 2, (B, N, 1), device="cuda", generator=g).float()  # router index 0 -> approximator
    assert 0 < int((idx == 0).sum()) < B * N
    res = {}
    for fused in (True, False):
        bpa.fused = fused
        xi = x.clone().requires_grad_(True)
        for p in m.parameters():
            p.grad = None
        out = bpa(xi, idx, [0])
        (out * w).sum().backward()
        res[fused] = (out.detach(), xi.grad.detach(), m.down_proj.weight.grad.clone(), m.up_proj.weight.grad.clone())
    for a, b in zip(res[True], res[False]):
        assert torch.equal(a, b)
    sel = (idx == 0).expand(B, N, D)
    assert torch.equal(res[True][0][~sel], x[~sel])  # unrouted rows pass through unchanged


@pytest.mark.parametrize("B,N,hdim,bs", [(3, 197, 64, 1), (2, 17, 512, 2), (2, 17, 48, 1), (2, 17, 40, 1)])
def test_fused_router_mlp_matches_per_op_path(B, N, hdim, bs):
    """vitmi.resvit_fused.router_mlp (RouterModule.out_conv as one node: GELU and GELU' written by the GEMM
    epilogues, GELU' multiplied in the data-gradient epilogues) against the per-op path (res-vit/model.py:
    150-156): the routing logits, the input gradient and all six parameter gradients. Not bit-identical:
    GELU' is rounded to bf16 (as in the ViT engine's MLP) and the hidden-bias gradients sum bf16 dU."""
    from vitmi import resvit
    torch.manual_seed(9)
    r = resvit.RouterModule(64, hdim, 1, 1e-5, block_size=bs).cuda()
    with torch.no_grad():  # a last layer with visible weights (the reference inits it at std 0.01)
        r.out_conv[-1].weight.normal_(0.0, 0.2)
    g = torch.Generator(device="cuda").manual_seed(13)
    x = torch.randn(B, N, 2 * hdim, device="cuda", generator=g)
    w = torch.randn(B, N, 2 * bs, device="cuda", generator=g)
    params = list(r.out_conv.parameters())
    res = {}
    for fused in (True, False):
        r.fused_mlp = fused
        xi = x.clone().requires_grad_(True)
        for p in params:
            p.grad = None
        from vitmi import resvit_fused
        if fused and not resvit_fused.router_mlp_supported(r.out_conv, xi):
            assert hdim % 16, hdim  # only widths the fused GEMM epilogues cannot take fall back
            out = r.out_conv(xi)
        else:
            out = resvit_fused.router_mlp(r.out_conv, xi) if fused else r.out_conv(xi)
        (out * w).sum().backward()
        res[fused] = (out.detach(), xi.grad.detach(), [p.grad.detach().clone() for p in params])
    (o1, dx1, g1), (o0, dx0, g0) = res[True], res[False]
    assert rel(o1, o0) < 1e-3
    assert rel(dx1, dx0) < 2e-2
    for a, b in zip(g1, g0):
        assert rel(a, b) < 2e-2, (rel(a, b), a.shape)


@pytest.mark.parametrize("B,N,hdim,reserve", [(3, 197, 64, 1), (2, 17, 512, 0), (2, 17, 48, 1), (2, 17, 40, 1),
                                             (2, 17, 100, 1)])
def test_fused_router_net_matches_per_op_path(B, N, hdim, reserve):
    """vitmi.resvit_fused.router_net (LN -> Linear -> GELU -> token mean -> concatenation -> out_conv as one node,
    the concatenated operand built in bf16 by the GEMM epilogue and a broadcast) against the per-op router
    (res-vit/model.py:186-190): soft routing probabilities and the gradients of the input and of every router
    parameter (the LayerNorm affine included). Tolerance-level against the fp32 per-op path: x_embed and its
    token mean enter out_conv as bf16 and GELU' is bf16; the bias gradients are signed sums over every token,
    so their relative error carries the cancellation (out_conv's first bias measured at 4e-2)."""
    from vitmi import resvit
    torch.manual_seed(21)
    r = resvit.RouterModule(64, hdim, reserve, 1e-5, block_size=1).cuda()
    with torch.no_grad():
        r.out_conv[-1].weight.normal_(0.0, 0.2)
        r.in_conv[0].layer_norm.weight.normal_(1.0, 0.1)
    g = torch.Generator(device="cuda").manual_seed(23)
    x = torch.randn(B, N, 64, device="cuda", generator=g)
    w = torch.randn(B, N, 1, 2, device="cuda", generator=g)
    params = list(r.parameters())
    from vitmi import resvit_fused
    # hdim 40 / 100 (hidden widths not multiples of 8): the router runs the per-op path instead of raising
    assert resvit_fused.router_net_supported(r, x) == (hdim % 16 == 0), hdim
    res = {}
    for fused in (True, False):
        r.fused_mlp = fused
        xi = x.clone().requires_grad_(True)
        for p in params:
            p.grad = None
        hard, idx, ent, soft = r(xi)
        (soft * w).sum().backward()
        res[fused] = [soft.detach(), xi.grad.detach()] + [p.grad.detach().clone() for p in params]
    names = ["soft", "dx"] + [n for n, _ in r.named_parameters()]
    tol = {"soft": 1e-3, "dx": 3e-2}
    for n, a, b in zip(names, res[True], res[False]):
        e = rel(a, b)
        print(f"{n}: {e:.2e}")
        assert e < tol.get(n, 6e-2), (n, e)


def test_fused_layer_refuses_backward_after_shared_operand_rewrite(gold):
    """The fused layer's LN1 | u operand and LoRA pack are per-block buffers shared by the block's forwards
    (SHARE_PACK): a backward whose forward's buffers were rewritten by a later grad-enabled forward of the same
    block raises instead of computing the LoRA gradients from the wrong activations; forward -> backward
    alternation (the training steps) is accepted."""
    from vitmi import resvit_fused
    m = build(gold).train()
    blk = m.layers[0]
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(2, 17, TINY["dim"], device="cuda", generator=g, requires_grad=True)
    resvit_fused.full_layer(blk, x).square().sum().backward()  # one forward, its backward: fine
    y1 = resvit_fused.full_layer(blk, x)
    y2 = resvit_fused.full_layer(blk, x)
    with pytest.raises(RuntimeError, match="another forward"):
        (y1.square().sum() + y2.square().sum()).backward()


def test_grad_sinks_only_inside_training_backward(gold):
    """vitmi.flat.grad_sink answers only inside flat.sinks() (train_step / GraphedTrainStep wrap their backward
    in it): a plain torch.autograd.grad over the router parameters of a FlatParams-managed model returns their
    gradients (none is None) and leaves .grad untouched."""
    from vitmi.optim import AdamW
    m = build(gold).train()
    opt = AdamW(m.parameters(), lr=1e-4, weight_decay=0.05, max_grad_norm=1.0)
    opt.zero_grad()
    routers = [l.router for l in m.layers if hasattr(l, "router")]
    params = [p for r in routers for p in r.parameters() if p.requires_grad]
    x = torch.from_numpy(gold["s0/x"]).cuda()
    y = torch.from_numpy(gold["s0/y"]).cuda()
    c_loss, a_loss, d_loss, _, _ = m(x, y)
    grads = torch.autograd.grad(c_loss + a_loss + d_loss, params, allow_unused=True)
    assert any(gr is not None for gr in grads)
    assert all(gr is None or torch.isfinite(gr).all() for gr in grads)
    assert float(opt.flat.grad.abs().sum()) == 0.0  # nothing was sunk into the flat gradient


def test_each_parameter_counted_once_per_backward(gold):
    """The data-parallel bucket count (FlatParams.on_grad) sees every trainable parameter exactly once per training
    backward, although the fused nodes sink their gradients into the flat .grad views and autograd's post hook
    still runs for the None they return (round 5: counted in both places, the reducer launched buckets early), and
    every parameter that took a gradient is flagged used."""
    from collections import Counter
    from vitmi.optim import AdamW
    from vitmi.resvit_train import train_step
    m = build(gold).train()
    opt = AdamW(m.parameters(), lr=1e-4, weight_decay=0.05, max_grad_norm=1.0)
    seen = []
    opt.flat.on_grad = seen.append
    x = torch.from_numpy(gold["s0/x"]).cuda()
    y = torch.from_numpy(gold["s0/y"]).cuda()
    train_step(m, x, y, opt, None, 10.0, 1.0, 10.0, True, None)
    torch.cuda.synchronize()
    c = Counter(seen)
    assert c and max(c.values()) == 1, {i: n for i, n in c.items() if n > 1}
    names = {id(p): n for n, p in m.named_parameters()}
    sunk_kinds = [names[id(opt.flat.params[i])] for i in c]
    assert any("lora_A" in n for n in sunk_kinds) and any("router" in n for n in sunk_kinds)
    assert all(opt.flat.used_host[i] for i in c)


def test_zero_grad_clears_stale_gates():
    """flat.gate ORs a forward's participation flag into an existing entry; FlatParams.zero_grad drops the
    entries of its parameters, so a flag left by a forward no step consumed cannot mark the next step used."""
    from vitmi.flat import FlatParams, _GATES, _take_gate, gate
    p = torch.nn.Parameter(torch.zeros(4, device="cuda"))
    f = FlatParams([p])
    gate([p], torch.tensor(True, device="cuda"))  # a train-mode forward whose step was skipped
    f.zero_grad()
    assert id(p) not in _GATES
    gate([p], torch.tensor(False, device="cuda"))  # the next step's forward routed no rows to p
    assert not bool(_take_gate(p))


def test_graphed_step_construction_leaves_state_untouched(gold):
    """GraphedTrainStep(warmup=1) runs its warm-up forward + backward without an optimizer or scheduler step
    (its Gumbel draws are taken from restored RNG states): parameters, the learning rate and the flat gradient are
    as before."""
    from vitmi.optim import AdamW, get_cosine_schedule_with_warmup
    from vitmi.resvit_train import GraphedTrainStep
    h = hp(gold)
    m = build(gold).train()
    opt = AdamW(m.parameters(), lr=h["lr"], weight_decay=h["wd"], betas=h["betas"], eps=h["eps"], max_grad_norm=1.0)
    sched = get_cosine_schedule_with_warmup(opt, h["warmup"], h["total"])
    p0 = opt.flat.data.clone()
    lr0 = opt.param_groups[0]["lr"]
    x = torch.from_numpy(gold["s0/x"]).cuda()
    y = torch.from_numpy(gold["s0/y"]).cuda()
    GraphedTrainStep(m, x, y, opt, sched, h["la"], h["ld"], h["lc"], True, warmup=1)
    assert torch.equal(opt.flat.data, p0)
    assert opt.param_groups[0]["lr"] == lr0
    assert float(opt.flat.grad.abs().sum()) == 0.0


def test_router_through_matches_autograd_add(gold, monkeypatch):
    """RouterModule.forward_through: the routed block's input handed to the layer through the fused router node, so
    the layer's input gradient is added inside the router's LayerNorm backward instead of by autograd — one reference
    step's losses equal and every trainable gradient within 1e-5 (one f32 add of the same two values, inside or after
    the LayerNorm backward's own arithmetic)"""
    from vitmi import resvit
    from vitmi.resvit_train import total_loss
    h = hp(gold)
    runs = []
    for through in (False, True):
        monkeypatch.setattr(resvit, "ROUTER_THROUGH", through)
        m = build(gold).train()
        for j, r in enumerate(l.router for l in m.layers if hasattr(l, "router")):
            hh = torch.from_numpy(gold[f"s0/router{j}_hard"]).cuda()
            gg = torch.from_numpy(gold[f"s0/gumbel{j}"]).cuda()
            r.hard_override = lambda logits, hh=hh: hh
            r.gumbel_noise = lambda logits, gg=gg: gg
        x = torch.from_numpy(gold["s0/x"]).cuda()
        y = torch.from_numpy(gold["s0/y"]).cuda()
        c, a, d, ent, _ = m(x, y)
        total = total_loss(m, c, a, d, h["la"], h["ld"], h["lc"])
        total.backward()
        runs.append((float(total), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}))
    (t0, g0), (t1, g1) = runs
    assert t0 == t1
    assert g0.keys() == g1.keys() and len(g0) > 0
    for k in g0:
        assert rel(g1[k], g0[k]) < 1e-5, (k, rel(g1[k], g0[k]))


def test_share_teacher_matches_two_pass(gold, monkeypatch):
    """SHARE_TEACHER (advisor, round 5): the first routed layer's teacher output taken from the student's grad-enabled
    layer forward equals the reference's separate teacher pass (res-vit/model.py:496-512) — the first routed layer's
    teacher and student outputs bit-identical, one reference step's losses equal and every trainable gradient (LoRA,
    router, approximators, head) within 1e-6 — while the layer is deterministic (no active dropout: the share is gated
    on that, vitmi.resvit._active_dropout)"""
    from vitmi import resvit
    from vitmi.resvit_train import total_loss
    h = hp(gold)
    runs, outs = [], []
    for share in (False, True):
        monkeypatch.setattr(resvit, "SHARE_TEACHER", share)
        m = build(gold).train()
        assert not resvit._active_dropout(m.layers[0])
        for j, r in enumerate(l.router for l in m.layers if hasattr(l, "router")):
            hh = torch.from_numpy(gold[f"s0/router{j}_hard"]).cuda()
            gg = torch.from_numpy(gold[f"s0/gumbel{j}"]).cuda()
            r.hard_override = lambda logits, hh=hh: hh
            r.gumbel_noise = lambda logits, gg=gg: gg
        first = next(l for l in m.layers if l.use_reslr and l.layer_id >= l.dynamic_start_layer)
        seen = []
        hook = first.register_forward_hook(lambda mod, inp, out: seen.append((out[0].detach().clone(),
                                                                              out[1].detach().clone())))
        x = torch.from_numpy(gold["s0/x"]).cuda()
        y = torch.from_numpy(gold["s0/y"]).cuda()
        c, a, d, ent, _ = m(x, y)
        hook.remove()
        total = total_loss(m, c, a, d, h["la"], h["ld"], h["lc"])
        total.backward()
        outs.append(seen[0])
        runs.append((float(total), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}))
    (t0, g0), (t1, g1) = runs
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert t0 == t1
    assert g0.keys() == g1.keys() and len(g0) > 0
    for k in g0:
        assert rel(g1[k], g0[k]) < 1e-6, (k, rel(g1[k], g0[k]))
