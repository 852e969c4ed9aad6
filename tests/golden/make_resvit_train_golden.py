"""Generate tests/golden/resvit_train3.npz: three Res-ViT training steps of the reference itself.

Run HERE (the container that has /root/reference mounted):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_resvit_train_golden.py

Imports the reference's own `res-vit/model.py` (as make_resvit_golden.py does) and runs the body of
`res-vit/train.py:train_epoch` (:23-68) for three batches on the tiny all-features configuration:
  optimizer.zero_grad(); c, a, d, ... = model(x, y)
  total = lambda_class * c + lambda_active * a + lambda_distill * d   (res-vit/config.py defaults 1, 1e-4, 1e-2)
  total.backward(); torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0, norm_type=2)
  optimizer.step(); lr_scheduler.step()
with the optimizer and schedule of res-vit/train.py:264-291: torch.optim.AdamW(model.parameters(), lr,
weight_decay, betas, eps) and transformers.get_cosine_schedule_with_warmup(optimizer, warmup, total)
(installed here: the reference's own dependency). The lr is raised from 1e-4 to 1e-2 so three steps move
the weights visibly; warmup 2 of 10 steps makes the first step's lr exactly 0.

Recorded per step: the batch, the three losses and the total, the Gumbel draws and hard decisions of every
router call (for replay on the GPU), clip_grad_norm_'s returned norm, every trainable parameter's gradient
before and after clipping, which parameters had a gradient (approximators no token was routed to have
none: AdamW skips them), the lr; and after the three steps every trainable parameter and its AdamW state
(exp_avg, exp_avg_sq, step). Weights: seed-42 constructor + make_resvit_golden.tame(). Data only.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_resvit_golden import CFG, _router_taps, load_ref, tame  # noqa: E402

BS = 3
STEPS = 3
LR, WD, BETAS, EPS = 1e-2, 0.05, (0.9, 0.999), 1e-8
WARMUP, TOTAL = 2, 10
LAMBDA_CLASS, LAMBDA_ACTIVE, LAMBDA_DISTILL = 1.0, 1e-4, 1e-2


def main():
    from transformers import get_cosine_schedule_with_warmup
    mod = load_ref()
    torch.manual_seed(42)
    model = mod.Transformer(mod.ModelArgs(**CFG))
    tame(model)
    out = {"p0/" + k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    trainable = [n for n, p in model.named_parameters() if p.requires_grad]
    out["trainable"] = np.array(trainable)
    out["hparams"] = np.array([LR, WD, BETAS[0], BETAS[1], EPS, WARMUP, TOTAL, LAMBDA_CLASS, LAMBDA_ACTIVE,
                               LAMBDA_DISTILL])
    optimizer = torch.optim.AdamW(params=model.parameters(), lr=LR, weight_decay=WD, betas=BETAS, eps=EPS)
    sched = get_cosine_schedule_with_warmup(optimizer, num_warmup_steps=WARMUP, num_training_steps=TOTAL)
    g = torch.Generator().manual_seed(21)
    orig = F.gumbel_softmax
    for step in range(STEPS):
        x = torch.randn(BS, 3, 32, 32, generator=g)
        y = torch.randint(0, CFG["num_classes"], (BS,), generator=g)
        noise, rec = [], []

        def recording_gumbel_softmax(logits, tau=1, hard=False, eps=1e-10, dim=-1):
            gumbels = -torch.empty_like(logits, memory_format=torch.legacy_contiguous_format).exponential_().log()
            noise.append(gumbels.detach().clone())
            y_soft = ((logits + gumbels) / tau).softmax(dim)
            if hard:
                index = y_soft.max(dim, keepdim=True)[1]
                y_hard = torch.zeros_like(logits, memory_format=torch.legacy_contiguous_format).scatter_(dim, index, 1.0)
                return y_hard - y_soft.detach() + y_soft
            return y_soft

        mod.F.gumbel_softmax = recording_gumbel_softmax
        hooks = _router_taps(model, rec)
        try:
            model.train()
            torch.manual_seed(100 + step)
            out[f"s{step}/lr"] = np.float64(optimizer.param_groups[0]["lr"])
            optimizer.zero_grad()
            c, a, d, ent, metric = model(x, y)
            total = LAMBDA_CLASS * c + LAMBDA_ACTIVE * a + LAMBDA_DISTILL * d
            total.backward()
        finally:
            mod.F.gumbel_softmax = orig
            for h_ in hooks:
                h_.remove()
        params = dict(model.named_parameters())
        for n in trainable:
            gr = params[n].grad
            out[f"s{step}/has_grad/{n}"] = np.bool_(gr is not None)
            if gr is not None:
                out[f"s{step}/grad/{n}"] = gr.detach().clone().numpy()
        norm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0, norm_type=2)
        for n in trainable:
            if params[n].grad is not None:
                out[f"s{step}/cgrad/{n}"] = params[n].grad.detach().clone().numpy()
        optimizer.step()
        sched.step()
        out[f"s{step}/x"] = x.numpy()
        out[f"s{step}/y"] = y.numpy()
        for k_, v_ in (("c_loss", c), ("a_loss", a), ("d_loss", d), ("total", total), ("r_entropy", ent)):
            out[f"s{step}/{k_}"] = np.float64(v_.detach())
        out[f"s{step}/norm"] = np.float64(norm)
        out[f"s{step}/logits"] = model.logits.detach().numpy()
        for i, n_ in enumerate(noise):
            out[f"s{step}/gumbel{i}"] = n_.numpy()
        for j, i in enumerate(range(0, len(rec), 2)):
            out[f"s{step}/router{j}_hard"] = rec[i + 1]["hard"].numpy()
    params = dict(model.named_parameters())
    for n in trainable:
        out["p3/" + n] = params[n].detach().numpy()
        st = optimizer.state.get(params[n], {})
        if st:
            out["m3/" + n] = st["exp_avg"].numpy()
            out["v3/" + n] = st["exp_avg_sq"].numpy()
            out["t3/" + n] = np.float64(st["step"])
    dst = os.path.join(HERE, "resvit_train3.npz")
    np.savez_compressed(dst, **out)
    unused = sum(1 for k in out if "/has_grad/" in k and not out[k])
    print(f"wrote {dst}: totals {[round(float(out[f's{s}/total']), 5) for s in range(STEPS)]}, norms "
          f"{[round(float(out[f's{s}/norm']), 4) for s in range(STEPS)]}, {unused} (step, param) pairs without grad")


if __name__ == "__main__":
    main()
