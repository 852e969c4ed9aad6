#!/usr/bin/env python3
"""Diagnostic: per-parameter gradient errors of the HIP step vs the fp32 oracle (ViT-B/16, tamed, bs 2)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from oracle.vit_oracle import ViTConfig, init_params, loss_and_grads, tame_params  # noqa: E402
from vitmi.model import VisionTransformer  # noqa: E402

cfg = ViTConfig()
params = tame_params(init_params(cfg, seed=42))
g = torch.Generator().manual_seed(7)
x = torch.randn(2, 3, 224, 224, generator=g)
y = torch.randint(0, 1000, (2,), generator=g)
rl, rloss, rg = loss_and_grads(params, x, y, cfg, dtype=torch.float64)
torch.manual_seed(42)
m = VisionTransformer(image_size=(224, 224), patch_size=(16, 16), num_classes=1000, dropout_rate=0.0)
m.load_state_dict(params)
m = m.cuda()
logits = m(x.cuda())
loss = torch.nn.functional.cross_entropy(logits, y.cuda())
loss.backward()
print("loss", float(loss), float(rloss), "logits rel", float((logits.detach().cpu().double() - rl).norm() / rl.norm()))
named = dict(m.named_parameters())
errs = []
for k, v in rg.items():
    mine = named[k].grad.detach().cpu().double()
    e = float((mine - v).norm() / v.norm().clamp_min(1e-30))
    errs.append((e, k, float(v.norm()), float(mine.norm())))
errs.sort(reverse=True)
for e in errs[:25]:
    print(f"{e[0]:.4e}  {e[1]:55s} ref_norm {e[2]:.4e} mine {e[3]:.4e}")
