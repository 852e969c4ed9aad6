#!/usr/bin/env python3
"""Per-step loss of bench.py's engine loop (B/16 bs 256, OneCycleLR from step 0) under the reference's seed-42 init and
under the tamed init (oracle.tame_params): does the timed step run on finite numbers? (diagnostic tool)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from vitmi import ops  # noqa: E402
from vitmi.model import VisionTransformer  # noqa: E402


def run(tamed, steps=25, b=256):
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = VisionTransformer(image_size=(224, 224), patch_size=(16, 16), emb_dim=768, mlp_dim=3072, num_heads=12,
                              num_layers=12, num_classes=1000, attn_dropout_rate=0.0, dropout_rate=0.0)
    if tamed:
        from oracle.vit_oracle import tame_params
        model.load_state_dict(tame_params(model.state_dict()))
    model = model.to(dev)
    eng = model.engine()
    eng.refresh_mirror()
    g = torch.Generator(device=dev).manual_seed(1000)
    x = torch.randn(b, 3, 224, 224, device=dev, generator=g)
    y = torch.randint(0, 1000, (b,), device=dev, generator=g)
    mom = torch.zeros_like(eng.flat)
    table = bench.onecycle_hyper_table(steps, dev)
    hyper = table[0].clone()
    out = []
    for k in range(steps):
        ops.copy2d(hyper, 12, table[k], 12, 12, 1)
        eng.forward(x)
        dl, st = eng.cross_entropy(y, grad_scale=1.0 / b)
        eng.backward(dl)
        ops.sgd_step_dev(eng.flat, eng.grad, mom, eng.mirror, eng.layout.numel, hyper, 0.0)
        eng.refresh_mirror(full=False)
        out.append((float(st[:, 0].mean()), int(torch.isnan(eng.flat).sum()), float(eng.grad.norm())))
    return out


if __name__ == "__main__":
    for tamed in (False, True):
        print("tamed" if tamed else "reference seed-42 init", flush=True)
        for k, (loss, nans, gn) in enumerate(run(tamed)):
            print(f"  step {k:2d} loss {loss:.5f} nan params {nans} grad norm {gn:.4e}", flush=True)
