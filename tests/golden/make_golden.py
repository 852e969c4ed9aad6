"""Generate the golden fixtures under tests/golden/ from the reference itself.

Run HERE (the container that has /root/reference mounted):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own `src/model.py` (VisionTransformer) and drives it
with torch.optim.SGD + OneCycleLR configured exactly as reference
src/train.py:151-163 does. Outputs are small data files (inputs + expected
outputs); no reference source is copied. The GPU box never runs this script.

Fixtures
  ctor_b16.json      per-tensor checksums of the seed-42 reference constructor, ViT-B/16 @224, 1000 cls
  ctor_tiny.json     same, tiny config
  tiny.npz           tiny config (img 32, P 8, D 64, M 128, H 2, L 2, C 10, bs 4), tamed init:
                     params, input, labels, logits, loss, grads, params after 3 SGD+OneCycleLR steps,
                     per-step lr/momentum
  b16_tamed.npz      ViT-B/16 @224 tamed init, bs 2: input seed, logits, loss, per-param grad norms
  onecycle.npz       OneCycleLR lr/momentum trace, reference defaults (lr .03, 15000 steps, 500 warmup)
"""
import importlib.util
import json
import math
import os
import sys
from collections import OrderedDict

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/src"
sys.path.insert(0, REPO)
from oracle.vit_oracle import ViTConfig, tame_params  # noqa: E402  (tame = protocol, not algorithm)

TINY = dict(image_size=32, patch_size=8, emb_dim=64, mlp_dim=128, num_heads=2, num_layers=2, num_classes=10)
B16 = dict(image_size=224, patch_size=16, emb_dim=768, mlp_dim=3072, num_heads=12, num_layers=12, num_classes=1000)


def load_ref_model_module():
    spec = importlib.util.spec_from_file_location("ref_vit_model", os.path.join(REF_SRC, "model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def ref_model(mod, cfg, seed=42):
    torch.manual_seed(seed)  # set_seed(42), reference src/data_loaders.py:13-29 / src/train.py:88
    return mod.VisionTransformer(
        image_size=(cfg["image_size"], cfg["image_size"]), patch_size=(cfg["patch_size"], cfg["patch_size"]),
        emb_dim=cfg["emb_dim"], mlp_dim=cfg["mlp_dim"], num_heads=cfg["num_heads"],
        num_layers=cfg["num_layers"], num_classes=cfg["num_classes"],
        attn_dropout_rate=0.0, dropout_rate=0.0)  # presets force 0.0 (reference src/config.py:64-65)


def checksums(sd):
    out = OrderedDict()
    for k, v in sd.items():
        a = v.detach().double().reshape(-1)
        out[k] = dict(shape=list(v.shape), sum=float(a.sum()), abs_sum=float(a.abs().sum()),
                      head=[float(t) for t in v.detach().reshape(-1)[:8]])
    return out


def main():
    torch.set_num_threads(8)
    mod = load_ref_model_module()

    # ---- constructor checksums ------------------------------------------------------------------
    for name, cfg in (("b16", B16), ("tiny", TINY)):
        m = ref_model(mod, cfg)
        with open(os.path.join(HERE, f"ctor_{name}.json"), "w") as f:
            json.dump(checksums(m.state_dict()), f)

    # ---- tiny config full trajectory (tamed init) -------------------------------------------------
    m = ref_model(mod, TINY)
    sd = tame_params(OrderedDict((k, v.detach().clone()) for k, v in m.state_dict().items()))
    m.load_state_dict(sd)
    g = torch.Generator().manual_seed(123)
    bs = 4
    x = torch.randn(bs, 3, TINY["image_size"], TINY["image_size"], generator=g)
    y = torch.randint(0, TINY["num_classes"], (bs,), generator=g)
    crit = torch.nn.CrossEntropyLoss()
    lr, wd, steps, warm = 0.03, 1e-4, 10, 2
    opt = torch.optim.SGD(params=m.parameters(), lr=lr, weight_decay=wd, momentum=0.9)
    sched = torch.optim.lr_scheduler.OneCycleLR(optimizer=opt, max_lr=lr, pct_start=warm / steps, total_steps=steps)
    data = {}
    for k, v in sd.items():
        data["p0/" + k] = v.numpy()
    data["x"] = x.numpy()
    data["y"] = y.numpy()
    lrs, moms, losses = [], [], []
    for step in range(3):
        lrs.append(opt.param_groups[0]["lr"])
        moms.append(opt.param_groups[0]["momentum"])
        opt.zero_grad()
        logits = m(x)
        loss = crit(logits, y)
        loss.backward()
        if step == 0:
            data["logits0"] = logits.detach().numpy()
            data["loss0"] = np.float32(loss.item())
            for k, v in m.named_parameters():
                data["g0/" + k] = v.grad.detach().numpy()
        losses.append(loss.item())
        opt.step()
        sched.step()
    for k, v in m.state_dict().items():
        data["p3/" + k] = v.detach().numpy()
    data["lrs"] = np.array(lrs)
    data["moms"] = np.array(moms)
    data["losses"] = np.array(losses)
    data["hparams"] = np.array([lr, wd, steps, warm])
    np.savez_compressed(os.path.join(HERE, "tiny.npz"), **data)

    # ---- ViT-B/16 tamed, bs 2 -------------------------------------------------------------------
    m = ref_model(mod, B16)
    sd = tame_params(OrderedDict((k, v.detach().clone()) for k, v in m.state_dict().items()))
    m.load_state_dict(sd)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 3, 224, 224, generator=g)
    y = torch.randint(0, 1000, (2,), generator=g)
    logits = m(x)
    loss = torch.nn.CrossEntropyLoss()(logits, y)
    loss.backward()
    names = [k for k, _ in m.named_parameters()]
    gn = np.array([float(p.grad.double().norm()) for _, p in m.named_parameters()])
    np.savez_compressed(os.path.join(HERE, "b16_tamed.npz"), input_seed=np.int64(7), labels=y.numpy(),
                        logits=logits.detach().numpy(), loss=np.float32(loss.item()), grad_norms=gn,
                        grad_names=np.array(names))

    # ---- OneCycleLR trace with the reference defaults (src/config.py:43-45) ----------------------
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=0.03, momentum=0.9, weight_decay=0.0)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=0.03, pct_start=500 / 15000, total_steps=15000)
    lrs, moms = [], []
    for _ in range(15000):
        lrs.append(opt.param_groups[0]["lr"])
        moms.append(opt.param_groups[0]["momentum"])
        opt.step()
        sched.step()
    np.savez_compressed(os.path.join(HERE, "onecycle.npz"), lrs=np.array(lrs), moms=np.array(moms))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
