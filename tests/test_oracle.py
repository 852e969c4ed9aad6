"""Pin the CPU oracle against golden vectors generated from the reference (tests/golden/make_golden.py)."""
import json
import os
from collections import OrderedDict

import numpy as np
import pytest
import torch

from oracle.vit_oracle import (OneCycle, ViTConfig, accuracy, cross_entropy, forward, init_params,
                               loss_and_grads, param_names, sgd_step, tame_params, train_flops_per_image)

TINY = ViTConfig(image_size=32, patch_size=8, emb_dim=64, mlp_dim=128, num_heads=2, num_layers=2, num_classes=10)
B16 = ViTConfig()


def _rel(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("name,cfg", [("tiny", TINY), ("b16", B16)])
def test_ctor_bit_exact(golden_dir, name, cfg):
    ref = json.load(open(os.path.join(golden_dir, f"ctor_{name}.json")))
    params = init_params(cfg, seed=42)
    assert list(params.keys()) == list(ref.keys()) == param_names(cfg)
    for k, v in params.items():
        r = ref[k]
        assert list(v.shape) == r["shape"], k
        assert [float(t) for t in v.reshape(-1)[:8]] == r["head"], k  # bit-exact first values
        assert float(v.double().sum()) == r["sum"], k
        assert float(v.double().abs().sum()) == r["abs_sum"], k


def _tiny_golden(golden_dir):
    z = np.load(os.path.join(golden_dir, "tiny.npz"))
    p0 = OrderedDict((k, torch.from_numpy(z["p0/" + k].copy())) for k in param_names(TINY))
    return z, p0


def test_tiny_tamed_matches_protocol(golden_dir):
    z, p0 = _tiny_golden(golden_dir)
    tamed = tame_params(init_params(TINY, seed=42))
    for k in p0:
        assert torch.equal(tamed[k], p0[k]), k


def test_tiny_forward_backward(golden_dir):
    z, p0 = _tiny_golden(golden_dir)
    x = torch.from_numpy(z["x"])
    y = torch.from_numpy(z["y"])
    logits, loss, grads = loss_and_grads(p0, x, y, TINY)
    assert _rel(logits, z["logits0"]) < 1e-5
    assert abs(float(loss) - float(z["loss0"])) <= 1e-5 * abs(float(z["loss0"]))
    for k, g in grads.items():
        assert _rel(g, z["g0/" + k]) < 1e-4 or float(torch.as_tensor(z["g0/" + k]).norm()) < 1e-7, k


def test_tiny_three_sgd_onecycle_steps(golden_dir):
    z, p0 = _tiny_golden(golden_dir)
    x = torch.from_numpy(z["x"])
    y = torch.from_numpy(z["y"])
    lr, wd, steps, warm = [float(t) for t in z["hparams"]]
    sched = OneCycle(lr, int(steps), warm / steps)
    params, bufs = OrderedDict((k, v.clone()) for k, v in p0.items()), {}
    for step in range(3):
        slr, smom = sched.at(step)
        assert abs(slr - z["lrs"][step]) < 1e-12 and abs(smom - z["moms"][step]) < 1e-12
        _, loss, grads = loss_and_grads(params, x, y, TINY)
        assert abs(float(loss) - z["losses"][step]) < 1e-5 * abs(z["losses"][step])
        params, bufs = sgd_step(params, grads, bufs, slr, smom, wd, first=(step == 0))
    for k in params:
        # attn.key.bias has a true gradient of 0 (softmax shift invariance): its update is
        # fp32 noise ~1e-11, so it is compared with an absolute tolerance instead.
        ref = torch.from_numpy(z["p3/" + k]).double()
        err = float((params[k].double() - ref).norm())
        assert err <= 1e-5 * float(ref.norm()) + 1e-8, k


def test_onecycle_trace(golden_dir):
    z = np.load(os.path.join(golden_dir, "onecycle.npz"))
    s = OneCycle(0.03, 15000, 500 / 15000)
    for step in list(range(0, 600)) + [1000, 5000, 14998, 14999]:
        lr, m = s.at(step)
        assert abs(lr - z["lrs"][step]) <= 1e-12 + 1e-9 * z["lrs"][step]
        assert abs(m - z["moms"][step]) <= 1e-12


@pytest.mark.slow
def test_b16_tamed_logits_loss_grads(golden_dir):
    z = np.load(os.path.join(golden_dir, "b16_tamed.npz"))
    params = tame_params(init_params(B16, seed=42))
    g = torch.Generator().manual_seed(int(z["input_seed"]))
    x = torch.randn(2, 3, 224, 224, generator=g)
    y = torch.from_numpy(z["labels"])
    logits, loss, grads = loss_and_grads(params, x, y, B16)
    assert _rel(logits, z["logits"]) < 1e-4
    assert abs(float(loss) - float(z["loss"])) < 1e-5 * float(z["loss"])
    names = list(z["grad_names"])
    gn = z["grad_norms"]
    tot = float(np.sqrt((gn ** 2).sum()))
    for n_, ref in zip(names, gn):
        mine = float(grads[n_].double().norm())
        assert abs(mine - ref) <= 1e-3 * ref + 1e-6 * tot, n_


def test_flops_formula():
    # validated against torch FlopCounterMode on the reference model
    assert abs(train_flops_per_image(B16) / 1e9 - 105.152) < 1e-3
    assert abs(train_flops_per_image(ViTConfig(image_size=32, patch_size=32, num_classes=100)) / 1e9 - 1.030) < 1e-3
    l16 = ViTConfig(emb_dim=1024, mlp_dim=4096, num_heads=16, num_layers=24)
    assert abs(train_flops_per_image(l16) / 1e9 - 369.020) < 1e-3


def test_accuracy_and_ce():
    logits = torch.tensor([[0.1, 2.0, 0.3], [1.0, 0.0, -1.0]])
    y = torch.tensor([1, 2])
    a1, = accuracy(logits, y, topk=(1,))
    assert float(a1) == 50.0
    ce = cross_entropy(logits, y)
    assert abs(float(ce) - float(torch.nn.functional.cross_entropy(logits, y))) < 1e-7
