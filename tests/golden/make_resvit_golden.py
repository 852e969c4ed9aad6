"""Generate tests/golden/resvit_tiny.npz from the reference Res-ViT itself (res-vit/model.py).

Run HERE (the container that has /root/reference mounted):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_resvit_golden.py          # resvit_tiny.npz
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_resvit_golden.py --b16    # resvit_b16.npz

Imports the reference's own `res-vit/model.py` (+ `model_utils.py`; einops is installed) and runs its
`Transformer` on a tiny configuration with every Res-ViT feature on (use_lora, use_reslr, two blocks of
block_size 2, router, low-rank approximators, teacher/student paths):
  * eval mode: the ragged inference path (router argmax, queries = active tokens, keys = all tokens,
    res-vit/model.py:494-529): logits, c_loss, router entropy, active ratio, per-block hard routing;
  * train mode: one forward/backward of 10 c_loss + 10 a_loss + 1 d_loss (res-vit/train.py:56) with the
    Gumbel noise of every router call recorded (F.gumbel_softmax is wrapped to draw its noise exactly as
    torch does and keep it), so the MI355X implementation can be fed the same noise: logits, the three
    losses, router entropy and the gradient of every trainable parameter.
Every router call's input tokens, decision logits and hard keep decisions are recorded too: the GPU
tests check the router on its own against them and replay the reference's discrete decisions into the
end-to-end comparison (a decision whose logit margin is below bf16 noise would otherwise flip).
Weights: the reference constructor under torch.manual_seed(42), then a deterministic well-conditioned
rescale (the parity protocol of SURVEY.md §8c, extended to the Res-ViT modules; see tame()). Data only;
no reference source is copied. The GPU box never runs this script.

--b16: BASELINE config C5's model, Res-ViT-B/16 @224 with the res-vit/config.py training defaults
(LoRA rank 8 + residual low-rank paths, router from layer 2, active target 0.6, block size 1, 100
classes), batch 2. Too large to store its weights, so the fixture holds per-tensor fingerprints
(f64 sum and sum of squares) of the seed-42 + tame() parameters, the eval / train outputs, every
router call's hard decisions and Gumbel draws (for replay), and per-parameter gradient norms; the
inputs are regenerated from a seeded CPU generator (INPUT_SEED).
"""
import importlib.util
import json
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/res-vit"

CFG = dict(dim=64, mlp_dim=128, n_layers=5, n_heads=2, n_kv_heads=2, norm_eps=1e-5, lora_rank=4,
           dynamic_active_target=0.4, dynamic_start_layer=1, dynamic_router_hdim=32, dynamic_reserve_initials=1,
           low_rank_dim=16, block_size=2, use_lora=True, use_reslr=True, image_size=(32, 32), patch_size=(8, 8),
           num_classes=10, device="cpu")
BS = 3

# Res-ViT-B/16 @224, res-vit/config.py get_train_config defaults (use_lora / use_reslr on)
B16 = dict(dim=768, mlp_dim=3072, n_layers=12, n_heads=12, n_kv_heads=12, norm_eps=1e-5, lora_rank=8,
           dynamic_active_target=0.6, dynamic_start_layer=2, dynamic_router_hdim=512, dynamic_reserve_initials=1,
           low_rank_dim=256, block_size=1, use_lora=True, use_reslr=True, image_size=(224, 224),
           patch_size=(16, 16), num_classes=100, device="cpu")
B16_BS = 2
INPUT_SEED = 7


def b16_inputs():
    g = torch.Generator().manual_seed(INPUT_SEED)
    x = torch.randn(B16_BS, 3, 224, 224, generator=g)
    y = torch.randint(0, B16["num_classes"], (B16_BS,), generator=g)
    return x, y


def load_ref():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    spec = importlib.util.spec_from_file_location("ref_resvit_model", os.path.join(REF, "model.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def tame(model, seed=1):
    """deterministic rescale in named_parameters() order: attention / LoRA / approximator / router weights
    to well-conditioned scales, the router's decision layer so that routing depends on the input."""
    g = torch.Generator().manual_seed(seed)
    rn = lambda t, s: torch.randn(t.shape, generator=g) * s
    with torch.no_grad():
        for n, p in model.named_parameters():
            if ".attention.w" in n and n.endswith("weight"):
                p.copy_(rn(p, 1.0 / math.sqrt(p.shape[1])))
            elif ".attention.w" in n and n.endswith("bias"):
                p.copy_(rn(p, 0.05))
            elif "lora_" in n or "approximators" in n:
                p.copy_(rn(p, 0.1 / math.sqrt(p.shape[1])))
            elif "router.out_conv.4" in n:  # decision layer: no bias, so routing follows the tokens
                p.copy_(rn(p, 8.0) if n.endswith("weight") else torch.zeros_like(p))
            elif n == "pos_embedding.pos_embedding" or n == "classifier.weight":
                p.copy_(rn(p, 0.02))
            elif "norm" in n:
                p.copy_((1.0 if n.endswith("weight") else 0.0) + rn(p, 0.05))


def _router_taps(model, rec):
    """record, per router call: its input tokens, its decision logits and its hard keep decisions"""
    hooks = []
    for l in model.layers:
        if hasattr(l, "router"):
            hooks.append(l.router.register_forward_hook(lambda m_, i_, o_: rec.append(
                {"x": i_[0].detach().clone(), "hard": o_[0].detach().clone()})))
            hooks.append(l.router.out_conv.register_forward_hook(lambda m_, i_, o_: rec.append(
                {"logits": o_.detach().clone()})))
    return hooks


def run_eval(model, x, y):
    rec = []
    hooks = _router_taps(model, rec)
    model.eval()
    with torch.no_grad():
        res = model(x, y)
    for h_ in hooks:
        h_.remove()
    return res, rec


def run_train(mod, model, x, y, seed):
    noise, rec = [], []
    orig = F.gumbel_softmax

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
        model.zero_grad()
        torch.manual_seed(seed)
        res = model(x, y)
        c, a, d = res[:3]
        (10.0 * c + 10.0 * a + 1.0 * d).backward()
    finally:
        mod.F.gumbel_softmax = orig
        for h_ in hooks:
            h_.remove()
    return res, noise, rec


def _save_router(out, tag, rec):
    """rec alternates {logits} (out_conv, fires first) and {x, hard} (router) per router call"""
    calls = [(rec[i]["logits"], rec[i + 1]) for i in range(0, len(rec), 2)]
    for j, (lg, r) in enumerate(calls):
        out[f"{tag}/router{j}_x"] = r["x"].numpy()
        out[f"{tag}/router{j}_logits"] = lg.numpy()
        out[f"{tag}/router{j}_hard"] = r["hard"].numpy()


def main():
    mod = load_ref()
    torch.manual_seed(42)
    args = mod.ModelArgs(**CFG)
    model = mod.Transformer(args)
    tame(model)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    g = torch.Generator().manual_seed(7)
    x = torch.randn(BS, 3, 32, 32, generator=g)
    y = torch.randint(0, CFG["num_classes"], (BS,), generator=g)
    (c, a, d, ent, metric), rec_e = run_eval(model, x, y)
    logits_eval = model.logits.clone()
    maps = {k: v.clone() for k, v in model.routing_maps.items()}
    (tc, ta, td, tent, tmetric), noise, rec_t = run_train(mod, model, x, y, 11)
    out = {"x": x.numpy(), "y": y.numpy()}
    out.update({"p/" + k: v.numpy() for k, v in sd.items()})
    out["trainable"] = np.array([n for n, p in model.named_parameters() if p.requires_grad])
    mu = sys.modules["model_utils"]
    out["lra_masks_json"] = np.array(json.dumps({bs: mu.get_indices_from_LRA_mask(bs) for bs in (1, 2, 4)}))
    out["eval/logits"] = logits_eval.numpy()
    out["eval/c_loss"] = np.float64(c)
    out["eval/r_entropy"] = np.float64(ent)
    out["eval/active_ratio"] = np.float64(metric["non_low_rank_ratio"])
    for k, v in maps.items():
        out[f"eval/routing{k}"] = v.numpy()
    _save_router(out, "eval", rec_e)
    _save_router(out, "train", rec_t)
    out["train/logits"] = model.logits.detach().numpy()
    for k, v in (("c_loss", tc), ("a_loss", ta), ("d_loss", td), ("r_entropy", tent)):
        out[f"train/{k}"] = np.float64(v.detach())
    out["train/active_ratio"] = np.float64(tmetric["non_low_rank_ratio"])
    for i, n_ in enumerate(noise):
        out[f"train/gumbel{i}"] = n_.numpy()
    for k, v in model.routing_maps.items():
        out[f"train/routing{k}"] = v.numpy()
    for n, p in model.named_parameters():
        if p.requires_grad:
            out["grad/" + n] = (p.grad if p.grad is not None else torch.zeros_like(p)).numpy()
    dst = os.path.join(HERE, "resvit_tiny.npz")
    np.savez_compressed(dst, **out)
    print(f"wrote {dst}: eval active ratio {float(out['eval/active_ratio']):.3f}; train losses c {float(tc):.4f} "
          f"a {float(ta):.4f} d {float(td):.6f}")


def main_b16():
    mod = load_ref()
    torch.manual_seed(42)
    model = mod.Transformer(mod.ModelArgs(**B16))
    tame(model)
    out = {"cfg_json": np.array(json.dumps({k: v for k, v in B16.items() if k != "device"}))}
    for k, v in model.state_dict().items():
        t = v.detach().double()
        out["fp/" + k] = np.array([float(t.sum()), float((t * t).sum())])
    x, y = b16_inputs()
    (c, a, d, ent, metric), rec_e = run_eval(model, x, y)
    out["eval/logits"] = model.logits.clone().numpy()
    out["eval/c_loss"] = np.float64(c)
    out["eval/r_entropy"] = np.float64(ent)
    out["eval/active_ratio"] = np.float64(metric["non_low_rank_ratio"])
    for k, v in model.routing_maps.items():
        out[f"eval/routing{k}"] = v.numpy()
    for j, i in enumerate(range(0, len(rec_e), 2)):
        out[f"eval/router{j}_hard"] = rec_e[i + 1]["hard"].numpy()
    (tc, ta, td, tent, tmetric), noise, rec_t = run_train(mod, model, x, y, 11)
    out["train/logits"] = model.logits.detach().numpy()
    for k, v in (("c_loss", tc), ("a_loss", ta), ("d_loss", td), ("r_entropy", tent)):
        out[f"train/{k}"] = np.float64(v.detach())
    for i, n_ in enumerate(noise):
        out[f"train/gumbel{i}"] = n_.numpy()
    for j, i in enumerate(range(0, len(rec_t), 2)):
        out[f"train/router{j}_hard"] = rec_t[i + 1]["hard"].numpy()
    out["trainable"] = np.array([n for n, p in model.named_parameters() if p.requires_grad])
    for n, p in model.named_parameters():
        if p.requires_grad:
            gr = p.grad if p.grad is not None else torch.zeros_like(p)
            out["gnorm/" + n] = np.float64(gr.double().norm())
    dst = os.path.join(HERE, "resvit_b16.npz")
    np.savez_compressed(dst, **out)
    print(f"wrote {dst}: eval active ratio {float(out['eval/active_ratio']):.3f}; train losses c {float(tc):.4f} "
          f"a {float(ta):.4f} d {float(td):.6f}; {len(noise)} router calls")


if __name__ == "__main__":
    if "--b16" in sys.argv[1:]:
        main_b16()
    else:
        main()
