"""Evaluation entry point, mirroring reference src/eval.py:12-77 on the MI355X HIP engine.

    python -m vitmi.eval --model-arch b16 --image-size 384 --checkpoint-path w.pth --synthetic

Same flow as the reference: get_eval_config (src/config.py:5-25, default 384 px, 1000 classes) ->
set_seed -> VisionTransformer -> load_checkpoint (.pth / JAX .npz) -> forward over the val split
under torch.no_grad() -> mean top-1 / top-5 over batches, printed in the reference's format.
Top-1 / top-5 come from the fused cross-entropy kernel's per-row hit counts (vit_cross_entropy,
src/utils.py:28-41 semantics) instead of a topk pass. Sequences above 320 tokens (384 px: 577 for
B/16 and L/16, 730 for H/14) run the K/V-tiled attention kernels. `--precision fp32` evaluates with
the reference's own f32 arithmetic (vit_gemm_f32 projections, f32 attention).
Data: torchvision is absent here, so the val split is synthetic (--synthetic), as in vitmi.train.
"""
from __future__ import annotations

import sys

import numpy as np
import torch

from . import ops
from .config import get_eval_config
from .train import SyntheticDataLoader, build_model, load_checkpoint, set_seed


def evaluate(model, data_loader, device):
    """Mean top-1 / top-5 (%) over batches (src/eval.py:56-75)."""
    acc1s, acc5s = [], []
    model.eval()
    with torch.no_grad():
        for data, target in data_loader:
            data = data.to(device)
            target = target.to(device, torch.int64)
            logits = model(data).float().contiguous()
            st = torch.empty(logits.shape[0], 3, device=device)
            ops.cross_entropy(logits, target.contiguous(), None, 1.0, st)
            acc1s.append(st[:, 1].mean() * 100.0)
            acc5s.append(st[:, 2].mean() * 100.0)
    return float(torch.stack(acc1s).mean()), float(torch.stack(acc5s).mean())


def main(argv=None):
    config = get_eval_config(argv)
    set_seed(config.seed)
    if not torch.cuda.is_available():
        raise SystemExit("vitmi.eval needs a ROCm GPU (MI355X)")
    device = torch.device("cuda", 0)
    model = build_model(config, device)
    if config.checkpoint_path:
        state_dict = load_checkpoint(config.checkpoint_path)
        model.load_state_dict(state_dict)
        print("Load pretrained weights from {}".format(config.checkpoint_path))
    model = model.to(device)
    model.precision = config.precision
    if not config.synthetic:
        raise SystemExit("torchvision datasets are not available in this environment; use --synthetic "
                         "(the input pipeline is outside the MI355X hot path, SURVEY.md §2 row 5)")
    data_loader = SyntheticDataLoader(config.batch_size, config.image_size, config.num_classes,
                                      config.steps_per_epoch, device, seed=config.seed)
    print("Starting evaluation")
    acc1, acc5 = evaluate(model, data_loader, device)
    print("Evaluation of model {:s} on dataset {:s}, Acc@1: {:.4f}, Acc@5: {:.4f}".format(
        config.model_arch, config.dataset, acc1, acc5))
    return acc1, acc5


if __name__ == "__main__":
    main(sys.argv[1:])
