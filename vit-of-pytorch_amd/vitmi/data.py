"""Device-side input pipeline: the reference's loader transforms run as one HIP kernel.

Reference `src/data_loaders.py:66-80` (CIFAR-10/100 train: `transforms.Compose([Resize(size),
RandomHorizontalFlip(), ToTensor(), Normalize([0.5]*3, [0.5]*3)])`, eval without the flip) and
`:100-112` (ImageNet: `Resize((size, size))`). torchvision is not part of this stack: uint8 HWC
batches (as decoded / as CIFAR stores them) go to the GPU once and `vit_preprocess_u8` produces
the f32 NCHW model input, with the resize bit-exact to Pillow's BILINEAR (the arithmetic under
torchvision's PIL path; oracle/preprocess.py, tests/test_preprocess_cpu.py and
tests/test_preprocess_gpu.py). Flip draws come from a torch.Generator: the per-worker RNG streams
of the reference's DataLoader are not reproducible, the decision rule (rand < p) is the same.
"""
from __future__ import annotations

import torch

from . import ops


def resized_size(h: int, w: int, size):
    """torchvision `Resize(size)` output (h, w): an int maps the shorter side to `size` keeping the
    aspect ratio (longer side truncated); a pair is (h, w)."""
    if isinstance(size, (tuple, list)):
        return int(size[0]), int(size[1])
    if w <= h:
        return int(size * h / w), int(size)
    return int(size), int(size * w / h)


class GPUTransform:
    """Compose([Resize(size), RandomHorizontalFlip(p)?, ToTensor(), Normalize(mean, std)]) over a
    uint8 [B, H, W, 3] batch on the device -> float32 [B, 3, h, w]."""

    def __init__(self, size, train: bool = True, flip_p: float = 0.5, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5),
                 generator: torch.Generator | None = None):
        self.size = size
        self.train = train
        self.flip_p = flip_p
        self.mean = tuple(mean)
        self.std = tuple(std)
        self.generator = generator

    def __call__(self, images: torch.Tensor, flips: torch.Tensor | None = None, out: torch.Tensor | None = None):
        if images.dtype != torch.uint8 or images.dim() != 4 or images.shape[3] != 3:
            raise ValueError(f"expected uint8 images [B, H, W, 3], got {images.dtype} {tuple(images.shape)}")
        if not images.is_cuda:
            raise ValueError("GPUTransform runs on the device: move the uint8 batch to the GPU first")
        images = images.contiguous()
        B, H, W, _ = images.shape
        h, w = resized_size(H, W, self.size)
        if flips is None and self.train and self.flip_p > 0:
            flips = torch.rand(B, generator=self.generator) < self.flip_p
        if flips is not None:
            flips = flips.to(device=images.device, dtype=torch.uint8)
        if out is None:
            out = torch.empty(B, 3, h, w, device=images.device, dtype=torch.float32)
        ops.preprocess_u8(images, out, flips, self.mean, self.std)
        return out
