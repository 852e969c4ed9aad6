#!/usr/bin/env python3
"""Throughput of vit_preprocess_u8 (uint8 HWC -> f32 NCHW, Pillow-exact bilinear resize + flip +
normalize) on a CIFAR batch at 32 -> 224 (bs 256) and an ImageNet-like 375x500 -> 224x298 batch
(bs 64), with HIP events; bytes = uint8 input read + f32 output written. Beside it, Pillow's resize
+ numpy ToTensor/Normalize on one host core for the same images (a bounded sample)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from vitmi.data import GPUTransform  # noqa: E402


def main():
    rng = np.random.default_rng(0)
    for b, h, w, size in [(256, 32, 32, 224), (64, 375, 500, 224)]:
        imgs = torch.from_numpy(rng.integers(0, 256, (b, h, w, 3), dtype=np.uint8)).cuda()
        t = GPUTransform(size, train=True, generator=torch.Generator().manual_seed(0))
        out = t(imgs)
        flips = torch.zeros(b, dtype=torch.uint8)
        for _ in range(3):
            t(imgs, flips=flips, out=out)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        s.record()
        for _ in range(n):
            t(imgs, flips=flips, out=out)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / n * 1e3
        byts = imgs.numel() + out.numel() * 4
        line = (f"{b}x{h}x{w} -> {tuple(out.shape[2:])}: {us:8.1f} us/batch  {b / us * 1e6:10.0f} img/s  "
                f"{byts / us / 1e3:7.1f} GB/s")
        try:
            from PIL import Image
            k = min(b, 16)
            arr = imgs[:k].cpu().numpy()
            oh, ow = out.shape[2], out.shape[3]
            t0 = time.perf_counter()
            for i in range(k):
                r = np.asarray(Image.fromarray(arr[i]).resize((ow, oh), Image.BILINEAR))
                x = (r.transpose(2, 0, 1).astype(np.float32) / np.float32(255) - np.float32(0.5)) / np.float32(0.5)
            cpu = k / (time.perf_counter() - t0)
            line += f"   | Pillow+numpy 1 core: {cpu:8.0f} img/s ({k} images)"
        except ImportError:
            pass
        print(line, flush=True)


if __name__ == "__main__":
    main()
