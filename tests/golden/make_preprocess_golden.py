"""Writes tests/golden/preprocess.npz: Pillow 12.2.0 `Image.resize(..., BILINEAR)` outputs (the
arithmetic under torchvision's `Resize` in the reference's loaders, src/data_loaders.py:66-80,
100-112) for seeded random uint8 RGB images. Run here (Pillow importable); the fixture travels.
    python tests/golden/make_preprocess_golden.py
"""
import os

import numpy as np
from PIL import Image

# (in_h, in_w, out_h, out_w): CIFAR 32 -> 224 (the C1/C2 upsample), odd up/down ratios, ImageNet-like
# non-square downsamples as torchvision Resize(224) sizes them, identity, a 1-pixel-wide source.
CASES = [(32, 32, 224, 224), (32, 32, 56, 56), (50, 40, 24, 30), (17, 33, 64, 64), (150, 100, 112, 74),
         (150, 200, 112, 149), (64, 64, 64, 64), (7, 9, 13, 5), (160, 160, 32, 32), (1, 6, 3, 1)]


def main():
    rng = np.random.default_rng(2024)
    out = {}
    for i, (h, w, oh, ow) in enumerate(CASES):
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        out[f"in{i}"] = img
        out[f"out{i}"] = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
    out["cases"] = np.array(CASES, np.int64)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "preprocess.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


if __name__ == "__main__":
    main()
