"""Training-input transform of the reference, restated on the CPU (test infrastructure only).

Reference: `src/data_loaders.py:66-80` (CIFAR-100 train: `Resize(image_size)`,
`RandomHorizontalFlip()`, `ToTensor()`, `Normalize([0.5]*3, [0.5]*3)`; eval drops the flip) and
`:100-112` (ImageNet: `Resize((image_size, image_size))`). The arithmetic lives in third-party
code that is not in /root/reference:
  * torchvision (absent here): `Resize` on a PIL image computes the output size
    (`_compute_resized_output_size`: int -> shorter side = size, longer = int(size * long / short))
    and calls `PIL.Image.resize(size, BILINEAR)`; `ToTensor` is `uint8 -> float32 / 255`;
    `Normalize` is `(x - mean) / std` in float32; `RandomHorizontalFlip` mirrors the resized
    image when `torch.rand(1) < 0.5`.
  * Pillow 12.2.0 (importable here; `libImaging/Resample.c`): separable two-pass resampling in
    8-bit fixed point. `precompute_coeffs`: scale = (in1 - in0) / outSize in double (a float32
    scale mismatches Pillow 12.2 on 32->56, 50x40->24x30, ...), filterscale = max(scale, 1), support = 1.0 * filterscale for
    the bilinear (triangle) filter, per output index xx: center = (xx + 0.5) * scale,
    xmin = max(int(center - support + 0.5), 0), xmax = min(int(center + support + 0.5), inSize)
    - xmin, w_x = tri((x + xmin - center + 0.5) / filterscale) normalised by their sum;
    `normalize_coeffs_8bpp`: k = int(w * 2**22 +- 0.5) (PRECISION_BITS = 32 - 8 - 2);
    horizontal pass first into an 8-bit image (accumulator starts at 2**21, `clip8` = clamp to
    [0, 255] of acc >> 22), then the vertical pass on that image with the same rounding.
This module restates exactly that (numpy int64) and is pinned bit-exactly against Pillow itself
by tests/test_preprocess_cpu.py (fixtures from tests/golden/make_preprocess_golden.py plus live
Pillow on random sizes). The flip decision is an input here: the per-sample draws of the
reference's DataLoader workers come from torch's global RNG and are not reproducible outside it.
"""
import numpy as np

PRECISION_BITS = 32 - 8 - 2


def resized_size(h, w, size):
    """torchvision Resize(size) output (h, w): an int scales the shorter side (aspect kept, longer
    side truncated); a pair is taken as (h, w)."""
    if isinstance(size, (tuple, list)):
        return int(size[0]), int(size[1])
    if w <= h:
        return int(size * h / w), int(size)
    return int(size), int(size * w / h)


def _tri(x):
    x = np.abs(x)
    return np.where(x < 1.0, 1.0 - x, 0.0)


def coeffs(in_size, out_size):
    """(bounds [out, 2] = (xmin, count), kk [out, ksize] int64) of Pillow's precompute_coeffs +
    normalize_coeffs_8bpp for the bilinear filter over the full box [0, in_size)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(np.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = np.array([_tri((x + xmin - center + 0.5) * ss) for x in range(xmax)], np.float64)
        ww = 0.0
        for v in w:  # sequential, as Pillow (numpy's pairwise sum reorders 8+ taps)
            ww += float(v)
        if ww != 0.0:
            w = w / ww
        k = np.where(w < 0, np.trunc(-0.5 + w * (1 << PRECISION_BITS)), np.trunc(0.5 + w * (1 << PRECISION_BITS)))
        kk[xx, :xmax] = k.astype(np.int64)
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(acc):
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_bilinear_u8(img, out_h, out_w):
    """Pillow Image.resize((out_w, out_h), BILINEAR) of a uint8 [H, W, C] image."""
    img = np.asarray(img, np.uint8)
    h, w, c = img.shape
    bx, kx = coeffs(w, out_w)
    by, ky = coeffs(h, out_h)
    src = img.astype(np.int64)
    tmp = np.empty((h, out_w, c), np.uint8)
    for xx in range(out_w):
        x0, n = bx[xx]
        acc = np.full((h, c), 1 << (PRECISION_BITS - 1), np.int64)
        acc += np.einsum("hkc,k->hc", src[:, x0:x0 + n, :], kx[xx, :n])
        tmp[:, xx, :] = _clip8(acc)
    t = tmp.astype(np.int64)
    out = np.empty((out_h, out_w, c), np.uint8)
    for yy in range(out_h):
        y0, n = by[yy]
        acc = np.full((out_w, c), 1 << (PRECISION_BITS - 1), np.int64)
        acc += np.einsum("kwc,k->wc", t[y0:y0 + n], ky[yy, :n])
        out[yy] = _clip8(acc)
    return out


def to_tensor_normalize(img_u8, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
    """ToTensor + Normalize: uint8 [H, W, 3] -> float32 [3, H, W], (v / 255 - mean) / std."""
    x = np.asarray(img_u8).transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    m = np.asarray(mean, np.float32).reshape(3, 1, 1)
    s = np.asarray(std, np.float32).reshape(3, 1, 1)
    return (x - m) / s


def transform_batch(images_u8, size, flips=None, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
    """The reference's train transform over a batch uint8 [B, H, W, 3] -> float32 [B, 3, h, w];
    flips[b] != 0 mirrors sample b horizontally after the resize."""
    images_u8 = np.asarray(images_u8, np.uint8)
    b, h, w, _ = images_u8.shape
    oh, ow = resized_size(h, w, size)
    out = np.empty((b, 3, oh, ow), np.float32)
    for i in range(b):
        r = resize_bilinear_u8(images_u8[i], oh, ow)
        if flips is not None and flips[i]:
            r = r[:, ::-1, :]
        out[i] = to_tensor_normalize(r, mean, std)
    return out
