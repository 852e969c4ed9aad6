"""vit_preprocess_u8 (the reference loader's Resize -> flip -> ToTensor -> Normalize,
src/data_loaders.py:66-80, 100-112) against the Pillow-pinned oracle: bit-exact f32 output on the
committed Pillow fixtures, random sizes (up- and downsampling, ragged aspect), flips, a CIFAR-sized
batch at 32 -> 224 (config C1/C2's input), and a full bs-256 batch checked on sampled images."""
import os

import numpy as np
import pytest
import torch

from oracle.preprocess import to_tensor_normalize, transform_batch

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "preprocess.npz")


def _run(imgs, size, flips=None, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
    from vitmi.data import GPUTransform
    t = GPUTransform(size, train=False, mean=mean, std=std)
    f = None if flips is None else torch.as_tensor(np.asarray(flips, np.uint8))
    return t(torch.from_numpy(np.ascontiguousarray(imgs)).cuda(), flips=f).cpu().numpy()


def test_matches_pillow_fixtures_bit_exact():
    z = np.load(GOLDEN)
    for i, (h, w, oh, ow) in enumerate(z["cases"]):
        got = _run(z[f"in{i}"][None], (int(oh), int(ow)))
        want = to_tensor_normalize(z[f"out{i}"])[None]
        assert np.array_equal(got, want), (h, w, oh, ow, np.abs(got - want).max())


def test_random_sizes_and_flips_match_oracle():
    rng = np.random.default_rng(1)
    for _ in range(8):
        b = int(rng.integers(1, 4))
        h, w = (int(v) for v in rng.integers(2, 90, 2))
        size = int(rng.integers(2, 80)) if rng.random() < 0.5 else tuple(int(v) for v in rng.integers(1, 80, 2))
        imgs = rng.integers(0, 256, (b, h, w, 3), dtype=np.uint8)
        flips = rng.integers(0, 2, b)
        mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
        got = _run(imgs, size, flips, mean, std)
        want = transform_batch(imgs, size, flips, mean, std)
        assert got.shape == want.shape and np.array_equal(got, want), (h, w, size)


def test_cifar_batch_to_224():
    rng = np.random.default_rng(2)
    imgs = rng.integers(0, 256, (6, 32, 32, 3), dtype=np.uint8)
    flips = [0, 1, 0, 1, 1, 0]
    got = _run(imgs, 224, flips)
    assert np.array_equal(got, transform_batch(imgs, 224, flips))
    assert got.min() >= -1.0 and got.max() <= 1.0


def test_full_batch_256_sampled():
    rng = np.random.default_rng(3)
    imgs = rng.integers(0, 256, (256, 32, 32, 3), dtype=np.uint8)
    flips = rng.integers(0, 2, 256)
    got = _run(imgs, 224, flips)
    for i in (0, 77, 255):
        assert np.array_equal(got[i:i + 1], transform_batch(imgs[i:i + 1], 224, flips[i:i + 1])), i


def test_train_transform_draws_flips_from_generator():
    from vitmi.data import GPUTransform
    rng = np.random.default_rng(4)
    imgs = torch.from_numpy(rng.integers(0, 256, (16, 20, 24, 3), dtype=np.uint8)).cuda()
    t = GPUTransform(12, train=True, generator=torch.Generator().manual_seed(9))
    got = t(imgs).cpu().numpy()
    flips = (torch.rand(16, generator=torch.Generator().manual_seed(9)) < 0.5).numpy()
    assert 0 < flips.sum() < 16
    assert np.array_equal(got, transform_batch(imgs.cpu().numpy(), 12, flips))


def test_bad_layout_raises():
    from vitmi import ops
    x = torch.zeros(2, 3, 8, 8, dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        ops.preprocess_u8(x, torch.empty(2, 3, 4, 4, device="cuda"))


@pytest.mark.parametrize("h,w,size", [(200, 40, (12, 40)), (45, 300, (45, 20)), (64, 64, (7, 9))])
def test_large_downsampling_ratios_generic_path(h, w, size):
    """more than 9 taps on an axis (ratio > 4) runs the generic kernel"""
    rng = np.random.default_rng(h * w)
    imgs = rng.integers(0, 256, (2, h, w, 3), dtype=np.uint8)
    assert np.array_equal(_run(imgs, size, [1, 0]), transform_batch(imgs, size, [1, 0]))
