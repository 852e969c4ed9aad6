"""Input-pipeline oracle (oracle/preprocess.py) pinned against Pillow, the library under the
reference's torchvision transforms (src/data_loaders.py:66-80, 100-112): bit-exact on the committed
fixtures (tests/golden/make_preprocess_golden.py) and on live Pillow for random sizes when Pillow is
importable."""
import os

import numpy as np
import pytest

from oracle.preprocess import resize_bilinear_u8, resized_size, to_tensor_normalize, transform_batch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "preprocess.npz")


def test_resize_matches_pillow_fixtures():
    z = np.load(GOLDEN)
    for i, (h, w, oh, ow) in enumerate(z["cases"]):
        mine = resize_bilinear_u8(z[f"in{i}"], int(oh), int(ow))
        assert np.array_equal(mine, z[f"out{i}"]), (h, w, oh, ow)


def test_resize_matches_live_pillow_random_sizes():
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(7)
    for _ in range(12):
        h, w = (int(v) for v in rng.integers(1, 120, 2))
        oh, ow = (int(v) for v in rng.integers(1, 120, 2))
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        ref = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
        assert np.array_equal(resize_bilinear_u8(img, oh, ow), ref), (h, w, oh, ow)


def test_resized_size_follows_torchvision_int_and_pair():
    assert resized_size(32, 32, 224) == (224, 224)
    assert resized_size(375, 500, 224) == (224, 298)   # landscape: shorter side (h) -> 224
    assert resized_size(500, 375, 224) == (298, 224)
    assert resized_size(300, 200, (224, 224)) == (224, 224)


def test_to_tensor_normalize_values():
    img = np.array([[[0, 128, 255]]], np.uint8)
    x = to_tensor_normalize(img)
    assert x.dtype == np.float32 and x.shape == (3, 1, 1)
    assert x[0, 0, 0] == -1.0 and x[2, 0, 0] == 1.0
    assert x[1, 0, 0] == (np.float32(128) / np.float32(255) - np.float32(0.5)) / np.float32(0.5)


def test_transform_batch_flip_mirrors_after_resize():
    rng = np.random.default_rng(3)
    imgs = rng.integers(0, 256, (2, 20, 30, 3), dtype=np.uint8)
    a = transform_batch(imgs, (16, 24), flips=[0, 1])
    b = transform_batch(imgs, (16, 24), flips=[0, 0])
    assert np.array_equal(a[0], b[0])
    assert np.array_equal(a[1], b[1][:, :, ::-1])
