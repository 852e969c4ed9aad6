"""JAX .npz checkpoint import (reference src/checkpoint.py) on CPU.

Pinned to the reference: tests/golden/jax_convert.npz holds the output of the reference's own
load_checkpoint -> load_jax -> convert_jax_pytorch (src/checkpoint.py:7-25, 80-115), run on a
synthetic Flax-named ViT parameter dump with a stub `tensorflow.io.gfile` (the only tensorflow use,
:3, :22); tests/golden/make_jax_golden.py is the generator. vitmi.checkpoint must reproduce it bit for
bit. The round trip below additionally pins every name and layout rule against the model itself.
"""
import os

import numpy as np
import pytest
import torch

from vitmi.checkpoint import convert_jax_pytorch, load_checkpoint, replace_names, save_jax_to_pytorch
from vitmi.model import VisionTransformer

ARCH = dict(image_size=(32, 32), patch_size=(8, 8), emb_dim=64, mlp_dim=128, num_heads=2, num_layers=2,
            num_classes=10, attn_dropout_rate=0.0, dropout_rate=0.0)


def _to_flax(sd, layers):
    """Inverse of the reference's conversion: a Flax-named, Flax-laid-out parameter dict."""
    out = {"cls": sd["cls_token"].numpy(),
           "embedding/kernel": sd["embedding.weight"].permute(2, 3, 1, 0).numpy(),   # OIHW -> HWIO
           "embedding/bias": sd["embedding.bias"].numpy(),
           "head/kernel": sd["classifier.weight"].t().numpy(),
           "head/bias": sd["classifier.bias"].numpy(),
           "Transformer/posembed_input/pos_embedding": sd["transformer.pos_embedding.pos_embedding"].numpy(),
           "Transformer/encoder_norm/scale": sd["transformer.norm.weight"].numpy(),
           "Transformer/encoder_norm/bias": sd["transformer.norm.bias"].numpy()}
    for i in range(layers):
        t, f = f"transformer.encoder_layers.{i}.", f"Transformer/encoderblock_{i}/"
        for j, n in ((0, "norm1"), (2, "norm2")):
            out[f + f"LayerNorm_{j}/scale"] = sd[t + n + ".weight"].numpy()
            out[f + f"LayerNorm_{j}/bias"] = sd[t + n + ".bias"].numpy()
        for j in (0, 1):
            out[f + f"MlpBlock_3/Dense_{j}/kernel"] = sd[t + f"mlp.fc{j + 1}.weight"].t().numpy()
            out[f + f"MlpBlock_3/Dense_{j}/bias"] = sd[t + f"mlp.fc{j + 1}.bias"].numpy()
        for n in ("query", "key", "value", "out"):
            out[f + f"MultiHeadDotProductAttention_1/{n}/kernel"] = sd[t + f"attn.{n}.weight"].numpy()
            out[f + f"MultiHeadDotProductAttention_1/{n}/bias"] = sd[t + f"attn.{n}.bias"].numpy()
    return out


def test_replace_names():
    assert replace_names("Transformer/encoderblock_11/MultiHeadDotProductAttention_1/query/kernel".split("/")) == \
        ["transformer", "encoder_layers", "11", "attn", "query", "weight"]
    assert replace_names("Transformer/encoderblock_3/LayerNorm_2/scale".split("/")) == \
        ["transformer", "encoder_layers", "3", "norm2", "weight"]
    assert replace_names("Transformer/encoderblock_0/MlpBlock_3/Dense_1/bias".split("/")) == \
        ["transformer", "encoder_layers", "0", "mlp", "fc2", "bias"]
    assert replace_names(["Transformer", "posembed_input", "pos_embedding"]) == \
        ["transformer", "pos_embedding", "pos_embedding"]
    assert replace_names(["head", "kernel"]) == ["classifier", "weight"]
    assert replace_names(["cls"]) == ["cls_token"]
    assert replace_names(["Transformer", "encoder_norm", "scale"]) == ["transformer", "norm", "weight"]


def test_npz_round_trip_into_model(tmp_path):
    torch.manual_seed(3)
    src = VisionTransformer(**ARCH)
    sd = {k: v.detach().clone() for k, v in src.state_dict().items()}
    flax = _to_flax(sd, ARCH["num_layers"])
    assert len(flax) == len(sd)
    path = tmp_path / "ViT-T_8.npz"
    np.savez(path, **flax)

    conv = load_checkpoint(str(path))
    assert set(conv) == set(sd)
    for k in sd:
        assert conv[k].dtype == torch.float32
        assert conv[k].shape == sd[k].shape, k
        assert torch.equal(conv[k], sd[k]), k

    torch.manual_seed(4)
    dst = VisionTransformer(**ARCH)
    dst.load_state_dict(conv)   # strict: every name and shape matches the model
    for k, v in dst.state_dict().items():
        assert torch.equal(v, sd[k]), k

    pth = save_jax_to_pytorch(str(path), str(tmp_path))
    assert pth.endswith("ViT-T_8.pth")
    again = load_checkpoint(pth)
    assert set(again) == set(sd) and all(torch.equal(again[k], sd[k]) for k in sd)


def test_layout_rules_and_errors(tmp_path):
    sd = convert_jax_pytorch(["embedding/kernel", "head/kernel", "encoder_norm/scale", "x/query/bias"],
                             [np.arange(2 * 2 * 3 * 5, dtype=np.float32).reshape(2, 2, 3, 5),
                              np.ones((4, 7), np.float64), np.ones((1,), np.float32), np.ones((2, 3), np.float32)])
    assert sd["embedding.weight"].shape == (5, 3, 2, 2)
    assert sd["embedding.weight"][4, 2, 1, 0] == float(np.arange(60).reshape(2, 2, 3, 5)[1, 0, 2, 4])
    assert sd["classifier.weight"].shape == (7, 4) and sd["classifier.weight"].dtype == torch.float32
    assert sd["norm.weight"].shape == ()          # rank-1 tensors are squeezed, as the reference does
    assert sd["x.query.bias"].shape == (2, 3)     # multi-head biases keep [H][hd]
    with pytest.raises(ValueError):
        load_checkpoint(str(tmp_path / "w.bin"))


def test_convert_matches_reference_converter_golden(golden_dir, tmp_path):
    """vitmi.checkpoint vs the reference's executed converter (tests/golden/jax_convert.npz)."""
    z = np.load(os.path.join(golden_dir, "jax_convert.npz"))
    order = [str(k) for k in z["order"]]
    values = [z["in/" + k] for k in order]
    expect = {k[4:]: z[k] for k in z.files if k.startswith("out/")}
    got = convert_jax_pytorch(order, values)
    assert list(got) == list(expect)  # same keys, same order
    for k, v in expect.items():
        assert got[k].dtype == torch.float32
        assert tuple(got[k].shape) == v.shape, k
        assert np.array_equal(got[k].numpy(), v), k
    # through the file path (load_checkpoint -> load_jax), as the reference reads it
    path = tmp_path / "ViT-tiny.npz"
    np.savez(path, **{k: z["in/" + k] for k in order})
    from_file = load_checkpoint(str(path))
    assert list(from_file) == list(expect)
    assert all(np.array_equal(from_file[k].numpy(), expect[k]) for k in expect)
    # and the converted weights load into the drop-in model (tiny config: D 64, H 2, P 8, 10 classes)
    m = VisionTransformer(**ARCH)
    m.load_state_dict(from_file)
