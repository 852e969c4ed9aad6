"""Host-side logic that needs no GPU: the C-ABI library exports, parameter layout, module surface."""
import ctypes
import os
import re

import pytest
import torch

from oracle.vit_oracle import ViTConfig, init_params, param_names

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "vit_hip.h")


def test_library_exports_every_header_symbol():
    from vitmi import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libvit_hip.so not built (run __graft_entry__.build())")
    text = open(HEADER).read()
    declared = set(re.findall(r"^\s*(?:const char\*|int64_t|int)\s+(vit_\w+)\s*\(", text, flags=re.M))
    assert declared, "no declarations parsed"
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(_lib.EXPORTED), declared ^ set(_lib.EXPORTED)
    assert lib.vit_abi_version() == _lib.ABI_VERSION


def test_library_build_id_matches_tree():
    """The library was built from exactly these sources: load() re-derives the fingerprint of csrc/,
    the Makefile and include/vit_hip.h and compares it with the stamped vit_build_id()."""
    from vitmi import _lib, buildid
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libvit_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.vit_build_id.restype = ctypes.c_char_p
    assert lib.vit_build_id().decode() == buildid.tree_id()
    _lib.check_build_id(lib, _lib.LIB_PATH)  # no raise
    assert _lib.load() is not None


def test_library_with_foreign_build_id_is_refused(tmp_path):
    """A library whose stamp differs from the tree (built from older sources) raises VitHipError: both a
    wrong expected id and a copy of the tree whose kernel source changed."""
    import shutil

    from vitmi import _lib, buildid
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libvit_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.vit_build_id.restype = ctypes.c_char_p
    with pytest.raises(_lib.VitHipError, match="built from other sources"):
        _lib.check_build_id(lib, _lib.LIB_PATH, expected="0123456789abcdef")
    # a tree that differs by one byte of one kernel source has another id
    pkg = tmp_path / "vit-of-pytorch_amd"
    shutil.copytree(os.path.join(buildid.PKG_ROOT, "csrc"), pkg / "csrc")
    shutil.copy(os.path.join(buildid.PKG_ROOT, "Makefile"), pkg / "Makefile")
    (tmp_path / "include").mkdir()
    shutil.copy(HEADER, tmp_path / "include" / "vit_hip.h")
    assert buildid.tree_id(str(pkg)) == buildid.tree_id()
    # editor swap / backup files beside the sources are not sources: same id
    (pkg / "csrc" / ".gemm.hip.swp").write_bytes(b"swap")
    (pkg / "csrc" / "gemm.hip~").write_text("backup")
    assert buildid.tree_id(str(pkg)) == buildid.tree_id()
    with open(pkg / "csrc" / "gemm.hip", "a") as f:
        f.write("\n// edited\n")
    other = buildid.tree_id(str(pkg))
    assert other != buildid.tree_id()
    with pytest.raises(_lib.VitHipError):
        _lib.check_build_id(lib, _lib.LIB_PATH, expected=other)


def test_flat_layout_and_buckets():
    from vitmi.engine import ArchConfig, FlatLayout
    cfg = ArchConfig()
    lay = FlatLayout(cfg)
    assert set(lay.offsets) == set(param_names(ViTConfig()))
    # every parameter 256-B aligned and non-overlapping
    spans = sorted((o, o + int(torch.tensor(lay.shapes[k]).prod())) for k, o in lay.offsets.items())
    for (a0, a1), (b0, _) in zip(spans, spans[1:]):
        assert a1 <= b0
    assert all(o % 64 == 0 for o in lay.offsets.values())
    # buckets tile [0, numel) contiguously in backward order: head, layer L-1 .. 0, embed
    assert lay.buckets[0][1] == 0 and lay.buckets[-1][2] == lay.numel
    for (_, _, e), (_, s, _) in zip(lay.buckets, lay.buckets[1:]):
        assert e == s
    assert [b[0] for b in lay.buckets[1:-1]] == [f"layer{i}" for i in reversed(range(12))]
    # q/k/v weights are equally strided (the batched wgrad / pack kernels rely on it)
    p = "transformer.encoder_layers.3.attn."
    q, k, v = (lay.offsets[p + s + ".weight"] for s in ("query", "key", "value"))
    assert k - q == v - k
    assert lay.offsets[p + "key.bias"] - lay.offsets[p + "query.bias"] == k - q


def test_module_surface_and_rng_order():
    from vitmi.model import MLPBlock, MlpBlock, VisionTransformer
    assert MLPBlock is MlpBlock
    cfg = ViTConfig(image_size=32, patch_size=8, emb_dim=64, mlp_dim=128, num_heads=2, num_layers=2, num_classes=10)
    torch.manual_seed(42)
    m = VisionTransformer(image_size=(32, 32), patch_size=(8, 8), emb_dim=64, mlp_dim=128, num_heads=2, num_layers=2,
                          num_classes=10, attn_dropout_rate=0.0, dropout_rate=0.0)
    ref = init_params(cfg, seed=42)
    sd = m.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k in ref:
        assert torch.equal(sd[k], ref[k]), k
    # default ctor keeps the reference's dropout modules (src/model.py defaults)
    d = VisionTransformer(image_size=(32, 32), patch_size=(8, 8), emb_dim=64, mlp_dim=128, num_heads=2, num_layers=1,
                          num_classes=10)
    assert sum(isinstance(x, torch.nn.Dropout) for x in d.modules()) == 4


def test_cpu_forward_refuses():
    from vitmi.model import VisionTransformer
    m = VisionTransformer(image_size=(32, 32), patch_size=(8, 8), emb_dim=64, mlp_dim=128, num_heads=2, num_layers=1,
                          num_classes=10, dropout_rate=0.0)
    with pytest.raises(RuntimeError, match="MI355X HIP path only"):
        m(torch.randn(1, 3, 32, 32))


def test_cpu_submodule_forwards_refuse():
    """standalone sub-modules run on the HIP kernels only (no PyTorch CPU fallback)"""
    from vitmi.model import EncoderBlock, LinearGeneral, MlpBlock
    with pytest.raises(RuntimeError, match="MI355X HIP path only"):
        EncoderBlock(64, 128, 2, dropout_rate=0.0)(torch.randn(1, 5, 64))
    with pytest.raises(RuntimeError, match="MI355X HIP path only"):
        MlpBlock(64, 128, 64, dropout_rate=0.0)(torch.randn(1, 5, 64))
    with pytest.raises(RuntimeError, match="MI355X HIP path only"):
        LinearGeneral((64,), (2, 32))(torch.randn(1, 5, 64), dims=([2], [0]))


def test_splitk_factor_one_wave_splits_and_h14_tail():
    """split-K choice of the weight gradients (engine._splitk / ops.wgrad): the ViT-B/16 and L/16 splits the
    sweeps picked (one wave of 256 x 256 workgroups), and ViT-H/14 bs 128's fc1 / fc2 weight gradients
    (100 tiles) at 5 splits = 500 workgroups rather than 3 = 300 (a second wave 17% full)."""
    from vitmi.ops import splitk_factor as f
    assert [f(3072, 768, 50432), f(768, 3072, 50432), f(2304, 768, 50432), f(768, 768, 50432)] == [7, 7, 9, 28]
    assert [f(4096, 1024, 12608), f(3072, 1024, 12608), f(1024, 1024, 12608)] == [4, 5, 16]
    assert [f(5120, 1280, 32896), f(1280, 5120, 32896), f(3840, 1280, 32896)] == [5, 5, 3]
    assert f(768, 768, 256) == 1 and f(768, 768, 64) == 1        # at least 8 k-tiles per split
    # one grid for a layer's out-projection + q|k|v weight gradients: B/16 one wave at 7, L/16 bs 64 one at 4
    from vitmi.ops import splitk_factor_group as fg
    assert fg([(768, 768, 1), (768, 768, 3)], 50432) == 7
    assert fg([(1024, 1024, 1), (1024, 1024, 3)], 12608) == 4
    for M, N, K in [(768, 768, 50432), (64, 64, 1 << 20), (5120, 1280, 32896)]:
        s = f(M, N, K)
        assert 1 <= s <= 32 and (s == 1 or K // 64 // s >= 8)


def test_bench_condition_init_is_the_parity_rescale():
    """bench.condition_init (the bench's weights: seed-42 reference draw, attention projections and pos-emb /
    classifier rescaled) equals the oracle's tame_params on the reference constructor's parameters, bit for bit"""
    import sys
    sys.path.insert(0, REPO)
    import bench
    from oracle.vit_oracle import tame_params
    from vitmi.model import VisionTransformer
    torch.manual_seed(42)
    m = VisionTransformer(image_size=(32, 32), patch_size=(4, 4), emb_dim=128, mlp_dim=256, num_heads=2, num_layers=2,
                          num_classes=10)
    ref = tame_params(m.state_dict())
    bench.condition_init(m)
    sd = m.state_dict()
    assert sd.keys() == ref.keys()
    assert all(torch.equal(sd[k], ref[k]) for k in ref)
