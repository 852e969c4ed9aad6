"""Generate tests/golden/jax_convert.npz by running the reference's own JAX -> PyTorch converter.

Run HERE (the container that has /root/reference mounted):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_jax_golden.py

reference src/checkpoint.py imports `tensorflow.io.gfile` (:3) only to open the `.npz` in
load_jax (:20-25); tensorflow is absent here, so a stub module whose `gfile.GFile` is the builtin
`open` is put in sys.modules, and the reference's load_checkpoint (:7-17) ->
load_jax -> convert_jax_pytorch (:80-115) runs unmodified on a synthetic Flax-named ViT parameter
dump (tiny config: D 64, H 2, hd 32, M 128, L 2, P 8, 10 classes; Flax layouts: HWIO conv
kernel, [in][out] Dense kernels, [D][H][hd] q/k/v kernels, [H][hd][D] out kernel).

Fixture: `in/<flax key>` = the input arrays (in file order), `out/<torch key>` = the reference's
converted state_dict, `order` = the Flax keys in the order the reference read them. Data only; no
reference source is copied. The GPU box never runs this script.
"""
import importlib.machinery
import importlib.util
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"

D, H, M, L, P, C, N = 64, 2, 128, 2, 8, 10, 17


def flax_params(rng):
    hd = D // H
    f = lambda *s: rng.standard_normal(s).astype(np.float32)
    p = {"cls": f(1, 1, D), "embedding/kernel": f(P, P, 3, D), "embedding/bias": f(D),
         "head/kernel": f(D, C), "head/bias": f(C),
         "Transformer/posembed_input/pos_embedding": f(1, N, D),
         "Transformer/encoder_norm/scale": f(D), "Transformer/encoder_norm/bias": f(D)}
    for i in range(L):
        b = f"Transformer/encoderblock_{i}/"
        for j in (0, 2):
            p[b + f"LayerNorm_{j}/scale"] = f(D)
            p[b + f"LayerNorm_{j}/bias"] = f(D)
        p[b + "MlpBlock_3/Dense_0/kernel"] = f(D, M)
        p[b + "MlpBlock_3/Dense_0/bias"] = f(M)
        p[b + "MlpBlock_3/Dense_1/kernel"] = f(M, D)
        p[b + "MlpBlock_3/Dense_1/bias"] = f(D)
        for n in ("query", "key", "value"):
            p[b + f"MultiHeadDotProductAttention_1/{n}/kernel"] = f(D, H, hd)
            p[b + f"MultiHeadDotProductAttention_1/{n}/bias"] = f(H, hd)
        p[b + "MultiHeadDotProductAttention_1/out/kernel"] = f(H, hd, D)
        p[b + "MultiHeadDotProductAttention_1/out/bias"] = f(D)
    return p


def stub_tensorflow():
    """tensorflow.io.gfile.GFile = open (each stub module carries a ModuleSpec: torch._dynamo's
    trace rules walk sys.modules and fail on modules without one)."""
    mods = {}
    for name in ("tensorflow", "tensorflow.io", "tensorflow.io.gfile"):
        m = types.ModuleType(name)
        m.__spec__ = importlib.machinery.ModuleSpec(name, None)
        mods[name] = m
    mods["tensorflow.io.gfile"].GFile = open
    mods["tensorflow.io"].gfile = mods["tensorflow.io.gfile"]
    mods["tensorflow"].io = mods["tensorflow.io"]
    sys.modules.update(mods)


def main():
    sys.dont_write_bytecode = True
    stub_tensorflow()
    spec = importlib.util.spec_from_file_location("ref_checkpoint", os.path.join(REF_SRC, "checkpoint.py"))
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    params = flax_params(np.random.default_rng(2024))
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "ViT-tiny.npz")
        np.savez(path, **params)
        keys, _ = ref.load_jax(path)
        sd = ref.load_checkpoint(path)
    out = {"order": np.array(list(keys))}
    out.update({"in/" + k: v for k, v in params.items()})
    out.update({"out/" + k: v.numpy() for k, v in sd.items()})
    dst = os.path.join(HERE, "jax_convert.npz")
    np.savez_compressed(dst, **out)
    print(f"wrote {dst}: {len(params)} Flax arrays -> {len(sd)} state_dict tensors")


if __name__ == "__main__":
    main()
