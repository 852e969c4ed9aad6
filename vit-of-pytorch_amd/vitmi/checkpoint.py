"""Checkpoint import: the reference's JAX `.npz` -> PyTorch state_dict conversion.

Follows reference src/checkpoint.py:
  load_checkpoint      :7-17   (.npz -> convert, .pth -> ['state_dict'])
  load_jax             :20-25  (np.load, allow_pickle=False; the reference opens the file through
                                tensorflow.io.gfile, absent here — a plain local open is used)
  save_jax_to_pytorch  :28-33
  replace_names        :36-77  (Flax module path -> reference module names)
  convert_jax_pytorch  :80-115 (per-tensor layout changes)

Layout rules, restated (reference :95-111): rank-1 tensors are squeezed; rank-2 `weight`s (Dense
kernels, stored [in][out] by Flax) are transposed to nn.Linear's [out][in]; the multi-head q/k/v
kernels [D][H][hd] / biases [H][hd] and the out kernel [H][hd][D] already match LinearGeneral and
are kept; the rank-4 conv kernel HWIO is permuted to OIHW. Everything else (cls token [1,1,D],
position embedding [1,N,D]) is kept as is.

Only safe loaders are used: numpy with allow_pickle=False, torch.load with weights_only=True.
The result feeds `VisionTransformer.load_state_dict`, whose parameters are views of the engine's
flat buffer; the bf16 GEMM mirror is rebuilt on the next forward (parameter versions change).
"""
import os

import numpy as np
import torch


def load_jax(path):
    """reference src/checkpoint.py:20-25 — (keys, values) of a Flax `.npz` parameter dump."""
    with open(path, "rb") as f:
        with np.load(f, allow_pickle=False) as ckpt:
            items = [(k, np.asarray(ckpt[k])) for k in ckpt.files]
    if not items:
        return (), ()
    keys, values = zip(*items)
    return keys, values


def replace_names(names):
    """reference src/checkpoint.py:36-77 — one Flax path component -> reference module name(s)."""
    out = []
    for name in names:
        if name == "Transformer":
            out.append("transformer")
        elif name == "encoder_norm":
            out.append("norm")
        elif "encoderblock" in name:
            out += ["encoder_layers", name.split("_")[-1]]
        elif "LayerNorm" in name:
            # LayerNorm_0 is the pre-attention norm, LayerNorm_2 the pre-MLP norm; the reference
            # drops any other index (none occurs inside an encoder block)
            idx = name.split("_")[-1]
            if idx == "0":
                out.append("norm1")
            elif idx == "2":
                out.append("norm2")
        elif "MlpBlock" in name:
            out.append("mlp")
        elif "Dense" in name:
            out.append("fc{}".format(int(name.split("_")[-1]) + 1))
        elif "MultiHeadDotProductAttention" in name:
            out.append("attn")
        elif name in ("kernel", "scale"):
            out.append("weight")
        elif name == "posembed_input":
            out.append("pos_embedding")
        elif name == "head":
            out.append("classifier")
        elif name == "cls":
            out.append("cls_token")
        else:  # bias, pos_embedding, embedding, query/key/value/out, ...
            out.append(name)
    return out


def convert_jax_pytorch(keys, values):
    """reference src/checkpoint.py:80-115 — Flax arrays -> fp32 tensors in the reference's layouts."""
    state_dict = {}
    for key, value in zip(keys, values):
        names = replace_names(key.split("/"))
        t = torch.tensor(np.asarray(value), dtype=torch.float)
        nd = t.dim()
        if nd == 1:
            t = t.squeeze()
        elif nd == 2 and names[-1] == "weight":
            t = t.T
        elif nd == 4 and names[-1] == "weight":
            t = t.permute(3, 2, 0, 1)
        # rank-3 q/k/v/out kernels and rank-2 q/k/v biases: LinearGeneral already uses Flax's layout
        state_dict[".".join(names)] = t.contiguous()
    return state_dict


def load_checkpoint(path):
    """reference src/checkpoint.py:7-17 — weights from a `.npz` (Flax) or `.pth` (reference) file."""
    if path.endswith("npz"):
        return convert_jax_pytorch(*load_jax(path))
    if path.endswith("pth"):
        return torch.load(path, map_location="cpu", weights_only=True)["state_dict"]
    raise ValueError("checkpoint format {} not supported yet!".format(path.split(".")[-1]))


def save_jax_to_pytorch(jax_path, save_path):
    """reference src/checkpoint.py:28-33 — write `<name>.pth` = {'state_dict': converted weights}."""
    model_name = os.path.basename(jax_path).split(".")[0]
    state_dict = convert_jax_pytorch(*load_jax(jax_path))
    out = os.path.join(save_path, model_name + ".pth")
    torch.save({"state_dict": state_dict}, out)
    return out
