"""ctypes binding of libvit_hip.so (the C ABI declared in include/vit_hip.h).

The library is built in-tree by `make -C vit-of-pytorch_amd` (or __graft_entry__.build()).
There is no fallback: if the library is missing, importing the GPU ops raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# VITMI_LIB: an alternate build of the same library (A/B timing of kernel variants in one process tree)
LIB_PATH = os.environ.get("VITMI_LIB") or os.path.join(_HERE, "libvit_hip.so")

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p

ABI_VERSION = 18  # vit_abi_version() of the library these prototypes describe

# enum vit_layout / vit_epilogue (include/vit_hip.h)
K_CONTIG, MN_CONTIG = 0, 1
(EPI_F32, EPI_BF16, EPI_BIAS_BF16, EPI_BIAS_GELU, EPI_BIAS_RESID_F32, EPI_GELU_BWD, EPI_PATCH, EPI_SPLITK,
 EPI_BIAS_GELU_DGELU, EPI_MUL_BF16) = range(10)


class Dropout(ctypes.Structure):
    """struct vit_dropout (include/vit_hip.h)"""
    _fields_ = [("p", c_f32), ("site", ctypes.c_uint32), ("seed", ctypes.c_uint64), ("offset", ctypes.c_uint64),
                ("row_stride", c_i64)]


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("M", c_i64), ("N", c_i64), ("K", c_i64),
        ("A", c_vp), ("lda", c_i64), ("a_batch_stride", c_i64),
        ("a_layout", c_i32), ("b_layout", c_i32),
        ("B", c_vp), ("ldb", c_i64), ("b_batch_stride", c_i64),
        ("C", c_vp), ("ldc", c_i64), ("c_batch_stride", c_i64),
        ("C2", c_vp), ("ldc2", c_i64),
        ("bias", c_vp), ("bias_batch_stride", c_i64),
        ("aux", c_vp), ("ldaux", c_i64), ("aux2", c_vp),
        ("batch", c_i64), ("split_k", c_i64), ("tokens", c_i64), ("col_partial", c_vp),
        ("epilogue", c_i32), ("tile", c_i32), ("dropout", ctypes.POINTER(Dropout)),
    ]


class ColsumJob(ctypes.Structure):
    """struct vit_colsum_job (include/vit_hip.h)"""
    _fields_ = [("inp", c_vp), ("rows", c_i64), ("cols", c_i64), ("ld", c_i64), ("seg", c_i64),
                ("out0", c_vp), ("out1", c_vp), ("out2", c_vp), ("accumulate", c_i32), ("reserved", c_i32)]


COLSUM_BATCH_MAX = 8  # VIT_COLSUM_BATCH_MAX


class SplitkJob(ctypes.Structure):
    """struct vit_splitk_job (include/vit_hip.h)"""
    _fields_ = [("ws", c_vp), ("batch", c_i64), ("split", c_i64), ("M", c_i64), ("N", c_i64), ("out", c_vp),
                ("ldo", c_i64), ("out_batch_stride", c_i64), ("accumulate", c_i32), ("reserved", c_i32)]


SPLITK_GROUP_MAX = 8  # VIT_SPLITK_GROUP_MAX


class CastJob(ctypes.Structure):
    """struct vit_cast_job (include/vit_hip.h)"""
    _fields_ = [("inp", c_vp), ("rows", c_i64), ("cols", c_i64), ("ldi", c_i64), ("out", c_vp), ("ldo", c_i64),
                ("rows_pad", c_i64), ("cols_pad", c_i64)]


CAST_BATCH_MAX = 8  # VIT_CAST_BATCH_MAX

# name -> (restype, argtypes)
_SIGS = {
    "vit_last_error": (ctypes.c_char_p, []),
    "vit_abi_version": (c_i32, []),
    "vit_gemm_bf16": (c_i32, [ctypes.POINTER(GemmArgs), c_vp]),
    "vit_gemm_tile_rows": (c_i64, [ctypes.POINTER(GemmArgs)]),
    "vit_gemm_partial_rows": (c_i64, [ctypes.POINTER(GemmArgs)]),
    "vit_gemm_split_rows": (c_i64, [ctypes.POINTER(GemmArgs)]),
    "vit_gemm_bf16_part": (c_i32, [ctypes.POINTER(GemmArgs), c_i32, c_vp]),
    "vit_gemm_splitk_group": (c_i32, [ctypes.POINTER(GemmArgs), c_i32, c_vp]),
    "vit_segment_colsum": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_f32, c_vp, c_i64, c_vp]),
    "vit_segment_colsum_bcast": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_f32, c_vp, c_i64,
                                         c_vp, c_i64, c_i64, c_vp]),
    "vit_router_dx_gate_partial_rows": (c_i64, [c_i64]),
    "vit_router_dx_gate": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_f32, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp,
                                   c_i64, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "vit_splitk_reduce_group": (c_i32, [ctypes.POINTER(SplitkJob), c_i32, c_vp]),
    "vit_cast_pad_batch": (c_i32, [ctypes.POINTER(CastJob), c_i32, c_vp]),
    "vit_router_head_partials": (c_i64, [c_i64]),
    "vit_cast_rows_masked": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "vit_router_select": (c_i32, [c_vp, c_i64, c_i32, ctypes.POINTER(ctypes.c_uint32), c_i32, c_vp, c_vp, c_vp, c_vp]),
    "vit_cls_mse": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "vit_cls_mse_bwd": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "vit_router_head_fwd": (c_i32, [c_vp, c_vp, c_i32, c_vp, c_i64, c_i64, c_i32, c_i64, c_i32, c_f32, c_vp, c_vp, c_vp,
                                    c_vp, c_vp, c_vp, c_vp]),
    "vit_router_head_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_i64, c_i64, c_i32, c_i64, c_i32, c_vp,
                                    c_vp]),
    "vit_splitk_reduce": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i32, c_vp]),
    "vit_layernorm_fwd": (c_i32, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_i64, c_i64, c_f32, c_vp]),
    "vit_layernorm_bwd_partial_rows": (c_i64, [c_i64]),
    "vit_layernorm_bwd_blocks": (c_i64, [c_i64]),
    "vit_layernorm_bwd": (c_i32, [c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64,
                                  c_vp, c_i64, c_vp, c_vp, c_vp, c_i32, c_i64, c_i64, ctypes.POINTER(Dropout),
                                  c_vp]),
    "vit_attention_fwd": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_f32, c_vp]),
    "vit_attention_bwd": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_f32, c_vp]),
    "vit_attention_fwd_rows": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_f32, c_i64, c_vp]),
    "vit_attention_bwd_rows": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_f32, c_i64,
                                       c_vp]),
    "vit_attention_bias_rows": (c_i64, [c_i64, c_i64, c_i32]),
    "vit_attention_workspace_elems": (c_i64, [c_i64, c_i64, c_i64, c_i32]),
    "vit_attention_fwd_ex": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_f32, c_i64, c_i32, c_vp]),
    "vit_attention_bwd_ex": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_f32, c_i64,
                                     c_i32, c_vp, c_vp]),
    "vit_im2col": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "vit_preprocess_u8": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "vit_embed_grad": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, ctypes.POINTER(Dropout), c_vp]),
    "vit_dropout_mask": (c_i32, [ctypes.POINTER(Dropout), c_i64, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "vit_colsum_partial_rows": (c_i64, [c_i64]),
    "vit_colsum": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_vp, c_i32, c_vp]),
    "vit_gemm_f32": (c_i32, [c_i64, c_i64, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_i32,
                             c_vp]),
    "vit_cross_entropy": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_vp, c_f32, c_vp, c_vp]),
    "vit_sgd_step": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_f32, c_f32, c_f32, c_i32, c_vp]),
    "vit_cast_f32_bf16": (c_i32, [c_vp, c_vp, c_i64, c_vp]),
    "vit_cast_pad_rows": (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "vit_axpby": (c_i32, [c_vp, c_vp, c_i64, c_f32, c_f32, c_vp]),
    "vit_pack_cols": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i32, c_vp]),
    "vit_pack_cols_batched": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i32, c_i64,
                                      c_vp]),
    "vit_transpose_f32_bf16": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "vit_colsum_batch": (c_i32, [ctypes.POINTER(ColsumJob), c_i32, c_vp]),
    "vit_colsum3": (c_i32, [c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp]),
    "vit_im2col_f32": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "vit_embed_fwd_f32": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "vit_gelu_f32": (c_i32, [c_vp, c_vp, c_i64, c_vp]),
    "vit_attention_fwd_f32": (c_i32, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_f32, c_vp]),
    "vit_gelu_bwd_f32": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    "vit_dropout_apply_f32": (c_i32, [ctypes.POINTER(Dropout), c_vp, c_vp, c_i64, c_i64, c_vp]),
    "vit_add_bcast_f32": (c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp]),
    "vit_unpack_bf16_f32": (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp]),
    "vit_attention_fwd_varlen": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_i64,
                                         c_i64, c_i64, c_f32, c_vp]),
    "vit_sqnorm_partial": (c_i32, [c_vp, c_i64, c_vp, c_i32, c_vp]),
    "vit_adamw_prep": (c_i32, [c_vp, c_i32, c_vp, c_vp, c_i32, c_f32, c_f32, c_f32, c_f32, c_vp, c_vp, c_vp]),
    "vit_adamw_update": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_f32, c_f32, c_f32, c_f32, c_f32,
                                 c_f32, c_i32, c_vp]),
    "vit_adamw_chunk_elems": (c_i32, []),
    "vit_scale_by_coef": (c_i32, [c_vp, c_i64, c_vp, c_vp]),
    "vit_zero": (c_i32, [c_vp, c_i64, c_vp]),
    "vit_copy2d": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "vit_rows_select": (c_i32, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp]),
    "vit_sgd_step_dev": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_f32, c_vp]),
    "vit_build_id": (ctypes.c_char_p, []),
}

EXPORTED = tuple(_SIGS)

_lib = None


class VitHipError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load the library once and attach prototypes. Raises if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise VitHipError(f"libvit_hip.so not built ({p}); run `make -C vit-of-pytorch_amd` or __graft_entry__.build()")
    lib = ctypes.CDLL(p)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.vit_abi_version() != ABI_VERSION:
        raise VitHipError(f"{p} has ABI {lib.vit_abi_version()}, the bindings expect {ABI_VERSION}: rebuild it "
                          "(make -C vit-of-pytorch_amd)")
    check_build_id(lib, p)
    _lib = lib
    return lib


def check_build_id(lib, path: str, expected: str | None = None):
    """Refuse a library built from other sources than the tree beside this package (vitmi/buildid.py):
    the stamped vit_build_id() must equal the fingerprint of csrc/, the Makefile and include/vit_hip.h
    as they are now. (A package installed without its sources has nothing to compare against.)"""
    from . import buildid
    if expected is None:
        if not buildid.have_sources():
            return
        expected = buildid.tree_id()
    got = lib.vit_build_id().decode()
    if got != expected:
        raise VitHipError(f"{path} was built from other sources (build id {got}, this tree {expected}): rebuild it "
                          "(make -C vit-of-pytorch_amd)")


def check(status: int, what: str):
    if status != 0:
        msg = _lib.vit_last_error().decode(errors="replace") if _lib is not None else "?"
        raise VitHipError(f"{what} failed (status {status}): {msg}")
