#!/usr/bin/env python3
"""Launch-gap probe (run under rocprofv3 --kernel-trace): B/16 bs 256 fc1 shapes in fixed sequences, so the
trace shows the idle time in front of each kernel kind: (a) dgrad GEMM x4, (b) weight-gradient GEMM (split-K
slabs) x4, (c) [wgrad, reduce, dgrad] x4, (d) wgrad with split 1 x4 (ws as the output)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_BF16, EPI_SPLITK, K_CONTIG, MN_CONTIG  # noqa: E402

T, D, M = 50432, 768, 3072
dU = torch.randn(T, M, device="cuda").bfloat16()
X = torch.randn(T, D, device="cuda").bfloat16()
W = torch.randn(D, M, device="cuda").bfloat16()      # fc1 dgrad: dX[T][D] = dU[T][M] W1[M][D] (B K-contiguous)
dX = torch.empty(T, D, device="cuda").bfloat16()
s = ops.splitk_factor(M, D, T)
ws = torch.empty(s * M * D, device="cuda")
dW = torch.empty(M, D, device="cuda")


def dgrad():
    ops.gemm(dU, W, dX, T, D, M, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=M, ldb=M, ldc=D, epilogue=EPI_BF16)


def wgrad(split=s):
    ops.gemm(dU, X, ws, M, D, T, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=M, ldb=D, ldc=D, epilogue=EPI_SPLITK,
             split_k=split)


def reduce():
    ops.splitk_reduce(ws, 1, s, M, D, dW, D)


for rep in range(2):
    torch.cuda.synchronize()
    for _ in range(4):
        dgrad()
    torch.cuda.synchronize()
    for _ in range(4):
        wgrad()
    torch.cuda.synchronize()
    for _ in range(4):
        wgrad()
        reduce()
        dgrad()
    torch.cuda.synchronize()
    for _ in range(4):
        wgrad(1)
    torch.cuda.synchronize()
print("split", s, flush=True)
