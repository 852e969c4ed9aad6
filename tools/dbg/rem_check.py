#!/usr/bin/env python3
"""Diagnostic: digests of production-path GEMM outputs (tile 0: whole-wave rows + wave-split remainder; split-K weight
gradients) on the B/16 bs-256 shapes, for comparing diagnostic knobs across processes (VIT_GEMM_REM_CFG, VIT_GEMM_ILV, ...
are read once per process).
    VITMI_LIB=vit-of-pytorch_amd/vitmi/diag/libvit_hip.so VIT_GEMM_REM_CFG=12 python3 tools/dbg/rem_check.py
"""
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_BF16, EPI_BIAS_RESID_F32, EPI_GELU_BWD, EPI_SPLITK, K_CONTIG, MN_CONTIG  # noqa: E402

T, D, F = 50432, 768, 3072
CASES = [("fc2", T, D, F, K_CONTIG, EPI_BIAS_RESID_F32), ("out", T, D, D, MN_CONTIG, EPI_BIAS_RESID_F32),
         ("qkvdg", T, D, 3 * D, K_CONTIG, EPI_BF16), ("fc1dg", T, D, F, MN_CONTIG, EPI_BF16),
         ("outdg", T, D, D, MN_CONTIG, EPI_BF16), ("fc2dg", T, F, D, MN_CONTIG, EPI_GELU_BWD),
         ("ragged", 12345, 768, 512, MN_CONTIG, EPI_BF16), ("fc1wg", D, F, T, -7, EPI_SPLITK),
         ("qkvwg", D, 3 * D, T, -9, EPI_SPLITK), ("wg_ragged", 520, 776, 3008, -3, EPI_SPLITK)]


def main():
    g = torch.Generator(device="cuda").manual_seed(3)
    for name, M, N, K, bl, epi in CASES:
        if epi == EPI_SPLITK:  # weight gradient: both operands M/N-contiguous ([K][M], [K][N]), split -bl
            S = -bl
            A = (torch.rand(K, M, device="cuda", generator=g) * 2 - 1).bfloat16()
            B = (torch.rand(K, N, device="cuda", generator=g) * 2 - 1).bfloat16()
            C = torch.empty(S, M, N, device="cuda")
            ops.gemm(A, B, C, M, N, K, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=M, ldb=N, ldc=N, epilogue=epi,
                     split_k=S)
            torch.cuda.synchronize()
            print(name, M, N, K, hashlib.sha256(C.view(torch.int32).cpu().numpy().tobytes()).hexdigest()[:16], flush=True)
            continue
        A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
        B = ((torch.rand(N, K, device="cuda", generator=g) if bl == K_CONTIG else
              torch.rand(K, N, device="cuda", generator=g)) * 2 - 1).bfloat16()
        ldb = K if bl == K_CONTIG else N
        if epi == EPI_BIAS_RESID_F32:
            C = torch.randn(M, N, device="cuda", generator=g)
            ops.gemm(A, B, C, M, N, K, a_layout=K_CONTIG, b_layout=bl, lda=K, ldb=ldb, ldc=N, epilogue=epi,
                     bias=torch.randn(N, device="cuda", generator=g), aux=C, ldaux=N)
        elif epi == EPI_GELU_BWD:
            U = torch.randn(M, N, device="cuda", generator=g).bfloat16()
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            ops.gemm(A, B, C, M, N, K, a_layout=K_CONTIG, b_layout=bl, lda=K, ldb=ldb, ldc=N, epilogue=epi, aux=U,
                     ldaux=N)
        else:
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            ops.gemm(A, B, C, M, N, K, a_layout=K_CONTIG, b_layout=bl, lda=K, ldb=ldb, ldc=N, epilogue=epi)
        torch.cuda.synchronize()
        print(name, M, N, K, hashlib.sha256(C.view(torch.int16 if C.dtype == torch.bfloat16 else torch.int32).cpu().numpy().tobytes()).hexdigest()[:16], flush=True)


if __name__ == "__main__":
    main()
