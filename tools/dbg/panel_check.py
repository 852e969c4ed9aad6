#!/usr/bin/env python3
"""Diagnostic: persistent row-panel GEMM (diagnostic tile config 12) against the one-shot half-tile kernel (config 9).

Bit-identity of the output (same per-tile arithmetic, only the tile -> workgroup walk differs) on the N = 768 B/16
shapes and ragged cases, for the plain bf16 and the bias + f32-residual epilogues, both B layouts.
    VITMI_LIB=vit-of-pytorch_amd/vitmi/diag/libvit_hip.so python3 tools/dbg/panel_check.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_BF16, EPI_BIAS_RESID_F32, K_CONTIG, MN_CONTIG  # noqa: E402


def main():
    torch.manual_seed(0)
    ok = True
    for (M, N, K) in [(300, 704, 256), (1000, 520, 640), (50432, 768, 768), (50432, 768, 3072), (70000, 768, 768)]:
        for bl in (K_CONTIG, MN_CONTIG):
            A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
            B = ((torch.rand(N, K, device="cuda") if bl == K_CONTIG else torch.rand(K, N, device="cuda")) * 2 - 1).bfloat16()
            ldb = K if bl == K_CONTIG else N
            bias = torch.randn(N, device="cuda")
            R = torch.randn(M, N, device="cuda")
            for epi in (EPI_BF16, EPI_BIAS_RESID_F32):
                outs = []
                for tile in (9, 12):
                    if epi == EPI_BF16:
                        C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
                        ops.gemm(A, B, C, M, N, K, a_layout=K_CONTIG, b_layout=bl, lda=K, ldb=ldb, ldc=N, epilogue=epi,
                                 tile=tile)
                    else:
                        C = R.clone()
                        ops.gemm(A, B, C, M, N, K, a_layout=K_CONTIG, b_layout=bl, lda=K, ldb=ldb, ldc=N, epilogue=epi,
                                 tile=tile, bias=bias, aux=C, ldaux=N)
                    outs.append(C)
                torch.cuda.synchronize()
                same = torch.equal(outs[0], outs[1])
                ok &= same
                print(f"M={M} N={N} K={K} b_layout={bl} epi={epi}: identical={same}", flush=True)
    if not ok:
        print("PARITY FAILED")
        sys.exit(1)


if __name__ == "__main__":
    main()
