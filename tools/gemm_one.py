#!/usr/bin/env python3
"""Run one vit_gemm_bf16 shape/config/epilogue N times (for rocprofv3 counter passes).

usage: gemm_one.py NAME TILE EPI [ITERS]   NAME in fc1, fc2, qkv, fc1dg, fc2dg
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_BF16, EPI_BIAS_GELU, EPI_GELU_BWD, K_CONTIG, MN_CONTIG  # noqa: E402

T = 50432
SHAPES = {"fc1": (T, 3072, 768, K_CONTIG, K_CONTIG), "fc2": (T, 768, 3072, K_CONTIG, K_CONTIG),
          "qkv": (T, 2304, 768, K_CONTIG, K_CONTIG), "fc1dg": (T, 768, 3072, K_CONTIG, MN_CONTIG),
          "fc2dg": (T, 3072, 768, K_CONTIG, MN_CONTIG), "sq8k": (8192, 8192, 8192, K_CONTIG, K_CONTIG),
          "sq4k": (4096, 4096, 4096, K_CONTIG, K_CONTIG), "fc1k4": (T, 3072, 3072, K_CONTIG, K_CONTIG)}


def main():
    name, tile, epi = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    M, N, K, al, bl = SHAPES[name]
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    B = ((torch.rand(N, K, device="cuda") if bl == K_CONTIG else torch.rand(K, N, device="cuda")) * 2 - 1).bfloat16()
    ldb = K if bl == K_CONTIG else N
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    extra = {}
    if epi == EPI_BIAS_GELU:
        extra = dict(bias=torch.randn(N, device="cuda"), C2=torch.empty_like(C), ldc2=N)
    elif epi == EPI_GELU_BWD:
        extra = dict(aux=torch.randn(M, N, device="cuda").bfloat16(), ldaux=N)
    fn = lambda: ops.gemm(A, B, C, M, N, K, a_layout=al, b_layout=bl, lda=K, ldb=ldb, ldc=N, epilogue=epi,  # noqa
                          tile=tile, **extra)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / iters * 1e3
    print(f"{name} tile={tile} epi={epi}: {us:.1f} us {2.0*M*N*K/us/1e6:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
