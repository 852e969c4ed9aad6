#!/usr/bin/env python3
"""Micro-benchmark of vit_gemm_bf16 tile configs / epilogues on the ViT-B/16 bs256 GEMM shapes."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_BF16, EPI_BIAS_GELU, EPI_SPLITK, EPI_F32, K_CONTIG, MN_CONTIG  # noqa: E402


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    dev = "cuda"
    T = 50432
    cases = []
    for (M, N, K, al, bl, name) in [(T, 3072, 768, K_CONTIG, K_CONTIG, "fc1 fwd"),
                                    (T, 768, 3072, K_CONTIG, K_CONTIG, "fc2 fwd"),
                                    (T, 2304, 768, K_CONTIG, MN_CONTIG, "qkv fwd"),
                                    (T, 768, 3072, K_CONTIG, MN_CONTIG, "fc1 dgrad"),
                                    (T, 768, 768, K_CONTIG, K_CONTIG, "out dgrad")]:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16() if bl == K_CONTIG else torch.randn(K, N, device=dev).bfloat16()
        ldb = K if bl == K_CONTIG else N
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        C2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        Cf = torch.empty(M, N, device=dev)
        bias = torch.randn(N, device=dev)
        flop = 2.0 * M * N * K
        for tile in (0, 1, 2, 3, 4):
            for epi, out, extra in ((EPI_BF16, C, {}), (EPI_BIAS_GELU, C, dict(bias=bias, C2=C2, ldc2=N)),
                                    (EPI_F32, Cf, {})):
                try:
                    us = bench(lambda: ops.gemm(A, B, out, M, N, K, a_layout=al, b_layout=bl, lda=K, ldb=ldb, ldc=N,
                                                epilogue=epi, tile=tile, **extra))
                except Exception as ex:  # noqa: BLE001
                    print(name, tile, epi, "ERR", ex)
                    continue
                print(f"{name:10s} M={M} N={N} K={K} tile={tile} epi={epi}: {us:8.1f} us  {flop/us/1e6:7.1f} TF/s",
                      flush=True)
    # wgrad shapes (TN, split-K)
    for (M, N, name) in [(768, 3072, "fc2 wgrad"), (3072, 768, "fc1 wgrad"), (768, 768, "out wgrad")]:
        K = T
        A = torch.randn(K, M, device=dev).bfloat16()
        B = torch.randn(K, N, device=dev).bfloat16()
        flop = 2.0 * M * N * K
        for tile in (0, 1, 3, 4):
            for S in (8, 16, 32):
                ws = torch.empty(S, M, N, device=dev)
                us = bench(lambda: ops.gemm(A, B, ws, M, N, K, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=M, ldb=N,
                                            ldc=N, epilogue=EPI_SPLITK, split_k=S, tile=tile))
                print(f"{name:10s} M={M} N={N} K={K} tile={tile} S={S}: {us:8.1f} us  {flop/us/1e6:7.1f} TF/s",
                      flush=True)


if __name__ == "__main__":
    main()
