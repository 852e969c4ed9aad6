#!/usr/bin/env python3
"""Diagnostic: the split-K weight-gradient GEMM with one operand K-contiguous (a feature-major copy of that
activation) against both M/N-contiguous (the production layout), same shapes, interleaved rounds.
    python3 tools/dbg/wgrad_layout_bench.py
"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_SPLITK, K_CONTIG, MN_CONTIG  # noqa: E402


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    T = 50432
    g = torch.Generator(device="cuda").manual_seed(1)
    for (M, N, S) in [(768, 3072, 7), (3072, 768, 7), (768, 768, 7), (768, 2304, 7)]:
        K = T
        fl = 2.0 * M * N * K
        fns = {}
        for al, bl in [(MN_CONTIG, MN_CONTIG), (K_CONTIG, MN_CONTIG), (MN_CONTIG, K_CONTIG)]:
            A = ((torch.rand(M, K, device="cuda", generator=g) if al == K_CONTIG else
                  torch.rand(K, M, device="cuda", generator=g)) * 2 - 1).bfloat16()
            B = ((torch.rand(N, K, device="cuda", generator=g) if bl == K_CONTIG else
                  torch.rand(K, N, device="cuda", generator=g)) * 2 - 1).bfloat16()
            lda = K if al == K_CONTIG else M
            ldb = K if bl == K_CONTIG else N
            ws = torch.empty(S, M, N, device="cuda")
            fns[(al, bl)] = (lambda A=A, B=B, al=al, bl=bl, lda=lda, ldb=ldb, ws=ws:
                             ops.gemm(A, B, ws, M, N, K, a_layout=al, b_layout=bl, lda=lda, ldb=ldb, ldc=N,
                                      epilogue=EPI_SPLITK, split_k=S))
        times = {k: [] for k in fns}
        for _ in range(3):
            for k, fn in fns.items():
                times[k].append(bench(fn))
        name = {(MN_CONTIG, MN_CONTIG): "A MN, B MN", (K_CONTIG, MN_CONTIG): "A K,  B MN",
                (MN_CONTIG, K_CONTIG): "A MN, B K "}
        for k, v in times.items():
            us = statistics.median(v)
            print(f"M={M} N={N} K={K} S={S} {name[k]}: {us:7.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
