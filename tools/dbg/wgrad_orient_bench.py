#!/usr/bin/env python3
"""Diagnostic: the split-K weight gradient (both operands M/N-contiguous, production layout) in both orientations,
dW = A^T B as [M][N] against dW^T = B^T A as [N][M] (operands swapped), interleaved rounds, production library.
    python3 tools/dbg/wgrad_orient_bench.py
"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_SPLITK, MN_CONTIG  # noqa: E402


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
    g = torch.Generator(device="cuda").manual_seed(2)
    for (M, N) in [(768, 3072), (768, 2304), (768, 768)]:
        A = (torch.rand(T, M, device="cuda", generator=g) * 2 - 1).bfloat16()
        B = (torch.rand(T, N, device="cuda", generator=g) * 2 - 1).bfloat16()
        fns = {}
        for name, (a, b, m, n) in {"dW  [M][N]": (A, B, M, N), "dW^T [N][M]": (B, A, N, M)}.items():
            S = ops.splitk_factor(m, n, T, 1, 256)
            ws = torch.empty(S, m, n, device="cuda")
            fns[name] = (S, lambda a=a, b=b, m=m, n=n, S=S, ws=ws: ops.gemm(
                a, b, ws, m, n, T, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=m, ldb=n, ldc=n, epilogue=EPI_SPLITK,
                split_k=S))
        times = {k: [] for k in fns}
        for _ in range(4):
            for k, (S, fn) in fns.items():
                times[k].append(bench(fn))
        for k, v in times.items():
            us = statistics.median(v)
            print(f"M={M} N={N} {k} split {fns[k][0]}: {us:7.1f} us {2.0 * M * N * T / us / 1e6:7.1f} TF/s "
                  f"(all: {' '.join(f'{x:.1f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main()
