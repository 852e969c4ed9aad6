#!/usr/bin/env python3
"""Wave-quantisation tail of the 256 x 256 GEMMs: what the remainder rows cost today (full call minus
the whole-wave rows alone) against running them as split-K 256 x 256 tiles plus a reduction.

    python tools/tail_bench.py [--shapes fc2:4,fc1dgk:1,qkvdg:1,outk:1,outk:4,fc1:8] [--splits 2,3,4]
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

from gemm_bench import bench, shapes  # noqa: E402
from vitmi import ops  # noqa: E402
from vitmi._lib import (EPI_BIAS_GELU_DGELU, EPI_BIAS_RESID_F32, EPI_SPLITK, K_CONTIG)  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="fc2:4,fc1dgk:1,qkvdg:1,outk:1,outk:4,fc1:8")
    ap.add_argument("--splits", default="2,3,4")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = "cuda"
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    SH = shapes(50432, 768, 3072)
    for spec in args.shapes.split(","):
        name, _, e = spec.partition(":")
        epi = int(e)
        M, N, K, al, bl = SH[name]
        tiles_n = (N + 255) // 256
        tiles = ((M + 255) // 256) * tiles_n
        full = tiles // ncu
        main_rows = (full * ncu // tiles_n) * 256
        rem = M - main_rows
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        B = ((torch.rand(N, K, device=dev) if bl == K_CONTIG else torch.rand(K, N, device=dev)) * 2 - 1).bfloat16()
        ldb = K if bl == K_CONTIG else N
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        C2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        Cf = torch.randn(M, N, device=dev)
        bias = torch.randn(N, device=dev)
        extra, out = {}, C
        if epi == EPI_BIAS_RESID_F32:
            extra, out = dict(bias=bias, aux=Cf, ldaux=N), Cf
        elif epi == EPI_BIAS_GELU_DGELU:
            extra = dict(bias=bias, C2=C2, ldc2=N)
        kw = dict(a_layout=al, b_layout=bl, lda=K, ldb=ldb, ldc=N, epilogue=epi)
        variants = [("full call", lambda: ops.gemm(A, B, out, M, N, K, **kw, **extra)),
                    ("whole-wave rows", lambda: ops.gemm(A, B, out, main_rows, N, K, **kw, **extra)),
                    ("tail rows alone", lambda: ops.gemm(A[main_rows:], B, out[main_rows:], rem, N, K, **kw, **extra))]
        for S in [int(s) for s in args.splits.split(",")]:
            ws = torch.empty(S, rem, N, device=dev)
            red = torch.empty(rem, N, device=dev)

            def sk(S=S, ws=ws, red=red):
                ops.gemm(A[main_rows:], B, ws, rem, N, K, a_layout=al, b_layout=bl, lda=K, ldb=ldb, ldc=N,
                         epilogue=EPI_SPLITK, split_k=S, tile=9 if bl == K_CONTIG else 5)
                ops.splitk_reduce(ws, 1, S, rem, N, red, N)
            variants.append((f"tail split-K {S} + reduce", sk))

            def sk_only(S=S, ws=ws):
                ops.gemm(A[main_rows:], B, ws, rem, N, K, a_layout=al, b_layout=bl, lda=K, ldb=ldb, ldc=N,
                         epilogue=EPI_SPLITK, split_k=S, tile=9 if bl == K_CONTIG else 5)
            variants.append((f"tail split-K {S} GEMM only", sk_only))
        times = {v: [] for v, _ in variants}
        for _ in range(args.rounds):
            for v, fn in variants:
                times[v].append(bench(fn))
        med = {v: statistics.median(t) for v, t in times.items()}
        print(f"{name} epi {epi}: M={M} N={N} K={K} tiles={tiles} main_rows={main_rows} tail_rows={rem}", flush=True)
        for v, _ in variants:
            print(f"   {v:28s} {med[v]:8.1f} us", flush=True)
        print(f"   {'tail cost in the full call':28s} {med['full call'] - med['whole-wave rows']:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
