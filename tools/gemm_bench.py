#!/usr/bin/env python3
"""Micro-benchmark of vit_gemm_bf16 tile configs / epilogues on the ViT GEMM shapes.

    python tools/gemm_bench.py [--tiles 3,5,6] [--epis 1,3] [--shapes fc1,fc2,...] [--wgrad] [--blas]
                               [--rounds 3] [--T 50432]

Random full-range operands (DVFS: zero data reads high). Variants are timed in interleaved rounds in
one process; the median over rounds is printed. --blas adds torch.matmul (hipBLASLt) on the same
shapes as a same-device reference point.
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import (EPI_BF16, EPI_BIAS_BF16, EPI_BIAS_GELU, EPI_BIAS_GELU_DGELU, EPI_BIAS_RESID_F32,  # noqa
                        EPI_GELU_BWD, EPI_MUL_BF16, EPI_SPLITK, K_CONTIG, MN_CONTIG)


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


def shapes(T, D, M):
    return {"fc1": (T, M, D, K_CONTIG, K_CONTIG), "fc2": (T, D, M, K_CONTIG, K_CONTIG),
            "qkv": (T, 3 * D, D, K_CONTIG, MN_CONTIG), "out": (T, D, D, K_CONTIG, MN_CONTIG),
            "fc2dg": (T, M, D, K_CONTIG, MN_CONTIG), "fc1dg": (T, D, M, K_CONTIG, MN_CONTIG),
            "qkvdg": (T, D, 3 * D, K_CONTIG, K_CONTIG), "sq8k": (8192, 8192, 8192, K_CONTIG, K_CONTIG),
            # the same GEMMs on K-contiguous (transposed) weight copies
            "qkvk": (T, 3 * D, D, K_CONTIG, K_CONTIG), "outk": (T, D, D, K_CONTIG, K_CONTIG),
            "fc2dgk": (T, M, D, K_CONTIG, K_CONTIG), "fc1dgk": (T, D, M, K_CONTIG, K_CONTIG)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="3,5,6")
    ap.add_argument("--epis", default="1")
    ap.add_argument("--shapes", default="fc1,fc2,qkv,out,fc2dg,fc1dg,qkvdg")
    ap.add_argument("--wgrad", action="store_true")
    ap.add_argument("--splits", default="8,16")
    ap.add_argument("--blas", action="store_true")
    ap.add_argument("--colpart", action="store_true", help="also write per-tile column partial sums")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--T", type=int, default=50432)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--M", type=int, default=3072)
    args = ap.parse_args()
    dev = "cuda"
    tiles = [int(t) for t in args.tiles.split(",")]
    epis = [int(e) for e in args.epis.split(",")]
    SH = shapes(args.T, args.D, args.M)
    for spec in args.shapes.split(","):
        if not spec:
            continue
        name, _, e = spec.partition(":")
        shape_epis = [int(x) for x in e.split("/")] if e else epis
        M, N, K, al, bl = SH[name]
        A = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        B = ((torch.rand(N, K, device=dev) if bl == K_CONTIG else torch.rand(K, N, device=dev)) * 2 - 1).bfloat16()
        ldb = K if bl == K_CONTIG else N
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        C2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        U = torch.randn(M, N, device=dev).bfloat16()
        Cf = torch.randn(M, N, device=dev)
        bias = torch.randn(N, device=dev)
        flop = 2.0 * M * N * K
        variants = []
        for tile in tiles:
            for epi in shape_epis:
                extra = {}
                out = C
                if epi == EPI_BIAS_BF16:
                    extra = dict(bias=bias)
                elif epi == EPI_BIAS_RESID_F32:
                    extra = dict(bias=bias, aux=Cf, ldaux=N)
                    out = Cf
                elif epi in (EPI_BIAS_GELU, EPI_BIAS_GELU_DGELU):
                    extra = dict(bias=bias, C2=C2, ldc2=N)
                elif epi in (EPI_GELU_BWD, EPI_MUL_BF16):
                    extra = dict(aux=U, ldaux=N)
                if args.colpart and epi in (EPI_BF16, EPI_GELU_BWD, EPI_MUL_BF16):
                    rows = ops.gemm_tile_rows(A, B, out, M, N, K, a_layout=al, b_layout=bl, lda=K, ldb=ldb, ldc=N,
                                              epilogue=epi, tile=tile, **extra)
                    extra = dict(extra, col_partial=torch.empty((M + rows - 1) // rows, N, device=dev))
                fn = (lambda tile=tile, epi=epi, extra=extra, out=out:
                      ops.gemm(A, B, out, M, N, K, a_layout=al, b_layout=bl, lda=K, ldb=ldb, ldc=N, epilogue=epi,
                               tile=tile, **extra))
                variants.append((f"tile={tile} epi={epi}", fn))
        if args.blas:
            Bt = B if bl == K_CONTIG else B.t()
            Bm = Bt.t() if bl == K_CONTIG else B  # [K, N] view
            variants.append(("torch.matmul", lambda: torch.matmul(A, Bm, out=C)))
        times = {v: [] for v, _ in variants}
        for _ in range(args.rounds):
            for v, fn in variants:
                try:
                    times[v].append(bench(fn))
                except Exception as ex:  # noqa: BLE001
                    times[v].append(float("nan"))
                    print(name, v, "ERR", ex, flush=True)
        for v, _ in variants:
            us = statistics.median(times[v])
            print(f"{name:6s} M={M} N={N} K={K} {v:16s}: {us:8.1f} us {flop / us / 1e6:7.1f} TF/s "
                  f"(min {min(times[v]):.1f})", flush=True)
    if args.wgrad:
        T = args.T
        for (M, N, name) in [(args.D, args.M, "fc2 wgrad"), (args.M, args.D, "fc1 wgrad"),
                             (args.D, args.D, "out wgrad"), (args.D, 3 * args.D, "qkv wgrad")]:
            K = T
            A = (torch.rand(K, M, device=dev) * 2 - 1).bfloat16()
            B = (torch.rand(K, N, device=dev) * 2 - 1).bfloat16()
            flop = 2.0 * M * N * K
            for tile in tiles:
                for S in [int(s) for s in args.splits.split(",")]:
                    ws = torch.empty(S, M, N, device=dev)
                    outw = torch.empty(M, N, device=dev)

                    def run(S=S, tile=tile, ws=ws, outw=outw):
                        ops.gemm(A, B, ws, M, N, K, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=M, ldb=N, ldc=N,
                                 epilogue=EPI_SPLITK, split_k=S, tile=tile)
                        ops.splitk_reduce(ws, 1, S, M, N, outw, N)
                    try:
                        us = bench(run)
                    except Exception as ex:  # noqa: BLE001
                        print(name, tile, S, "ERR", ex, flush=True)
                        continue
                    print(f"{name:10s} M={M} N={N} K={K} tile={tile} S={S} (+reduce): {us:8.1f} us  {flop / us / 1e6:7.1f} TF/s",
                          flush=True)
            if args.blas:
                us = bench(lambda: torch.matmul(A.t(), B))
                print(f"{name:10s} M={M} N={N} K={K} torch.matmul: {us:8.1f} us  {flop / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
