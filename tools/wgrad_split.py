#!/usr/bin/env python3
"""Split-K sweep of the engine's weight-gradient GEMMs exactly as ViTEngine._wgrad issues them
(split-K 256x256 ping-pong into f32 slabs + fixed-order reduce), including the batched q|k|v call.
    python tools/wgrad_split.py [--T 50432] [--D 768] [--M 3072] [--splits 7,9,14,28]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402
from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_SPLITK, MN_CONTIG  # noqa: E402


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
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=50432)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--M", type=int, default=3072)
    ap.add_argument("--splits", default="4,7,9,12,14,18,21,28")
    a = ap.parse_args()
    T, D, M = a.T, a.D, a.M
    dev = "cuda"
    # (name, M, N, lda, ldb, batch, b batch stride): A is [T][lda], B is [T][ldb]
    cases = [("fc2", D, M, D, M, 1, 0), ("fc1", M, D, M, D, 1, 0), ("out", D, D, D, D, 1, 0),
             ("qkv x3", D, D, D, 3 * D, 3, D)]
    for name, m, n, lda, ldb, batch, bbs in cases:
        A = (torch.rand(T, lda, device=dev) * 2 - 1).bfloat16()
        B = (torch.rand(T, ldb, device=dev) * 2 - 1).bfloat16()
        out = torch.empty(batch, m, n, device=dev)
        flop = 2.0 * m * n * T * batch
        for s in [int(x) for x in a.splits.split(",")]:
            ws = torch.empty(batch * s * m * n, device=dev)

            def run(s=s, ws=ws):
                ops.gemm(A, B, ws, m, n, T, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=lda, ldb=ldb, ldc=n,
                         epilogue=EPI_SPLITK, batch=batch, b_bs=bbs, split_k=s)
                ops.splitk_reduce(ws, batch, s, m, n, out, n, m * n)
            us = bench(run)
            print(f"{name:7s} {m}x{n}x{T} batch {batch} split {s:3d}: {us:8.1f} us {flop / us / 1e6:7.1f} TF/s",
                  flush=True)


if __name__ == "__main__":
    main()
