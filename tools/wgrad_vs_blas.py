#!/usr/bin/env python3
"""Weight-gradient GEMM shapes of the B/16 bs256 step: the split-K HIP kernel (+ reduction) against
hipBLASLt through torch.mm(out_dtype=float32) on the same bf16 operands (HIP events)."""
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


T = 50432
for name, M, N in (("fc1", 3072, 768), ("fc2", 768, 3072), ("qkv", 2304, 768), ("out", 768, 768)):
    dy = torch.randn(T, M, device="cuda").bfloat16()
    x = torch.randn(T, N, device="cuda").bfloat16()
    out = torch.empty(M, N, device="cuda")
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    s = max(1, min(round(256 / tiles), T // 64 // 8, 32))
    ws = torch.empty(s * M * N, device="cuda")

    def ours():
        ops.gemm(dy, x, ws, M, N, T, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=M, ldb=N, ldc=N,
                 epilogue=EPI_SPLITK, split_k=s)
        ops.splitk_reduce(ws, 1, s, M, N, out, N, 0)

    def blas():
        torch.mm(dy.t(), x, out_dtype=torch.float32)

    ref = torch.mm(dy.t().float(), x.float())
    ours()
    err = float((out - ref).norm() / ref.norm())
    t1 = bench(ours)
    try:
        if os.environ.get("SKIP_BLAS"):
            raise RuntimeError("skipped (SKIP_BLAS)")
        t2 = bench(blas)
    except Exception as ex:  # noqa: BLE001
        t2 = float("nan")
        print("hipBLASLt path failed:", ex)
    fl = 2 * M * N * T
    print(f"{name:4s} M{M} N{N} K{T} split {s}: ours {t1:7.1f} us ({fl / t1 / 1e6:6.1f} TF/s, rel err {err:.1e}) "
          f"| hipBLASLt {t2:7.1f} us ({fl / t2 / 1e6:6.1f} TF/s)", flush=True)
