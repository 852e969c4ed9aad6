#!/usr/bin/env python3
"""Diagnostic: the 8-phase GEMM schedule (diagnostic tile config 12) against config 9 (gemm_pp2).

Bit-identity of the bf16 output on K-contiguous operands (the same per-accumulator MFMA order), ragged and short-K
cases included, then interleaved timings on the ViT-B/16 bs256 forward / data-gradient shapes.
    VITMI_LIB=vit-of-pytorch_amd/vitmi/diag/libvit_hip.so python3 tools/dbg/ph8_check.py
"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_BF16, K_CONTIG  # noqa: E402


def run(A, B, M, N, K, tile):
    C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    ops.gemm(A, B, C, M, N, K, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=K, ldb=K, ldc=N, epilogue=EPI_BF16,
             tile=tile)
    return C


def main():
    torch.manual_seed(0)
    ok = True
    for (M, N, K) in [(256, 256, 64), (256, 256, 128), (512, 256, 192), (300, 700, 256), (1000, 520, 640),
                      (4096, 3072, 768), (2048, 768, 3072)]:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        c9, c12 = run(A, B, M, N, K, 9), run(A, B, M, N, K, 12)
        ref = (A.float() @ B.float().t())
        same = torch.equal(c9, c12)
        err = float((c12.float() - ref).abs().max())
        ok &= same and err < 0.05 * float(ref.abs().max())
        print(f"M={M} N={N} K={K}: identical={same} max|c12-ref|={err:.4f}", flush=True)
    if not ok:
        print("PARITY FAILED")
        sys.exit(1)
    T, D, F = 50432, 768, 3072
    shapes = {"fc1": (T, F, D), "fc2": (T, D, F), "qkvk": (T, 3 * D, D), "outk": (T, D, D), "qkvdg": (T, D, 3 * D),
              "fc1dgk": (T, D, F), "fc2dgk": (T, F, D)}
    for name, (M, N, K) in shapes.items():
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fns = {t: (lambda t=t: ops.gemm(A, B, C, M, N, K, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=K, ldb=K, ldc=N,
                                         epilogue=EPI_BF16, tile=t)) for t in (9, 12)}
        times = {t: [] for t in fns}
        for _ in range(5):
            for t, fn in fns.items():
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[t].append(s.elapsed_time(e) / 20 * 1e3)
        fl = 2.0 * M * N * K
        line = "  ".join(f"tile{t}: {statistics.median(v):7.1f} us {fl / statistics.median(v) / 1e6:6.1f} TF/s"
                         for t, v in times.items())
        print(f"{name:7s} M={M} N={N} K={K}  {line}", flush=True)


if __name__ == "__main__":
    main()
