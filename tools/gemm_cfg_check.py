#!/usr/bin/env python3
"""Bit-exactness of alternative GEMM tile configs against config 9 (the half-tile ping-pong) on random operands:
    VITMI_LIB=vit-of-pytorch_amd/vitmi/diag/libvit_hip.so python tools/gemm_cfg_check.py 10,11
Diagnostic tool (not a test): prints max |diff| per config and shape, exits non-zero on any difference."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402
from vitmi._lib import EPI_BF16, EPI_F32, K_CONTIG  # noqa: E402


def main():
    cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "10,11").split(",")]
    bad = 0
    g = torch.Generator(device="cuda").manual_seed(0)
    for (M, N, K) in [(50432, 768, 768), (4096, 3072, 768), (2304, 768, 3072), (700, 520, 448), (513, 300, 128)]:
        A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda", generator=g) * 2 - 1).bfloat16()
        for epi, dt in ((EPI_F32, torch.float32), (EPI_BF16, torch.bfloat16)):
            outs = {}
            for t in [9] + cfgs:
                C = torch.full((M, N), float("nan"), device="cuda", dtype=dt)
                ops.gemm(A, B, C, M, N, K, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=K, ldb=K, ldc=N, epilogue=epi,
                         tile=t)
                outs[t] = C
            for t in cfgs:
                d = (outs[t].float() - outs[9].float()).abs().max().item()
                same = torch.equal(outs[t], outs[9])
                bad += not same
                print(f"M={M} N={N} K={K} epi={epi} tile {t} vs 9: {'bit-exact' if same else 'DIFF'} (max |d| {d:.3g})",
                      flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
