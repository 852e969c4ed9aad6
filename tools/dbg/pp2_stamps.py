#!/usr/bin/env python3
"""Diagnostic: slot timeline of the half-tile ping-pong GEMM (gemm_pp2) from s_memtime stamps.

Diagnostic library (make DIAG=1: VIT_PP2_STAMPS), VIT_GEMM_DIAG=4: waves 0 (group 0) and 4 (group 1) of the launch-index-0
workgroup stamp 8 points of k-tile nk/2: 0 slot start, 1 fragment reads issued, 2 DMA issued, 3 reads back
(lgkmcnt 0), 4 own DMA of two slots ago landed (vmcnt), 5 past the barrier = multiply start, 6 the 64 MFMAs issued,
7 past the next barrier. Prints cycles relative to group 0's point 0, per shape and run.
    VITMI_LIB=vit-of-pytorch_amd/vitmi/diag/libvit_hip.so VIT_GEMM_DIAG=4 python3 tools/dbg/pp2_stamps.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import _lib, ops  # noqa: E402
from vitmi._lib import EPI_BF16, EPI_SPLITK, K_CONTIG, MN_CONTIG  # noqa: E402

NAMES = ["start", "reads", "dma", "lgkm0", "vmcnt", "bar1", "mfma", "bar2"]


def main():
    assert os.environ.get("VIT_GEMM_DIAG") == "4", "run with VIT_GEMM_DIAG=4"
    lib = _lib.load()
    buf = torch.zeros(16, dtype=torch.int64, device="cuda")
    lib.vit_gemm_set_stamps(ctypes.c_void_p(buf.data_ptr()))
    T, D, F = 50432, 768, 3072
    g = torch.Generator(device="cuda").manual_seed(5)
    for name, M, N, K, al, bl, split in [("fc2 fwd (K,K)", T, D, F, K_CONTIG, K_CONTIG, 1),
                                         ("fc1 dgrad (K,MN)", T, D, F, K_CONTIG, MN_CONTIG, 1),
                                         ("qkv dgrad (K,K)", T, D, 3 * D, K_CONTIG, K_CONTIG, 1),
                                         ("fc1 wgrad (MN,MN) split 7", D, F, T, MN_CONTIG, MN_CONTIG, 7)]:
        A = ((torch.rand(M, K, device="cuda", generator=g) if al == K_CONTIG else
              torch.rand(K, M, device="cuda", generator=g)) * 2 - 1).bfloat16()
        B = ((torch.rand(N, K, device="cuda", generator=g) if bl == K_CONTIG else
              torch.rand(K, N, device="cuda", generator=g)) * 2 - 1).bfloat16()
        lda = K if al == K_CONTIG else M
        ldb = K if bl == K_CONTIG else N
        if split > 1:
            C = torch.empty(split, M, N, device="cuda")
            kw = dict(epilogue=EPI_SPLITK, split_k=split)
        else:
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            kw = dict(epilogue=EPI_BF16, tile=9)
        for run in range(4):
            buf.zero_()
            for _ in range(3):
                ops.gemm(A, B, C, M, N, K, a_layout=al, b_layout=bl, lda=lda, ldb=ldb, ldc=N, **kw)
            torch.cuda.synchronize()
            s = buf.cpu().tolist()
            if run == 0:
                continue
            t0 = s[0]
            rows = []
            for grp in range(2):
                v = s[grp * 8:(grp + 1) * 8]
                rows.append(f"g{grp}: " + " ".join(f"{NAMES[k]}={v[k] - t0:6d}" for k in range(8)))
                d = [v[k + 1] - v[k] for k in range(7)]
                rows.append(f"    deltas " + " ".join(f"{NAMES[k + 1]}+{d[k]}" for k in range(7)))
            print(f"{name} run {run}:\n  " + "\n  ".join(rows), flush=True)


if __name__ == "__main__":
    main()
