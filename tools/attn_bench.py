#!/usr/bin/env python3
"""Micro-benchmark of the fused attention kernels (HIP events, warm L2 excluded by size).

    python tools/attn_bench.py [B N H hd path] ...      default: ViT-B/16 bs256 (256 197 12 64 0)
path: 0 auto, 1 LDS-resident, 2 K/V-tiled, 3 LDS-resident one-shot (no persistent kernels). Algorithmic FLOPs: 4 B H N^2 hd forward, 2.5x that backward
(5 products); bytes: q|k|v read + o written forward, q|k|v + dO read + dq|dk|dv written backward.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402


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


def run(B, N, H, hd, path):
    D = H * hd
    qkv = (torch.randn(B * N, 3 * D, device="cuda") * 0.5).bfloat16()
    o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * N, device="cuda")
    do = torch.randn(B * N, D, device="cuda").bfloat16()
    dqkv = torch.empty_like(qkv)
    bp = torch.empty(B * ops.attention_bias_rows(N, hd, path), 3 * D, device="cuda")
    ws = torch.empty(max(1, ops.attention_workspace_elems(B, N, H, path)), device="cuda")
    fl = 4 * B * H * N * N * hd
    by_f = (3 + 1) * B * N * D * 2
    by_b = (3 + 1 + 3) * B * N * D * 2
    us = bench(lambda: ops.attention_fwd(qkv, o, lse, B, N, H, hd, hd ** -0.5, path=path))
    print(f"B{B} N{N} H{H} hd{hd} path{path} fwd {us:7.1f} us {fl / us / 1e6:6.1f} TF/s {by_f / us / 1e6:5.2f} TB/s",
          flush=True)
    nq = int(os.environ.get("ATTN_QROWS", N))  # q_rows (1: the pruned last layer's cls query pair)
    us = bench(lambda: ops.attention_bwd(qkv, o, do, lse, dqkv, B, N, H, hd, hd ** -0.5, bias_partial=bp, path=path,
                                         workspace=ws, q_rows=nq))
    print(f"B{B} N{N} H{H} hd{hd} path{path} bwd {us:7.1f} us {2.5 * fl / us / 1e6:6.1f} TF/s "
          f"{by_b / us / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:]]
    cases = [a[i:i + 5] for i in range(0, len(a), 5)] or [[256, 197, 12, 64, 0]]
    for c in cases:
        run(*c)
