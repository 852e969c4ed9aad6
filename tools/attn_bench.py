#!/usr/bin/env python3
"""Micro-benchmark of the fused attention kernels on the ViT-B/16 bs256 shape (N=197, H=12, hd=64)."""
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


B, N, H, hd = 256, 197, 12, 64
D = H * hd
qkv = (torch.randn(B * N, 3 * D, device="cuda") * 0.5).bfloat16()
o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B * H * N, device="cuda")
do = torch.randn(B * N, D, device="cuda").bfloat16()
dqkv = torch.empty_like(qkv)
bp = torch.empty(B, 3 * D, device="cuda")
fl = 4 * B * H * N * N * hd
us = bench(lambda: ops.attention_fwd(qkv, o, lse, B, N, H, hd, hd ** -0.5))
print(f"attn_fwd {us:7.1f} us  {fl/us/1e6:6.1f} TFLOP/s")
us = bench(lambda: ops.attention_bwd(qkv, o, do, lse, dqkv, B, N, H, hd, hd ** -0.5, bias_partial=bp))
print(f"attn_bwd {us:7.1f} us  {2.5*fl/us/1e6:6.1f} TFLOP/s (2.5x fwd flops)", flush=True)
