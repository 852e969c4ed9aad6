#!/usr/bin/env python3
"""Attention backward phase probe: full backward vs q_rows = 1 (stage 1 writes zero dQ strips, stage 2
visits one query pair) vs forward, per (B, N, H, hd) given on the command line.
    python tools/attn_phase.py B N H hd [B N H hd ...]"""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402


def timeit(fn, iters=20):
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


args = [int(v) for v in sys.argv[1:]]
for k in range(0, len(args), 4):
    B, N, H, hd = args[k:k + 4]
    D = H * hd
    sc = 1.0 / math.sqrt(hd)
    qkv = (torch.randn(B * N, 3 * D, device="cuda") * 1.5).bfloat16()
    o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device="cuda")
    dout = torch.randn(B * N, D, device="cuda").bfloat16()
    dqkv = torch.empty(B * N, 3 * D, device="cuda", dtype=torch.bfloat16)
    ops.attention_fwd(qkv, o, lse, B, N, H, hd, sc)
    tf = timeit(lambda: ops.attention_fwd(qkv, o, lse, B, N, H, hd, sc))
    tb = timeit(lambda: ops.attention_bwd(qkv, o, dout, lse, dqkv, B, N, H, hd, sc))
    t1 = timeit(lambda: ops.attention_bwd(qkv, o, dout, lse, dqkv, B, N, H, hd, sc, q_rows=1))
    items = B * H
    print(f"B{B} N{N} H{H} hd{hd}: fwd {tf:7.1f} us  bwd {tb:7.1f} us  bwd(q_rows=1) {t1:7.1f} us  "
          f"bwd per item-slot {tb / max(1, items / 256):.1f} us", flush=True)
