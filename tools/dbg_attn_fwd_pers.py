#!/usr/bin/env python3
"""Run-to-run and cross-kernel bit comparison of the persistent attention forward (path 0) and the one-shot
kernel (path 3) on a few shapes."""
import sys, math, torch
sys.path.insert(0, "vit-of-pytorch_amd")
from vitmi import ops


def run(qkv, B, N, H, hd, path):
    D = H * hd
    o = torch.full((B * N, D), float("nan"), device="cuda", dtype=torch.bfloat16)
    lse = torch.full((B, H, N), float("nan"), device="cuda")
    ops.attention_fwd(qkv, o, lse, B, N, H, hd, 1.0 / math.sqrt(hd), path=path)
    torch.cuda.synchronize()
    return o, lse


def cmp(tag, a, b):
    (o1, l1), (o0, l0) = a, b
    ne = (o1 != o0)
    d = (o1.float() - o0.float()).abs()
    print(f"  {tag}: o ne frac {ne.float().mean().item():.5f} max {d.max().item():.3g} nan {o1.isnan().sum().item()} "
          f"lse ne {(l1 != l0).float().mean().item():.5f} max {(l1 - l0).abs().max().item():.3g}", flush=True)
    if ne.any():
        rows = ne.any(1).nonzero().flatten()
        print("    rows:", rows[:16].tolist(), "count", rows.numel(), flush=True)


for (B, N, H, hd) in [(2, 197, 12, 64), (2, 208, 3, 64), (1, 5, 3, 64), (24, 197, 12, 64)]:
    D = H * hd
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + N)
    qkv = (torch.randn(B * N, 3 * D, device="cuda", generator=g) * 1.5).bfloat16()
    p1, p2, s1, s2 = run(qkv, B, N, H, hd, 0), run(qkv, B, N, H, hd, 0), run(qkv, B, N, H, hd, 3), run(qkv, B, N, H, hd, 3)
    print(B, N, H, hd, flush=True)
    cmp("pers vs pers", p1, p2)
    cmp("oneshot vs oneshot", s1, s2)
    cmp("pers vs oneshot", p1, s1)
