#!/usr/bin/env python3
"""Known-good ceiling: torch.matmul (hipBLASLt) bf16 on the ViT-B/16 bs256 GEMM shapes (reference only;
the product path never calls it)."""
import torch


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
for name, (M, N, K) in {"fc1 fwd": (T, 3072, 768), "fc2 fwd": (T, 768, 3072), "qkv fwd": (T, 2304, 768),
                        "out": (T, 768, 768), "fc wgrad": (768, 3072, T), "out wgrad": (768, 768, T)}.items():
    if "wgrad" in name:
        A = torch.randn(K, M, device="cuda").bfloat16().t()
        B = torch.randn(K, N, device="cuda").bfloat16()
    else:
        A = torch.randn(M, K, device="cuda").bfloat16()
        B = torch.randn(N, K, device="cuda").bfloat16().t()
    us = bench(lambda: torch.matmul(A, B))
    print(f"hipBLASLt {name:10s} M={M} N={N} K={K}: {us:8.1f} us  {2*M*N*K/us/1e6:7.1f} TF/s", flush=True)
