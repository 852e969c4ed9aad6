#!/usr/bin/env python3
"""Micro-benchmark of the LayerNorm kernels on the ViT-B/16 bs256 shape."""
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


T, D = 50432, 768
x = torch.randn(T, D, device="cuda")
g = torch.randn(D, device="cuda")
b = torch.randn(D, device="cuda")
y = torch.empty(T, D, device="cuda", dtype=torch.bfloat16)
mu = torch.empty(T, device="cuda")
rs = torch.empty(T, device="cuda")
dy = torch.randn(T, D, device="cuda").bfloat16()
dh = torch.randn(T, D, device="cuda")
dhb = torch.empty(T, D, device="cuda", dtype=torch.bfloat16)
part = torch.empty(ops.layernorm_bwd_partial_rows(T), 3 * D, device="cuda")
dgb = torch.empty(2 * D, device="cuda")
ds = torch.empty(D, device="cuda")
us = bench(lambda: ops.layernorm_fwd(x, D, g, b, y, D, mu, rs, T, D))
print(f"ln_fwd  {us:7.1f} us  {T*D*6/us/1e3:6.0f} GB/s")
for name, kw in [("bwd full", dict(dres=dh, lddres=D, dx_bf16=dhb, lddxb=D, dgamma_dbeta=dgb, dx_colsum=ds)),
                 ("bwd no colsum", dict(dres=dh, lddres=D, dx_bf16=dhb, lddxb=D, dgamma_dbeta=dgb)),
                 ("bwd no params", dict(dres=dh, lddres=D, dx_bf16=dhb, lddxb=D))]:
    us = bench(lambda: ops.layernorm_bwd(dy, D, x, D, mu, rs, g, dh, D, part, T, D, **kw))
    print(f"ln_{name:14s} {us:7.1f} us  {T*D*16/us/1e3:6.0f} GB/s", flush=True)
