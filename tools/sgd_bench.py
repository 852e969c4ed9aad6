#!/usr/bin/env python3
"""Micro-benchmark of the device-hyper SGD step (vit_sgd_step_dev) over ViT-B/16's 86.6 M parameters and ViT-L/16's
304 M (HIP events), and a check of the update against torch: python tools/sgd_bench.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

for n in (86_567_656, 304_326_632):
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    buf = torch.randn(n, device="cuda")
    pb = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    hyper = torch.tensor([0.01, 0.9, 0.0], device="cuda")
    p0, b0 = p.clone(), buf.clone()
    ops.sgd_step_dev(p, g, buf, pb, n, hyper, 1e-4)
    d = 0.9 * b0 + (g + 1e-4 * p0)
    ok = torch.allclose(buf, d, rtol=1e-6, atol=1e-6) and torch.allclose(p, p0 - 0.01 * d, rtol=1e-6, atol=1e-6) \
        and torch.equal(pb, p.bfloat16())
    for _ in range(3):
        ops.sgd_step_dev(p, g, buf, pb, n, hyper, 1e-4)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        ops.sgd_step_dev(p, g, buf, pb, n, hyper, 1e-4)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    print(f"n {n}: {us:8.1f} us  {22 * n / us / 1e6:5.2f} TB/s  update ok {ok}", flush=True)
    del p, g, buf, pb, p0, b0
