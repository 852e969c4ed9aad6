#!/usr/bin/env python3
"""Print the backward's relative errors (dq, dk, dv, bias partials) against torch fp32 for a few shapes."""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


CASES = [(2, 2, 2, 64, 1.5, None), (2, 17, 2, 64, 1.5, None), (2, 197, 2, 64, 1.5, None), (3, 17, 2, 32, 1.5, None),
         (24, 197, 12, 64, 1.5, None), (32, 2, 12, 64, 30.0, None), (32, 2, 12, 64, 30.0, 1), (32, 2, 12, 64, 1.5, 1),
         (24, 197, 12, 64, 1.5, 1)]
for B, N, H, hd, amp, nq in CASES:
    torch.manual_seed(0)
    D = H * hd
    qkv = (torch.randn(B * N, 3 * D, device="cuda") * amp).bfloat16()
    o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device="cuda")
    ops.attention_fwd(qkv, o, lse, B, N, H, hd, 1.0 / math.sqrt(hd))
    qf = qkv.float().requires_grad_(True)
    q, k, v = qf.view(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    p = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(hd), -1)
    oref = (p @ v).permute(0, 2, 1, 3).reshape(B * N, D)
    dout = torch.randn(B * N, D, device="cuda").bfloat16()
    dqkv = torch.full((B * N, 3 * D), float("nan"), device="cuda", dtype=torch.bfloat16)
    bpart = torch.full((B * ops.attention_bias_rows(N, hd), 3 * D), float("nan"), device="cuda")
    if nq is not None:
        dout.view(B, N, D)[:, nq:] = 0
    ops.attention_bwd(qkv, o, dout, lse, dqkv, B, N, H, hd, 1.0 / math.sqrt(hd), bias_partial=bpart, q_rows=nq)
    gref, = torch.autograd.grad(oref, qf, dout.float())
    bpart = bpart.view(B, -1, 3 * D).sum(1)
    m = dqkv.float().view(B * N, 3, D)
    gr = gref.view(B * N, 3, D)
    bref = gref.view(B, N, 3 * D).sum(1)
    print(f"B{B} N{N} H{H} hd{hd} amp{amp} nq{nq}: dq {rel(m[:, 0], gr[:, 0]):.2e} dk {rel(m[:, 1], gr[:, 1]):.2e} "
          f"dv {rel(m[:, 2], gr[:, 2]):.2e} | bias q {rel(bpart[:, :D], bref[:, :D]):.2e} "
          f"v {rel(bpart[:, 2 * D:], bref[:, 2 * D:]):.2e} k-abs {float((bpart[:, D:2 * D] - bref[:, D:2 * D]).abs().max()):.2e}"
          f" nan {int(torch.isnan(dqkv.float()).sum())}", flush=True)
    if N == 2 and amp < 2 and nq is None:
        print("  bias q got ", bpart[0, :8].tolist())
        print("  bias q want", bref[0, :8].tolist())
