#!/usr/bin/env python3
"""Run the attention backward once under the VIT_ATTN_STAMPS diagnostic build (VITMI_LIB=.../ab/libvit_hip.so)
and print workgroup 0's per-item phase durations (cycles) for waves 0 and 7."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import _lib, ops  # noqa: E402

B, N, H, hd = 256, 197, 12, 64
nq = int(os.environ.get("ATTN_QROWS", N))
D = H * hd
qkv = (torch.randn(B * N, 3 * D, device="cuda") * 0.5).bfloat16()
o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B * H * N, device="cuda")
do = torch.randn(B * N, D, device="cuda").bfloat16()
dqkv = torch.empty_like(qkv)
bp = torch.empty(B * ops.attention_bias_rows(N, hd), 3 * D, device="cuda")
ops.attention_fwd(qkv, o, lse, B, N, H, hd, hd ** -0.5)
for _ in range(3):
    ops.attention_bwd(qkv, o, do, lse, dqkv, B, N, H, hd, hd ** -0.5, bias_partial=bp, q_rows=nq)
torch.cuda.synchronize()
lib = _lib.load()
buf = (ctypes.c_ulonglong * 128)()
lib.vit_attn_stamps(buf)
names = ["wait_vm", "barrier_a", "stage1", "barrier_1_2", "stage2_prologue", "stage2", "bias", "next"]
for w in range(2):
    for it in range(4):
        t = [buf[w * 32 + it * 8 + k] for k in range(8)]
        # point order in time: 0 (start), 1, 2, 3 (end stage 1), 4, 7 (after stage-2 prologue), 5 (end stage 2), 6 (end)
        seq = [t[0], t[1], t[2], t[3], t[4], t[7], t[5], t[6]]
        d = [seq[k + 1] - seq[k] for k in range(7)]
        nxt = buf[w * 32 + (it + 1) * 8] - t[6] if it < 3 else 0
        print(f"wave {'0' if w == 0 else '7'} item {it}: " + " ".join(f"{n}={v}" for n, v in zip(names, d + [nxt])))
names1 = ["q_do_lse_reads", "s_dp_products", "delta", "dq_products"]
for w in range(2):
    for it in range(4):
        t = [buf[64 + w * 32 + it * 8 + k] for k in range(5)]
        t2 = buf[w * 32 + it * 8 + 2]  # after barrier (a)
        t7 = buf[64 + w * 32 + it * 8 + 7]  # after the DMA issue
        print(f"wave {'0' if w == 0 else '7'} item {it} first strip: dma_issue={t7 - t2} to_strip={t[0] - t7} " +
              " ".join(f"{n}={t[k + 1] - t[k]}" for k, n in enumerate(names1)))
