#!/usr/bin/env python3
"""Debug helper: per (image, head, 16-query strip) relative error of the LDS-resident attention forward
against an fp32 torch reference.   python tools/dbg_attn80.py B N H hd"""
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import ops  # noqa: E402

B, N, H, hd = (int(v) for v in sys.argv[1:5])
D = H * hd
torch.manual_seed(0)
qkv = (torch.randn(B * N, 3 * D, device="cuda") * 1.5).bfloat16()
o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B, H, N, device="cuda")
ops.attention_fwd(qkv, o, lse, B, N, H, hd, 1.0 / math.sqrt(hd), path=1)
x = qkv.float().view(B, N, 3, H, hd)
q, k, v = (x[:, :, z].permute(0, 2, 1, 3) for z in range(3))
s = q @ k.transpose(-1, -2) / math.sqrt(hd)
ref = (s.softmax(-1) @ v).permute(0, 2, 1, 3)  # B N H hd
got = o.float().view(B, N, H, hd)
lref = torch.logsumexp(s, -1)
for b in range(B):
    for h in range(H):
        errs = []
        for t in range((N + 15) // 16):
            a, r = got[b, t * 16:(t + 1) * 16, h], ref[b, t * 16:(t + 1) * 16, h]
            errs.append(float((a - r).norm() / r.norm()))
        le = float((lse[b, h] - lref[b, h]).abs().max())
        print(f"b{b} h{h} lse-err {le:.2e} strip errs " + " ".join(f"{e:.3f}" for e in errs))
# per-dim error of the first strip of image 0 head 0
a, r = got[0, :, 0], ref[0, :, 0]
print("per-dim err (all rows, b0 h0):", " ".join(f"{float((a[:, d] - r[:, d]).norm() / r[:, d].norm()):.2f}"
                                               for d in range(hd)))
