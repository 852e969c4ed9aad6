#!/usr/bin/env python3
"""Phase durations of the two-stage attention backward (attention.hip attn_bwd_kernel) from the diagnostic
library's stamps (make DIAG=1; VITMI_LIB=vit-of-pytorch_amd/vitmi/diag/libvit_hip.so):
    python tools/attn2_stamps.py B N H hd [bias]
s_memtime ticks (100 MHz) for workgroups 0 and gridDim-1, their first and last waves."""
import ctypes
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vit-of-pytorch_amd"))
import torch  # noqa: E402

from vitmi import _lib, ops  # noqa: E402

B, N, H, hd = (int(v) for v in sys.argv[1:5])
bias = len(sys.argv) > 5 and sys.argv[5] == "bias"
D = H * hd
sc = 1.0 / math.sqrt(hd)
qkv = (torch.randn(B * N, 3 * D, device="cuda") * 1.5).bfloat16()
o = torch.empty(B * N, D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B, H, N, device="cuda")
do = torch.randn(B * N, D, device="cuda").bfloat16()
dqkv = torch.empty_like(qkv)
bp = torch.empty(B * ops.attention_bias_rows(N, hd), 3 * D, device="cuda") if bias else None
ops.attention_fwd(qkv, o, lse, B, N, H, hd, sc)
for _ in range(3):
    ops.attention_bwd(qkv, o, do, lse, dqkv, B, N, H, hd, sc, bias_partial=bp)
torch.cuda.synchronize()
lib = _lib.load()
buf = (ctypes.c_ulonglong * 32)()
lib.vit_attn2_stamps(buf)
names = ["kv_images", "stage1", "qdo_images", "stage2", "bias+end"]
t00 = buf[0]
for blk in range(2):
    for w in range(2):
        t = [buf[blk * 16 + w * 8 + k] for k in range(6)]
        d = [t[k + 1] - t[k] for k in range(5)]
        print(f"{'first' if blk == 0 else 'last '} wg, {'first' if w == 0 else 'last '} wave: start +{t[0] - t00:6d} "
              + " ".join(f"{n}={v:5d}" for n, v in zip(names, d)) + f"  total={t[5] - t[0]}")
