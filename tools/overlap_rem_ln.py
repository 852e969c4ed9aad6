"""Does the wave-split remainder of a GEMM overlap the row-local LayerNorm that follows it? (diagnostic)

ViT-B/16 bs 256 (T = 50 432 rows): the out-projection / fc2 forwards and the fc1 / q|k|v data gradients split into
whole-wave rows (256 x 256 tiles) and a remainder (128 x 128 tiles); the next op is a LayerNorm, row-local. Serial:
GEMM, then LayerNorm. Overlapped: whole-wave rows; then the remainder on a side stream beside the LayerNorm of the
whole-wave rows on the compute stream; join; LayerNorm of the remainder rows. Prints us per pair.

  python3 tools/overlap_rem_ln.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "vit-of-pytorch_amd"))
from vitmi import ops  # noqa: E402
from vitmi._lib import (EPI_BF16, EPI_BIAS_RESID_F32, K_CONTIG, MN_CONTIG)  # noqa: E402

dev = torch.device("cuda")
T, D, M = 50432, 768, 3072
bf = torch.bfloat16
r = lambda *s, dt=bf: (torch.randn(*s, device=dev) * 0.05).to(dt)


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


main = torch.cuda.current_stream()
side = torch.cuda.Stream()
evs = [torch.cuda.Event() for _ in range(2)]
gamma, beta = torch.ones(D, device=dev), torch.zeros(D, device=dev)
mean, rstd = torch.empty(T, device=dev), torch.empty(T, device=dev)
nb = ops.layernorm_bwd_blocks(T)
part = torch.empty(2 * nb + 8, 3 * D, device=dev)


def case(name, A, B, C, K, kw, ln):
    ms = ops.gemm_split_rows(A, B, C, T, D, K, **kw)

    def serial():
        ops.gemm(A, B, C, T, D, K, **kw)
        ln(0, T, 0)

    def overlap():
        ops.gemm(A, B, C, T, D, K, part=1, **kw)
        evs[0].record(main)
        side.wait_event(evs[0])
        with torch.cuda.stream(side):
            ops.gemm(A, B, C, T, D, K, part=2, **kw)
        evs[1].record(side)
        ln(0, ms, 0)
        main.wait_event(evs[1])
        ln(ms, T - ms, ops.layernorm_bwd_blocks(ms))

    def gemm_only():
        ops.gemm(A, B, C, T, D, K, **kw)

    def ln_only():
        ln(0, T, 0)

    def events_only():  # the serial pair plus the event traffic of the overlapped one, all on the compute stream
        ops.gemm(A, B, C, T, D, K, part=1, **kw)
        evs[0].record(main)
        side.wait_event(evs[0])
        evs[1].record(side)
        ops.gemm(A, B, C, T, D, K, part=2, **kw)
        ln(0, ms, 0)
        main.wait_event(evs[1])
        ln(ms, T - ms, ops.layernorm_bwd_blocks(ms))

    serial()
    torch.cuda.synchronize()
    ref = C.clone()
    C.zero_()
    overlap()
    torch.cuda.synchronize()
    assert torch.equal(C, ref), f"{name}: parts 1 + 2 differ from the whole GEMM"
    if os.environ.get("OVERLAP_TRACE"):  # a few overlapped pairs only, for a kernel-trace timeline
        for _ in range(3):
            overlap()
        torch.cuda.synchronize()
        return
    res = {k: timeit(f) for k, f in (("gemm", gemm_only), ("ln", ln_only), ("serial", serial),
                                       ("split_serial_events", events_only), ("overlap", overlap))}
    print(f"{name:28s} split_rows={ms}: " + "  ".join(f"{k} {v:7.1f}" for k, v in res.items()), flush=True)


# forward: out-projection (+ bias + residual, f32) -> LayerNorm 2
o, wo = r(T, D), r(D, D)
hres, hm = r(T, D, dt=torch.float32), torch.empty(T, D, device=dev)
bias = torch.zeros(D, device=dev)
y = torch.empty(T, D, device=dev, dtype=bf)
kw = dict(a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=D, ldb=D, ldc=D, epilogue=EPI_BIAS_RESID_F32, bias=bias, aux=hres,
          ldaux=D)
lnf = lambda r0, n, _p: ops.layernorm_fwd(hm[r0:], D, gamma, beta, y[r0:], D, mean[r0:], rstd[r0:], n, D)
case("out-proj fwd -> LN2 fwd", o, wo, hm, D, kw, lnf)
# forward: fc2 (+ bias + residual) -> next layer's LayerNorm 1
g, w2 = r(T, M), r(D, M)
kw2 = dict(a_layout=K_CONTIG, b_layout=K_CONTIG, lda=M, ldb=M, ldc=D, epilogue=EPI_BIAS_RESID_F32, bias=bias, aux=hres,
           ldaux=D)
case("fc2 fwd -> LN1 fwd", g, w2, hm, M, kw2, lnf)
# backward: fc1 data gradient (bf16) -> LayerNorm 2 backward (dx f32 += residual, bf16 copy, block partials)
dg, w1 = r(T, M), r(M, D)
dyln = torch.empty(T, D, device=dev, dtype=bf)
x = r(T, D, dt=torch.float32)
ops.layernorm_fwd(x, D, gamma, beta, y, D, mean, rstd, T, D)
dh, dhb = r(T, D, dt=torch.float32), torch.empty(T, D, device=dev, dtype=bf)
kw3 = dict(a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=M, ldb=D, ldc=D, epilogue=EPI_BF16)
lnb = lambda r0, n, p0: ops.layernorm_bwd(dyln[r0:], D, x[r0:], D, mean[r0:], rstd[r0:], gamma, dh[r0:], D, part[p0:],
                                          n, D, dres=dh[r0:], lddres=D, dx_bf16=dhb[r0:], lddxb=D)
case("fc1 dgrad -> LN2 bwd", dg, w1, dyln, M, kw3, lnb)
# backward: q|k|v data gradient -> LayerNorm 1 backward
dqkv, wqkv = r(T, 3 * D), r(D, 3 * D)
kw4 = dict(a_layout=K_CONTIG, b_layout=K_CONTIG, lda=3 * D, ldb=3 * D, ldc=D, epilogue=EPI_BF16)
case("qkv dgrad -> LN1 bwd", dqkv, wqkv, dyln, 3 * D, kw4, lnb)
