"""Per-kernel numerics of libvit_hip.so against plain PyTorch fp32 references (GPU only)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from vitmi import ops
from vitmi._lib import (EPI_BF16, EPI_BIAS_BF16, EPI_BIAS_GELU, EPI_BIAS_GELU_DGELU, EPI_BIAS_RESID_F32, EPI_F32,
                        EPI_GELU_BWD, EPI_MUL_BF16, EPI_PATCH, EPI_SPLITK, K_CONTIG, MN_CONTIG)

DEV = "cuda"


def rel(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _mats(M, N, K, al, bl, ints=False, gen=None):
    if ints:
        A = torch.randint(-4, 5, (M, K), device=DEV).float()
        B = torch.randint(-4, 5, (K, N), device=DEV).float()
    else:
        A = torch.randn(M, K, device=DEV)
        B = torch.randn(K, N, device=DEV)
    A = A.bfloat16()
    B = B.bfloat16()
    # MN-contiguous operands get their rows padded to a multiple of 8 elements (16 B)
    pad = lambda n: (n + 7) // 8 * 8
    if al == K_CONTIG:
        Am, lda = A.contiguous(), K                                  # [M][K]
    else:
        lda = pad(M)
        Am = torch.zeros(K, lda, device=DEV, dtype=torch.bfloat16)   # [K][lda]
        Am[:, :M] = A.t()
    if bl == K_CONTIG:
        Bm, ldb = B.t().contiguous(), K                              # [N][K]
    else:
        ldb = pad(N)
        Bm = torch.zeros(K, ldb, device=DEV, dtype=torch.bfloat16)   # [K][ldb]
        Bm[:, :N] = B
    return A, B, Am, Bm, lda, ldb


LAYOUTS = [(K_CONTIG, K_CONTIG), (K_CONTIG, MN_CONTIG), (MN_CONTIG, MN_CONTIG), (MN_CONTIG, K_CONTIG)]


@pytest.mark.parametrize("al,bl", LAYOUTS)
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 384, 192), (200, 136, 128), (37, 300, 64)])
def test_gemm_exact_integers(al, bl, M, N, K):
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, al, bl, ints=True)
    C = torch.full((M, N), float("nan"), device=DEV)
    ops.gemm(Am, Bm, C, M, N, K, a_layout=al, b_layout=bl, lda=lda, ldb=ldb, ldc=N, epilogue=EPI_F32)
    ref = A.float() @ B.float()
    assert torch.equal(C, ref)


@pytest.mark.parametrize("al,bl", LAYOUTS)
@pytest.mark.parametrize("tile,M,N,K", [(1, 600, 520, 128), (2, 600, 300, 192), (0, 300, 200, 128), (1, 2100, 1600, 64),
                                        (2, 2100, 768, 128), (6, 600, 520, 128), (6, 2100, 768, 64),
                                        (6, 700, 300, 320), (5, 600, 520, 192), (7, 600, 520, 192),
                                        (8, 2100, 768, 320), (7, 300, 256, 64), (9, 600, 520, 192),
                                        (9, 2100, 768, 320), (9, 300, 256, 64), (9, 513, 300, 128)])
def test_gemm_tiles_exact(al, bl, tile, M, N, K):
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, al, bl, ints=True)
    C = torch.full((M, N), float("nan"), device=DEV)
    ops.gemm(Am, Bm, C, M, N, K, a_layout=al, b_layout=bl, lda=lda, ldb=ldb, ldc=N, epilogue=EPI_F32, tile=tile)
    assert torch.equal(C, A.float() @ B.float())


@pytest.mark.parametrize("tile", [0, 3, 6, 9])
def test_gemm_col_partial(tile):
    M, N, K = 1000, 384, 256
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, K_CONTIG, MN_CONTIG)
    U = torch.randn(M, N, device=DEV).bfloat16()
    C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    kw = dict(a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=lda, ldb=ldb, ldc=N, epilogue=EPI_GELU_BWD, aux=U, ldaux=N,
              tile=tile)
    rows = ops.gemm_tile_rows(Am, Bm, C, M, N, K, **kw)
    part = torch.full(((M + rows - 1) // rows, N), float("nan"), device=DEV)
    ops.gemm(Am, Bm, C, M, N, K, col_partial=part, **kw)
    u = U.float().requires_grad_(True)
    gref, = torch.autograd.grad(torch.nn.functional.gelu(u), u, A.float() @ B.float())
    assert rel(part.sum(0), gref.sum(0)) < 1e-3
    assert rel(C.float(), gref) < 5e-3


def test_gemm_col_partial_wave_split():
    """The production dispatch of a col_partial GEMM whose last wave of 256 x 256 tiles would run nearly empty
    (20 x 13 = 260 tiles on 256 CUs): the whole-wave rows on the ping-pong kernel, the remaining 256 rows on two
    128-row tiles, their column partials continuing after the main ones (vit_gemm_partial_rows rows); the
    fc2-dgrad x GELU' shape family (EPI_MUL_BF16, both operands K-contiguous)."""
    from vitmi._lib import EPI_MUL_BF16
    M, N, K = 5120, 3328, 128
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, K_CONTIG, K_CONTIG)
    U = torch.randn(M, N, device=DEV).bfloat16()
    C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    kw = dict(a_layout=K_CONTIG, b_layout=K_CONTIG, lda=lda, ldb=ldb, ldc=N, epilogue=EPI_MUL_BF16, aux=U, ldaux=N)
    rows = ops.gemm_partial_rows(Am, Bm, C, M, N, K, **kw)
    assert rows == 19 + 2  # 19 whole-wave 256-row tiles, then 2 remainder 128-row tiles
    part = torch.full((rows + 1, N), float("nan"), device=DEV)
    ops.gemm(Am, Bm, C, M, N, K, col_partial=part, **kw)
    assert torch.isnan(part[rows]).all()  # nothing past the reported rows
    ref = (A.float() @ B.float()) * U.float()
    assert rel(C.float(), ref) < 5e-3
    assert rel(part[:rows].sum(0), ref.sum(0)) < 1e-4  # the partials sum the f32 values before bf16 rounding
    assert rel(part[19:rows].sum(0), ref[19 * 256:].sum(0)) < 1e-4


def test_gemm_parts_equal_whole():
    """vit_gemm_bf16_part: the whole-wave rows (part 1) and the wave-split remainder (part 2), on two streams,
    write exactly what one vit_gemm_bf16 call writes (bias + f32 residual epilogue, the out-projection shape
    family); a GEMM that does not split runs whole as part 1 and not at all as part 2."""
    M, N, K = 5120, 3328, 128
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, K_CONTIG, K_CONTIG)
    bias, res = torch.randn(N, device=DEV), torch.randn(M, N, device=DEV)
    kw = dict(a_layout=K_CONTIG, b_layout=K_CONTIG, lda=lda, ldb=ldb, ldc=N, epilogue=EPI_BIAS_RESID_F32, bias=bias,
              aux=res, ldaux=N)
    whole, parts = torch.empty(M, N, device=DEV), torch.full((M, N), float("nan"), device=DEV)
    assert ops.gemm_split_rows(Am, Bm, whole, M, N, K, **kw) == 19 * 256
    ops.gemm(Am, Bm, whole, M, N, K, **kw)
    ops.gemm(Am, Bm, parts, M, N, K, part=1, **kw)
    assert torch.isnan(parts[19 * 256:]).all() and not torch.isnan(parts[:19 * 256]).any()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ops.gemm(Am, Bm, parts, M, N, K, part=2, **kw)
    torch.cuda.current_stream().wait_stream(side)
    assert torch.equal(parts, whole)
    assert rel(whole, A.float() @ B.float() + bias + res) < 5e-3
    small = torch.full((256, N), float("nan"), device=DEV)
    assert ops.gemm_split_rows(Am, Bm, small, 256, N, K, **kw) == 0
    ops.gemm(Am, Bm, small, 256, N, K, part=2, **kw)
    assert torch.isnan(small).all()
    ops.gemm(Am, Bm, small, 256, N, K, part=1, **kw)
    assert torch.equal(small, whole[:256])


def test_gemm_splitk_group_equals_members():
    """vit_gemm_splitk_group: an out-projection-like member (batch 1) and a q|k|v-like one (batch 3, B columns
    strided) in one launch write bit-identical f32 slabs to their own vit_gemm_bf16 calls at the same split, and the
    slabs sum to the f32 products; a member that breaks the contract (K-contiguous A) is refused."""
    from vitmi._lib import EPI_SPLITK, VitHipError
    g = torch.Generator(device="cpu").manual_seed(7)
    K, D, S = 1024, 256, 3
    A1 = torch.randn(K, D, generator=g).bfloat16().to(DEV)       # [tokens][M]: M/N-contiguous
    B1 = torch.randn(K, D, generator=g).bfloat16().to(DEV)
    A2 = torch.randn(K, D, generator=g).bfloat16().to(DEV)
    B2 = torch.randn(K, 3 * D, generator=g).bfloat16().to(DEV)   # three [tokens][D] column blocks
    kw1 = dict(a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=D, ldb=D, ldc=D, epilogue=EPI_SPLITK, split_k=S)
    kw2 = dict(a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=D, ldb=3 * D, ldc=D, epilogue=EPI_SPLITK, split_k=S,
               batch=3, b_bs=D)
    w1, w2 = torch.empty(S, D, D, device=DEV), torch.empty(3, S, D, D, device=DEV)
    ops.gemm(A1, B1, w1, D, D, K, **kw1)
    ops.gemm(A2, B2, w2, D, D, K, **kw2)
    g1, g2 = torch.full_like(w1, float("nan")), torch.full_like(w2, float("nan"))
    ops.gemm_splitk_group([(A1, B1, g1, D, D, K, kw1), (A2, B2, g2, D, D, K, kw2)])
    assert torch.equal(g1, w1) and torch.equal(g2, w2)
    ref1 = A1.float().t() @ B1.float()
    assert rel(g1.sum(0), ref1) < 1e-5
    for z in range(3):
        assert rel(g2[z].sum(0), A2.float().t() @ B2[:, z * D:(z + 1) * D].float()) < 1e-5
    bad = dict(kw1, a_layout=K_CONTIG, lda=K)
    with pytest.raises(VitHipError, match="split-K weight gradient"):
        ops.gemm_splitk_group([(A1.t().contiguous(), B1, g1, D, D, K, bad)])


def test_gemm_splitk_group_small_members():
    """the Res-ViT router's weight gradients as one group: members narrower than a tile (M = 2: the 2-logit layer;
    N = 512) run as partial 256 x 256 tiles and match their own calls bit for bit"""
    from vitmi._lib import EPI_SPLITK
    g = torch.Generator(device="cpu").manual_seed(11)
    K, S = 640, 2
    shapes = [(2, 256, 64, 256), (256, 512, 256, 512), (512, 768, 512, 768)]  # (M, N, lda, ldb)
    members, refs = [], []
    for M, N, lda, ldb in shapes:
        A = torch.randn(K, lda, generator=g).bfloat16().to(DEV)
        B = torch.randn(K, ldb, generator=g).bfloat16().to(DEV)
        kw = dict(a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=lda, ldb=ldb, ldc=N, epilogue=EPI_SPLITK, split_k=S)
        w = torch.empty(S, M, N, device=DEV)
        ops.gemm(A, B, w, M, N, K, **kw)
        refs.append((w, A[:, :M].float().t() @ B[:, :N].float()))
        members.append((A, B, torch.full_like(w, float("nan")), M, N, K, kw))
    ops.gemm_splitk_group(members)
    for (_, _, out, *_), (w, ref) in zip(members, refs):
        assert torch.equal(out, w)
        assert rel(out.sum(0), ref) < 1e-5


def test_splitk_reduce_group_equals_single_reductions():
    """vit_splitk_reduce_group: jobs of different shapes, splits, batches, strides and accumulate flags in one launch
    write what their own vit_splitk_reduce calls write, bit for bit (a scalar-form job falls back per job)"""
    g = torch.Generator(device="cpu").manual_seed(3)
    specs = [(1, 7, 768, 256, 256, 0, False), (3, 5, 64, 96, 104, 64 * 104, True), (1, 3, 10, 6, 6, 0, False)]
    jobs, refs = [], []
    for batch, split, M, N, ldo, obs, acc in specs:
        ws = torch.randn(batch * split * M * N, generator=g).to(DEV)
        init = torch.randn(max(1, batch) * max(M * ldo, obs or 0) + 8, generator=g).to(DEV)
        a, b = init.clone(), init.clone()
        ops.splitk_reduce(ws, batch, split, M, N, a, ldo, obs, acc)
        refs.append(a)
        jobs.append((ws, batch, split, M, N, b, ldo, obs, acc))
    ops.splitk_reduce_group(jobs)
    for (_, _, _, _, _, b, _, _, _), a in zip(jobs, refs):
        assert torch.equal(a, b)
    ops.splitk_reduce_group(jobs[:2])  # all vector form: one launch
    for (_, _, _, _, _, b, _, _, acc), a in zip(jobs[:2], refs[:2]):
        assert acc or torch.equal(a, b)


def test_cast_pad_batch_matches_single_casts():
    """vit_cast_pad_batch: jobs of different shapes (a strided column block, row and column padding, an empty
    source) in one launch equal their bf16 casts with zeros in the padding, bit for bit"""
    g = torch.Generator(device="cpu").manual_seed(13)
    src = [torch.randn(5, 37, generator=g).to(DEV), torch.randn(64, 8, generator=g).to(DEV)[:, :6],
           torch.randn(3, 100, generator=g).to(DEV)]
    outs = [torch.full((8, 64), float("nan"), device=DEV).bfloat16(), torch.full((64, 16), float("nan"),
                                                                                  device=DEV).bfloat16(),
            torch.full((4, 128), float("nan"), device=DEV).bfloat16()]
    jobs = [(src[0], 5, 37, 37, outs[0], 64, 8, 64), (src[1], 64, 6, 8, outs[1], 16, 64, 8),
            (src[2], 0, 0, 100, outs[2], 128, 4, 100)]
    ops.cast_pad_batch(jobs)
    ref0 = torch.zeros(8, 64, device=DEV).bfloat16()
    ref0[:5, :37] = src[0].bfloat16()
    assert torch.equal(outs[0], ref0)
    assert torch.equal(outs[1][:, :6], src[1].bfloat16()) and (outs[1][:, 6:8].float() == 0).all()
    assert torch.isnan(outs[1][:, 8:].float()).all()  # past cols_pad: untouched
    assert (outs[2][:, :100].float() == 0).all() and torch.isnan(outs[2][:, 100:].float()).all()


def test_cast_rows_masked():
    """vit_cast_rows_masked: the bf16 rounding of the masked rows, zeros for the others (bit-identical to a cast then
    vit_rows_select), the padding columns of the output untouched; no mask: every row"""
    g = torch.Generator(device="cpu").manual_seed(8)
    rows, cols, ldi, ldo = 301, 96, 100, 104
    x = torch.randn(rows, ldi, generator=g).to(DEV)
    mask = (torch.rand(rows, generator=g) < 0.6).to(DEV)
    out = torch.full((rows, ldo), float("nan"), device=DEV).bfloat16()
    ops.cast_rows_masked(x, ldi, rows, cols, mask, out, ldo)
    ref = torch.where(mask[:, None], x[:, :cols], torch.zeros_like(x[:, :cols])).bfloat16()
    assert torch.equal(out[:, :cols], ref)
    assert torch.isnan(out[:, cols:].float()).all()
    ops.cast_rows_masked(x, ldi, rows, cols, None, out, ldo)
    assert torch.equal(out[:, :cols], x[:, :cols].bfloat16())


@pytest.mark.parametrize("C", [200, 199])
def test_segment_colsum_bcast(C):
    """vit_segment_colsum_bcast (the router forward's token mean, broadcast as bf16 into the global half of out_conv's
    operand): the means as segment_colsum's, bit for bit, and each image's rows of the right half equal to their bf16
    rounding; the left half (the input) and the padding rows untouched"""
    g = torch.Generator(device="cpu").manual_seed(6)
    Bn, N, reserve, ld = 3, 50, 1, 2 * 256
    buf = torch.randn(Bn * N + 6, ld, generator=g).bfloat16().to(DEV)
    before = buf.clone()
    ref = torch.empty(Bn, C, device=DEV)
    ops.segment_colsum(buf, ld, Bn, N - reserve, C, ref, C, seg_stride=N, row0=reserve, scale=1.0 / (N - reserve))
    out = torch.full((Bn, C), float("nan"), device=DEV)
    ops.segment_colsum_bcast(buf, ld, Bn, N - reserve, C, out, C, buf[:, 256:], ld, N, seg_stride=N, row0=reserve,
                             scale=1.0 / (N - reserve))
    assert torch.equal(out, ref)
    got = buf[:Bn * N, 256:256 + C].view(Bn, N, C)
    assert torch.equal(got, ref.bfloat16()[:, None, :].expand(Bn, N, C))
    assert torch.equal(buf[:, :256], before[:, :256])
    assert torch.equal(buf[Bn * N:], before[Bn * N:])
    assert torch.equal(buf[:, 256 + C:], before[:, 256 + C:])


def test_segment_colsum_and_router_dx_gate():
    """the Res-ViT router backward helpers against torch: per-image token sums (bf16 and f32 inputs), and
    bf16((dx + [t % N >= reserve] s g[t // N]) * gp) with zero padding and per-row-block column partials of the
    rounded values"""
    g = torch.Generator(device="cpu").manual_seed(5)
    Bn, N, C, ld = 3, 50, 200, 264
    x = torch.randn(Bn * N, ld, generator=g).to(DEV)
    for inp in (x, x.bfloat16()):
        out = torch.full((Bn, C + 8), float("nan"), device=DEV)
        ops.segment_colsum(inp, ld, Bn, N, C, out, C + 8)
        ref = inp[:, :C].float().view(Bn, N, C).sum(1)
        assert torch.allclose(out[:, :C], ref, rtol=1e-5, atol=1e-4)
        assert torch.isnan(out[:, C:]).all()
        # the router forward's mean over the non-reserved tokens (odd column count: the last pair half empty)
        mean = torch.empty(Bn, C - 1, device=DEV)
        ops.segment_colsum(inp, ld, Bn, N - 2, C - 1, mean, C - 1, seg_stride=N, row0=2, scale=1.0 / (N - 2))
        assert torch.allclose(mean, inp[:, :C - 1].float().view(Bn, N, C - 1)[:, 2:].mean(1), rtol=1e-5, atol=1e-5)
    T, reserve, scale = Bn * N, 2, 1.0 / 48
    rows_pad, cols_pad = 192, 256
    dx = torch.randn(T, C, generator=g).to(DEV)
    gs = torch.randn(Bn, C, generator=g).to(DEV)
    gp = torch.randn(rows_pad, cols_pad, generator=g).bfloat16().to(DEV)
    out = torch.full((rows_pad, cols_pad), float("nan"), device=DEV).bfloat16()
    nb = ops.router_dx_gate_partial_rows(rows_pad)
    part = torch.full((nb, C), float("nan"), device=DEV)
    ops.router_dx_gate(dx, C, gs, C, scale, gp, cols_pad, T, N, reserve, C, out, cols_pad, part, C)
    keep = (torch.arange(T, device=DEV) % N >= reserve).float()[:, None]
    ref = ((dx + keep * scale * gs.repeat_interleave(N, 0)) * gp[:T, :C].float()).bfloat16()
    assert torch.equal(out[:T, :C], ref)
    assert (out[T:].float() == 0).all() and (out[:, C:].float() == 0).all()
    full = torch.zeros(rows_pad, C, device=DEV)
    full[:T] = ref.float()
    rb = -(-rows_pad // nb)  # rows per partial block
    assert rb * nb == rows_pad
    assert torch.allclose(part, full.view(nb, rb, C).sum(1), rtol=1e-5, atol=1e-4)
    # the branch-free column-pair kernel (even width, no padding columns): the same values
    out2 = torch.full((rows_pad, C), float("nan"), device=DEV).bfloat16()
    gp2 = gp[:, :C].contiguous()
    part2 = torch.full((nb, C), float("nan"), device=DEV)
    ops.router_dx_gate(dx, C, gs, C, scale, gp2, C, T, N, reserve, C, out2, C, part2, C)
    assert torch.equal(out2[:T], ref) and (out2[T:].float() == 0).all()
    assert torch.equal(part2, part)


@pytest.mark.parametrize("tile", [1, 2, 6, 9])
def test_gemm_tiles_epilogue_splitk(tile):
    M, N, K = 700, 520, 512
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, K_CONTIG, MN_CONTIG)
    ref = A.float() @ B.float()
    bias = torch.randn(N, device=DEV)
    C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    C2 = torch.empty_like(C)
    ops.gemm(Am, Bm, C, M, N, K, a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=lda, ldb=ldb, ldc=N,
             epilogue=EPI_BIAS_GELU, bias=bias, C2=C2, ldc2=N, tile=tile)
    assert rel(C.float(), ref + bias) < 5e-3
    assert rel(C2.float(), torch.nn.functional.gelu(ref + bias)) < 5e-3
    S = 3
    ws = torch.empty(S, M, N, device=DEV)
    ops.gemm(Am, Bm, ws, M, N, K, a_layout=K_CONTIG, b_layout=MN_CONTIG, lda=lda, ldb=ldb, ldc=N,
             epilogue=EPI_SPLITK, split_k=S, tile=tile)
    assert rel(ws.sum(0), ref) < 1e-5


@pytest.mark.parametrize("al,bl", LAYOUTS)
def test_gemm_random_f32(al, bl):
    M, N, K = 1000, 768, 768
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, al, bl)
    C = torch.empty(M, N, device=DEV)
    ops.gemm(Am, Bm, C, M, N, K, a_layout=al, b_layout=bl, lda=lda, ldb=ldb, ldc=N, epilogue=EPI_F32)
    assert rel(C, A.float() @ B.float()) < 1e-5


def test_gemm_epilogues():
    M, N, K = 300, 256, 128
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, K_CONTIG, K_CONTIG)
    ref = A.float() @ B.float()
    bias = torch.randn(N, device=DEV)
    kw = dict(a_layout=K_CONTIG, b_layout=K_CONTIG, lda=lda, ldb=ldb, ldc=N)
    C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.gemm(Am, Bm, C, M, N, K, epilogue=EPI_BF16, **kw)
    assert rel(C.float(), ref) < 5e-3
    ops.gemm(Am, Bm, C, M, N, K, epilogue=EPI_BIAS_BF16, bias=bias, **kw)
    assert rel(C.float(), ref + bias) < 5e-3
    C2 = torch.empty_like(C)
    ops.gemm(Am, Bm, C, M, N, K, epilogue=EPI_BIAS_GELU, bias=bias, C2=C2, ldc2=N, **kw)
    assert rel(C.float(), ref + bias) < 5e-3
    assert rel(C2.float(), torch.nn.functional.gelu(ref + bias)) < 5e-3
    R = torch.randn(M, N, device=DEV)
    Cf = R.clone()
    ops.gemm(Am, Bm, Cf, M, N, K, epilogue=EPI_BIAS_RESID_F32, bias=bias, aux=Cf, ldaux=N, **kw)
    assert rel(Cf, ref + bias + R) < 1e-5
    U = torch.randn(M, N, device=DEV).bfloat16()
    ops.gemm(Am, Bm, C, M, N, K, epilogue=EPI_GELU_BWD, aux=U, ldaux=N, **kw)
    u = U.float().requires_grad_(True)
    gref, = torch.autograd.grad(torch.nn.functional.gelu(u), u, ref)
    assert rel(C.float(), gref) < 5e-3


def test_gemm_patch_epilogue():
    tokens, D, Kp = 5, 128, 64
    M = 3 * tokens
    A = torch.randn(M, Kp, device=DEV).bfloat16()
    A[::tokens] = 0
    W = torch.randn(D, Kp, device=DEV).bfloat16()
    bias, pos, cls = torch.randn(D, device=DEV), torch.randn(tokens, D, device=DEV), torch.randn(D, device=DEV)
    C = torch.empty(M, D, device=DEV)
    ops.gemm(A, W, C, M, D, Kp, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=Kp, ldb=Kp, ldc=D, epilogue=EPI_PATCH,
             bias=bias, aux=pos, ldaux=D, aux2=cls, tokens=tokens)
    ref = A.float() @ W.float().t() + bias + pos.repeat(3, 1)
    ref[::tokens] = cls + pos[0]
    assert rel(C, ref) < 1e-5


def test_gemm_batched_splitk():
    M, N, K, Z, S = 256, 192, 1024, 3, 4
    A = torch.randn(Z, K, M, device=DEV).bfloat16()      # MN-contig A (wgrad style)
    B = torch.randn(Z, K, N, device=DEV).bfloat16()
    ws = torch.empty(Z, S, M, N, device=DEV)
    ops.gemm(A, B, ws, M, N, K, a_layout=MN_CONTIG, b_layout=MN_CONTIG, lda=M, ldb=N, ldc=N, epilogue=EPI_SPLITK,
             batch=Z, a_bs=K * M, b_bs=K * N, split_k=S)
    out = torch.empty(Z, M, N + 8, device=DEV)
    ops.splitk_reduce(ws, Z, S, M, N, out, N + 8, M * (N + 8))
    ref = torch.einsum("zkm,zkn->zmn", A.float(), B.float())
    assert rel(out[..., :N], ref) < 1e-5


@pytest.mark.parametrize("D", [64, 768, 1024, 1280])
def test_layernorm(D):
    rows = 333
    x = (torch.randn(rows, D, device=DEV) * 3 + 1).requires_grad_(True)
    g = torch.randn(D, device=DEV).requires_grad_(True)
    b = torch.randn(D, device=DEV).requires_grad_(True)
    y = torch.empty(rows, D, device=DEV, dtype=torch.bfloat16)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    ops.layernorm_fwd(x.detach(), D, g.detach(), b.detach(), y, D, mean, rstd, rows, D)
    ref = torch.nn.functional.layer_norm(x, (D,), g, b, 1e-5)
    assert rel(y.float(), ref.detach()) < 5e-3
    dy = torch.randn(rows, D, device=DEV).bfloat16()
    dres = torch.randn(rows, D, device=DEV)
    gx, gg, gb = torch.autograd.grad(ref, (x, g, b), dy.float())
    dx = torch.empty(rows, D, device=DEV)
    dxb = torch.empty(rows, D, device=DEV, dtype=torch.bfloat16)
    part = torch.empty(ops.layernorm_bwd_partial_rows(rows), 3 * D, device=DEV)
    dgb = torch.empty(2 * D, device=DEV)
    dsum = torch.empty(D, device=DEV)
    ops.layernorm_bwd(dy, D, x.detach(), D, mean, rstd, g.detach(), dx, D, part, rows, D, dres=dres, lddres=D,
                      dx_bf16=dxb, lddxb=D, dgamma_dbeta=dgb, dx_colsum=dsum)
    assert rel(dsum, (gx + dres).sum(0)) < 1e-4
    assert rel(dx, gx + dres) < 1e-4
    assert rel(dxb.float(), gx + dres) < 5e-3
    assert rel(dgb[:D], gg) < 1e-4
    assert rel(dgb[D:], gb) < 1e-4


def _attn_ref(qkv, B, N, H, hd):
    q, k, v = qkv.float().view(B, N, 3, H, hd).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
    p = torch.softmax(s, -1)
    o = (p @ v).permute(0, 2, 1, 3).reshape(B * N, H * hd)
    lse = torch.logsumexp(s, -1)
    return o, lse


ATTN_CASES = [(2, 2, 2, 64, 0),  # (config C1: 2 tokens)
              (2, 197, 12, 64, 0), (3, 17, 2, 32, 0), (2, 50, 4, 64, 0), (1, 5, 3, 64, 0), (2, 257, 2, 64, 0),
              (2, 257, 3, 80, 0), (1, 197, 2, 48, 0), (2, 33, 2, 96, 0),
              # K/V-tiled path (ops.ATTN_TILED): forced at ViT-224 sizes, and the 384-px sequences it exists for
              # (B/16, L/16 @384: 577 tokens; H/14 @384: 730 tokens, hd 80)
              (2, 197, 3, 64, 2), (2, 257, 2, 80, 2), (3, 17, 2, 32, 2), (1, 65, 2, 48, 2), (2, 33, 2, 96, 2),
              (2, 577, 3, 64, 0), (1, 730, 2, 80, 0), (1, 321, 2, 64, 0),
              # more (image, head) items than CUs: the persistent backward's workgroups walk several items
              # (its Q / dO slots double as bias scratch: tiny N exercises the padded slot size)
              (24, 197, 12, 64, 0), (23, 50, 12, 64, 0), (32, 2, 12, 64, 0), (30, 17, 12, 32, 0),
              # hd <= 32 past 256 tokens: more key pairs than the persistent backward's 8 waves (two-stage
              # kernel), and exactly 8 pairs (the persistent kernel with no idle wave)
              (1, 300, 2, 32, 0), (2, 256, 2, 32, 0),
              # 80-wide images (hd 80, ViT-H/14): odd tile counts (the 16-k P V / dQ / dK-dV steps), a single
              # tile, 10 key pairs on 8 waves (the second pair's K / V loaded in stage 2), many items
              (2, 5, 2, 80, 0), (3, 17, 2, 80, 0), (1, 241, 2, 80, 0), (1, 320, 2, 80, 0), (20, 50, 4, 80, 0)]


@pytest.mark.parametrize("B,N,H,hd,path", ATTN_CASES)
def test_attention(B, N, H, hd, path):
    D = H * hd
    qkv = (torch.randn(B * N, 3 * D, device=DEV) * 1.5).bfloat16().requires_grad_(True)

    o = torch.empty(B * N, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attention_fwd(qkv.detach(), o, lse, B, N, H, hd, 1.0 / math.sqrt(hd), path=path)
    qf = qkv.float().detach().requires_grad_(True)
    oref, lref = _attn_ref(qf, B, N, H, hd)
    assert rel(o.float(), oref.detach()) < 1e-2
    assert rel(lse, lref.detach()) < 1e-4
    dout = torch.randn(B * N, D, device=DEV).bfloat16()
    dqkv = torch.full((B * N, 3 * D), float("nan"), device=DEV, dtype=torch.bfloat16)
    rows = ops.attention_bias_rows(N, hd, path)
    bpart = torch.full((B * rows, 3 * D), float("nan"), device=DEV)
    ops.attention_bwd(qkv.detach(), o, dout, lse, dqkv, B, N, H, hd, 1.0 / math.sqrt(hd), bias_partial=bpart,
                      path=path)
    bpart = bpart.view(B, rows, 3 * D).sum(1)
    gref, = torch.autograd.grad(oref, qf, dout.float())
    gq, gk, gv = gref.view(B * N, 3, D).unbind(1)
    mq, mk, mv = dqkv.float().view(B * N, 3, D).unbind(1)
    # per-image column sums (bias-gradient partials), dq | dk | dv; dk sums are ~0 (shift invariance)
    bref = gref.view(B, N, 3 * D).sum(1)
    assert rel(bpart[:, :D], bref[:, :D]) < 2e-2 and rel(bpart[:, 2 * D:], bref[:, 2 * D:]) < 2e-2
    assert float((bpart[:, D:2 * D] - bref[:, D:2 * D]).abs().max()) < 1e-2 * float(bref.abs().max())
    assert rel(mq, gq) < 2e-2
    assert rel(mk, gk) < 2e-2
    assert rel(mv, gv) < 2e-2


@pytest.mark.parametrize("B,N,H,hd", [(2, 197, 12, 64), (24, 197, 12, 64), (3, 17, 2, 32), (1, 5, 3, 64), (2, 2, 2, 64),
                                       (23, 50, 12, 64), (2, 208, 3, 64), (1, 197, 2, 48), (7, 300, 4, 32),
                                       (2, 320, 2, 32), (40, 33, 8, 64)])
@pytest.mark.parametrize("q_rows", [None, 1])
def test_attention_persistent_forward_matches_oneshot(B, N, H, hd, q_rows):
    """the persistent forward (attention_fwd_pers.hip: K / V / Q of the next (image, head) by LDS-DMA while the
    current one runs) does attn_fwd2_kernel's arithmetic per strip: o and lse bit-identical to the
    one-workgroup-per-item kernel (ops.ATTN_ONESHOT) and run to run, also past 256 items (several per
    workgroup), for odd tile counts, hd 48 on 64-wide images, and the cls-only query pair (q_rows = 1). (Run
    to run is what caught the row max once read from MFMA registers by an inline-asm v_max3 too early:
    attn_common.h max3f.)"""
    D = H * hd
    g = torch.Generator(device=DEV).manual_seed(B * 1000 + N)
    qkv = (torch.randn(B * N, 3 * D, device=DEV, generator=g) * 1.5).bfloat16()
    outs = []
    for path in (ops.ATTN_AUTO, ops.ATTN_ONESHOT, ops.ATTN_AUTO):
        o = torch.full((B * N, D), float("nan"), device=DEV, dtype=torch.bfloat16)
        lse = torch.full((B, H, N), float("nan"), device=DEV)
        ops.attention_fwd(qkv, o, lse, B, N, H, hd, 1.0 / math.sqrt(hd), q_rows=q_rows, path=path)
        outs.append((o, lse))
    (o1, l1), (o0, l0), (o2, l2) = outs
    rows = N if q_rows is None else min(N, 32)
    for o, lse in ((o0, l0), (o2, l2)):
        assert torch.equal(o1.view(B, N, D)[:, :rows], o.view(B, N, D)[:, :rows])
        assert torch.equal(l1[:, :, :rows], lse[:, :, :rows])
    if q_rows is None:
        oref, lref = _attn_ref(qkv, B, N, H, hd)
        assert rel(o1.float(), oref) < 1e-2 and rel(l1, lref) < 1e-4


@pytest.mark.parametrize("N,B,hd", [(2, 2, 64), (17, 2, 64), (197, 2, 64), (2, 32, 64), (257, 2, 80), (5, 2, 80)])
def test_attention_backward_saturated_scores_finite(N, B, hd):
    """scores of |s| ~ 1e3 (the reference's std-1 init, config C1's 2 tokens): the LSE of a query can be far
    below 0, and the zero-padded keys of its last computed key tile must still get P = 0, not 2^-LSE = inf
    (inf * dP 0 = NaN); B = 32 x H = 12 puts several items on each workgroup of the persistent backward"""
    H = 2 if B == 2 else 12
    D = H * hd
    g = torch.Generator(device=DEV).manual_seed(1)
    qkv = (torch.randn(B * N, 3 * D, device=DEV, generator=g) * 8.0).bfloat16()
    qkv[:, :D] = -qkv[:, :D].abs()  # q < 0 < k elementwise: every score q.k is very negative
    qkv[:, D:2 * D] = qkv[:, D:2 * D].abs()
    o = torch.empty(B * N, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attention_fwd(qkv, o, lse, B, N, H, hd, 1.0 / math.sqrt(hd))
    assert float(lse.min()) < -100.0
    dout = torch.randn(B * N, D, device=DEV).bfloat16()
    dqkv = torch.zeros(B * N, 3 * D, device=DEV, dtype=torch.bfloat16)
    bp = torch.zeros(B * ops.attention_bias_rows(N, hd), 3 * D, device=DEV)
    ops.attention_bwd(qkv, o, dout, lse, dqkv, B, N, H, hd, 1.0 / math.sqrt(hd), bias_partial=bp)
    assert torch.isfinite(o.float()).all() and torch.isfinite(dqkv.float()).all() and torch.isfinite(bp).all()


@pytest.mark.parametrize("N,path,hd", [(197, 0, 64), (197, 2, 64), (257, 0, 64), (2, 0, 64), (17, 0, 64),
                                       (257, 0, 80), (17, 0, 80)])
def test_attention_backward_keeps_nan(N, path, hd):
    """a NaN in one query row (a diverging run) must surface as NaN in that row's dQ, not be clamped into a
    finite gradient by the padded-key exponent clamp"""
    B, H = 2, 2
    D = H * hd
    qkv = torch.randn(B * N, 3 * D, device=DEV).bfloat16()
    qkv[min(5, N - 1), 3] = float("nan")  # image 0, token 5 (or the last), head 0: q
    o = torch.empty(B * N, D, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attention_fwd(qkv, o, lse, B, N, H, hd, 1.0 / math.sqrt(hd), path=path)
    dout = torch.randn(B * N, D, device=DEV).bfloat16()
    dqkv = torch.zeros(B * N, 3 * D, device=DEV, dtype=torch.bfloat16)
    ops.attention_bwd(qkv, o, dout, lse, dqkv, B, N, H, hd, 1.0 / math.sqrt(hd), path=path)
    dq = dqkv.float()[:, :D]
    assert torch.isnan(dq[min(5, N - 1), :hd]).any()
    # other images and the other head are untouched by the NaN
    assert torch.isfinite(dq[N:]).all() and torch.isfinite(dq[:, hd:]).all()


@pytest.mark.parametrize("B,img,P,D", [(2, 32, 8, 64), (3, 224, 16, 768), (2, 224, 14, 1280), (2, 64, 32, 1024)])
def test_im2col_and_embed_grad(B, img, P, D):
    """vector paths (P % 8 == 0, D % 4 == 0) and the scalar fallback (P = 14)"""
    g = img // P
    N = g * g + 1
    K = 3 * P * P
    x = torch.randn(B, 3, img, img, device=DEV)
    out = torch.empty(B * N, K, device=DEV, dtype=torch.bfloat16)
    ops.im2col(x, out, B, img, P, K)
    cols = x.unfold(2, P, P).unfold(3, P, P)  # B,3,g,g,P,P
    cols = cols.permute(0, 2, 3, 1, 4, 5).reshape(B, g * g, K)
    ref = torch.zeros(B, N, K, device=DEV)
    ref[:, 1:] = cols
    assert torch.equal(out.float(), ref.reshape(B * N, K).bfloat16().float())
    dh0 = torch.randn(B * N, D, device=DEV)
    dpos = torch.empty(N, D, device=DEV)
    dcls = torch.empty(D, device=DEV)
    dcb = torch.empty(D, device=DEV)
    ops.embed_grad(dh0, B, N, D, dpos, dcls, dcb)
    r = dh0.view(B, N, D).sum(0)
    assert rel(dpos, r) < 1e-6
    assert rel(dcls, r[0]) < 1e-6
    assert rel(dcb, r[1:].sum(0)) < 1e-6


def test_colsum_ce_gemm_f32_sgd():
    x = torch.randn(5000, 300, device=DEV)
    part = torch.empty(ops.colsum_partial_rows(5000), 300, device=DEV)
    out = torch.empty(300, device=DEV)
    ops.colsum(x, 5000, 300, 300, part, out)
    assert rel(out, x.sum(0)) < 1e-5
    xb = x.bfloat16()
    ops.colsum(xb, 5000, 300, 300, part, out)
    assert rel(out, xb.float().sum(0)) < 1e-5
    for rows, cols in ((50432, 768), (333, 3072), (7, 64)):   # vector path (cols % 8 == 0)
        xv = torch.randn(rows, cols + 16, device=DEV)
        pv = torch.empty(ops.colsum_partial_rows(rows), cols, device=DEV)
        ov = torch.full((cols,), 1.0, device=DEV)
        ops.colsum(xv, rows, cols, cols + 16, pv, ov, accumulate=True)
        assert rel(ov, 1.0 + xv[:, :cols].sum(0)) < 1e-5
        ops.colsum(xv.bfloat16(), rows, cols, cols + 16, pv, ov)
        assert rel(ov, xv[:, :cols].bfloat16().float().sum(0)) < 1e-5

    logits = torch.randn(64, 1000, device=DEV) * 3
    y = torch.randint(0, 1000, (64,), device=DEV)
    dl = torch.empty_like(logits)
    st = torch.empty(64, 3, device=DEV)
    ops.cross_entropy(logits, y, dl, 1.0 / 64, st)
    lr = logits.clone().requires_grad_(True)
    loss = torch.nn.functional.cross_entropy(lr, y)
    loss.backward()
    assert abs(float(st[:, 0].mean()) - float(loss.detach())) < 1e-5
    assert rel(dl, lr.grad) < 1e-5
    top5 = logits.topk(5, 1).indices
    assert float(st[:, 1].sum()) == float((top5[:, 0] == y).sum())
    assert float(st[:, 2].sum()) == float((top5 == y[:, None]).any(1).sum())

    A = torch.randn(70, 33, device=DEV)
    Bm = torch.randn(50, 33, device=DEV)
    bias = torch.randn(50, device=DEV)
    C = torch.empty(70, 50, device=DEV)
    ops.gemm_f32(70, 50, 33, A, 33, False, Bm, 33, True, C, 50, bias)
    assert rel(C, A @ Bm.t() + bias) < 1e-5
    C2 = torch.empty(33, 50, device=DEV)
    ops.gemm_f32(33, 50, 70, A, 33, True, C, 50, False, C2, 50)
    assert rel(C2, A.t() @ C) < 1e-5

    n = 1003
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    buf = torch.zeros(n, device=DEV)
    pb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    p0 = p.clone()
    ops.sgd_step(p, g, buf, pb, n, 0.1, 0.9, 1e-2, True)
    d = g + 1e-2 * p0
    assert rel(p, p0 - 0.1 * d) < 1e-6 and rel(buf, d) < 1e-6
    assert torch.equal(pb, p.bfloat16())
    p1 = p.clone()
    ops.sgd_step(p, g, buf, pb, n, 0.1, 0.9, 1e-2, False)
    d2 = 0.9 * d + g + 1e-2 * p1
    assert rel(p, p1 - 0.1 * d2) < 1e-6


@pytest.mark.parametrize("rows,cols", [(768, 3072), (3072, 768), (100, 70), (64, 64)])
@pytest.mark.parametrize("aligned", [False, True])
def test_transpose_bf16(rows, cols, aligned):
    # aligned: ldo a multiple of 8 (the 16-B store path; rows 100 also takes its row-tail path)
    ldo = (rows + 7) // 8 * 8 if aligned else rows + 3
    x = torch.randn(rows, cols + 5, device=DEV)
    out = torch.full((cols, ldo), float("nan"), device=DEV).bfloat16()
    ops.transpose_bf16(x, rows, cols, cols + 5, out, ldo)
    assert torch.equal(out[:, :rows], x[:, :cols].t().bfloat16())


@pytest.mark.parametrize("tile", [0, 3, 9])
def test_gemm_gelu_dgelu_and_mul(tile):
    """fc1 forward epilogue writing GELU(u) and GELU'(u); backward multiply by the saved GELU'."""
    M, N, K = 700, 512, 256
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, K_CONTIG, K_CONTIG)
    bias = torch.randn(N, device=DEV)
    u = (A.float() @ B.float() + bias).requires_grad_(True)
    g = torch.nn.functional.gelu(u)
    gp, = torch.autograd.grad(g.sum(), u)
    C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    C2 = torch.empty_like(C)
    ops.gemm(Am, Bm, C, M, N, K, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=lda, ldb=ldb, ldc=N,
             epilogue=EPI_BIAS_GELU_DGELU, bias=bias, C2=C2, ldc2=N, tile=tile)
    assert rel(C.float(), gp) < 5e-3
    assert rel(C2.float(), g.detach()) < 5e-3
    D = torch.empty_like(C)
    ops.gemm(Am, Bm, D, M, N, K, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=lda, ldb=ldb, ldc=N,
             epilogue=EPI_MUL_BF16, aux=C, ldaux=N, tile=tile)
    assert rel(D.float(), (A.float() @ B.float()) * C.float()) < 5e-3


@pytest.mark.parametrize("at,bt", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm_f32_layouts(at, bt):
    M, N, K = 300, 200, 150
    A = torch.randn(M, K, device=DEV)
    B = torch.randn(K, N, device=DEV)
    Am = A.t().contiguous() if at else A
    Bm = B.t().contiguous() if bt else B
    bias = torch.randn(N, device=DEV)
    C = torch.randn(M, N, device=DEV)
    C0 = C.clone()
    ops.gemm_f32(M, N, K, Am, M if at else K, at, Bm, K if bt else N, bt, C, N, bias=bias, accumulate=True)
    assert rel(C, C0 + A @ B + bias) < 1e-5


def test_attention_fwd_f32():
    B, N, H, hd = 2, 197, 3, 80
    D = H * hd
    qkv = torch.randn(B * N, 3 * D, device=DEV) * 1.5
    o = torch.empty(B * N, D, device=DEV)
    ops.attention_fwd_f32(qkv, o, B, N, H, hd, 1.0 / math.sqrt(hd))
    ref, _ = _attn_ref(qkv, B, N, H, hd)
    assert rel(o, ref) < 1e-5


@pytest.mark.parametrize("epi,K", [(EPI_BF16, 64), (EPI_BIAS_RESID_F32, 2048)])
def test_gemm_wave_split_rows(epi, K):
    """M = 50 432, N = 768 (591 tiles of 256x256 = 2.3 waves): the auto path splits the rows between the
    256x256 kernel (whole waves) and 128x128 tiles; every row must come out right."""
    M, N = 50432, 768
    A, B, Am, Bm, lda, ldb = _mats(M, N, K, K_CONTIG, K_CONTIG, ints=True)
    ref = A.double() @ B.double()
    if epi == EPI_BF16:
        C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.gemm(Am, Bm, C, M, N, K, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=lda, ldb=ldb, ldc=N, epilogue=epi)
        assert torch.equal(C.double(), ref.bfloat16().double())
    else:
        bias = torch.randint(-3, 4, (N,), device=DEV).float()
        R = torch.randint(-9, 10, (M, N), device=DEV).float()
        C = R.clone()
        ops.gemm(Am, Bm, C, M, N, K, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=lda, ldb=ldb, ldc=N, epilogue=epi,
                 bias=bias, aux=C, ldaux=N)
        assert torch.equal(C.double(), ref + bias.double() + R.double())


@pytest.mark.parametrize("B,N,H,hd,path", [(2, 197, 3, 64, 0), (2, 257, 2, 80, 0), (1, 50, 2, 32, 0),
                                           (2, 197, 3, 64, 2), (1, 577, 2, 80, 0), (24, 197, 12, 64, 0)])
def test_attention_query_rows_match_full(B, N, H, hd, path):
    """q_rows = 1 (the last layer's cls query): o / lse of the first 32-query pair equal the full
    run; with dO zero past row 0, dK / dV / bias partials are bit-identical to the full backward and
    every other dQ row is written as 0 (buffers start as NaN)."""
    D = H * hd
    sc = 1.0 / math.sqrt(hd)
    qkv = (torch.randn(B * N, 3 * D, device=DEV) * 1.5).bfloat16()
    o_f, o_r = (torch.empty(B * N, D, device=DEV, dtype=torch.bfloat16) for _ in range(2))
    l_f, l_r = torch.empty(B, H, N, device=DEV), torch.full((B, H, N), float("nan"), device=DEV)
    ops.attention_fwd(qkv, o_f, l_f, B, N, H, hd, sc, path=path)
    ops.attention_fwd(qkv, o_r, l_r, B, N, H, hd, sc, q_rows=1, path=path)
    tiled = path == 2 or (path == 0 and N > 320)
    rows = min(N, 64 if tiled else 32)  # whole 64-row blocks (tiled) / query pairs (resident)
    ov_f, ov_r = o_f.view(B, N, D)[:, :rows], o_r.view(B, N, D)[:, :rows]
    assert torch.equal(ov_f, ov_r) and torch.equal(l_f[:, :, :rows], l_r[:, :, :rows])
    dout = torch.zeros(B, N, D, device=DEV)
    dout[:, 0] = torch.randn(B, D, device=DEV)
    dout = dout.view(B * N, D).bfloat16()
    outs = []
    for qr in (None, 1):
        dqkv = torch.full((B * N, 3 * D), float("nan"), device=DEV, dtype=torch.bfloat16)
        bpart = torch.full((B * ops.attention_bias_rows(N, hd, path), 3 * D), float("nan"), device=DEV)
        ops.attention_bwd(qkv, o_f, dout, l_f, dqkv, B, N, H, hd, sc, bias_partial=bpart, q_rows=qr, path=path)
        outs.append((dqkv, bpart))
    (g_f, b_f), (g_r, b_r) = outs
    assert torch.equal(g_f.view(B * N, 3, D)[:, 1:], g_r.view(B * N, 3, D)[:, 1:])   # dK, dV
    assert torch.equal(g_f.view(B * N, 3, D)[:, 0], g_r.view(B * N, 3, D)[:, 0])     # dQ (0 past row 0)
    assert torch.equal(b_f, b_r)


@pytest.mark.parametrize("counts,Nkv,H,hd", [((5, 0, 17, 1), 17, 2, 32), ((197, 60, 3), 197, 3, 64),
                                             ((70, 577), 577, 2, 64), ((100, 257), 257, 2, 80)])
def test_attention_varlen_ragged_queries(counts, Nkv, H, hd):
    """vit_attention_fwd_varlen (Res-ViT inference, res-vit/model.py:494-529): sample b's queries are its
    own rows of a packed q (any count, 0 included), its keys / values all Nkv of its tokens."""
    B = len(counts)
    D = H * hd
    total = sum(counts)
    q = torch.randn(max(total, 1), D, device=DEV).bfloat16()
    k = torch.randn(B * Nkv, D, device=DEV).bfloat16()
    v = torch.randn(B * Nkv, D, device=DEV).bfloat16()
    o = torch.full((max(total, 1), D), float("nan"), device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), device=DEV, dtype=torch.int32)
    ops.attention_fwd_varlen(q, D, k, D, v, D, o, D, cu, B, max(counts), Nkv, H, hd, 1.0 / math.sqrt(hd))
    for b in range(B):
        s, e = int(cu[b]), int(cu[b + 1])
        if s == e:
            continue
        qb = q[s:e].float().view(e - s, H, hd).transpose(0, 1)
        kb = k[b * Nkv:(b + 1) * Nkv].float().view(Nkv, H, hd).transpose(0, 1)
        vb = v[b * Nkv:(b + 1) * Nkv].float().view(Nkv, H, hd).transpose(0, 1)
        ref = (torch.softmax(qb @ kb.transpose(-1, -2) / math.sqrt(hd), -1) @ vb).transpose(0, 1).reshape(e - s, D)
        assert rel(o[s:e].float(), ref) < 1e-2, b


def test_colsum_batch_exact_integers():
    """vit_colsum_batch: several jobs in one launch (segments, dropped outputs, accumulate, unaligned
    widths / strides) against torch sums; integer data, so every order of summation is exact"""
    g = torch.Generator(device=DEV).manual_seed(5)
    mk = lambda r, ld: torch.randint(-64, 65, (r, ld), device=DEV, generator=g).float()
    a, b_, c, d = mk(512, 2304), mk(197, 3072), mk(3, 10), mk(130, 13)
    o = [torch.full((768,), 7.0, device=DEV) for _ in range(3)]
    ob = torch.zeros(3072, device=DEV)
    oc = torch.zeros(10, device=DEV)
    od = torch.full((12,), 1.0, device=DEV)
    jobs = [(a, 512, 2304, 2304, 768, (o[0], None, o[2]), False),
            (b_, 197, 3072, 3072, 0, (ob,), False),
            (c, 3, 10, 10, 0, (oc,), False),
            (d, 130, 12, 13, 0, (od,), True)]   # 12 of 13 columns, accumulated
    ops.colsum_batch(jobs)
    torch.cuda.synchronize()
    s = a.sum(0)
    assert torch.equal(o[0], s[:768]) and torch.equal(o[2], s[1536:])
    assert torch.equal(o[1], torch.full((768,), 7.0, device=DEV))  # NULL segment: untouched
    assert torch.equal(ob, b_.sum(0)) and torch.equal(oc, c.sum(0))
    assert torch.equal(od, 1.0 + d[:, :12].sum(0))


def test_colsum_batch_random_matches_torch():
    x = torch.randn(394, 3072, device=DEV)
    out = torch.empty(3072, device=DEV)
    ops.colsum_batch([(x, 394, 3072, 3072, 0, (out,), False)])
    torch.cuda.synchronize()
    assert rel(out, x.double().sum(0).float()) < 1e-6
