"""The persistent ping-pong GEMM (config 10, csrc/gemm_ps.inc) against the one-shot ping-pong kernel (config 9)
and plain torch, GPU only.

The persistent kernel runs the forward / dgrad GEMMs of the step (src/model.py:43-48,61-63,99 and their
autograd dgrads, src/train.py:23): rounds of whole 256 x 256 tiles per CU, the last round's tiles split
along K over idle workgroups (f32 partials summed in part order by the last-arriving part), and a register
epilogue (transposed MFMA + v_permlane16_swap). On small-integer operands every f32 sum is exact whatever
its order, so its output must equal the reference kernel's bit for bit, for every epilogue, with and
without the split tail, at tile-row tails and at the benchmarked B/16 shapes."""
import pytest
import torch

from vitmi import ops
from vitmi._lib import (EPI_BF16, EPI_BIAS_BF16, EPI_BIAS_GELU, EPI_BIAS_GELU_DGELU, EPI_F32, EPI_MUL_BF16,
                        K_CONTIG)

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ints(*shape, gen):
    return torch.randint(-4, 5, shape, device=DEV, generator=gen).float().bfloat16()


def _run(A, Bt, M, N, K, epi, tile, workspace=True, **extra):
    """C (and C2) of one call; A [M][K], Bt [N][K] (both K-contiguous)"""
    f32 = epi == EPI_F32
    C = torch.full((M, N), float("nan"), device=DEV, dtype=torch.float32 if f32 else torch.bfloat16)
    kw = dict(a_layout=K_CONTIG, b_layout=K_CONTIG, lda=K, ldb=K, ldc=N, epilogue=epi, tile=tile, workspace=workspace)
    if epi in (EPI_BIAS_GELU, EPI_BIAS_GELU_DGELU):
        extra = dict(extra, C2=torch.full_like(C, float("nan")), ldc2=N)
    ops.gemm(A, Bt, C, M, N, K, **kw, **extra)
    return C, extra.get("C2")


def _counters_zero():
    ws = ops.gemm_workspace()
    return int(ws[:4096].count_nonzero()) == 0


# (M, N, K): a single partial round (fewer tiles than CUs), several rounds + a K-split tail, row tails,
# K of one / two k-tiles (no room to split), long K
SHAPES = [(1100, 512, 256), (17820, 1024, 512), (50432, 768, 768), (33000, 768, 64), (20000, 1024, 128),
          (12800, 2304, 3072)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_ps_exact_integers_f32(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A, Bt = _ints(M, K, gen=g), _ints(N, K, gen=g)
    ref = A.float() @ Bt.float().t()
    C, _ = _run(A, Bt, M, N, K, EPI_F32, 10)
    assert torch.equal(C, ref)
    C1, _ = _run(A, Bt, M, N, K, EPI_F32, 10, workspace=None)  # last round unsplit
    assert torch.equal(C1, ref)
    assert _counters_zero()


@pytest.mark.parametrize("epi", [EPI_BF16, EPI_BIAS_BF16, EPI_BIAS_GELU, EPI_BIAS_GELU_DGELU, EPI_MUL_BF16])
@pytest.mark.parametrize("M,N,K", [(17820, 1024, 512), (2000, 768, 256)])
def test_ps_epilogues_match_pp2(epi, M, N, K):
    """every register epilogue bit-identical to the LDS-staged one of the one-shot kernel (config 9)"""
    g = torch.Generator(device=DEV).manual_seed(7 * epi + M)
    A, Bt = _ints(M, K, gen=g), _ints(N, K, gen=g)
    extra = {}
    if epi in (EPI_BIAS_BF16, EPI_BIAS_GELU, EPI_BIAS_GELU_DGELU):
        extra["bias"] = torch.randn(N, device=DEV, generator=g) * 8
    if epi == EPI_MUL_BF16:
        extra.update(aux=torch.randn(M, N, device=DEV, generator=g).bfloat16(), ldaux=N)
    C9, C29 = _run(A, Bt, M, N, K, epi, 9, **extra)
    C10, C210 = _run(A, Bt, M, N, K, epi, 10, **extra)
    assert torch.equal(C10, C9)
    if C29 is not None:
        assert torch.equal(C210, C29)
    assert _counters_zero()


@pytest.mark.parametrize("name,M,N,K,epi", [("fc1 fwd", 50432, 3072, 768, EPI_BIAS_GELU_DGELU),
                                            ("qkv fwd", 50432, 2304, 768, EPI_BIAS_BF16),
                                            ("fc1 dgrad", 50432, 768, 3072, EPI_BF16),
                                            ("fc2 dgrad", 50432, 3072, 768, EPI_MUL_BF16)])
def test_ps_b16_shapes_match_pp2(name, M, N, K, epi):
    """the benchmarked ViT-B/16 bs-256 shapes (T = 50 432 tokens): auto dispatch (the persistent kernel)
    equals config 9 bit for bit on integer operands"""
    g = torch.Generator(device=DEV).manual_seed(11)
    A, Bt = _ints(M, K, gen=g), _ints(N, K, gen=g)
    extra = {}
    if epi in (EPI_BIAS_BF16, EPI_BIAS_GELU_DGELU):
        extra["bias"] = torch.randn(N, device=DEV, generator=g)
    if epi == EPI_MUL_BF16:
        extra.update(aux=torch.randn(M, N, device=DEV, generator=g).bfloat16(), ldaux=N)
    C9, C29 = _run(A, Bt, M, N, K, epi, 9, **extra)
    C0, C20 = _run(A, Bt, M, N, K, epi, 0, **extra)
    assert torch.equal(C0, C9), name
    if C29 is not None:
        assert torch.equal(C20, C29), name
    assert _counters_zero()


def test_ps_random_f32_close():
    M, N, K = 9000, 768, 3072
    A = torch.randn(M, K, device=DEV).bfloat16()
    Bt = torch.randn(N, K, device=DEV).bfloat16()
    C, _ = _run(A, Bt, M, N, K, EPI_F32, 10)
    ref = A.float() @ Bt.float().t()
    assert float((C.double() - ref.double()).norm() / ref.double().norm()) < 1e-5
