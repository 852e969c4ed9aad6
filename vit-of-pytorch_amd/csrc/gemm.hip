// bf16 MFMA GEMM for gfx950 with fused ViT epilogues.
//
// Replaces the ATen GEMMs of the reference hot path (LinearGeneral tensordot src/model.py:61-63,
// nn.Linear fc1/fc2 src/model.py:43-48, Conv2d patch embedding src/model.py:179,197) and their
// autograd dgrad / wgrad (src/train.py:23).
//
// Design:
//   * BM x BN x 64 workgroup tile, WM x WN waves, each wave a (BM/WM) x (BN/WN) sub-tile of
//     v_mfma_f32_16x16x32_bf16 accumulators (fp32).
//   * Operands are staged HBM -> LDS with LDS-DMA (buffer_load ... lds, 16 B per lane), two LDS
//     stages: the load of k-tile t+1 is in flight while k-tile t is multiplied.
//   * A K-contiguous operand is kept [rows][64] (128-B rows) with a 16-B-chunk XOR swizzle and is
//     read with ds_read_b128. An M/N-contiguous operand is kept [64][rows] and read with the
//     gfx950 transpose read ds_read_b64_tr_b16, with a 32-B-granule XOR swizzle. The swizzles are
//     applied to the per-lane global SOURCE address (LDS-DMA writes lane-linearly).
//   * Buffer descriptors bound every operand, so M/N tails read zeros instead of faulting.
//   * XCD-aware bijective block remap so consecutive tiles (same A rows) share an XCD's L2.
#include "gemm_decl.h"

namespace {
using vitg::GemmDev;
using vitg::EPI_DROP;

int pick_tile(const vit_gemm_args* a) {
  if (a->tile > 0) return (int)a->tile;
  // measured on MI355X (tools/gemm_bench.py, ViT-B/16 bs256 shapes, profiles/r01/gemm_*):
  //  * split-K weight gradients: the 256x256 ping-pong kernel with the split sized to one wave
  //    (fc1/fc2 wgrad 244 us vs 340 us for 256x128 at split 16);
  //  * wide outputs (N >= 2048: fc1 fwd, qkv fwd) and long-K MN-contiguous-B dgrads (fc1 dgrad):
  //    ping-pong; the GELU-backward epilogue (fc2 dgrad) and the N = 768 K-contiguous-B shapes
  //    are faster on 256x128x32 with 2 resident workgroups per CU (one's epilogue under the
  //    other's MFMAs);
  //  * 128x128 for small problems.
  //  * both operands K-contiguous (fc1 / fc2 fwd, qkv and out-proj dgrad): the half-tile scheduled
  //    ping-pong (fc2 fwd 260 vs 309 us, qkv dgrad 167 vs 195 us); with an M/N-contiguous operand
  //    it loses to the plain ping-pong, so those keep config 5 / 3.
  const bool ak = a->a_layout == VIT_K_CONTIG, bk = a->b_layout == VIT_K_CONTIG;
  if (a->epilogue == VIT_EPI_SPLITK && a->M >= 256 && a->N >= 256) {
    // round 5: the half-tile ping-pong with inline-asm transposed reads (both operands M/N-contiguous) beats
    // gemm_pp_kernel on the split-K weight gradients: B/16 step 8178 / 8187 -> 8256 / 8265 img/s, same box
    // (profiles/r05/splitk_pp2_ab.txt)
    static const int env_sk = vit::knob("VIT_GEMM_SPLITK_CFG", 9);
    return env_sk == 5 || env_sk == 6 || env_sk == 7 || env_sk == 8 ? env_sk : 9;
  }
  if (a->M >= 1024 && a->N >= 256) {
    // (short-K f32 residual outputs keep 2 workgroups per CU; the aux-reading epilogues run on the
    // half-tile kernel since their operand is prefetched a staging pass ahead: fc2 dgrad x GELU'
    // 286 us vs 356 us on 256x128)
    // (short-K f32 residual outputs — the out-projection — also run here: 7418 vs 7385 img/s over
    // the 256x128 two-workgroup kernel, profiles/r02/gemm_epilogue_diag.txt; VIT_GEMM_RESID_PP2=0
    // restores that)
    // (round 5: with its M/N-contiguous fragments read by inline asm the half-tile kernel runs a B operand in
    // either layout at the same speed — fc2 dgrad on W2 as it is 269 vs 268 us on the transposed copy,
    // profiles/r05/gemm_mn_b_pp2.txt — so the forward / data-gradient GEMMs read the weights in place)
    static const int env_rs = vit::knob("VIT_GEMM_RESID_PP2", 1);
    if (ak && (env_rs || !(a->epilogue == VIT_EPI_BIAS_RESID_F32 && a->K < 2048))) return 9;
    if (a->N >= 2048 && a->epilogue != VIT_EPI_GELU_BWD && a->epilogue != VIT_EPI_MUL_BF16) return 5;
    if (!bk && a->K >= 3072) return 5;
    return 3;
  }
  return 0;
}

int tile_rows_of(int cfg) {
  switch (cfg) {
    case 1: case 2: case 3: case 5: case 6: case 7: case 8: case 9: case 10: case 11: return 256;
    default: return 128;
  }
}

// Wave quantisation of the one-workgroup-per-CU 256 x 256 kernels: when the last wave of tiles would run less
// than half full (M = 50 432, N = 768: 591 tiles = 2.3 waves on 256 CUs), the rows that fill whole waves run
// on them and the remaining rows on 128 x 128 tiles (several workgroups per CU), ~2.4 instead of 3 wave-times.
// Row-local epilogues only; per-tile column partials (col_partial) continue after the whole-wave tiles' rows,
// one row per 128-row tile of the remainder. Returns the rows of the whole-wave part, 0 for one launch.
long wave_split_rows(const vit_gemm_args* a, int cfg) {
  if (!((cfg == 5 || cfg == 9) && a->batch == 1 && a->split_k == 1 && a->epilogue != VIT_EPI_PATCH && a->tile == 0))
    return 0;
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                               hipSuccess)
      return 0;
    return n;
  }();
  if (ncu <= 0) return 0;
  const long tiles_n = (a->N + 255) / 256, tiles = ((a->M + 255) / 256) * tiles_n;
  const long full = tiles / ncu, rem = tiles - full * ncu;
  const long main_rows = (full * ncu / tiles_n) * 256;
  return full >= 1 && rem > 0 && 2 * rem <= ncu && main_rows > 0 && main_rows < a->M ? main_rows : 0;
}

// tile config of the wave-split remainder launch (128 x 128; VIT_GEMM_REM_CFG in diagnostic builds)
int rem_config() {
  static const int rem_cfg = vit::knob("VIT_GEMM_REM_CFG", 0);
  return rem_cfg >= 0 && rem_cfg <= 9 && rem_cfg != 1 ? rem_cfg : 0;
}

}  // namespace

extern "C" int64_t vit_gemm_tile_rows(const vit_gemm_args* a) {
  if (!a) return 0;
  return tile_rows_of(pick_tile(a));
}

extern "C" int64_t vit_gemm_partial_rows(const vit_gemm_args* a) {
  if (!a) return 0;
  const int cfg = pick_tile(a);
  const long main_rows = wave_split_rows(a, cfg);
  if (main_rows > 0) {
    const long rr = tile_rows_of(rem_config());
    return main_rows / 256 + (a->M - main_rows + rr - 1) / rr;
  }
  const long tr = tile_rows_of(cfg);
  return (a->M + tr - 1) / tr;
}

extern "C" int64_t vit_gemm_split_rows(const vit_gemm_args* a) {
  if (!a) return 0;
  return wave_split_rows(a, pick_tile(a));
}

#ifdef VIT_PP2_STAMPS
// diagnostic build: device buffer of 2 x 8 u64 for gemm_pp2's slot stamps (taken when VIT_GEMM_DIAG = 4)
static unsigned long long* g_pp2_stamp_buf = nullptr;
extern "C" int vit_gemm_set_stamps(void* dev_buf) {
  g_pp2_stamp_buf = (unsigned long long*)dev_buf;
  return 0;
}
#endif

namespace {
// validated device descriptor of a call's arguments; `empty`: M or N is 0 (nothing to launch)
int make_dev(const vit_gemm_args* a, GemmDev& d, bool& empty) {
  empty = false;
  VIT_CHECK_ARG(a != nullptr, "vit_gemm_bf16: null args");
  VIT_CHECK_ARG(a->M >= 0 && a->N >= 0 && a->K >= 0, "vit_gemm_bf16: negative size");
  VIT_CHECK_ARG(a->K % 64 == 0, "vit_gemm_bf16: K=%lld must be a multiple of 64", (long long)a->K);
  VIT_CHECK_ARG(a->M < (1 << 30) && a->N < (1 << 30), "vit_gemm_bf16: M/N too large");
  VIT_CHECK_ARG(a->A && a->B && a->C, "vit_gemm_bf16: null operand");
  VIT_CHECK_ARG(a->batch >= 1 && a->split_k >= 1, "vit_gemm_bf16: batch/split_k must be >= 1");
  VIT_CHECK_ARG(a->split_k == 1 || a->epilogue == VIT_EPI_SPLITK, "vit_gemm_bf16: split_k>1 needs VIT_EPI_SPLITK");
  VIT_CHECK_ARG(a->a_layout == VIT_K_CONTIG || a->a_layout == VIT_MN_CONTIG, "vit_gemm_bf16: bad a_layout");
  VIT_CHECK_ARG(a->b_layout == VIT_K_CONTIG || a->b_layout == VIT_MN_CONTIG, "vit_gemm_bf16: bad b_layout");
  if (a->M == 0 || a->N == 0) {
    empty = true;
    return VIT_OK;
  }
  const bool ak = a->a_layout == VIT_K_CONTIG, bk = a->b_layout == VIT_K_CONTIG;
  // valid extents (bytes) of one batch of each operand
  const long a_rows = ak ? a->M : a->K, a_cols = ak ? a->K : a->M;
  const long b_rows = bk ? a->N : a->K, b_cols = bk ? a->K : a->N;
  VIT_CHECK_ARG(a->lda >= a_cols && a->ldb >= b_cols, "vit_gemm_bf16: leading dimension too small");
  // 16-B granularity of the LDS-DMA loads: rows must start 16-B aligned, and the last row is read
  // up to its next 16-B boundary (which lies inside the row stride).
  VIT_CHECK_ARG(a->lda % 8 == 0 && a->ldb % 8 == 0, "vit_gemm_bf16: lda/ldb must be multiples of 8");
  VIT_CHECK_ARG(((uintptr_t)a->A | (uintptr_t)a->B) % 16 == 0 && (a->a_batch_stride | a->b_batch_stride) % 8 == 0,
                "vit_gemm_bf16: A/B must be 16-byte aligned");
  const long a_bytes = ((a_rows - 1) * a->lda + ((a_cols + 7) & ~7L)) * 2;
  const long b_bytes = ((b_rows - 1) * a->ldb + ((b_cols + 7) & ~7L)) * 2;
  VIT_CHECK_ARG(a_bytes < (1L << 31) && b_bytes < (1L << 31), "vit_gemm_bf16: operand larger than 2 GiB");
  switch (a->epilogue) {
    case VIT_EPI_BIAS_GELU: VIT_CHECK_ARG(a->C2 != nullptr, "GELU epilogue needs C2"); break;
    case VIT_EPI_BIAS_RESID_F32: VIT_CHECK_ARG(a->aux != nullptr, "RESID epilogue needs aux"); break;
    case VIT_EPI_GELU_BWD: VIT_CHECK_ARG(a->aux != nullptr, "GELU_BWD epilogue needs aux"); break;
    case VIT_EPI_MUL_BF16: VIT_CHECK_ARG(a->aux != nullptr, "MUL epilogue needs aux"); break;
    case VIT_EPI_BIAS_GELU_DGELU: VIT_CHECK_ARG(a->C2 != nullptr, "GELU_DGELU epilogue needs C2"); break;
    case VIT_EPI_PATCH:
      VIT_CHECK_ARG(a->aux && a->aux2 && a->bias && a->tokens > 0 && a->batch == 1, "PATCH epilogue args");
      break;
    default: break;
  }
  d = GemmDev{};
  d.M = (int)a->M; d.N = (int)a->N; d.K = (int)a->K;
  d.A = (const char*)a->A; d.lda = a->lda; d.a_bs = a->a_batch_stride; d.a_bytes = (uint32_t)a_bytes;
  d.B = (const char*)a->B; d.ldb = a->ldb; d.b_bs = a->b_batch_stride; d.b_bytes = (uint32_t)b_bytes;
  d.C = a->C; d.ldc = a->ldc; d.c_bs = a->c_batch_stride;
  d.C2 = a->C2; d.ldc2 = a->ldc2;
  d.bias = a->bias; d.bias_bs = a->bias_batch_stride;
  d.aux = a->aux; d.ldaux = a->ldaux; d.aux2 = a->aux2;
  d.split_k = (int)a->split_k; d.tokens = (int)a->tokens;
  {
    // 8-column vector epilogue: every row start of every touched array must be 32-B aligned
    auto al = [](const void* q) { return ((uintptr_t)q % 32) == 0; };
    bool v = al(a->C) && a->ldc % 8 == 0 && a->c_batch_stride % 8 == 0;
    if (a->C2) v = v && al(a->C2) && a->ldc2 % 8 == 0;
    if (a->bias) v = v && al(a->bias) && a->bias_batch_stride % 8 == 0;
    if (a->aux) v = v && al(a->aux) && a->ldaux % 8 == 0;
    if (a->aux2) v = v && al(a->aux2);
    if (a->epilogue == VIT_EPI_SPLITK) v = al(a->C) && a->N % 8 == 0;
    d.vec = v ? 1 : 0;
  }
  d.col_partial = a->col_partial;
  d.drop = make_drop(a->dropout);
  VIT_CHECK_ARG(!d.drop.thr || a->epilogue == VIT_EPI_PATCH || a->epilogue == VIT_EPI_BIAS_RESID_F32 ||
                    a->epilogue == VIT_EPI_BIAS_GELU_DGELU,
                "vit_gemm_bf16: dropout is supported on the PATCH, BIAS_RESID_F32 and BIAS_GELU_DGELU epilogues");
  VIT_CHECK_ARG(!d.drop.thr || (a->a_layout == VIT_K_CONTIG &&
                                  (a->b_layout == VIT_K_CONTIG || a->epilogue == VIT_EPI_BIAS_RESID_F32)),
                "vit_gemm_bf16: dropout epilogues need a K-contiguous A (and B, except BIAS_RESID_F32)");
  {
    // tile order: groups of 8 tile rows, column-major inside, so the workgroups resident at once
    // share A row panels and B column panels in L2 (fc1 fwd 326 -> 306 us; VIT_GEMM_GROUP_M=1:
    // row-major)
    static const int env_gm = vit::knob("VIT_GEMM_GROUP_M", 8);
    static const int env_nt = vit::knob("VIT_GEMM_NT", 0);
    d.group_m = env_gm;
    d.nt = env_nt;
    static const int env_diag = vit::knob("VIT_GEMM_DIAG", 0);
    d.diag = env_diag;
    static const int env_sx = vit::knob("VIT_GEMM_SPLIT_XCD", 1);
    d.split_xcd = env_sx;
    static const int env_prio = vit::knob("VIT_GEMM_PRIO", 1);
    d.prio = env_prio;
    static const int env_ilv = vit::knob("VIT_GEMM_ILV", -1);
    d.ilv = env_ilv;
#ifdef VIT_PP2_STAMPS
    d.stamps = g_pp2_stamp_buf;
#endif
  }
  return VIT_OK;
}

// part 0: the whole GEMM; 1: its whole-wave rows (all of it when it does not split); 2: the wave-split remainder
// rows (nothing when it does not split)
int gemm_bf16_impl(const vit_gemm_args* a, int part, vit_stream_t stream) {
  GemmDev d;
  bool empty = false;
  if (const int rc = make_dev(a, d, empty)) return rc;
  if (empty) return VIT_OK;
  const bool ak = a->a_layout == VIT_K_CONTIG, bk = a->b_layout == VIT_K_CONTIG;
  if (a->col_partial) {
    VIT_CHECK_ARG(a->batch == 1 && a->split_k == 1 && d.vec && a->N % 8 == 0 &&
                      (a->epilogue == VIT_EPI_F32 || a->epilogue == VIT_EPI_BF16 || a->epilogue == VIT_EPI_GELU_BWD ||
                       a->epilogue == VIT_EPI_MUL_BF16 ||
                       a->epilogue == VIT_EPI_BIAS_BF16 || a->epilogue == VIT_EPI_BIAS_RESID_F32),
                  "vit_gemm_bf16: col_partial needs batch 1, split_k 1, aligned N%%8==0 operands and a plain epilogue");
  }
  hipStream_t s = (hipStream_t)stream;
  const int batch = (int)a->batch, split = (int)a->split_k;
  const int cfg = pick_tile(a);
#ifdef VIT_DIAG_KNOBS
  VIT_CHECK_ARG(cfg >= 0 && cfg <= 11, "vit_gemm_bf16: bad tile config %d", cfg);
#else
  VIT_CHECK_ARG(cfg >= 0 && cfg <= 9, "vit_gemm_bf16: bad tile config %d", cfg);
#endif
  VIT_CHECK_ARG(cfg != 1 || a->K % 32 == 0, "vit_gemm_bf16: K");
  auto run = [&](int c, const GemmDev& g) -> hipError_t {
    switch (a->epilogue) {
      case VIT_EPI_F32: return vitg::launch_layout_x<VIT_EPI_F32>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BF16: return vitg::launch_layout_x<VIT_EPI_BF16>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BIAS_BF16: return vitg::launch_layout_x<VIT_EPI_BIAS_BF16>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BIAS_GELU: return vitg::launch_layout_x<VIT_EPI_BIAS_GELU>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BIAS_RESID_F32:
        if (g.drop.thr) return vitg::launch_kk_x<VIT_EPI_BIAS_RESID_F32 | EPI_DROP>(c, g, bk, batch, split, s);
        return vitg::launch_layout_x<VIT_EPI_BIAS_RESID_F32>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_GELU_BWD: return vitg::launch_layout_x<VIT_EPI_GELU_BWD>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BIAS_GELU_DGELU:
        if (g.drop.thr) return vitg::launch_kk_x<VIT_EPI_BIAS_GELU_DGELU | EPI_DROP>(c, g, bk, batch, split, s);
        return vitg::launch_layout_x<VIT_EPI_BIAS_GELU_DGELU>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_MUL_BF16: return vitg::launch_layout_x<VIT_EPI_MUL_BF16>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_PATCH:
        if (g.drop.thr) return vitg::launch_kk_x<VIT_EPI_PATCH | EPI_DROP>(c, g, bk, batch, split, s);
        return vitg::launch_layout_x<VIT_EPI_PATCH>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_SPLITK: return vitg::launch_layout_x<VIT_EPI_SPLITK>(c, g, ak, bk, batch, split, s);
      default: return hipErrorInvalidValue;
    }
  };
  if (a->epilogue < 0 || a->epilogue > VIT_EPI_MUL_BF16) {
    vit::set_error("vit_gemm_bf16: unknown epilogue %d", a->epilogue);
    return VIT_ERR_INVALID_ARG;
  }
  // wave quantisation: whole-wave rows on the 256 x 256 kernel, the remainder on 128 x 128 tiles
  if (const long main_rows = wave_split_rows(a, cfg)) {
    GemmDev g1 = d, g2 = d;
    g1.M = (int)main_rows;
    g2.M = (int)(a->M - main_rows);
    const long r0 = main_rows;
    const long a_off = ak ? r0 * a->lda * 2 : r0 * 2;
    g2.A = d.A + a_off;
    g2.a_bytes = d.a_bytes > a_off ? (uint32_t)(d.a_bytes - a_off) : 0u;
    const int csz = (a->epilogue == VIT_EPI_F32 || a->epilogue == VIT_EPI_BIAS_RESID_F32) ? 4 : 2;
    g2.C = (char*)d.C + r0 * a->ldc * csz;
    if (d.C2) g2.C2 = (char*)d.C2 + r0 * a->ldc2 * 2;
    if (d.aux) g2.aux = (const char*)d.aux + r0 * a->ldaux * (a->epilogue == VIT_EPI_BIAS_RESID_F32 ? 4 : 2);
    if (d.col_partial) g2.col_partial = d.col_partial + (main_rows / 256) * a->N;
    g2.drop.row0 = (int)r0;  // dropout masks are indexed by the absolute row
    hipError_t e = hipSuccess;
    if (part != 2) e = run(cfg, g1);
    if (e == hipSuccess && part != 1) e = run(rem_config(), g2);
    return vit::check_hip(e, "vit_gemm_bf16 launch");
  }
  if (part == 2) return VIT_OK;
  return vit::check_hip(run(cfg, d), "vit_gemm_bf16 launch");
}
}  // namespace

extern "C" int vit_gemm_bf16(const vit_gemm_args* a, vit_stream_t stream) { return gemm_bf16_impl(a, 0, stream); }

extern "C" int vit_gemm_bf16_part(const vit_gemm_args* a, int32_t part, vit_stream_t stream) {
  VIT_CHECK_ARG(part == 1 || part == 2, "vit_gemm_bf16_part: part %d (1 = whole-wave rows, 2 = remainder)", part);
  return gemm_bf16_impl(a, part, stream);
}

extern "C" int vit_gemm_splitk_group(const vit_gemm_args* args, int32_t n, vit_stream_t stream) {
  VIT_CHECK_ARG(args != nullptr && n >= 1 && n <= vitg::GEMM_GROUP_MAX, "vit_gemm_splitk_group: 1..%d members, got %d",
                vitg::GEMM_GROUP_MAX, n);
  vitg::GemmGroup g{};
  long total = 0;
  for (int i = 0; i < n; ++i) {
    const vit_gemm_args* a = args + i;
    VIT_CHECK_ARG(a->epilogue == VIT_EPI_SPLITK && a->a_layout == VIT_MN_CONTIG && a->b_layout == VIT_MN_CONTIG &&
                      a->tile == 0 && !a->col_partial && !a->dropout,
                  "vit_gemm_splitk_group: member %d must be a split-K weight gradient (VIT_EPI_SPLITK, both operands "
                  "M/N-contiguous, no tile / col_partial / dropout)", i);
    bool empty = false;
    if (const int rc = make_dev(a, g.g[i], empty)) return rc;
    VIT_CHECK_ARG(!empty, "vit_gemm_splitk_group: member %d is empty", i);
    g.start[i] = (int)total;
    total += ((a->M + 255) / 256) * ((a->N + 255) / 256) * a->split_k * a->batch;
    VIT_CHECK_ARG(total < (1L << 30), "vit_gemm_splitk_group: grid too large");
  }
  g.start[n] = (int)total;
  g.n = n;
  return vit::check_hip(vitg::launch_splitk_group(g, (hipStream_t)stream), "vit_gemm_splitk_group launch");
}

// ---- split-K reduction -------------------------------------------------------------------------
namespace {
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int split, long M, long N, float* __restrict__ out,
                                     long ldo, long obs, int accumulate) {
  const int z = blockIdx.y;
  const long total = M * N;
  const float* w = ws + (long)z * split * total;
  float* o = out + z * obs;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < split; ++k) s += w[k * total + i];
    const long m = i / N, n = i - m * N;
    float* dst = o + m * ldo + n;
    *dst = accumulate ? *dst + s : s;
  }
}
// 4 columns per thread, the slabs read 4 at a time with independent 16-B loads (memory-level
// parallelism: the scalar loop above issued one dependent load per slab); N, ldo multiples of 4.
__global__ void splitk_reduce4_kernel(const float* __restrict__ ws, int split, long M, long N, float* __restrict__ out,
                                      long ldo, long obs, int accumulate) {
  const int z = blockIdx.y;
  const long total = M * N, total4 = total / 4;
  const float4* w = reinterpret_cast<const float4*>(ws + (long)z * split * total);
  float* o = out + z * obs;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += (long)gridDim.x * blockDim.x) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int k = 0;
    for (; k + 4 <= split; k += 4) {
      const float4 a = w[(long)k * total4 + i], b = w[(long)(k + 1) * total4 + i];
      const float4 c = w[(long)(k + 2) * total4 + i], d = w[(long)(k + 3) * total4 + i];
      s.x += (a.x + b.x) + (c.x + d.x);
      s.y += (a.y + b.y) + (c.y + d.y);
      s.z += (a.z + b.z) + (c.z + d.z);
      s.w += (a.w + b.w) + (c.w + d.w);
    }
    for (; k < split; ++k) {
      const float4 a = w[(long)k * total4 + i];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
    const long e = i * 4, m = e / N, n = e - m * N;
    float4* dst = reinterpret_cast<float4*>(o + m * ldo + n);
    if (accumulate) {
      const float4 p = *dst;
      s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
    }
    *dst = s;
  }
}

// several vit_splitk_reduce jobs (vector form) in one launch: workgroups [blk0_j, blk0_{j+1}) are job j's, batch-major;
// the same 4-at-a-time slab order as splitk_reduce4_kernel, so each output equals its own launch's bit for bit
struct SplitkJobDev {
  const float* ws;
  float* out;
  long M, N, ldo, obs;
  int split, batch, nb, blk0, acc;
};
struct SplitkGroupDev {
  SplitkJobDev j[VIT_SPLITK_GROUP_MAX];
  int n;
};
__global__ void splitk_reduce4_group_kernel(const SplitkGroupDev G) {
  int jx = 0;
#pragma unroll
  for (int k = 1; k < VIT_SPLITK_GROUP_MAX; ++k)
    if (k < G.n && (int)blockIdx.x >= G.j[k].blk0) jx = k;
  const SplitkJobDev& J = G.j[jx];
  const int local = blockIdx.x - J.blk0;
  const int z = local / J.nb, bx = local - z * J.nb;
  const long total = J.M * J.N, total4 = total / 4;
  const float4* w = reinterpret_cast<const float4*>(J.ws + (long)z * J.split * total);
  float* o = J.out + z * J.obs;
  for (long i = (long)bx * blockDim.x + threadIdx.x; i < total4; i += (long)J.nb * blockDim.x) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int k = 0;
    for (; k + 4 <= J.split; k += 4) {
      const float4 a = w[(long)k * total4 + i], b = w[(long)(k + 1) * total4 + i];
      const float4 c = w[(long)(k + 2) * total4 + i], d = w[(long)(k + 3) * total4 + i];
      s.x += (a.x + b.x) + (c.x + d.x);
      s.y += (a.y + b.y) + (c.y + d.y);
      s.z += (a.z + b.z) + (c.z + d.z);
      s.w += (a.w + b.w) + (c.w + d.w);
    }
    for (; k < J.split; ++k) {
      const float4 a = w[(long)k * total4 + i];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
    const long e = i * 4, m = e / J.N, n = e - m * J.N;
    float4* dst = reinterpret_cast<float4*>(o + m * J.ldo + n);
    if (J.acc) {
      const float4 p = *dst;
      s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
    }
    *dst = s;
  }
}
}  // namespace

extern "C" int vit_splitk_reduce_group(const vit_splitk_job* jobs, int32_t n, vit_stream_t stream) {
  VIT_CHECK_ARG(jobs && n >= 1 && n <= VIT_SPLITK_GROUP_MAX, "vit_splitk_reduce_group: 1..%d jobs, got %d",
                VIT_SPLITK_GROUP_MAX, (int)n);
  bool vec = true;
  for (int k = 0; k < n; ++k) {
    const vit_splitk_job& j = jobs[k];
    VIT_CHECK_ARG(j.ws && j.out && j.batch >= 1 && j.split >= 1 && j.M >= 1 && j.N >= 1 && j.ldo >= j.N,
                  "vit_splitk_reduce_group: job %d: bad args", k);
    vec = vec && j.N % 4 == 0 && j.ldo % 4 == 0 && j.out_batch_stride % 4 == 0 && ((uintptr_t)j.ws % 16) == 0 &&
          ((uintptr_t)j.out % 16) == 0;
  }
  if (!vec) {  // any job outside the vector form: one launch each
    for (int k = 0; k < n; ++k) {
      const vit_splitk_job& j = jobs[k];
      if (const int rc = vit_splitk_reduce(j.ws, j.batch, j.split, j.M, j.N, j.out, j.ldo, j.out_batch_stride,
                                           j.accumulate, stream))
        return rc;
    }
    return VIT_OK;
  }
  SplitkGroupDev g{};
  long blk = 0;
  for (int k = 0; k < n; ++k) {
    const vit_splitk_job& j = jobs[k];
    long nb = (j.M * j.N / 4 + 255) / 256;
    if (nb > 4096) nb = 4096;
    SplitkJobDev& d = g.j[k];
    d.ws = j.ws; d.out = j.out; d.M = j.M; d.N = j.N; d.ldo = j.ldo; d.obs = j.out_batch_stride;
    d.split = (int)j.split; d.batch = (int)j.batch; d.nb = (int)nb; d.blk0 = (int)blk; d.acc = j.accumulate ? 1 : 0;
    blk += nb * j.batch;
  }
  g.n = n;
  VIT_CHECK_ARG(blk < (1L << 31), "vit_splitk_reduce_group: grid too large");
  hipLaunchKernelGGL(splitk_reduce4_group_kernel, dim3((unsigned)blk), dim3(256), 0, (hipStream_t)stream, g);
  VIT_LAUNCH_CHECK("vit_splitk_reduce_group");
}

extern "C" int vit_splitk_reduce(const float* ws, int64_t batch, int64_t split, int64_t M, int64_t N, float* out,
                                 int64_t ldo, int64_t out_batch_stride, int32_t accumulate, vit_stream_t stream) {
  VIT_CHECK_ARG(ws && out && batch >= 1 && split >= 1 && ldo >= N, "vit_splitk_reduce: bad args");
  if (M * N == 0) return VIT_OK;
  const bool vec = N % 4 == 0 && ldo % 4 == 0 && out_batch_stride % 4 == 0 && ((uintptr_t)ws % 16) == 0 &&
                   ((uintptr_t)out % 16) == 0;
  long blocks = (M * N / (vec ? 4 : 1) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (vec)
    hipLaunchKernelGGL(splitk_reduce4_kernel, dim3((unsigned)blocks, (unsigned)batch), dim3(256), 0,
                       (hipStream_t)stream, ws, (int)split, (long)M, (long)N, out, (long)ldo, (long)out_batch_stride,
                       (int)accumulate);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)blocks, (unsigned)batch), dim3(256), 0, (hipStream_t)stream,
                       ws, (int)split, (long)M, (long)N, out, (long)ldo, (long)out_batch_stride, (int)accumulate);
  VIT_LAUNCH_CHECK("vit_splitk_reduce");
}
