// bf16 MFMA GEMM kernels (included by gemm.hip and the per-epilogue instantiation units gemm_e*.hip).
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
#pragma once
#include "common.h"
#include <stdlib.h>

namespace vitg {

struct GemmDev {
  int M, N, K;
  const char* A;
  long lda;
  long a_bs;
  uint32_t a_bytes;  // valid bytes of one batch of A
  const char* B;
  long ldb;
  long b_bs;
  uint32_t b_bytes;
  void* C;
  long ldc;
  long c_bs;
  void* C2;
  long ldc2;
  const float* bias;
  long bias_bs;
  const void* aux;
  long ldaux;
  const float* aux2;
  int split_k;
  int tokens;
  int vec;  // every pointer / leading dim allows 8-column (16/32-B) vector access
  float* col_partial;  // optional per-M-tile column sums of the output
  int group_m;         // tile order: groups of group_m tile rows, column-major inside (0: row-major)
  int nt;              // non-temporal output stores (keep the operands resident in L2)
  DropDev drop;        // dropout on the PATCH / BIAS_RESID_F32 / BIAS_GELU_DGELU output (thr 0 = off)
  int diag;            // diagnostics (VIT_GEMM_DIAG): 1 = skip the half-tile kernel's global stores, 2 = its epilogue
  int split_xcd;       // split-K grids: place each XCD's workgroups on one or two K-chunks (VIT_GEMM_SPLIT_XCD)
  int prio;            // s_setprio(1) around the ping-pong kernels' MFMA clusters (VIT_GEMM_PRIO)
  int ilv;             // diagnostic builds: gemm_pp2's interleaved read slot, -1 auto (M/N-contiguous pairs), 0 off, 1 on
#ifdef VIT_PP2_STAMPS
  unsigned long long* stamps;  // diagnostic build: gemm_pp2's slot stamps (VIT_GEMM_DIAG = 4, vit_gemm_set_stamps)
#endif
};

// a group of split-K GEMMs launched as one grid (vit_gemm_splitk_group): member i owns workgroup positions
// [start[i], start[i + 1])
constexpr int GEMM_GROUP_MAX = 4;
struct GemmGroup {
  GemmDev g[GEMM_GROUP_MAX];
  int start[GEMM_GROUP_MAX + 1];
  int n;
};
hipError_t launch_splitk_group(const GemmGroup& g, hipStream_t s);

// Internal epilogue flag: the dropout variant of PATCH / BIAS_RESID_F32 / BIAS_GELU_DGELU (its own
// instantiation, so the dropout-free kernels carry none of the Philox code)
constexpr int EPI_DROP = 16;

// launchers, one translation unit per epilogue (gemm_e<EPI>.hip) so the build parallelises
template <int EPI>
hipError_t launch_layout_x(int cfg, const GemmDev& d, bool ak, bool bk, int batch, int split, hipStream_t s);
template <int EPI>  // A K-contiguous (the dropout variants); B K-contiguous, or M/N-contiguous when bk is false
hipError_t launch_kk_x(int cfg, const GemmDev& d, bool bk, int batch, int split, hipStream_t s);
template <> hipError_t launch_layout_x<0>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_layout_x<1>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_layout_x<2>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_layout_x<3>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_layout_x<4>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_layout_x<5>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_layout_x<6>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_layout_x<7>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_layout_x<8>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_layout_x<9>(int, const GemmDev&, bool, bool, int, int, hipStream_t);
template <> hipError_t launch_kk_x<20>(int, const GemmDev&, bool, int, int, hipStream_t);
template <> hipError_t launch_kk_x<22>(int, const GemmDev&, bool, int, int, hipStream_t);
template <> hipError_t launch_kk_x<24>(int, const GemmDev&, bool, int, int, hipStream_t);
}  // namespace vitg

