// Fused multi-head self-attention (forward + backward) for gfx950.
//
// Replaces SelfAttention.forward's core (reference src/model.py:90-97: permute, q@k^T, / sqrt(hd),
// softmax(-1), @v, permute back) and its autograd backward.
//
// One workgroup per (image, head). ViT sequences are short (197 tokens for B/16 @224, 257 for
// H/14), so every K/V row of a head fits in LDS and softmax is exact (no online rescaling).
//   fwd: per 16-query strip, S^T = K Q^T on v_mfma_f32_16x16x32_bf16 (query on the lane, keys in
//        registers), masked wavefront softmax, O^T = V^T P^T with V read by ds_read_b64_tr_b16.
//        The P fragment is the S accumulator itself (keys permuted consistently on both MFMA
//        operands), so P never touches LDS. Saves LSE (f32) for the backward.
//   bwd: stage 1 (K, V in LDS), each wave owns 16-query strips: P and dP of the strip for all keys
//        stay in registers, delta = sum P dP, dS = P (dP - delta), dQ = dS K. stage 2 (Q, dO in
//        LDS), each wave owns pairs of 16-key tiles: recompute P, dS and accumulate dV = P^T dO,
//        dK = dS^T Q in registers. No atomics, deterministic (details above attn_bwd_kernel).
// LDS images: [rows][HD] bf16 with a 16-B-chunk XOR swizzle that is conflict-free for both the
// row read (ds_read_b128) and the transposed read (ds_read_b64_tr_b16) at HD = 64.
#include "attn_common.h"
#include <stdlib.h>

#ifdef VIT_ATTN_STAMPS
// DIAGNOSTIC build only: s_memtime stamps of the two-stage backward, workgroups 0 and gridDim - 1, their first
// and last waves, 6 points (start, K / V images in, stage 1 done, Q / dO images in, stage 2 done, end);
// read back with vit_attn2_stamps()
__device__ unsigned long long g_attn2_stamps[2][2][8];
#define A2STAMP(k)                                                                                          \
  do {                                                                                                      \
    const int w_ = threadIdx.x >> 6, lw_ = blockDim.x / 64 - 1;                                             \
    const bool blk_ = blockIdx.x == 0 || blockIdx.x == gridDim.x - 1;                                        \
    if (blk_ && (w_ == 0 || w_ == lw_)) {                                                                   \
      unsigned long long t_;                                                                                \
      __builtin_amdgcn_sched_barrier(0);                                                                    \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                          \
      __builtin_amdgcn_sched_barrier(0);                                                                    \
      if ((threadIdx.x & 63) == 0) g_attn2_stamps[blockIdx.x != 0][w_ != 0][k] = t_;                         \
    }                                                                                                       \
  } while (0)
extern "C" int vit_attn2_stamps(unsigned long long* out) {  // 32 values: [block first/last][wave first/last][point]
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_attn2_stamps), sizeof(g_attn2_stamps));
}
#else
#define A2STAMP(k) \
  do {             \
  } while (0)
#endif

namespace {
using namespace vit_attn;

// ------------------------------------------------------------------------------------------------
template <int HD, int NKT, int NW>
__global__ void __launch_bounds__(NW * 64) attn_fwd_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o,
                                                           float* __restrict__ lse, int N, int H, int hd,
                                                           float scale, int nq) {
  constexpr int NP = NKT * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ki = smem;
  char* Vi = smem + NP * HD * 2;
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * hd;
  const long rs = 3L * D;
  const bf16_t* base = qkv + (long)b * N * rs + (long)h * hd;
  load_images<HD, NP, NW * 64>(Ki, base + D, rs, Vi, base + 2 * D, rs, N, hd);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const float c = scale * LOG2E;
  // queries [0, nq) are needed (nq < N: the last layer's cls rows); whole 32-row pairs are kept so
  // the backward's stage 2 (query pairs) finds lse for every row it touches
  const int nqa = min(N, (nq + 31) / 32 * 32);
  const int nqt = (nqa + 15) / 16;
  // Q fragments come straight from HBM; the next strip's are requested before this strip's math
  v8bf qn[HD / 32];
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) qn[kk] = gl_row<HD>(base, rs, wave * 16, kk, N, hd, lane);
  for (int qt = wave; qt < nqt; qt += NW) {
    const int q = qt * 16 + i;
    v8bf qf[HD / 32];
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) {
      qf[kk] = qn[kk];
      qn[kk] = gl_row<HD>(base, rs, (qt + NW) * 16, kk, N, hd, lane);  // rows >= N read as zero
    }
    v4f s[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      s[kt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk) s[kt] = mfma(rd_row<HD>(Ki, kt * 16, kk, lane), qf[kk], s[kt]);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kt * 16 + 4 * g + r;
        const float v = key < N ? s[kt][r] : -INFINITY;
        s[kt][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mc = mx * c;
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = ex2(s[kt][r] * c - mc);
        s[kt][r] = p;
        l += p;
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    if (g == 0 && q < N) lse[(long)bh * N + q] = mx * scale + logf(l);
    const float inv_l = 1.0f / l;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKT / 2; ++ks)
        acc = mfma(rd_tr<HD>(Vi, 2 * ks, 2 * ks + 1, dt * 16, lane), pack8(s[2 * ks], s[2 * ks + 1]), acc);
      const int d = dt * 16 + 4 * g;
      if (q < N && d < hd) store4(o + ((long)b * N + q) * D + (long)h * hd + d, acc, inv_l);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Forward, lean form: one (image, head) per workgroup, keys padded to whole 16-row tiles only (an odd
// last tile takes v_mfma_f32_16x16x16_bf16 in P V), so B/16's 197 tokens need 2 x 208 x 64 x 2 B =
// 53 KB of LDS and three workgroups share a CU. Per 16-query strip and lane: S^T = K Q^T accumulators
// (keys 4g + r of every tile, query i), masking only on the last tile, max via max3, p = exp2(s c - m c)
// (one fma + one v_exp), bf16 packing of the accumulators as the P^T operand. LDS addresses are
// per-lane bases + immediates (ImgLane), so the inner loops carry no address arithmetic.
template <int HD, int NP, int NT>
__device__ __forceinline__ void load_images_lds(lds_t* imgA, const bf16_t* srcA, long strideA, lds_t* imgB,
                                                const bf16_t* srcB, long strideB, int N, int hd) {
  constexpr int CPR = HD / 8;
  constexpr int TOTAL = NP * CPR;
  constexpr int PER = (TOTAL + NT - 1) / NT;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(srcA, (uint32_t)(((long)(N - 1) * strideA + hd) * 2));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(srcB, (uint32_t)(((long)(N - 1) * strideB + hd) * 2));
  v4u a[PER], b[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = threadIdx.x + k * NT;
    const int row = c / CPR, ch = c % CPR;
    const bool ok = c < TOTAL && row < N && ch * 8 < hd;
    const int offa = ok ? (int)(((long)row * strideA + ch * 8) * 2) : 0x7ffffff0;
    const int offb = ok ? (int)(((long)row * strideB + ch * 8) * 2) : 0x7ffffff0;
    a[k] = __builtin_amdgcn_raw_buffer_load_b128(ra, offa, 0, 0);
    b[k] = __builtin_amdgcn_raw_buffer_load_b128(rb, offb, 0, 0);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = threadIdx.x + k * NT;
    if (TOTAL % NT == 0 || c < TOTAL) {
      const int row = c / CPR, ch = c % CPR;
      lds_st(imgA + img_off<HD>(row, ch), a[k]);
      lds_st(imgB + img_off<HD>(row, ch), b[k]);
    }
  }
}

template <int HD, int NKT, int NW>
__global__ void __launch_bounds__(NW * 64, NW == 8 ? (k_tail<HD> ? 1 : 2) : 3) attn_fwd2_kernel(const bf16_t* __restrict__ qkv,
                                                               bf16_t* __restrict__ o, float* __restrict__ lse,
                                                               int N, int H, int hd, float scale, int nq) {
  constexpr int NP = NKT * 16;
  constexpr int IMG = NP * HD * 2;
  constexpr int T = ImgLane<HD>::TILE;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lds_t* Ki = (lds_t*)smem;
  lds_t* Vi = Ki + IMG;
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * hd;
  const long rs = 3L * D;
  const bf16_t* base = qkv + (long)b * N * rs + (long)h * hd;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const ImgLane<HD> L(lane);
  load_images_lds<HD, NP, NW * 64>(Ki, base + D, rs, Vi, base + 2 * D, rs, N, hd);
  const float c = scale * LOG2E;
  const int nqa = min(N, (nq + 31) / 32 * 32);  // whole 32-row pairs (the backward's stage 2 reads their lse)
  const int nqt = (nqa + 15) / 16;
  // every Q fragment of this wave's strips is requested up front, beside the K / V image loads: one HBM
  // latency per workgroup instead of one per strip
  constexpr int MAXS = (NKT + NW - 1) / NW;
  v8bf qa[MAXS][HD / 32];
  v4s qa16[MAXS];  // hd 80: the 16-k tail
#pragma unroll
  for (int u = 0; u < MAXS; ++u) {
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) qa[u][kk] = gl_row<HD>(base, rs, (wave + u * NW) * 16, kk, N, hd, lane);
    if constexpr (k_tail<HD>) qa16[u] = gl_row16<HD>(base, rs, (wave + u * NW) * 16, N, hd, lane);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < MAXS; ++u) {
    const int qt = wave + u * NW;
    if (qt >= nqt) break;
    const v8bf* qf = qa[u];
    v4f s[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      s[kt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk)
        s[kt] = mfma(__builtin_bit_cast(v8bf, lds_ld<v8s>(Ki + kt * T + L.row[kk])), qf[kk], s[kt]);
      if constexpr (k_tail<HD>) s[kt] = mfma16_add(lds_ld<v4s>(Ki + kt * T + L.row16), qa16[u], s[kt]);
    }
    if (N < NP) {  // only the last tile holds padded keys
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if ((NKT - 1) * 16 + 4 * g + r >= N) s[NKT - 1][r] = -INFINITY;
    }
    // row max: two v_max3 per tile (max(mx, a, b))
    float mx = max3f(s[0][0], s[0][1], s[0][2]);
    mx = fmaxf(mx, s[0][3]);
#pragma unroll
    for (int kt = 1; kt < NKT; ++kt) {
      mx = max3f(mx, s[kt][0], s[kt][1]);
      mx = max3f(mx, s[kt][2], s[kt][3]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mc = mx * c;
    float l = 0.f;  // f32 row sum of the unrounded P (the reference's normalisation)
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[kt][r] = ex2(fmaf(s[kt][r], c, -mc));
        l += s[kt][r];
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    v4f acc[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) acc[dt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKT / 2; ++ks) {
      const v8bf pp = pack8(s[2 * ks], s[2 * ks + 1]);
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        v8s vt;
        vt.lo = lds_tr(Vi + 2 * ks * T + L.tr[dt]);
        vt.hi = lds_tr(Vi + (2 * ks + 1) * T + L.tr[dt]);
        acc[dt] = mfma(__builtin_bit_cast(v8bf, vt), pp, acc[dt]);
      }
    }
    if constexpr (NKT % 2 == 1) {
      const v4s pp = pack4(s[NKT - 1]);
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) acc[dt] = mfma16_add(lds_tr(Vi + (NKT - 1) * T + L.tr[dt]), pp, acc[dt]);
    }
    const int q = qt * 16 + i;
    if (g == 0 && q < N) lse[(long)bh * N + q] = mx * scale + logf(l);
    const float inv_l = 1.0f / l;
    {  // whole 2*hd-byte rows through the wave's LDS strip (StripOut)
      lds_t* so = Vi + IMG + wave * StripOut<HD>::BYTES;
      StripOut<HD>::stage(so, acc, inv_l, lane);
      StripOut<HD>::store(so, o + ((long)b * N + qt * 16) * D + (long)h * hd, D, N - qt * 16, hd, lane);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Backward, two LDS images at a time (56 KB at N = 197, hd = 64: two workgroups per CU, so one
// workgroup's image loads overlap the other's MFMA work).
//   stage 1 (K, V images): each wave owns 16-query strips, Q / dO rows in registers (the next
//     strip's requested one strip ahead). HD <= 80: P and dP of the strip for all keys are kept in
//     registers, so delta_q = sum_j P_qj dP_qj (from the recomputed P and dP themselves:
//     FlashAttention-2's rowsum(dO * O) differs from it by bf16 O's rounding, and dS = P (dP - delta)
//     is a small difference: that turned into 10-25% errors on the q/k weight gradients under
//     near-uniform attention), dS and dQ = dS K come from one pass. HD = 96 (too many registers):
//     pairs of strips, pass A for delta, pass B recomputing S / dP for dS and dQ.
//   stage 2 (Q, dO images): each wave owns pairs of 16-key tiles, K / V rows in registers; dV =
//     P^T dO, dK = dS^T Q, with delta from stage 1.
// Deterministic (no atomics). Optionally writes per-image column sums of dQ | dK | dV (q/k/v bias
// gradient partials) to bias_partial[b][3*D].
template <int HD, int NKT, int NW>
__global__ void __launch_bounds__(NW * 64, NW == 8 ? 1 : 2) attn_bwd_kernel(const bf16_t* __restrict__ qkv,
                                                              const bf16_t* __restrict__ dout,
                                                              const float* __restrict__ lse, bf16_t* __restrict__ dqkv,
                                                              float* __restrict__ bias_partial, int N, int H, int hd,
                                                              float scale, int nq) {
  constexpr int NP = NKT * 16;
  constexpr int IMG = NP * HD * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ImA = smem;        // K, then Q
  char* ImB = smem + IMG;  // V, then dO
  float* lse_s = reinterpret_cast<float*>(smem + 2 * IMG);
  float* dlt_s = lse_s + NP;
  float* bsum = dlt_s + NP;  // [NW][3][HD]

  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * hd;
  const long rs = 3L * D;
  const bf16_t* base = qkv + (long)b * N * rs + (long)h * hd;
  const bf16_t* dob = dout + (long)b * N * D + (long)h * hd;
  bf16_t* dq_base = dqkv + (long)b * N * rs + (long)h * hd;

  A2STAMP(0);
  load_images<HD, NP, NW * 64>(ImA, base + D, rs, ImB, base + 2 * D, rs, N, hd);
  for (int r = threadIdx.x; r < NP; r += blockDim.x) {
    // padded queries: P = 2^-1e30 = 0 (finite, so that nan_of() of their exponent stays 0)
    lse_s[r] = r < N ? lse[(long)bh * N + r] * LOG2E : 1e30f;
    dlt_s[r] = 0.f;
  }
  __syncthreads();
  A2STAMP(1);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const float c = scale * LOG2E;
  const int npair = (N + 31) / 32;  // pairs of 16-row tiles holding valid rows
  // queries [0, nq) carry a gradient (nq < N: dO is zero on every other row); the 32-row pairs
  // holding them are processed, the other rows get dQ = 0 and contribute nothing to dK / dV
  const int nqa = min(N, (nq + 31) / 32 * 32);
  const int npair_q = (nqa + 31) / 32;
  // bias partials: each wave adds the column sums of every dQ strip / dK, dV tile it finishes to its own
  // LDS rows bsum[wave][3][HD] (nothing long-lived in registers); summed over waves at the end
  float* bs_w = bsum + wave * 3 * HD;
  if (bias_partial)
    for (int e = lane; e < 3 * HD; e += 64) bs_w[e] = 0.f;

  // ---- stage 1: delta and dQ ----
  if constexpr (HD != 96) {
    // one 16-query strip at a time with P and dP of ALL keys kept in registers (2 x NKT x 4 f32):
    // delta = sum_j P dP comes out of the same pass, so dS and dQ need no recompute of S / dP
    const int nqt = (N + 15) / 16;
    v8bf qn[HD / 32], dn[HD / 32];  // next strip's Q / dO rows, requested one strip ahead
    v4s qn16 = {0, 0, 0, 0}, dn16 = {0, 0, 0, 0};  // hd 80: their 16-k tails
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) {
      qn[kk] = gl_row<HD>(base, rs, wave * 16, kk, N, hd, lane);
      dn[kk] = gl_row<HD>(dob, D, wave * 16, kk, N, hd, lane);
    }
    if constexpr (k_tail<HD>) {
      qn16 = gl_row16<HD>(base, rs, wave * 16, N, hd, lane);
      dn16 = gl_row16<HD>(dob, D, wave * 16, N, hd, lane);
    }
    for (int qt = wave; qt < nqt; qt += NW) {
      if (qt * 16 >= nqa) {  // no gradient reaches these queries: dQ = 0, delta = 0
        const int q = qt * 16 + i;
        if (g == 0) dlt_s[q] = 0.f;
        if (q < N) {
#pragma unroll
          for (int dt = 0; dt < HD / 16; ++dt) {
            const int d = dt * 16 + 4 * g;
            if (d < hd) store4(dq_base + (long)q * rs + d, v4f{0.f, 0.f, 0.f, 0.f}, 1.f);
          }
        }
        continue;
      }
      v8bf qf[HD / 32], df[HD / 32];
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk) {
        qf[kk] = qn[kk];
        df[kk] = dn[kk];
        qn[kk] = gl_row<HD>(base, rs, (qt + NW) * 16, kk, N, hd, lane);
        dn[kk] = gl_row<HD>(dob, D, (qt + NW) * 16, kk, N, hd, lane);
      }
      const v4s qf16 = qn16, df16 = dn16;
      if constexpr (k_tail<HD>) {
        qn16 = gl_row16<HD>(base, rs, (qt + NW) * 16, N, hd, lane);
        dn16 = gl_row16<HD>(dob, D, (qt + NW) * 16, N, hd, lane);
      }
      const float ls = lse_s[qt * 16 + i];
      v4f P[NKT], DP[NKT];
      float dlr[4] = {0.f, 0.f, 0.f, 0.f};  // four independent chains (one fma chain per row r)
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        if (kt == NKT - 1 && kt * 16 >= N) {  // a wholly padded last key tile (N % 32 in 1..16)
          P[kt] = DP[kt] = v4f{0.f, 0.f, 0.f, 0.f};
          continue;
        }
        v4f st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk) {
          st = mfma(rd_row<HD>(ImA, kt * 16, kk, lane), qf[kk], st);
          dpt = mfma(rd_row<HD>(ImB, kt * 16, kk, lane), df[kk], dpt);
        }
        if constexpr (k_tail<HD>) {
          st = mfma16_add(rd_row16<HD>(ImA, kt * 16, lane), qf16, st);
          dpt = mfma16_add(rd_row16<HD>(ImB, kt * 16, lane), df16, dpt);
        }
        // Padded keys (rows N.. of the zero-filled K / V images) need no mask here: their dP = dO V^T
        // is 0, so they add nothing to delta, and their dS only meets the zero K rows in dQ = dS K.
        // Their exponent -LSE is clamped at 0 so that P stays finite whatever the query's LSE (unclamped,
        // LSE << 0 gives 2^-LSE = inf and P dP = inf * 0 = NaN); a real key's exponent is <= 0 up to
        // rounding (LSE >= every score), so the clamp is applied to every key without a mask (the
        // per-(tile, row) masks it replaces were spilled SGPR lane masks: 2 v_readlane + 2 v_cndmask per
        // element). nan_of(e) = e - e in hardware (0, or NaN for a NaN score) keeps a diverging run's NaN
        // visible in dQ: v_min alone returns the non-NaN operand.
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = st[r] * c - ls;
          // only the last two tiles can hold padded keys (N > 16 (NKT - 2)): the others skip the clamp
          const float pv = kt >= NKT - 2 ? ex2(fminf(e, 0.f) + nan_of(e)) : ex2(e);
          P[kt][r] = pv;
          dlr[r] += pv * dpt[r];
        }
        DP[kt] = dpt;
      }
      float dl = (dlr[0] + dlr[1]) + (dlr[2] + dlr[3]);
      dl += __shfl_xor(dl, 16, 64);
      dl += __shfl_xor(dl, 32, 64);
      const int q = qt * 16 + i;
      if (q >= N) dl = 0.f;
      if (g == 0) dlt_s[q] = dl;
      v4f dq[HD / 16];
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) dq[dt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKT / 2; ++ks) {
        v4f d0, d1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          d0[r] = P[2 * ks][r] * (DP[2 * ks][r] - dl);
          d1[r] = P[2 * ks + 1][r] * (DP[2 * ks + 1][r] - dl);
        }
        const v8bf bD = pack8(d0, d1);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) dq[dt] = mfma(rd_tr<HD>(ImA, 2 * ks, 2 * ks + 1, dt * 16, lane), bD, dq[dt]);
      }
      if constexpr (NKT % 2 == 1) {  // odd tile count (hd 80 images hold ceil(N / 16) tiles): a 16-k step
        v4f d0;
#pragma unroll
        for (int r = 0; r < 4; ++r) d0[r] = P[NKT - 1][r] * (DP[NKT - 1][r] - dl);
        const v4s bD = pack4(d0);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) dq[dt] = mfma16_add(rd_tr1<HD>(ImA, NKT - 1, dt * 16, lane), bD, dq[dt]);
      }
      if (q < N) {
        uint2 pk[HD / 16];
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) pk[dt] = pack4bf(dq[dt], scale);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
          const int d = dt * 16 + 4 * g;
          if (d < hd) *reinterpret_cast<uint2*>(dq_base + (long)q * rs + d) = pk[dt];
        }
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) keep_live2(pk[dt]);
      }
      if (bias_partial) add_colsums<HD>(bs_w, dq, scale, lane);  // padded queries: dS = 0
    }
  } else {
    for (int qp = wave; qp < npair; qp += NW) {
      if (qp >= npair_q) {  // no gradient reaches these queries: dQ = 0, delta = 0
        for (int u = 0; u < 2; ++u) {
          const int q = (2 * qp + u) * 16 + i;
          if (g == 0) dlt_s[q] = 0.f;
          if (q < N) {
            for (int dt = 0; dt < HD / 16; ++dt) {
              const int d = dt * 16 + 4 * g;
              if (d < hd) store4(dq_base + (long)q * rs + d, v4f{0.f, 0.f, 0.f, 0.f}, 1.f);
            }
          }
        }
        continue;
      }
      v8bf qf[2][HD / 32], df[2][HD / 32];
      float ls[2], dl[2] = {0.f, 0.f};
  #pragma unroll
      for (int u = 0; u < 2; ++u) {
  #pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk) {
          qf[u][kk] = gl_row<HD>(base, rs, (2 * qp + u) * 16, kk, N, hd, lane);
          df[u][kk] = gl_row<HD>(dob, D, (2 * qp + u) * 16, kk, N, hd, lane);
        }
        ls[u] = lse_s[(2 * qp + u) * 16 + i];
      }
      // pass A: delta
      for (int kt = 0; kt < 2 * npair; ++kt) {
        v8bf kr[HD / 32], vr[HD / 32];
  #pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk) {
          kr[kk] = rd_row<HD>(ImA, kt * 16, kk, lane);
          vr[kk] = rd_row<HD>(ImB, kt * 16, kk, lane);
        }
  #pragma unroll
        for (int u = 0; u < 2; ++u) {
          v4f st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
  #pragma unroll
          for (int kk = 0; kk < HD / 32; ++kk) {
            st = mfma(kr[kk], qf[u][kk], st);
            dpt = mfma(vr[kk], df[u][kk], dpt);
          }
  #pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kt * 16 + 4 * g + r;
            if (key < N) dl[u] += ex2(st[r] * c - ls[u]) * dpt[r];
          }
        }
      }
  #pragma unroll
      for (int u = 0; u < 2; ++u) {
        dl[u] += __shfl_xor(dl[u], 16, 64);
        dl[u] += __shfl_xor(dl[u], 32, 64);
        const int q = (2 * qp + u) * 16 + i;
        if (q >= N) dl[u] = 0.f;
        if (g == 0) dlt_s[q] = dl[u];
      }
      // pass B: dQ
      v4f dq[2][HD / 16];
  #pragma unroll
      for (int u = 0; u < 2; ++u)
  #pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) dq[u][dt] = v4f{0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < npair; ++ks) {
        v4f DS[2][2];  // [query tile][key tile]
  #pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int kt = 2 * ks + t;
          v8bf kr[HD / 32], vr[HD / 32];
  #pragma unroll
          for (int kk = 0; kk < HD / 32; ++kk) {
            kr[kk] = rd_row<HD>(ImA, kt * 16, kk, lane);
            vr[kk] = rd_row<HD>(ImB, kt * 16, kk, lane);
          }
  #pragma unroll
          for (int u = 0; u < 2; ++u) {
            v4f st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
  #pragma unroll
            for (int kk = 0; kk < HD / 32; ++kk) {
              st = mfma(kr[kk], qf[u][kk], st);
              dpt = mfma(vr[kk], df[u][kk], dpt);
            }
  #pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int key = kt * 16 + 4 * g + r;
              const float p = key < N ? ex2(st[r] * c - ls[u]) : 0.f;
              DS[u][t][r] = p * (dpt[r] - dl[u]);
            }
          }
        }
        const v8bf bD0 = pack8(DS[0][0], DS[0][1]), bD1 = pack8(DS[1][0], DS[1][1]);
  #pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
          const v8bf kt_ = rd_tr<HD>(ImA, 2 * ks, 2 * ks + 1, dt * 16, lane);
          dq[0][dt] = mfma(kt_, bD0, dq[0][dt]);
          dq[1][dt] = mfma(kt_, bD1, dq[1][dt]);
        }
      }
  #pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int q = (2 * qp + u) * 16 + i;
        if (q < N) {
  #pragma unroll
          for (int dt = 0; dt < HD / 16; ++dt) {
            const int d = dt * 16 + 4 * g;
            if (d < hd) store4(dq_base + (long)q * rs + d, dq[u][dt], scale);
          }
        }
        if (bias_partial) add_colsums<HD>(bs_w, dq[u], scale, lane);  // padded queries: dS = 0
      }
    }

  }
  // stage 2's first key pair per wave (kp = wave) takes its K / V rows from the stage-1 images before
  // they are overwritten (rows past N are the images' zero padding): K and V of those pairs are read
  // from HBM once instead of twice; later pairs are requested from HBM one pair ahead as before
  v8bf kn[2][HD / 32], vn[2][HD / 32];  // next pair's K / V rows
  v4s kn16[2] = {}, vn16[2] = {};       // hd 80: their 16-k tails
  asm volatile("" ::: "memory");
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    // an odd image has no tile 2 npair - 1 (its keys are all padding: zeros)
    const bool in = wave < npair && 2 * wave + t < NKT;
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) {
      kn[t][kk] = in ? rd_row<HD>(ImA, (2 * wave + t) * 16, kk, lane) : v8bf{};
      vn[t][kk] = in ? rd_row<HD>(ImB, (2 * wave + t) * 16, kk, lane) : v8bf{};
    }
    if constexpr (k_tail<HD>) {
      kn16[t] = in ? rd_row16<HD>(ImA, (2 * wave + t) * 16, lane) : v4s{0, 0, 0, 0};
      vn16[t] = in ? rd_row16<HD>(ImB, (2 * wave + t) * 16, lane) : v4s{0, 0, 0, 0};
    }
  }
  A2STAMP(2);
  __syncthreads();  // K / V images no longer read; delta complete

  // ---- stage 2: dK and dV, key-tile pairs ----
  // Q, dO: only the query pairs stage 2 visits (rows past nqa read as zeros without a memory access)
  load_images<HD, NP, NW * 64>(ImA, base, rs, ImB, dob, D, min(N, 32 * npair_q), hd);
  __syncthreads();
  A2STAMP(3);
  // the last query pair may hold one wholly padded 16-row tile (N % 32 in 1..16): its S / dP
  // products are skipped (P = dS = 0 there)
  const bool last_half = (2 * npair - 1) * 16 >= N;
  // 8 waves: at most two pairs a wave at N <= 320; the pair after the first is loaded when it starts
  // (no prefetch registers)
  v8bf kf[2][HD / 32], vf[2][HD / 32];
  v4s kf16[2] = {}, vf16[2] = {};
  if constexpr (NW == 8) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk) {
        kf[t][kk] = kn[t][kk];
        vf[t][kk] = vn[t][kk];
      }
      kf16[t] = kn16[t];
      vf16[t] = vn16[t];
    }
  }
  for (int kp = wave; kp < npair; kp += NW) {
    if constexpr (NW == 4) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk) {
          kf[t][kk] = kn[t][kk];
          vf[t][kk] = vn[t][kk];
          kn[t][kk] = gl_row<HD>(base + D, rs, (2 * (kp + NW) + t) * 16, kk, N, hd, lane);
          vn[t][kk] = gl_row<HD>(base + 2 * D, rs, (2 * (kp + NW) + t) * 16, kk, N, hd, lane);
        }
    } else if (kp != wave) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk) {
          kf[t][kk] = gl_row<HD>(base + D, rs, (2 * kp + t) * 16, kk, N, hd, lane);
          vf[t][kk] = gl_row<HD>(base + 2 * D, rs, (2 * kp + t) * 16, kk, N, hd, lane);
        }
        if constexpr (k_tail<HD>) {
          kf16[t] = gl_row16<HD>(base + D, rs, (2 * kp + t) * 16, N, hd, lane);
          vf16[t] = gl_row16<HD>(base + 2 * D, rs, (2 * kp + t) * 16, N, hd, lane);
        }
      }
    }
    v4f dv[2][HD / 16], dk[2][HD / 16];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        dv[t][dt] = v4f{0.f, 0.f, 0.f, 0.f};
        dk[t][dt] = v4f{0.f, 0.f, 0.f, 0.f};
      }
    for (int qs = 0; qs < npair_q; ++qs) {
      v4f P[2][2], DS[2][2];  // [key tile][query tile]
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qt = 2 * qs + u;
        if (u == 1 && last_half && qs == npair - 1) {
          P[0][1] = P[1][1] = DS[0][1] = DS[1][1] = v4f{0.f, 0.f, 0.f, 0.f};
          continue;
        }
        v8bf qr[HD / 32], orow[HD / 32];
#pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk) {
          qr[kk] = rd_row<HD>(ImA, qt * 16, kk, lane);
          orow[kk] = rd_row<HD>(ImB, qt * 16, kk, lane);
        }
        v4s qr16 = {0, 0, 0, 0}, or16 = {0, 0, 0, 0};
        if constexpr (k_tail<HD>) {
          qr16 = rd_row16<HD>(ImA, qt * 16, lane);
          or16 = rd_row16<HD>(ImB, qt * 16, lane);
        }
        // queries 16qt + 4g + r, r = 0..3: one 16-B read each of lse and delta
        const v4f lq = *reinterpret_cast<const v4f*>(lse_s + qt * 16 + 4 * g);
        const v4f dq4 = *reinterpret_cast<const v4f*>(dlt_s + qt * 16 + 4 * g);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          v4f sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < HD / 32; ++kk) {
            sv = mfma(qr[kk], kf[t][kk], sv);
            dp = mfma(orow[kk], vf[t][kk], dp);
          }
          if constexpr (k_tail<HD>) {
            sv = mfma16_add(qr16, kf16[t], sv);
            dp = mfma16_add(or16, vf16[t], dp);
          }
          const bool kvalid = (2 * kp + t) * 16 + i < N;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = kvalid ? ex2(sv[r] * c - lq[r]) : 0.f;
            P[t][u][r] = p;
            DS[t][u][r] = p * (dp[r] - dq4[r]);
          }
        }
      }
      if (NKT % 2 == 1 && qs == npair - 1) {  // odd image: query tile 2 qs alone (a 16-k step)
        const v4s bP0 = pack4(P[0][0]), bP1 = pack4(P[1][0]);
        const v4s bD0 = pack4(DS[0][0]), bD1 = pack4(DS[1][0]);
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
          const v4s ot = rd_tr1<HD>(ImB, 2 * qs, dt * 16, lane);
          const v4s qt = rd_tr1<HD>(ImA, 2 * qs, dt * 16, lane);
          dv[0][dt] = mfma16_add(ot, bP0, dv[0][dt]);
          dv[1][dt] = mfma16_add(ot, bP1, dv[1][dt]);
          dk[0][dt] = mfma16_add(qt, bD0, dk[0][dt]);
          dk[1][dt] = mfma16_add(qt, bD1, dk[1][dt]);
        }
        continue;
      }
      const v8bf bP0 = pack8(P[0][0], P[0][1]), bP1 = pack8(P[1][0], P[1][1]);
      const v8bf bD0 = pack8(DS[0][0], DS[0][1]), bD1 = pack8(DS[1][0], DS[1][1]);
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        const v8bf ot = rd_tr<HD>(ImB, 2 * qs, 2 * qs + 1, dt * 16, lane);
        const v8bf qt = rd_tr<HD>(ImA, 2 * qs, 2 * qs + 1, dt * 16, lane);
        dv[0][dt] = mfma(ot, bP0, dv[0][dt]);
        dv[1][dt] = mfma(ot, bP1, dv[1][dt]);
        dk[0][dt] = mfma(qt, bD0, dk[0][dt]);
        dk[1][dt] = mfma(qt, bD1, dk[1][dt]);
      }
    }
    uint2 pk[2][HD / 16], pv[2][HD / 16];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        pk[t][dt] = pack4bf(dk[t][dt], scale);
        pv[t][dt] = pack4bf(dv[t][dt], 1.0f);
      }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = (2 * kp + t) * 16 + i;
      if (key < N) {
#pragma unroll
        for (int dt = 0; dt < HD / 16; ++dt) {
          const int d = dt * 16 + 4 * g;
          if (d < hd) {
            *reinterpret_cast<uint2*>(dq_base + (long)key * rs + D + d) = pk[t][dt];
            *reinterpret_cast<uint2*>(dq_base + (long)key * rs + 2 * D + d) = pv[t][dt];
          }
        }
      }
      if (bias_partial) {  // invalid keys hold exact zeros (P = 0)
        add_colsums<HD>(bs_w + HD, dk[t], scale, lane);
        add_colsums<HD>(bs_w + 2 * HD, dv[t], 1.0f, lane);
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        keep_live2(pk[t][dt]);
        keep_live2(pv[t][dt]);
      }
  }

  A2STAMP(4);
  if (bias_partial) {
    __syncthreads();
    for (int e = threadIdx.x; e < 3 * HD; e += blockDim.x) {
      const int z = e / HD, d = e % HD;
      if (d >= hd) continue;
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) acc += bsum[(w * 3 + z) * HD + d];
      bias_partial[(long)b * 3 * D + z * D + h * hd + d] = acc;
    }
  }
  A2STAMP(5);
}

template <int HD, int NKT, int NW>
hipError_t launch_fwd_nw(const bf16_t* qkv, bf16_t* o, float* lse, int B, int N, int H, int hd, float scale,
                         int nq, hipStream_t s) {
  const size_t lds = (size_t)2 * NKT * 16 * HD * 2;
  auto kern = attn_fwd_kernel<HD, NKT, NW>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(B * H), dim3(NW * 64), lds, s, qkv, o, lse, N, H, hd, scale, nq);
  return hipGetLastError();
}

template <int HD, int NKT16, int NW = 8>
hipError_t launch_fwd2(const bf16_t* qkv, bf16_t* o, float* lse, int B, int N, int H, int hd, float scale, int nq,
                       hipStream_t s) {
  const size_t lds = (size_t)2 * NKT16 * 16 * HD * 2 + (size_t)NW * StripOut<HD>::BYTES;
  auto kern = attn_fwd2_kernel<HD, NKT16, NW>;
  if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(B * H), dim3(NW * 64), lds, s, qkv, o, lse, N, H, hd, scale, nq);
  return hipGetLastError();
}

// Forward: the lean 8-wave kernel (attn_fwd2_kernel) for image widths 32, 64 and 80 (ViT-H/14's hd 80:
// one workgroup per CU); 96 on the 4-wave kernel, whose registers hold one 16-query strip at a time
template <int HD, int NKT>
hipError_t launch_fwd(const bf16_t* qkv, bf16_t* o, float* lse, int B, int N, int H, int hd, float scale,
                      int nq, hipStream_t s) {
  if constexpr (HD != 96) {  // NKT = 2 * ceil(N / 32); the lean kernel takes ceil(N / 16) tiles
    if ((N + 15) / 16 == NKT) return launch_fwd2<HD, NKT>(qkv, o, lse, B, N, H, hd, scale, nq, s);
    return launch_fwd2<HD, NKT - 1>(qkv, o, lse, B, N, H, hd, scale, nq, s);
  } else {
    return launch_fwd_nw<HD, NKT, 4>(qkv, o, lse, B, N, H, hd, scale, nq, s);
  }
}

// Backward: the two-stage kernel, 4 waves (two workgroups per CU); 80-wide images (hd 80): 8 waves and
// ceil(N / 16) tiles (97 KB at N = 257: one workgroup per CU, two waves per SIMD)
template <int HD, int NKT>
hipError_t launch_bwd1(const bf16_t* qkv, const bf16_t* dout, const float* lse, bf16_t* dqkv, float* bias_partial,
                       int B, int N, int H, int hd, float scale, int nq, hipStream_t s) {
  constexpr int NW = k_tail<HD> ? 8 : 4;
  const size_t lds = (size_t)2 * NKT * 16 * HD * 2 + 2 * NKT * 16 * 4 + (size_t)NW * 3 * HD * 4;
  auto kern = attn_bwd_kernel<HD, NKT, NW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(B * H), dim3(NW * 64), lds, s, qkv, dout, lse, dqkv, bias_partial, N, H, hd, scale, nq);
  return hipGetLastError();
}
template <int HD, int NKT>
hipError_t launch_bwd(const bf16_t* qkv, const bf16_t* dout, const float* lse, bf16_t* dqkv, float* bias_partial,
                      int B, int N, int H, int hd, float scale, int nq, hipStream_t s) {
  if constexpr (k_tail<HD>)
    if ((N + 15) / 16 < NKT) return launch_bwd1<HD, NKT - 1>(qkv, dout, lse, dqkv, bias_partial, B, N, H, hd, scale, nq, s);
  return launch_bwd1<HD, NKT>(qkv, dout, lse, dqkv, bias_partial, B, N, H, hd, scale, nq, s);
}

#define VIT_NKT_CASES(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20)

template <int HD>
hipError_t dispatch_fwd(int nkt, const bf16_t* qkv, bf16_t* o, float* lse, int B, int N, int H, int hd, float scale,
                        int nq, hipStream_t s) {
  switch (nkt) {
#define C(n) \
  case n: return launch_fwd<HD, n>(qkv, o, lse, B, N, H, hd, scale, nq, s);
    VIT_NKT_CASES(C)
#undef C
  }
  return hipErrorInvalidValue;
}
template <int HD>
hipError_t dispatch_bwd(int nkt, const bf16_t* qkv, const bf16_t* dout, const float* lse, bf16_t* dqkv,
                        float* bias_partial, int B, int N, int H, int hd, float scale, int nq, hipStream_t s) {
  switch (nkt) {
#define C(n) \
  case n: return launch_bwd<HD, n>(qkv, dout, lse, dqkv, bias_partial, B, N, H, hd, scale, nq, s);
    VIT_NKT_CASES(C)
#undef C
  }
  return hipErrorInvalidValue;
}

int check_shape(int64_t B, int64_t N, int64_t H, int64_t hd) {
  VIT_CHECK_ARG(B >= 1 && H >= 1 && N >= 1, "attention: bad sizes B=%lld N=%lld H=%lld", (long long)B, (long long)N,
                (long long)H);
  VIT_CHECK_ARG(N <= 16384 && B * H <= 0x7fffffff, "attention: N=%lld too large", (long long)N);
  VIT_CHECK_ARG(hd >= 16 && hd <= 96 && hd % 16 == 0, "attention: head_dim %lld unsupported (multiple of 16, <= 96)",
                (long long)hd);
  return VIT_OK;
}

// LDS image width: the head dim rounded up to the MFMA k-depth (32): 32, 64 or 96, except hd 80
// (ViT-H/14), whose 80-wide images take a 16-k tail step (v_mfma_f32_16x16x16_bf16).
int image_width(int64_t hd) { return hd <= 32 ? 32 : hd <= 64 ? 64 : hd == 80 ? 80 : 96; }

constexpr int64_t RESIDENT_MAX_N = 320;  // all keys of a head in LDS (attn_fwd_kernel / attn_bwd_kernel)

// 1: LDS-resident kernels, 2: K/V-tiled kernels (attention_tiled.hip); 0 picks by N; 3: the LDS-resident
// kernels in their one-workgroup-per-item forms only (no persistent forward / backward; A/B and parity checks)
constexpr int32_t PATH_ONESHOT = 3;
int resolve_path(int32_t path, int64_t N) {
  if (path == 1 || path == 2) return path;
  if (path == PATH_ONESHOT) return 1;
  return N <= RESIDENT_MAX_N ? 1 : 2;
}

}  // namespace

hipError_t vit_attn_tiled_fwd(const void* qkv, void* o, float* lse, int B, int N, int H, int hd, float scale, int nq,
                              hipStream_t s);
hipError_t vit_attn_tiled_bwd(const void* qkv, const void* dout, const float* lse, float* delta, void* dqkv,
                              float* bias_partial, int B, int N, int H, int hd, float scale, int nq, hipStream_t s);
size_t vit_attn_bwd_pers_lds(int N, int hd);
int vit_attn_bwd_pers_bias_rows();
hipError_t vit_attn_bwd_pers(const void* qkv, const void* dout, const float* lse, void* dqkv, float* bias_partial,
                             int B, int N, int H, int hd, float scale, int nq, hipStream_t s);
bool vit_attn_fwd_pers_ok(int N, int hd);
hipError_t vit_attn_fwd_pers(const void* qkv, void* o, float* lse, int B, int N, int H, int hd, float scale, int nq,
                             hipStream_t s);

extern "C" int64_t vit_attention_bias_rows(int64_t N, int64_t hd, int32_t path) {
  if (resolve_path(path, N) == 2) return (N + 63) / 64;  // one per 64-row block
  // persistent kernel: one per wave; two-stage kernel: one per image
  return path != PATH_ONESHOT && vit_attn_bwd_pers_lds((int)N, (int)hd) > 0 ? vit_attn_bwd_pers_bias_rows() : 1;
}

extern "C" int64_t vit_attention_workspace_elems(int64_t B, int64_t N, int64_t H, int32_t path) {
  (void)path;  // both paths hand delta from their dQ kernel to their dK / dV kernel
  return B * H * N;
}

extern "C" int vit_attention_fwd_ex(const void* qkv, void* o, float* lse, int64_t B, int64_t N, int64_t H, int64_t hd,
                                    float scale, int64_t q_rows, int32_t path, vit_stream_t stream) {
  int st = check_shape(B, N, H, hd);
  if (st) return st;
  VIT_CHECK_ARG(qkv && o && lse, "vit_attention_fwd: null pointer");
  VIT_CHECK_ARG(q_rows >= 1 && q_rows <= N, "vit_attention_fwd: q_rows=%lld outside [1, N]", (long long)q_rows);
  VIT_CHECK_ARG(path >= 0 && path <= 3, "vit_attention_fwd: path %d", (int)path);
  const int p = resolve_path(path, N);
  VIT_CHECK_ARG(p == 2 || N <= RESIDENT_MAX_N, "vit_attention_fwd: N=%lld > %lld on the LDS-resident path",
                (long long)N, (long long)RESIDENT_MAX_N);
  const bf16_t* q = (const bf16_t*)qkv;
  hipStream_t s = (hipStream_t)stream;
  const int nq = (int)q_rows;
  hipError_t e;
  if (p == 2) {
    e = vit_attn_tiled_fwd(qkv, o, lse, (int)B, (int)N, (int)H, (int)hd, scale, nq, s);
    return vit::check_hip(e, "vit_attention_fwd (tiled) launch");
  }
  if (path != PATH_ONESHOT && vit_attn_fwd_pers_ok((int)N, (int)hd)) {  // persistent kernel (attention_fwd_pers.hip)
    e = vit_attn_fwd_pers(qkv, o, lse, (int)B, (int)N, (int)H, (int)hd, scale, nq, s);
    return vit::check_hip(e, "vit_attention_fwd (persistent) launch");
  }
  const int nkt = (int)((N + 31) / 32) * 2;
  switch (image_width(hd)) {
    case 32: e = dispatch_fwd<32>(nkt, q, (bf16_t*)o, lse, (int)B, (int)N, (int)H, (int)hd, scale, nq, s); break;
    case 64: e = dispatch_fwd<64>(nkt, q, (bf16_t*)o, lse, (int)B, (int)N, (int)H, (int)hd, scale, nq, s); break;
    case 80: e = dispatch_fwd<80>(nkt, q, (bf16_t*)o, lse, (int)B, (int)N, (int)H, (int)hd, scale, nq, s); break;
    default: e = dispatch_fwd<96>(nkt, q, (bf16_t*)o, lse, (int)B, (int)N, (int)H, (int)hd, scale, nq, s); break;
  }
  return vit::check_hip(e, "vit_attention_fwd launch");
}

extern "C" int vit_attention_fwd_rows(const void* qkv, void* o, float* lse, int64_t B, int64_t N, int64_t H,
                                      int64_t hd, float scale, int64_t q_rows, vit_stream_t stream) {
  return vit_attention_fwd_ex(qkv, o, lse, B, N, H, hd, scale, q_rows, 0, stream);
}

extern "C" int vit_attention_fwd(const void* qkv, void* o, float* lse, int64_t B, int64_t N, int64_t H, int64_t hd,
                                 float scale, vit_stream_t stream) {
  return vit_attention_fwd_rows(qkv, o, lse, B, N, H, hd, scale, N, stream);
}

extern "C" int vit_attention_bwd_ex(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv,
                                    float* bias_partial, int64_t B, int64_t N, int64_t H, int64_t hd, float scale,
                                    int64_t q_rows, int32_t path, float* workspace, vit_stream_t stream) {
  int st = check_shape(B, N, H, hd);
  if (st) return st;
  VIT_CHECK_ARG(qkv && o && dout && lse && dqkv, "vit_attention_bwd: null pointer");
  VIT_CHECK_ARG(q_rows >= 1 && q_rows <= N, "vit_attention_bwd: q_rows=%lld outside [1, N]", (long long)q_rows);
  VIT_CHECK_ARG(path >= 0 && path <= 3, "vit_attention_bwd: path %d", (int)path);
  const int p = resolve_path(path, N);
  VIT_CHECK_ARG(p == 2 || N <= RESIDENT_MAX_N, "vit_attention_bwd: N=%lld > %lld on the LDS-resident path",
                (long long)N, (long long)RESIDENT_MAX_N);
  hipStream_t s = (hipStream_t)stream;
  const int nq = (int)q_rows;
  hipError_t e;
  if (p == 2) {
    VIT_CHECK_ARG(workspace, "vit_attention_bwd: the tiled path (N=%lld) needs a workspace of "
                  "vit_attention_workspace_elems() floats", (long long)N);
    e = vit_attn_tiled_bwd(qkv, dout, lse, workspace, dqkv, bias_partial, (int)B, (int)N, (int)H, (int)hd, scale, nq,
                           s);
    return vit::check_hip(e, "vit_attention_bwd (tiled) launch");
  }
  if (path != PATH_ONESHOT && vit_attn_bwd_pers_lds((int)N, (int)hd) > 0) {  // persistent kernel (attention_bwd.hip)
    e = vit_attn_bwd_pers(qkv, dout, lse, dqkv, bias_partial, (int)B, (int)N, (int)H, (int)hd, scale, nq, s);
    return vit::check_hip(e, "vit_attention_bwd (persistent) launch");
  }
  const int nkt = (int)((N + 31) / 32) * 2;
  const bf16_t *q = (const bf16_t*)qkv, *d = (const bf16_t*)dout;
  switch (image_width(hd)) {
    case 32:
      e = dispatch_bwd<32>(nkt, q, d, lse, (bf16_t*)dqkv, bias_partial, (int)B, (int)N, (int)H, (int)hd, scale, nq, s);
      break;
    case 64:
      e = dispatch_bwd<64>(nkt, q, d, lse, (bf16_t*)dqkv, bias_partial, (int)B, (int)N, (int)H, (int)hd, scale, nq, s);
      break;
    case 80:
      e = dispatch_bwd<80>(nkt, q, d, lse, (bf16_t*)dqkv, bias_partial, (int)B, (int)N, (int)H, (int)hd, scale, nq, s);
      break;
    default:
      e = dispatch_bwd<96>(nkt, q, d, lse, (bf16_t*)dqkv, bias_partial, (int)B, (int)N, (int)H, (int)hd, scale, nq, s);
      break;
  }
  return vit::check_hip(e, "vit_attention_bwd launch");
}

extern "C" int vit_attention_bwd_rows(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv,
                                      float* bias_partial, int64_t B, int64_t N, int64_t H, int64_t hd, float scale,
                                      int64_t q_rows, vit_stream_t stream) {
  return vit_attention_bwd_ex(qkv, o, dout, lse, dqkv, bias_partial, B, N, H, hd, scale, q_rows, 0, nullptr, stream);
}

extern "C" int vit_attention_bwd(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv,
                                 float* bias_partial, int64_t B, int64_t N, int64_t H, int64_t hd, float scale,
                                 vit_stream_t stream) {
  return vit_attention_bwd_rows(qkv, o, dout, lse, dqkv, bias_partial, B, N, H, hd, scale, N, stream);
}

// ---- fp32 (exact) attention forward -------------------------------------------------------------
// The reference's SelfAttention core (src/model.py:90-97) in f32 operands and f32 accumulation, for
// the exact-parity forward (no bf16 anywhere): one query row per thread, keys streamed through LDS in
// chunks of 32 with an online softmax; S = (q . k) / sqrt(hd), as the reference divides after the
// matmul. qkv f32 [B*N, 3, H, hd] -> o f32 [B*N, H, hd].
namespace {
template <int HD>
__global__ void __launch_bounds__(256) attn_fwd_f32_kernel(const float* __restrict__ qkv, float* __restrict__ o, int N,
                                                           int H, int hd, float inv_sqrt) {
  constexpr int KC = 32;
  __shared__ float Ks[KC][HD + 1], Vs[KC][HD + 1];
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * hd;
  const long rs = 3L * D;
  const float* base = qkv + (long)b * N * rs + (long)h * hd;
  const int qi = blockIdx.y * 256 + threadIdx.x;
  const bool valid = qi < N;
  float q[HD], acc[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) {
    q[d] = (valid && d < hd) ? base[(long)qi * rs + d] : 0.f;
    acc[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < N; k0 += KC) {
    __syncthreads();
    for (int e = threadIdx.x; e < KC * HD; e += 256) {
      const int j = e / HD, d = e % HD;
      const bool ok = k0 + j < N && d < hd;
      Ks[j][d] = ok ? base[(long)(k0 + j) * rs + D + d] : 0.f;
      Vs[j][d] = ok ? base[(long)(k0 + j) * rs + 2 * D + d] : 0.f;
    }
    __syncthreads();
    float s[KC];
    float cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      float dot = 0.f;
#pragma unroll
      for (int d = 0; d < HD; ++d) dot = fmaf(q[d], Ks[j][d], dot);
      s[j] = k0 + j < N ? dot * inv_sqrt : -INFINITY;
      cm = fmaxf(cm, s[j]);
    }
    const float mn = fmaxf(m, cm);
    const float corr = expf(m - mn);
    l *= corr;
#pragma unroll
    for (int d = 0; d < HD; ++d) acc[d] *= corr;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const float p = expf(s[j] - mn);
      l += p;
#pragma unroll
      for (int d = 0; d < HD; ++d) acc[d] = fmaf(p, Vs[j][d], acc[d]);
    }
    m = mn;
  }
  if (valid) {
    const float inv = 1.0f / l;
    float* dst = o + ((long)b * N + qi) * D + (long)h * hd;
#pragma unroll
    for (int d = 0; d < HD; ++d)
      if (d < hd) dst[d] = acc[d] * inv;
  }
}
}  // namespace

extern "C" int vit_attention_fwd_f32(const float* qkv, float* o, int64_t B, int64_t N, int64_t H, int64_t hd,
                                     float inv_sqrt_hd, vit_stream_t stream) {
  VIT_CHECK_ARG(qkv && o && B >= 1 && N >= 1 && H >= 1 && hd >= 1 && hd <= 96, "vit_attention_fwd_f32: bad args");
  dim3 grid((unsigned)(B * H), (unsigned)((N + 255) / 256));
  hipStream_t s = (hipStream_t)stream;
  if (hd <= 32)
    hipLaunchKernelGGL(attn_fwd_f32_kernel<32>, grid, dim3(256), 0, s, qkv, o, (int)N, (int)H, (int)hd, inv_sqrt_hd);
  else if (hd <= 64)
    hipLaunchKernelGGL(attn_fwd_f32_kernel<64>, grid, dim3(256), 0, s, qkv, o, (int)N, (int)H, (int)hd, inv_sqrt_hd);
  else
    hipLaunchKernelGGL(attn_fwd_f32_kernel<96>, grid, dim3(256), 0, s, qkv, o, (int)N, (int)H, (int)hd, inv_sqrt_hd);
  return vit::check_hip(hipGetLastError(), "vit_attention_fwd_f32");
}
