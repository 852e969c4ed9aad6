// K/V-tiled multi-head self-attention for sequences longer than the LDS-resident kernels take
// (N > 320: ViT-B/16 and L/16 at 384 px have 577 tokens, H/14 at 384 px 730; src/config.py:12,37).
//
// Same math and the same operands / outputs as attention.hip (reference SelfAttention core,
// src/model.py:90-97: q @ k^T, / sqrt(hd), softmax(-1), @ v), but no kernel needs a whole head's
// keys on chip:
//   fwd   one workgroup per (image, head, 64-query block); 64-key blocks of K and V stream through
//         a double-buffered LDS ring (register-staged: the next block's loads are in flight during
//         the current block's MFMAs), online softmax with the running max / sum per query row.
//   bwd   two kernels, deterministic (no atomics):
//         dq    per (image, head, 64-query block): pass 1 over the key blocks accumulates
//               delta_q = sum_j P_qj dP_qj exactly (from the recomputed P and dP, not from the bf16 O;
//               see attention.hip), pass 2 recomputes S, dP and accumulates dQ = dS K. Writes delta.
//         dkdv  per (image, head, 64-key block): K / V rows in registers, 64-query blocks of Q, dO,
//               lse, delta streamed through LDS; dV = P^T dO, dK = dS^T Q.
// Bias-gradient partials (optional): per (image, 64-row block) column sums of dQ | dK | dV,
// bias_partial[(b * nblk + blk) * 3D + ...], nblk = ceil(N / 64) (vit_attention_bias_rows).
// MFMA fragment conventions and LDS images: attn_common.h.
#include "attn_common.h"

namespace {
using namespace vit_attn;

constexpr int BLK = 64;  // rows of every streamed block (keys or queries) and of every workgroup's own block

// Register-staged copy of rows [row0, row0 + BLK) x [0, HD) of two strided bf16 matrices into two LDS
// images (rows >= N and columns >= hd read as zero through the buffer descriptors' bounds).
template <int HD, int NT>
struct Stage2 {
  static constexpr int CPR = HD / 8;
  static constexpr int TOTAL = BLK * CPR;
  static constexpr int PER = (TOTAL + NT - 1) / NT;
  v4u a[PER], b[PER];

  __device__ __forceinline__ void issue(const bf16_t* srcA, long strideA, const bf16_t* srcB, long strideB, int row0,
                                        int N, int hd) {
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(srcA, (uint32_t)(((long)(N - 1) * strideA + hd) * 2));
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(srcB, (uint32_t)(((long)(N - 1) * strideB + hd) * 2));
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = threadIdx.x + k * NT;
      const int row = row0 + c / CPR, ch = c % CPR;
      const bool ok = c < TOTAL && row < N && ch * 8 < hd;
      const int offa = ok ? (int)(((long)row * strideA + ch * 8) * 2) : 0x7ffffff0;
      const int offb = ok ? (int)(((long)row * strideB + ch * 8) * 2) : 0x7ffffff0;
      a[k] = __builtin_amdgcn_raw_buffer_load_b128(ra, offa, 0, 0);
      b[k] = __builtin_amdgcn_raw_buffer_load_b128(rb, offb, 0, 0);
    }
  }
  __device__ __forceinline__ void write(char* imgA, char* imgB) const {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = threadIdx.x + k * NT;
      if (c < TOTAL) {
        const int row = c / CPR, ch = c % CPR;
        *reinterpret_cast<v4u*>(imgA + img_off<HD>(row, ch)) = a[k];
        *reinterpret_cast<v4u*>(imgB + img_off<HD>(row, ch)) = b[k];
      }
    }
  }
};

// ---- forward ------------------------------------------------------------------------------------
template <int HD, int NW>
__global__ void __launch_bounds__(NW * 64) attn_fwd_tiled_kernel(const bf16_t* __restrict__ qkv,
                                                                 bf16_t* __restrict__ o, float* __restrict__ lse,
                                                                 int N, int H, int hd, float scale) {
  static_assert(NW * 16 == BLK, "one 16-query strip per wave");
  constexpr int IMG = BLK * HD * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [2 buffers][K image, V image]
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * hd;
  const long rs = 3L * D;
  const bf16_t* base = qkv + (long)b * N * rs + (long)h * hd;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int q0 = blockIdx.y * BLK + wave * 16;
  v8bf qf[HD / 32];
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) qf[kk] = gl_row<HD>(base, rs, q0, kk, N, hd, lane);

  const int nkb = (N + BLK - 1) / BLK;
  Stage2<HD, NW * 64> st;
  st.issue(base + D, rs, base + 2 * D, rs, 0, N, hd);
  st.write(smem, smem + IMG);
  __syncthreads();

  const float c = scale * LOG2E;
  float m = -INFINITY, l = 0.f;  // running max (raw score units) and this lane's partial sum
  v4f oacc[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) oacc[dt] = v4f{0.f, 0.f, 0.f, 0.f};

  for (int j = 0; j < nkb; ++j) {
    if (j + 1 < nkb) st.issue(base + D, rs, base + 2 * D, rs, (j + 1) * BLK, N, hd);
    const char* Ki = smem + (j & 1) * 2 * IMG;
    const char* Vi = Ki + IMG;
    v4f s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk) s[kt] = mfma(rd_row<HD>(Ki, kt * 16, kk, lane), qf[kk], s[kt]);
    }
    if ((j + 1) * BLK > N) {  // the last block: keys >= N take no weight
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (j * BLK + kt * 16 + 4 * g + r >= N) s[kt][r] = -INFINITY;
    }
    float mx = fmaxf(fmaxf(fmaxf(s[0][0], s[0][1]), fmaxf(s[0][2], s[0][3])),
                     fmaxf(fmaxf(s[1][0], s[1][1]), fmaxf(s[1][2], s[1][3])));
    mx = fmaxf(mx, fmaxf(fmaxf(fmaxf(s[2][0], s[2][1]), fmaxf(s[2][2], s[2][3])),
                         fmaxf(fmaxf(s[3][0], s[3][1]), fmaxf(s[3][2], s[3][3]))));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);  // finite: every block holds at least one valid key
    const float alpha = ex2((m - mn) * c);
    m = mn;
    const float mc = mn * c;
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) oacc[dt] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = ex2(fmaf(s[kt][r], c, -mc));
        s[kt][r] = p;
        l += p;
      }
    const v8bf p01 = pack8(s[0], s[1]), p23 = pack8(s[2], s[3]);
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      oacc[dt] = mfma(rd_tr<HD>(Vi, 0, 1, dt * 16, lane), p01, oacc[dt]);
      oacc[dt] = mfma(rd_tr<HD>(Vi, 2, 3, dt * 16, lane), p23, oacc[dt]);
    }
    if (j + 1 < nkb) st.write(smem + ((j + 1) & 1) * 2 * IMG, smem + ((j + 1) & 1) * 2 * IMG + IMG);
    __syncthreads();
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const int q = q0 + i;
  if (q < N) {
    if (g == 0) lse[(long)bh * N + q] = m * scale + logf(l);
    const float inv_l = 1.0f / l;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      const int d = dt * 16 + 4 * g;
      if (d < hd) store4(o + ((long)b * N + q) * D + (long)h * hd + d, oacc[dt], inv_l);
    }
  }
}

// ---- backward: dQ (and delta) ---------------------------------------------------------------------
template <int HD, int NW>
__global__ void __launch_bounds__(NW * 64) attn_bwd_dq_tiled_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    bf16_t* __restrict__ dqkv, float* __restrict__ delta, float* __restrict__ bias_partial, int N, int H, int hd,
    float scale, int nq_blocks) {
  constexpr int IMG = BLK * HD * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [2][K, V] + bias scratch [NW][HD]
  float* bsum = reinterpret_cast<float*>(smem + 4 * IMG);
  const int bh = blockIdx.x, b = bh / H, h = bh % H, qb = blockIdx.y;
  const int D = H * hd;
  const long rs = 3L * D;
  const int nblk = (N + BLK - 1) / BLK;
  const bf16_t* base = qkv + (long)b * N * rs + (long)h * hd;
  const bf16_t* dob = dout + (long)b * N * D + (long)h * hd;
  bf16_t* dq_base = dqkv + (long)b * N * rs + (long)h * hd;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int q = qb * BLK + wave * 16 + i;
  const float c = scale * LOG2E;

  if (qb >= nq_blocks) {  // no gradient reaches these queries (the last layer's pruned rows): dQ = 0
    if (q < N) {
      if (g == 0) delta[(long)bh * N + q] = 0.f;
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        const int d = dt * 16 + 4 * g;
        if (d < hd) store4(dq_base + (long)q * rs + d, v4f{0.f, 0.f, 0.f, 0.f}, 1.f);
      }
    }
    if (bias_partial)
      for (int d = threadIdx.x; d < hd; d += NW * 64) bias_partial[((long)b * nblk + qb) * 3 * D + h * hd + d] = 0.f;
    return;
  }

  v8bf qf[HD / 32], df[HD / 32];
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) {
    qf[kk] = gl_row<HD>(base, rs, qb * BLK + wave * 16, kk, N, hd, lane);
    df[kk] = gl_row<HD>(dob, D, qb * BLK + wave * 16, kk, N, hd, lane);
  }
  const float ls = q < N ? lse[(long)bh * N + q] * LOG2E : INFINITY;  // padded queries: P = 0

  Stage2<HD, NW * 64> st;
  st.issue(base + D, rs, base + 2 * D, rs, 0, N, hd);
  st.write(smem, smem + IMG);
  __syncthreads();

  float dl = 0.f;
  v4f dq[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) dq[dt] = v4f{0.f, 0.f, 0.f, 0.f};
  // iterations [0, nblk): pass 1 (delta); [nblk, 2 nblk): pass 2 (dS, dQ), over the same key blocks
  for (int it = 0; it < 2 * nblk; ++it) {
    const int j = it < nblk ? it : it - nblk;
    if (it + 1 < 2 * nblk) {
      const int jn = it + 1 < nblk ? it + 1 : it + 1 - nblk;
      st.issue(base + D, rs, base + 2 * D, rs, jn * BLK, N, hd);
    }
    if (it == nblk) {  // delta complete (every lane of a query holds a partial over its key rows)
      dl += __shfl_xor(dl, 16, 64);
      dl += __shfl_xor(dl, 32, 64);
    }
    const char* Ki = smem + (it & 1) * 2 * IMG;
    const char* Vi = Ki + IMG;
    v4f P[4], DP[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      v4f sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk) {
        sv = mfma(rd_row<HD>(Ki, kt * 16, kk, lane), qf[kk], sv);
        dp = mfma(rd_row<HD>(Vi, kt * 16, kk, lane), df[kk], dp);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) P[kt][r] = ex2(fmaf(sv[r], c, -ls));
      DP[kt] = dp;
    }
    if ((j + 1) * BLK > N) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (j * BLK + kt * 16 + 4 * g + r >= N) P[kt][r] = 0.f;
    }
    if (it < nblk) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) dl = fmaf(P[kt][r], DP[kt][r], dl);
    } else {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) P[kt][r] *= DP[kt][r] - dl;  // dS
      const v8bf d01 = pack8(P[0], P[1]), d23 = pack8(P[2], P[3]);
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        dq[dt] = mfma(rd_tr<HD>(Ki, 0, 1, dt * 16, lane), d01, dq[dt]);
        dq[dt] = mfma(rd_tr<HD>(Ki, 2, 3, dt * 16, lane), d23, dq[dt]);
      }
    }
    if (it + 1 < 2 * nblk) st.write(smem + ((it + 1) & 1) * 2 * IMG, smem + ((it + 1) & 1) * 2 * IMG + IMG);
    __syncthreads();
  }
  if (q < N) {
    if (g == 0) delta[(long)bh * N + q] = dl;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      const int d = dt * 16 + 4 * g;
      if (d < hd) store4(dq_base + (long)q * rs + d, dq[dt], scale);
    }
  }
  if (bias_partial) {  // padded queries hold dS = 0, so their dQ is exactly zero
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sum16(dq[dt][r]);
        if (i == 0) bsum[wave * HD + dt * 16 + 4 * g + r] = v * scale;
      }
    __syncthreads();
    for (int d = threadIdx.x; d < hd; d += NW * 64) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) acc += bsum[w * HD + d];
      bias_partial[((long)b * nblk + qb) * 3 * D + h * hd + d] = acc;
    }
  }
}

// ---- backward: dK, dV --------------------------------------------------------------------------
template <int HD, int NW>
__global__ void __launch_bounds__(NW * 64) attn_bwd_dkdv_tiled_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dqkv, float* __restrict__ bias_partial, int N, int H,
    int hd, float scale, int nq_blocks) {
  static_assert(NW * 16 == BLK, "one 16-key tile per wave");
  constexpr int IMG = BLK * HD * 2;
  constexpr int BUF = 2 * IMG + 2 * BLK * 4;  // Q image, dO image, lse, delta
  extern __shared__ __attribute__((aligned(16))) char smem[];  // [2][BUF] + bias scratch [NW][2][HD]
  float* bsum = reinterpret_cast<float*>(smem + 2 * BUF);
  const int bh = blockIdx.x, b = bh / H, h = bh % H, kb = blockIdx.y;
  const int D = H * hd;
  const long rs = 3L * D;
  const int nblk = (N + BLK - 1) / BLK;
  const bf16_t* base = qkv + (long)b * N * rs + (long)h * hd;
  const bf16_t* dob = dout + (long)b * N * D + (long)h * hd;
  bf16_t* dk_base = dqkv + (long)b * N * rs + (long)h * hd + D;
  const float* lse_bh = lse + (long)bh * N;
  const float* dlt_bh = delta + (long)bh * N;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int k0 = kb * BLK + wave * 16;
  const float c = scale * LOG2E;
  v8bf kf[HD / 32], vf[HD / 32];
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) {
    kf[kk] = gl_row<HD>(base + D, rs, k0, kk, N, hd, lane);
    vf[kk] = gl_row<HD>(base + 2 * D, rs, k0, kk, N, hd, lane);
  }
  const bool kvalid = k0 + i < N;

  Stage2<HD, NW * 64> st;
  float rowv = 0.f;  // thread t < 64: lse(q0 + t) * log2e; 64 <= t < 128: delta(q0 + t - 64)
  auto issue_rows = [&](int blk) {
    st.issue(base, rs, dob, D, blk * BLK, N, hd);
    const int t = threadIdx.x;
    if (t < 2 * BLK) {
      const int qq = blk * BLK + (t & (BLK - 1));
      rowv = t < BLK ? (qq < N ? lse_bh[qq] * LOG2E : INFINITY) : (qq < N ? dlt_bh[qq] : 0.f);
    }
  };
  auto write_rows = [&](char* buf) {
    st.write(buf, buf + IMG);
    if (threadIdx.x < 2 * BLK) reinterpret_cast<float*>(buf + 2 * IMG)[threadIdx.x] = rowv;
  };
  issue_rows(0);
  write_rows(smem);
  __syncthreads();

  v4f dv[HD / 16], dk[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) dv[dt] = dk[dt] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < nq_blocks; ++j) {
    if (j + 1 < nq_blocks) issue_rows(j + 1);
    const char* Qi = smem + (j & 1) * BUF;
    const char* Oi = Qi + IMG;
    const float* lse_s = reinterpret_cast<const float*>(Qi + 2 * IMG);
    const float* dlt_s = lse_s + BLK;
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      v4f P[2], DS[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qt = 2 * qs + u;
        v4f sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk) {
          sv = mfma(rd_row<HD>(Qi, qt * 16, kk, lane), kf[kk], sv);
          dp = mfma(rd_row<HD>(Oi, qt * 16, kk, lane), vf[kk], dp);
        }
        const v4f lq = *reinterpret_cast<const v4f*>(lse_s + qt * 16 + 4 * g);
        const v4f dq4 = *reinterpret_cast<const v4f*>(dlt_s + qt * 16 + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = kvalid ? ex2(fmaf(sv[r], c, -lq[r])) : 0.f;
          P[u][r] = p;
          DS[u][r] = p * (dp[r] - dq4[r]);
        }
      }
      const v8bf bP = pack8(P[0], P[1]), bD = pack8(DS[0], DS[1]);
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        dv[dt] = mfma(rd_tr<HD>(Oi, 2 * qs, 2 * qs + 1, dt * 16, lane), bP, dv[dt]);
        dk[dt] = mfma(rd_tr<HD>(Qi, 2 * qs, 2 * qs + 1, dt * 16, lane), bD, dk[dt]);
      }
    }
    if (j + 1 < nq_blocks) write_rows(smem + ((j + 1) & 1) * BUF);
    __syncthreads();
  }
  if (kvalid) {
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      const int d = dt * 16 + 4 * g;
      if (d < hd) {
        store4(dk_base + (long)(k0 + i) * rs + d, dk[dt], scale);
        store4(dk_base + (long)(k0 + i) * rs + D + d, dv[dt], 1.0f);
      }
    }
  }
  if (bias_partial) {  // invalid keys hold exact zeros (P = dS = 0)
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = sum16(dk[dt][r]), v = sum16(dv[dt][r]);
        if (i == 0) {
          bsum[(wave * 2 + 0) * HD + dt * 16 + 4 * g + r] = a * scale;
          bsum[(wave * 2 + 1) * HD + dt * 16 + 4 * g + r] = v;
        }
      }
    __syncthreads();
    for (int e = threadIdx.x; e < 2 * HD; e += NW * 64) {
      const int z = e / HD, d = e % HD;
      if (d >= hd) continue;
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) acc += bsum[(w * 2 + z) * HD + d];
      bias_partial[((long)b * nblk + kb) * 3 * D + (1 + z) * D + h * hd + d] = acc;
    }
  }
}

// ---- forward, ragged queries (Res-ViT inference, res-vit/model.py:494-529) ------------------------
// Sample b's queries are rows [cu_q[b], cu_q[b+1]) of q (its active tokens, any count), its keys and
// values rows [b * Nkv, (b+1) * Nkv) of k / v (all tokens). One launch replaces the reference's
// per-sample loop of asymmetric attention calls; same online-softmax body as attn_fwd_tiled_kernel.
template <int HD, int NW>
__global__ void __launch_bounds__(NW * 64) attn_fwd_varlen_kernel(
    const bf16_t* __restrict__ q, long ldq, const bf16_t* __restrict__ k, long ldk, const bf16_t* __restrict__ v,
    long ldv, bf16_t* __restrict__ o, long ldo, const int* __restrict__ cu_q, int Nkv, int H, int hd, float scale) {
  static_assert(NW * 16 == BLK, "one 16-query strip per wave");
  constexpr int IMG = BLK * HD * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int qs = cu_q[b], nqb = cu_q[b + 1] - qs;
  if ((int)blockIdx.y * BLK >= nqb) return;  // uniform over the workgroup
  const bf16_t* qb = q + (long)qs * ldq + (long)h * hd;
  const bf16_t* kb = k + (long)b * Nkv * ldk + (long)h * hd;
  const bf16_t* vb = v + (long)b * Nkv * ldv + (long)h * hd;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const int q0 = blockIdx.y * BLK + wave * 16;
  v8bf qf[HD / 32];
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) qf[kk] = gl_row<HD>(qb, ldq, q0, kk, nqb, hd, lane);
  const int nkb = (Nkv + BLK - 1) / BLK;
  Stage2<HD, NW * 64> st;
  st.issue(kb, ldk, vb, ldv, 0, Nkv, hd);
  st.write(smem, smem + IMG);
  __syncthreads();
  const float c = scale * LOG2E;
  float m = -INFINITY, l = 0.f;
  v4f oacc[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) oacc[dt] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < nkb; ++j) {
    if (j + 1 < nkb) st.issue(kb, ldk, vb, ldv, (j + 1) * BLK, Nkv, hd);
    const char* Ki = smem + (j & 1) * 2 * IMG;
    const char* Vi = Ki + IMG;
    v4f s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk) s[kt] = mfma(rd_row<HD>(Ki, kt * 16, kk, lane), qf[kk], s[kt]);
    }
    if ((j + 1) * BLK > Nkv) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (j * BLK + kt * 16 + 4 * g + r >= Nkv) s[kt][r] = -INFINITY;
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) mx = fmaxf(mx, fmaxf(fmaxf(s[kt][0], s[kt][1]), fmaxf(s[kt][2], s[kt][3])));
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = ex2((m - mn) * c);
    m = mn;
    const float mc = mn * c;
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) oacc[dt] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = ex2(fmaf(s[kt][r], c, -mc));
        s[kt][r] = p;
        l += p;
      }
    const v8bf p01 = pack8(s[0], s[1]), p23 = pack8(s[2], s[3]);
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      oacc[dt] = mfma(rd_tr<HD>(Vi, 0, 1, dt * 16, lane), p01, oacc[dt]);
      oacc[dt] = mfma(rd_tr<HD>(Vi, 2, 3, dt * 16, lane), p23, oacc[dt]);
    }
    if (j + 1 < nkb) st.write(smem + ((j + 1) & 1) * 2 * IMG, smem + ((j + 1) & 1) * 2 * IMG + IMG);
    __syncthreads();
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const int qq = q0 + i;
  if (qq < nqb) {
    const float inv_l = 1.0f / l;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      const int d = dt * 16 + 4 * g;
      if (d < hd) store4(o + (long)(qs + qq) * ldo + (long)h * hd + d, oacc[dt], inv_l);
    }
  }
}

constexpr int NWT = BLK / 16;  // 4 waves per workgroup

template <int HD>
hipError_t launch_tiled_fwd(const bf16_t* qkv, bf16_t* o, float* lse, int B, int N, int H, int hd, float scale,
                            int nq, hipStream_t s) {
  const size_t lds = (size_t)4 * BLK * HD * 2;
  const int nqb = (nq + BLK - 1) / BLK;
  hipLaunchKernelGGL((attn_fwd_tiled_kernel<HD, NWT>), dim3(B * H, nqb), dim3(NWT * 64), lds, s, qkv, o, lse, N, H,
                     hd, scale);
  return hipGetLastError();
}

template <int HD>
hipError_t launch_tiled_bwd(const bf16_t* qkv, const bf16_t* dout, const float* lse, float* delta, bf16_t* dqkv,
                            float* bias_partial, int B, int N, int H, int hd, float scale, int nq, hipStream_t s) {
  const int nblk = (N + BLK - 1) / BLK;
  const int nqb = (nq + BLK - 1) / BLK;  // query blocks that carry a gradient
  const size_t lds_dq = (size_t)4 * BLK * HD * 2 + (size_t)NWT * HD * 4;
  hipLaunchKernelGGL((attn_bwd_dq_tiled_kernel<HD, NWT>), dim3(B * H, nblk), dim3(NWT * 64), lds_dq, s, qkv, dout,
                     lse, dqkv, delta, bias_partial, N, H, hd, scale, nqb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t lds_kv = (size_t)2 * (2 * BLK * HD * 2 + 2 * BLK * 4) + (size_t)NWT * 2 * HD * 4;
  hipLaunchKernelGGL((attn_bwd_dkdv_tiled_kernel<HD, NWT>), dim3(B * H, nblk), dim3(NWT * 64), lds_kv, s, qkv, dout,
                     lse, delta, dqkv, bias_partial, N, H, hd, scale, nqb);
  return hipGetLastError();
}

}  // namespace

// Entry points used by attention.hip's dispatch (path selection lives there).
hipError_t vit_attn_tiled_fwd(const void* qkv, void* o, float* lse, int B, int N, int H, int hd, float scale, int nq,
                              hipStream_t s) {
  const bf16_t* q = (const bf16_t*)qkv;
  if (hd <= 32) return launch_tiled_fwd<32>(q, (bf16_t*)o, lse, B, N, H, hd, scale, nq, s);
  if (hd <= 64) return launch_tiled_fwd<64>(q, (bf16_t*)o, lse, B, N, H, hd, scale, nq, s);
  return launch_tiled_fwd<96>(q, (bf16_t*)o, lse, B, N, H, hd, scale, nq, s);
}

hipError_t vit_attn_tiled_bwd(const void* qkv, const void* dout, const float* lse, float* delta, void* dqkv,
                              float* bias_partial, int B, int N, int H, int hd, float scale, int nq, hipStream_t s) {
  const bf16_t *q = (const bf16_t*)qkv, *d = (const bf16_t*)dout;
  if (hd <= 32) return launch_tiled_bwd<32>(q, d, lse, delta, (bf16_t*)dqkv, bias_partial, B, N, H, hd, scale, nq, s);
  if (hd <= 64) return launch_tiled_bwd<64>(q, d, lse, delta, (bf16_t*)dqkv, bias_partial, B, N, H, hd, scale, nq, s);
  return launch_tiled_bwd<96>(q, d, lse, delta, (bf16_t*)dqkv, bias_partial, B, N, H, hd, scale, nq, s);
}

hipError_t vit_attn_varlen_fwd(const void* q, long ldq, const void* k, long ldk, const void* v, long ldv, void* o,
                               long ldo, const int* cu_q, int B, int max_q, int Nkv, int H, int hd, float scale,
                               hipStream_t s) {
  const dim3 grid(B * H, (max_q + BLK - 1) / BLK);
  const auto* qq = (const bf16_t*)q;
  const auto* kk = (const bf16_t*)k;
  const auto* vv = (const bf16_t*)v;
  auto* oo = (bf16_t*)o;
  if (hd <= 32)
    hipLaunchKernelGGL((attn_fwd_varlen_kernel<32, NWT>), grid, dim3(NWT * 64), (size_t)4 * BLK * 32 * 2, s, qq, ldq, kk,
                       ldk, vv, ldv, oo, ldo, cu_q, Nkv, H, hd, scale);
  else if (hd <= 64)
    hipLaunchKernelGGL((attn_fwd_varlen_kernel<64, NWT>), grid, dim3(NWT * 64), (size_t)4 * BLK * 64 * 2, s, qq, ldq, kk,
                       ldk, vv, ldv, oo, ldo, cu_q, Nkv, H, hd, scale);
  else
    hipLaunchKernelGGL((attn_fwd_varlen_kernel<96, NWT>), grid, dim3(NWT * 64), (size_t)4 * BLK * 96 * 2, s, qq, ldq, kk,
                       ldk, vv, ldv, oo, ldo, cu_q, Nkv, H, hd, scale);
  return hipGetLastError();
}

extern "C" int vit_attention_fwd_varlen(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                                        int64_t ldv, void* o, int64_t ldo, const int32_t* cu_q, int64_t B,
                                        int64_t max_q, int64_t Nkv, int64_t H, int64_t hd, float scale,
                                        vit_stream_t stream) {
  VIT_CHECK_ARG(q && k && v && o && cu_q && B >= 1 && H >= 1 && Nkv >= 1 && max_q >= 0,
                "vit_attention_fwd_varlen: bad args");
  VIT_CHECK_ARG(hd >= 16 && hd <= 96 && hd % 16 == 0, "vit_attention_fwd_varlen: head_dim %lld unsupported",
                (long long)hd);
  VIT_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0,
                "vit_attention_fwd_varlen: row strides must keep 16-B (q/k/v) and 8-B (o) alignment");
  if (max_q == 0) return VIT_OK;
  return vit::check_hip(vit_attn_varlen_fwd(q, ldq, k, ldk, v, ldv, o, ldo, cu_q, (int)B, (int)max_q, (int)Nkv,
                                            (int)H, (int)hd, scale, (hipStream_t)stream),
                        "vit_attention_fwd_varlen launch");
}
