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
//   bwd: phase 1, each wave owns 16-key tiles: recompute P (key on the lane), dP, dS and
//        accumulate dV^T, dK^T in registers over all queries. phase 2, each wave owns 16-query
//        tiles: recompute S^T, dP^T and accumulate dQ^T. No atomics, deterministic.
// LDS images: [rows][HD] bf16 with a 16-B-chunk XOR swizzle that is conflict-free for both the
// row read (ds_read_b128) and the transposed read (ds_read_b64_tr_b16) at HD = 64.
#include "common.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;

template <int HD>
__device__ __forceinline__ int aswz(int row) {
  if constexpr (HD == 64) return ((row >> 1) & 3) << 1;
  return 0;
}

template <int HD>
__device__ __forceinline__ int img_off(int row, int chunk) {
  return row * HD * 2 + ((chunk ^ aswz<HD>(row)) << 4);
}

// Load rows [0, NP) x [0, HD) of a strided bf16 matrix into a swizzled LDS image (zero padded).
template <int HD>
__device__ __forceinline__ void load_image(char* img, const bf16_t* __restrict__ src, long row_stride, int N, int hd,
                                           int NP) {
  constexpr int CPR = HD / 8;
  const int total = NP * CPR;
  for (int c = threadIdx.x; c < total; c += blockDim.x) {
    const int row = c / CPR, ch = c % CPR;
    v8s v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (row < N && ch * 8 < hd) v = *reinterpret_cast<const v8s*>(src + (long)row * row_stride + ch * 8);
    *reinterpret_cast<v8s*>(img + img_off<HD>(row, ch)) = v;
  }
}

// 16 rows x 32 k fragment: lane holds row r0 + (lane&15), k = kk*32 + 8*(lane>>4) + j.
template <int HD>
__device__ __forceinline__ v8bf rd_row(const char* img, int r0, int kk, int lane) {
  const int row = r0 + (lane & 15);
  const int ch = kk * 4 + (lane >> 4);
  return __builtin_bit_cast(v8bf, *reinterpret_cast<const v8s*>(img + img_off<HD>(row, ch)));
}

// Transposed fragment: lane (g, i) gets column d0+i of image rows {16ta+4g+0..3, 16tb+4g+0..3}.
template <int HD>
__device__ __forceinline__ v8bf rd_tr(const char* img, int ta, int tb, int d0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int colb = (d0 + 4 * p) * 2;
  const int ch = colb >> 4, within = colb & 15;
  const int ra = 16 * ta + 4 * g + q, rb = 16 * tb + 4 * g + q;
  v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, img + img_off<HD>(ra, ch) + within));
  v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(v4s, img + img_off<HD>(rb, ch) + within));
  v8s r;
  r.lo = lo;
  r.hi = hi;
  return __builtin_bit_cast(v8bf, r);
}

__device__ __forceinline__ v8bf pack8(const v4f& a, const v4f& b) {
  v8s r;
  r[0] = (short)f2bf(a[0]); r[1] = (short)f2bf(a[1]); r[2] = (short)f2bf(a[2]); r[3] = (short)f2bf(a[3]);
  r[4] = (short)f2bf(b[0]); r[5] = (short)f2bf(b[1]); r[6] = (short)f2bf(b[2]); r[7] = (short)f2bf(b[3]);
  return __builtin_bit_cast(v8bf, r);
}

__device__ __forceinline__ v4f mfma(const v8bf& a, const v8bf& b, const v4f& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void store4(bf16_t* dst, const v4f& v, float s) {
  uint2 u;
  u.x = pack2bf(v[0] * s, v[1] * s);
  u.y = pack2bf(v[2] * s, v[3] * s);
  *reinterpret_cast<uint2*>(dst) = u;
}

// ------------------------------------------------------------------------------------------------
template <int HD, int NKT, int NW>
__global__ void __launch_bounds__(NW * 64) attn_fwd_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ o,
                                                           float* __restrict__ lse, int N, int H, int hd,
                                                           float scale) {
  constexpr int NP = NKT * 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ki = smem;
  char* Vi = smem + NP * HD * 2;
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * hd;
  const long rs = 3L * D;
  const bf16_t* base = qkv + (long)b * N * rs + (long)h * hd;
  load_image<HD>(Ki, base + D, rs, N, hd, NP);
  load_image<HD>(Vi, base + 2 * D, rs, N, hd, NP);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const float c = scale * LOG2E;
  const int nqt = (N + 15) / 16;
  for (int qt = wave; qt < nqt; qt += NW) {
    const int q = qt * 16 + i;
    v8bf qf[HD / 32];
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) {
      v8s v = {0, 0, 0, 0, 0, 0, 0, 0};
      const int d = kk * 32 + 8 * g;
      if (q < N && d < hd) v = *reinterpret_cast<const v8s*>(base + (long)q * rs + d);
      qf[kk] = __builtin_bit_cast(v8bf, v);
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
        const float p = exp2f(s[kt][r] * c - mc);
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
template <int HD, int NKT, int NW>
__global__ void __launch_bounds__(NW * 64) attn_bwd_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o,
                                                           const bf16_t* __restrict__ dout,
                                                           const float* __restrict__ lse, bf16_t* __restrict__ dqkv,
                                                           int N, int H, int hd, float scale) {
  constexpr int NP = NKT * 16;
  constexpr int IMG = NP * HD * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Qi = smem;
  char* Ki = smem + IMG;
  char* Vi = smem + 2 * IMG;
  char* Oi = smem + 3 * IMG;  // dO image
  float* lse_s = reinterpret_cast<float*>(smem + 4 * IMG);
  float* dlt_s = lse_s + NP;

  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * hd;
  const long rs = 3L * D;
  const bf16_t* base = qkv + (long)b * N * rs + (long)h * hd;
  const bf16_t* dob = dout + (long)b * N * D + (long)h * hd;
  const bf16_t* ob = o + (long)b * N * D + (long)h * hd;
  load_image<HD>(Qi, base, rs, N, hd, NP);
  load_image<HD>(Ki, base + D, rs, N, hd, NP);
  load_image<HD>(Vi, base + 2 * D, rs, N, hd, NP);
  load_image<HD>(Oi, dob, D, N, hd, NP);
  for (int r = threadIdx.x; r < NP; r += blockDim.x) {
    float d = 0.f, ls = INFINITY;
    if (r < N) {
      ls = lse[(long)bh * N + r] * LOG2E;
      for (int k = 0; k < hd; k += 8) {
        v8s a = *reinterpret_cast<const v8s*>(dob + (long)r * D + k);
        v8s bb = *reinterpret_cast<const v8s*>(ob + (long)r * D + k);
#pragma unroll
        for (int j = 0; j < 8; ++j) d += bf2f((bf16_t)a[j]) * bf2f((bf16_t)bb[j]);
      }
    }
    lse_s[r] = ls;
    dlt_s[r] = d;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  const float c = scale * LOG2E;
  const int nt_valid = (N + 15) / 16;       // 16-row tiles holding valid rows
  const int ns_valid = (N + 31) / 32;       // 32-row steps holding valid rows
  bf16_t* dq_base = dqkv + (long)b * N * rs + (long)h * hd;

  // ---- phase 1: dK, dV (key tiles owned by waves) ----
  for (int kt = wave; kt < nt_valid; kt += NW) {
    v8bf kf[HD / 32], vf[HD / 32];
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) {
      kf[kk] = rd_row<HD>(Ki, kt * 16, kk, lane);
      vf[kk] = rd_row<HD>(Vi, kt * 16, kk, lane);
    }
    v4f dv[HD / 16], dk[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      dv[dt] = v4f{0.f, 0.f, 0.f, 0.f};
      dk[dt] = v4f{0.f, 0.f, 0.f, 0.f};
    }
    const int key = kt * 16 + i;
    const bool kvalid = key < N;
    for (int qs = 0; qs < ns_valid; ++qs) {
      v4f P[2], DS[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qt = 2 * qs + u;
        v4f s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk) {
          s = mfma(rd_row<HD>(Qi, qt * 16, kk, lane), kf[kk], s);
          dp = mfma(rd_row<HD>(Oi, qt * 16, kk, lane), vf[kk], dp);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = qt * 16 + 4 * g + r;
          const float p = kvalid ? exp2f(s[r] * c - lse_s[q]) : 0.f;
          P[u][r] = p;
          DS[u][r] = p * (dp[r] - dlt_s[q]);
        }
      }
      const v8bf bP = pack8(P[0], P[1]);
      const v8bf bD = pack8(DS[0], DS[1]);
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        dv[dt] = mfma(rd_tr<HD>(Oi, 2 * qs, 2 * qs + 1, dt * 16, lane), bP, dv[dt]);
        dk[dt] = mfma(rd_tr<HD>(Qi, 2 * qs, 2 * qs + 1, dt * 16, lane), bD, dk[dt]);
      }
    }
    if (kvalid) {
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        const int d = dt * 16 + 4 * g;
        if (d < hd) {
          store4(dq_base + (long)key * rs + D + d, dk[dt], scale);
          store4(dq_base + (long)key * rs + 2 * D + d, dv[dt], 1.0f);
        }
      }
    }
  }

  // ---- phase 2: dQ (query tiles owned by waves) ----
  for (int qt = wave; qt < nt_valid; qt += NW) {
    v8bf qf[HD / 32], df[HD / 32];
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) {
      qf[kk] = rd_row<HD>(Qi, qt * 16, kk, lane);
      df[kk] = rd_row<HD>(Oi, qt * 16, kk, lane);
    }
    const int q = qt * 16 + i;
    const float ls = lse_s[q], dl = dlt_s[q];
    v4f dq[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) dq[dt] = v4f{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < ns_valid; ++ks) {
      v4f DS[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int kt = 2 * ks + u;
        v4f st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk) {
          st = mfma(rd_row<HD>(Ki, kt * 16, kk, lane), qf[kk], st);
          dpt = mfma(rd_row<HD>(Vi, kt * 16, kk, lane), df[kk], dpt);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kt * 16 + 4 * g + r;
          const float p = key < N ? exp2f(st[r] * c - ls) : 0.f;
          DS[u][r] = p * (dpt[r] - dl);
        }
      }
      const v8bf bD = pack8(DS[0], DS[1]);
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt)
        dq[dt] = mfma(rd_tr<HD>(Ki, 2 * ks, 2 * ks + 1, dt * 16, lane), bD, dq[dt]);
    }
    if (q < N) {
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) {
        const int d = dt * 16 + 4 * g;
        if (d < hd) store4(dq_base + (long)q * rs + d, dq[dt], scale);
      }
    }
  }
}

template <int HD, int NKT>
hipError_t launch_fwd(const bf16_t* qkv, bf16_t* o, float* lse, int B, int N, int H, int hd, float scale,
                      hipStream_t s) {
  constexpr int NW = 4;
  const size_t lds = (size_t)2 * NKT * 16 * HD * 2;
  hipLaunchKernelGGL((attn_fwd_kernel<HD, NKT, NW>), dim3(B * H), dim3(NW * 64), lds, s, qkv, o, lse, N, H, hd, scale);
  return hipGetLastError();
}

template <int HD, int NKT>
hipError_t launch_bwd(const bf16_t* qkv, const bf16_t* o, const bf16_t* dout, const float* lse, bf16_t* dqkv, int B,
                      int N, int H, int hd, float scale, hipStream_t s) {
  constexpr int NW = 8;
  const size_t lds = (size_t)4 * NKT * 16 * HD * 2 + 2 * NKT * 16 * 4;
  auto kern = attn_bwd_kernel<HD, NKT, NW>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(B * H), dim3(NW * 64), lds, s, qkv, o, dout, lse, dqkv, N, H, hd, scale);
  return hipGetLastError();
}

#define VIT_NKT_CASES(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20)

template <int HD>
hipError_t dispatch_fwd(int nkt, const bf16_t* qkv, bf16_t* o, float* lse, int B, int N, int H, int hd, float scale,
                        hipStream_t s) {
  switch (nkt) {
#define C(n) \
  case n: return launch_fwd<HD, n>(qkv, o, lse, B, N, H, hd, scale, s);
    VIT_NKT_CASES(C)
#undef C
  }
  return hipErrorInvalidValue;
}
template <int HD>
hipError_t dispatch_bwd(int nkt, const bf16_t* qkv, const bf16_t* o, const bf16_t* dout, const float* lse,
                        bf16_t* dqkv, int B, int N, int H, int hd, float scale, hipStream_t s) {
  switch (nkt) {
#define C(n) \
  case n: return launch_bwd<HD, n>(qkv, o, dout, lse, dqkv, B, N, H, hd, scale, s);
    VIT_NKT_CASES(C)
#undef C
  }
  return hipErrorInvalidValue;
}

int check_shape(int64_t B, int64_t N, int64_t H, int64_t hd) {
  VIT_CHECK_ARG(B >= 1 && H >= 1 && N >= 1, "attention: bad sizes B=%lld N=%lld H=%lld", (long long)B, (long long)N,
                (long long)H);
  VIT_CHECK_ARG(N <= 320, "attention: N=%lld > 320 unsupported", (long long)N);
  VIT_CHECK_ARG(hd == 32 || hd == 64, "attention: head_dim %lld unsupported (32, 64)", (long long)hd);
  return VIT_OK;
}

}  // namespace

extern "C" int vit_attention_fwd(const void* qkv, void* o, float* lse, int64_t B, int64_t N, int64_t H, int64_t hd,
                                 float scale, vit_stream_t stream) {
  int st = check_shape(B, N, H, hd);
  if (st) return st;
  VIT_CHECK_ARG(qkv && o && lse, "vit_attention_fwd: null pointer");
  const int nkt = (int)((N + 31) / 32) * 2;
  hipError_t e = hd == 64 ? dispatch_fwd<64>(nkt, (const bf16_t*)qkv, (bf16_t*)o, lse, (int)B, (int)N, (int)H, (int)hd,
                                             scale, (hipStream_t)stream)
                          : dispatch_fwd<32>(nkt, (const bf16_t*)qkv, (bf16_t*)o, lse, (int)B, (int)N, (int)H, (int)hd,
                                             scale, (hipStream_t)stream);
  return vit::check_hip(e, "vit_attention_fwd launch");
}

extern "C" int vit_attention_bwd(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv,
                                 int64_t B, int64_t N, int64_t H, int64_t hd, float scale, vit_stream_t stream) {
  int st = check_shape(B, N, H, hd);
  if (st) return st;
  VIT_CHECK_ARG(qkv && o && dout && lse && dqkv, "vit_attention_bwd: null pointer");
  const int nkt = (int)((N + 31) / 32) * 2;
  hipError_t e = hd == 64
                     ? dispatch_bwd<64>(nkt, (const bf16_t*)qkv, (const bf16_t*)o, (const bf16_t*)dout, lse,
                                        (bf16_t*)dqkv, (int)B, (int)N, (int)H, (int)hd, scale, (hipStream_t)stream)
                     : dispatch_bwd<32>(nkt, (const bf16_t*)qkv, (const bf16_t*)o, (const bf16_t*)dout, lse,
                                        (bf16_t*)dqkv, (int)B, (int)N, (int)H, (int)hd, scale, (hipStream_t)stream);
  return vit::check_hip(e, "vit_attention_bwd launch");
}
