// LayerNorm forward/backward (nn.LayerNorm(D), eps 1e-5, reference src/model.py:108,114,146).
// One wavefront per row, the row held in registers as float4 chunks (HBM-bound kernels: each
// row is read once and written once; 16-B loads per lane). Statistics in fp32.
#include "common.h"

#include <cstdlib>

namespace {

// NV = float4 chunks per lane (D <= NV * 256).
// FULL: D == NV * 256, every chunk in range: no per-chunk guards, so a row's loads (and the gamma /
// beta loads) issue back to back instead of one guarded load and its wait at a time
template <int NV, bool FULL>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const float* __restrict__ x, long ldx, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, void* __restrict__ y, long ldy,
                                                     int y_f32, float* __restrict__ mean, float* __restrict__ rstd,
                                                     int rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (long)row * ldx;
  float4 v[NV], gmv[NV], btv[NV];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {  // gamma / beta requested with the row, not after its reductions
    const int c = (k * 64 + lane) * 4;
    if (FULL || c < D) {
      gmv[k] = *reinterpret_cast<const float4*>(gamma + c);
      btv[k] = *reinterpret_cast<const float4*>(beta + c);
    }
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 4;
    if (FULL || c < D) {
      v[k] = *reinterpret_cast<const float4*>(xr + c);
      s += v[k].x + v[k].y + v[k].z + v[k].w;
    } else {
      v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const float mu = wave_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 4;
    if (FULL || c < D) {
      const float a = v[k].x - mu, b = v[k].y - mu, cc = v[k].z - mu, d = v[k].w - mu;
      ss += a * a + b * b + cc * cc + d * d;
    }
  }
  const float var = wave_sum(ss) / D;
  const float rs = rsqrtf(var + eps);
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = (k * 64 + lane) * 4;
    if (FULL || c < D) {
      const float4 gm = gmv[k], bt = btv[k];
      const float o0 = (v[k].x - mu) * rs * gm.x + bt.x;
      const float o1 = (v[k].y - mu) * rs * gm.y + bt.y;
      const float o2 = (v[k].z - mu) * rs * gm.z + bt.z;
      const float o3 = (v[k].w - mu) * rs * gm.w + bt.w;
      if (y_f32) {
        *reinterpret_cast<float4*>((float*)y + (long)row * ldy + c) = make_float4(o0, o1, o2, o3);
      } else {
        uint2 u;
        u.x = pack2bf(o0, o1);
        u.y = pack2bf(o2, o3);
        *reinterpret_cast<uint2*>((bf16_t*)y + (long)row * ldy + c) = u;
      }
    }
  }
}

// The row-pipelined backward needs 187 VGPRs (2 waves per SIMD): 512 four-wave blocks are all
// resident at once on 256 CUs, and each wave walks ~25 rows (B/16 bs256: 123 vs 129 us isolated
// at 1024 blocks, +0.3% step; VIT_LN_BWD_BLOCKS overrides).
constexpr int LN_BWD_MAX_BLOCKS = 512;

template <int NV, bool FULL>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const void* __restrict__ dy, long lddy, int dy_f32,
                                                     const float* __restrict__ x, long ldx, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                     const float* __restrict__ dres, long lddres, float* __restrict__ dx,
                                                     long lddx, bf16_t* __restrict__ dxb, long lddxb,
                                                     float* __restrict__ partial, int rows, int D, DropDev drop) {
  __shared__ float red[4][NV * 256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float4 pg[NV], pb[NV], ps[NV];
  float4 gm[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    pg[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    pb[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    ps[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int c = (k * 64 + lane) * 4;
    gm[k] = FULL || c < D ? *reinterpret_cast<const float4*>(gamma + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // rows are software-pipelined: the next row's loads (dy, x, residual grad, stats) are issued
  // before this row's math and stores, so each wave keeps two rows of HBM reads in flight
  auto load_row = [&](int row, float4* d4, float4* x4, float4* r4, float& mu, float& rs) {
    mu = mean[row];
    rs = rstd[row];
    if constexpr (FULL) {
      // wave-uniform choices outside the chunk loops: each loop is straight-line, so the row's loads
      // issue together (a per-chunk branch made hipcc wait for each chunk's loads in turn)
      if (dy_f32) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
          d4[k] = *reinterpret_cast<const float4*>((const float*)dy + (long)row * lddy + (k * 64 + lane) * 4);
      } else {
        uint2 u[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k)
          u[k] = *reinterpret_cast<const uint2*>((const bf16_t*)dy + (long)row * lddy + (k * 64 + lane) * 4);
#pragma unroll
        for (int k = 0; k < NV; ++k)
          d4[k] = make_float4(bf2f(u[k].x & 0xffff), bf2f(u[k].x >> 16), bf2f(u[k].y & 0xffff), bf2f(u[k].y >> 16));
      }
#pragma unroll
      for (int k = 0; k < NV; ++k) x4[k] = *reinterpret_cast<const float4*>(x + (long)row * ldx + (k * 64 + lane) * 4);
      if (dres) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
          r4[k] = *reinterpret_cast<const float4*>(dres + (long)row * lddres + (k * 64 + lane) * 4);
      } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) r4[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      if (FULL || c < D) {
        if (dy_f32) {
          d4[k] = *reinterpret_cast<const float4*>((const float*)dy + (long)row * lddy + c);
        } else {
          const uint2 u = *reinterpret_cast<const uint2*>((const bf16_t*)dy + (long)row * lddy + c);
          d4[k] = make_float4(bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16));
        }
        x4[k] = *reinterpret_cast<const float4*>(x + (long)row * ldx + c);
        r4[k] = dres ? *reinterpret_cast<const float4*>(dres + (long)row * lddres + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        d4[k] = x4[k] = r4[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  const int stride = gridDim.x * 4;
  float4 d4[NV], x4[NV], r4[NV];
  float mu = 0.f, rs = 0.f;
  int row = blockIdx.x * 4 + wave;
  if (row < rows) load_row(row, d4, x4, r4, mu, rs);
  for (; row < rows; row += stride) {
    float4 dn[NV], xn[NV], rn[NV];
    float mun = 0.f, rsn = 0.f;
    if (row + stride < rows) load_row(row + stride, dn, xn, rn, mun, rsn);
    float4 xh[NV], g[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      xh[k] = make_float4((x4[k].x - mu) * rs, (x4[k].y - mu) * rs, (x4[k].z - mu) * rs, (x4[k].w - mu) * rs);
      g[k] = make_float4(d4[k].x * gm[k].x, d4[k].y * gm[k].y, d4[k].z * gm[k].z, d4[k].w * gm[k].w);
      s1 += g[k].x + g[k].y + g[k].z + g[k].w;
      s2 += g[k].x * xh[k].x + g[k].y * xh[k].y + g[k].z * xh[k].z + g[k].w * xh[k].w;
      pg[k].x += d4[k].x * xh[k].x; pg[k].y += d4[k].y * xh[k].y; pg[k].z += d4[k].z * xh[k].z;
      pg[k].w += d4[k].w * xh[k].w;
      pb[k].x += d4[k].x; pb[k].y += d4[k].y; pb[k].z += d4[k].z; pb[k].w += d4[k].w;
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      if (FULL || c < D) {
        float4 o;
        o.x = rs * (g[k].x - m1 - xh[k].x * m2) + r4[k].x;
        o.y = rs * (g[k].y - m1 - xh[k].y * m2) + r4[k].y;
        o.z = rs * (g[k].z - m1 - xh[k].z * m2) + r4[k].z;
        o.w = rs * (g[k].w - m1 - xh[k].w * m2) + r4[k].w;
        *reinterpret_cast<float4*>(dx + (long)row * lddx + c) = o;
        if (drop.thr) {  // the copy / column sums feed the dropout-ed branch: gradient x mask
          float m8[8];
          drop_mult8(drop, row, c >> 3, m8);
          const bool hi = c & 4;
          o.x *= hi ? m8[4] : m8[0];
          o.y *= hi ? m8[5] : m8[1];
          o.z *= hi ? m8[6] : m8[2];
          o.w *= hi ? m8[7] : m8[3];
        }
        ps[k].x += o.x; ps[k].y += o.y; ps[k].z += o.z; ps[k].w += o.w;
        if (dxb) {
          uint2 u;
          u.x = pack2bf(o.x, o.y);
          u.y = pack2bf(o.z, o.w);
          *reinterpret_cast<uint2*>(dxb + (long)row * lddxb + c) = u;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      d4[k] = dn[k];
      x4[k] = xn[k];
      r4[k] = rn[k];
    }
    mu = mun;
    rs = rsn;
  }
  // block partials [dgamma | dbeta | dsum]: sum dy*xhat, sum dy, sum of the written dx (the
  // bias gradient of the linear layer that produced this residual stream)
#pragma unroll
  for (int q = 0; q < 3; ++q) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = (k * 64 + lane) * 4;
      *reinterpret_cast<float4*>(&red[wave][c]) = q == 0 ? pg[k] : (q == 1 ? pb[k] : ps[k]);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256)
      partial[(long)blockIdx.x * 3 * D + q * D + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    __syncthreads();
  }
}

int nv_for(int64_t D) { return (int)((D + 255) / 256); }

}  // namespace

extern "C" int vit_layernorm_fwd(const float* x, int64_t ldx, const float* gamma, const float* beta, void* y,
                                 int64_t ldy, int32_t y_f32, float* mean, float* rstd, int64_t rows, int64_t D,
                                 float eps, vit_stream_t stream) {
  VIT_CHECK_ARG(x && gamma && beta && y && mean && rstd, "vit_layernorm_fwd: null pointer");
  VIT_CHECK_ARG(D > 0 && D % 4 == 0 && D <= 2048, "vit_layernorm_fwd: D=%lld unsupported", (long long)D);
  VIT_CHECK_ARG(ldx % 4 == 0 && ldy % 4 == 0, "vit_layernorm_fwd: strides must be multiples of 4");
  if (rows <= 0) return VIT_OK;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  hipStream_t s = (hipStream_t)stream;
  switch (nv_for(D)) {
#define C(n)                                                                                                        \
  case n:                                                                                                           \
    if (D == n * 256)                                                                                               \
      hipLaunchKernelGGL((ln_fwd_kernel<n, true>), grid, block, 0, s, x, (long)ldx, gamma, beta, y, (long)ldy,       \
                         (int)y_f32, mean, rstd, (int)rows, (int)D, eps);                                           \
    else                                                                                                            \
      hipLaunchKernelGGL((ln_fwd_kernel<n, false>), grid, block, 0, s, x, (long)ldx, gamma, beta, y, (long)ldy,      \
                         (int)y_f32, mean, rstd, (int)rows, (int)D, eps);                                           \
    break;
    C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8)
#undef C
  }
  VIT_LAUNCH_CHECK("vit_layernorm_fwd");
}

static int64_t ln_bwd_blocks(int64_t rows) {
  static const int64_t cap = [] {
    const int k = vit::knob("VIT_LN_BWD_BLOCKS", 0);
    return k > 0 ? (int64_t)k : (int64_t)LN_BWD_MAX_BLOCKS;
  }();
  int64_t b = (rows + 3) / 4;
  if (b > cap) b = cap;
  return b < 1 ? 1 : b;
}

// rows of block partials the backward writes (the rows a deferred vit_colsum3 of them reduces)
extern "C" int64_t vit_layernorm_bwd_blocks(int64_t rows) { return ln_bwd_blocks(rows); }

// rows of 3*D floats the `partial` workspace must hold (block partials + their column reduction)
extern "C" int64_t vit_layernorm_bwd_partial_rows(int64_t rows) {
  const int64_t nb = ln_bwd_blocks(rows);
  return nb + vit_colsum_partial_rows(nb);
}

extern "C" int vit_layernorm_bwd(const void* dy, int64_t lddy, int32_t dy_f32, const float* x, int64_t ldx,
                                 const float* mean, const float* rstd, const float* gamma, const float* dres,
                                 int64_t lddres, float* dx, int64_t lddx, void* dx_bf16, int64_t lddxb, float* partial,
                                 float* dgamma_dbeta, float* dx_colsum, int32_t accumulate_params, int64_t rows,
                                 int64_t D, const vit_dropout* dx_dropout, vit_stream_t stream) {
  VIT_CHECK_ARG(dy && x && mean && rstd && gamma && dx && partial, "vit_layernorm_bwd: null pointer");
  const DropDev drop = make_drop(dx_dropout);
  VIT_CHECK_ARG(D > 0 && D % 4 == 0 && D <= 2048, "vit_layernorm_bwd: D=%lld unsupported", (long long)D);
  if (rows <= 0) return VIT_OK;
  const int64_t nblk = ln_bwd_blocks(rows);
  hipStream_t s = (hipStream_t)stream;
  switch (nv_for(D)) {
#define C(n)                                                                                                        \
  case n:                                                                                                           \
    if (D == n * 256)                                                                                               \
      hipLaunchKernelGGL((ln_bwd_kernel<n, true>), dim3((unsigned)nblk), dim3(256), 0, s, dy, (long)lddy, (int)dy_f32, \
                         x, (long)ldx, mean, rstd, gamma, dres, (long)lddres, dx, (long)lddx, (bf16_t*)dx_bf16,      \
                         (long)lddxb, partial, (int)rows, (int)D, drop);                                            \
    else                                                                                                            \
      hipLaunchKernelGGL((ln_bwd_kernel<n, false>), dim3((unsigned)nblk), dim3(256), 0, s, dy, (long)lddy,           \
                         (int)dy_f32, x, (long)ldx, mean, rstd, gamma, dres, (long)lddres, dx, (long)lddx,          \
                         (bf16_t*)dx_bf16, (long)lddxb, partial, (int)rows, (int)D, drop);                          \
    break;
    C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8)
#undef C
  }
  int st = vit::check_hip(hipGetLastError(), "vit_layernorm_bwd");
  if (st) return st;
  float* ws = partial + nblk * 3 * D;
  if (!dgamma_dbeta && !dx_colsum) return VIT_OK;
  if (D % 8 == 0)  // one reduction for [dgamma | dbeta | dx colsum]
    return vit_colsum3(partial, 0, nblk, D, 3 * D, ws, dgamma_dbeta, dgamma_dbeta ? dgamma_dbeta + D : nullptr,
                       dx_colsum, accumulate_params, stream);
  if (dgamma_dbeta) st = vit_colsum(partial, 0, nblk, 2 * D, 3 * D, ws, dgamma_dbeta, accumulate_params, stream);
  if (st) return st;
  if (dx_colsum) st = vit_colsum(partial + 2 * D, 0, nblk, D, 3 * D, ws, dx_colsum, accumulate_params, stream);
  return st;
}
