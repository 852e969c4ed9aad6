// HBM-bound helper kernels of the ViT training step: patch im2col, embedding grads, column sums
// (bias / LayerNorm-affine grads), the small f32 classifier GEMM, fused cross entropy + accuracy,
// fused SGD-momentum with the bf16 weight mirror, and casts.
#include "common.h"

namespace {

// ---- im2col for Conv2d(3, D, k=P, s=P) (reference src/model.py:179,197-200) ----------------------
// out[b*N + 1 + py*g + px][c*P*P + ky*P + kx] = x[b][c][py*P+ky][px*P+kx]; cls rows and pad cols = 0.
template <typename OUT>
__global__ void im2col_kernel(const float* __restrict__ x, OUT* __restrict__ out, int B, int img, int P, int Kpad) {
  const int g = img / P;
  const int N = g * g + 1;
  const long total = (long)B * N * Kpad;
  const int K = 3 * P * P;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int col = (int)(i % Kpad);
    const long row = i / Kpad;
    const int t = (int)(row % N);
    const int b = (int)(row / N);
    float v = 0.f;
    if (t > 0 && col < K) {
      const int patch = t - 1, py = patch / g, px = patch % g;
      const int c = col / (P * P), rem = col % (P * P), ky = rem / P, kx = rem % P;
      v = x[(((long)b * 3 + c) * img + (py * P + ky)) * img + (px * P + kx)];
    }
    if constexpr (sizeof(OUT) == 2)
      out[i] = f2bf(v);
    else
      out[i] = v;
  }
}

// dpos[n][d] = sum_b dh0[(b*N+n)*D + d]
__global__ void pos_grad_kernel(const float* __restrict__ dh0, int B, int N, int D, float* __restrict__ dpos,
                                DropDev drop) {
  const int n = blockIdx.y;
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  float s = 0.f;
  if (drop.thr) {  // gradient through the position-embedding dropout
    for (int b = 0; b < B; ++b) s += dh0[((long)b * N + n) * D + d] * drop_mult1(drop, (long)b * N + n, d);
  } else {
    for (int b = 0; b < B; ++b) s += dh0[((long)b * N + n) * D + d];
  }
  dpos[(long)n * D + d] = s;
}

__global__ void dropout_mask_kernel(DropDev drop, long row0, long rows, int cols, float* __restrict__ out, long ld) {
  const long r = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows || c >= cols) return;
  out[r * ld + c] = drop.thr ? drop_mult1(drop, row0 + r, c) : 1.0f;
}

// Vector forms of the two embedding kernels above (the common shapes: P % 8 == 0, D % 4 == 0).
// im2col: one thread per 8 consecutive patch columns (8 adjacent pixels of one image row: two
// 16-B loads, one 16-B bf16 store); the division chain runs once per 8 outputs instead of per output.
template <typename OUT>
__global__ void im2col8_kernel(const float* __restrict__ x, OUT* __restrict__ out, int B, int img, int P) {
  const int g = img / P, N = g * g + 1, K8 = 3 * P * P / 8;
  const long total = (long)B * N * K8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % K8);
    const long row = i / K8;
    const int t = (int)(row % N), b = (int)(row / N);
    float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
    if (t > 0) {
      const int patch = t - 1, py = patch / g, px = patch % g;
      const int col = c8 * 8, c = col / (P * P), rem = col % (P * P), ky = rem / P, kx = rem % P;
      const float4* src =
          reinterpret_cast<const float4*>(x + (((long)b * 3 + c) * img + (py * P + ky)) * img + (px * P + kx));
      lo = src[0];
      hi = src[1];
    }
    if constexpr (sizeof(OUT) == 2) {
      uint4 v;
      v.x = (uint32_t)f2bf(lo.x) | ((uint32_t)f2bf(lo.y) << 16);
      v.y = (uint32_t)f2bf(lo.z) | ((uint32_t)f2bf(lo.w) << 16);
      v.z = (uint32_t)f2bf(hi.x) | ((uint32_t)f2bf(hi.y) << 16);
      v.w = (uint32_t)f2bf(hi.z) | ((uint32_t)f2bf(hi.w) << 16);
      reinterpret_cast<uint4*>(out)[i] = v;
    } else {
      reinterpret_cast<float4*>(out)[2 * i] = lo;
      reinterpret_cast<float4*>(out)[2 * i + 1] = hi;
    }
  }
}

// dpos[n][d] = sum_b dh0[(b*N+n)*D + d]: workgroup (n, column slice) = 8 image groups x C4 float4
// columns, the 8 partial rows summed through LDS. gridDim.y slices keep > 256 workgroups in flight.
__global__ void __launch_bounds__(768) pos_grad4_kernel(const float* __restrict__ dh0, int B, int N, int D,
                                                        float* __restrict__ dpos, DropDev drop) {
  __shared__ float4 red[8][96];
  const int C4 = D / 4 / gridDim.y;
  const int n = blockIdx.x, c = threadIdx.x % C4, grp = threadIdx.x / C4;
  const int d = (blockIdx.y * C4 + c) * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* base = dh0 + (long)n * D + d;
  const long bstride = (long)N * D;
#pragma unroll 4
  for (int b = grp; b < B; b += 8) {
    float4 v = *reinterpret_cast<const float4*>(base + b * bstride);
    if (drop.thr) {
      const long r = (long)b * N + n;
      v.x *= drop_mult1(drop, r, d);
      v.y *= drop_mult1(drop, r, d + 1);
      v.z *= drop_mult1(drop, r, d + 2);
      v.w *= drop_mult1(drop, r, d + 3);
    }
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  }
  red[grp][c] = s;
  __syncthreads();
  if (grp == 0) {
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      s.x += red[k][c].x;
      s.y += red[k][c].y;
      s.z += red[k][c].z;
      s.w += red[k][c].w;
    }
    *reinterpret_cast<float4*>(dpos + (long)n * D + d) = s;
  }
}

// dcls = dpos[0]; dconv_bias = sum_{n>=1} dpos[n]: 16 columns x 16 row lanes per workgroup
__global__ void __launch_bounds__(256) cls_bias_grad16_kernel(const float* __restrict__ dpos, int N, int D,
                                                              float* __restrict__ dcls, float* __restrict__ dbias) {
  __shared__ float red[16][17];
  const int c = threadIdx.x & 15, r = threadIdx.x >> 4;
  const int d = blockIdx.x * 16 + c;
  float s = 0.f;
  if (d < D)
    for (int n = 1 + r; n < N; n += 16) s += dpos[(long)n * D + d];
  red[r][c] = s;
  __syncthreads();
  if (r == 0 && d < D) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][c];
    dbias[d] = t;
    dcls[d] = dpos[d];
  }
}

// ---- column sums --------------------------------------------------------------------------------
// Vector path: a thread owns 8 consecutive columns (one 16-B bf16 / 32-B f32 load per row), a
// 256-thread block = 32 column groups x 8 row lanes; each block reduces a chunk of rows into one
// partial row, a second pass of the same kernel reduces the partial rows.
constexpr int COLSUM_MAX_CHUNKS = 256;
constexpr int COLSUM_MIN_ROWS_PER_CHUNK = 64;

// Final destination of column `col`: with seg > 0 the columns are split into segments of `seg`
// columns written to out / out1 / out2 (segment k -> its own array, NULL = dropped).
__device__ __forceinline__ float* seg_dst(float* out, float* out1, float* out2, long seg, long ch, int cols, int col) {
  if (seg <= 0) return out + ch * cols + col;
  const int k = (int)(col / seg);
  float* base = k == 0 ? out : (k == 1 ? out1 : out2);
  return base ? base + (col - k * seg) : nullptr;
}

template <bool BF16>
__global__ void __launch_bounds__(256) colsum8_kernel(const void* __restrict__ in, long rows, int cols, long ld,
                                                      int chunks, float* __restrict__ out, int accumulate,
                                                      long seg = 0, float* out1 = nullptr, float* out2 = nullptr) {
  __shared__ float red[8][32][9];
  const int cgl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int cg = blockIdx.x * 32 + cgl;
  const int ch = blockIdx.y;
  const long per = (rows + chunks - 1) / chunks;
  const long r0 = ch * per, r1 = r0 + per < rows ? r0 + per : rows;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (cg * 8 < cols) {
    for (long r = r0 + rl; r < r1; r += 8) {
      if constexpr (BF16) {
        const uint4 u = *reinterpret_cast<const uint4*>((const bf16_t*)in + r * ld + cg * 8);
        acc[0] += bf2f(u.x & 0xffff); acc[1] += bf2f(u.x >> 16); acc[2] += bf2f(u.y & 0xffff); acc[3] += bf2f(u.y >> 16);
        acc[4] += bf2f(u.z & 0xffff); acc[5] += bf2f(u.z >> 16); acc[6] += bf2f(u.w & 0xffff); acc[7] += bf2f(u.w >> 16);
      } else {
        const float4 a = *reinterpret_cast<const float4*>((const float*)in + r * ld + cg * 8);
        const float4 b = *reinterpret_cast<const float4*>((const float*)in + r * ld + cg * 8 + 4);
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
        acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rl][cgl][k] = acc[k];
  __syncthreads();
  const int ocg = threadIdx.x >> 3, k = threadIdx.x & 7;
  const int col = (blockIdx.x * 32 + ocg) * 8 + k;
  if (col < cols) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) s += red[q][ocg][k];
    float* dst = seg_dst(out, out1, out2, seg, ch, cols, col);
    if (dst) *dst = accumulate ? *dst + s : s;
  }
}

// Scalar fallback (odd widths / alignment).
__device__ __forceinline__ float ld_elem(const void* p, long i, int is_bf16) {
  return is_bf16 ? bf2f(((const bf16_t*)p)[i]) : ((const float*)p)[i];
}
__global__ void colsum_partial_kernel(const void* __restrict__ in, int in_bf16, long rows, int cols, long ld,
                                      int chunks, float* __restrict__ partial) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  const int ch = blockIdx.y;
  const long per = (rows + chunks - 1) / chunks;
  const long r0 = ch * per, r1 = r0 + per < rows ? r0 + per : rows;
  float s = 0.f;
  // (one loop per input type, unrolled: eight loads in flight — a short job, the 100-class head's bias gradient over
  // 128 rows in one chunk, is otherwise one HBM round trip per row; the additions keep their row order)
  if (in_bf16) {
    const bf16_t* p = (const bf16_t*)in + c;
#pragma unroll 8
    for (long r = r0; r < r1; ++r) s += bf2f(p[r * ld]);
  } else {
    const float* p = (const float*)in + c;
#pragma unroll 8
    for (long r = r0; r < r1; ++r) s += p[r * ld];
  }
  partial[(long)ch * cols + c] = s;
}
__global__ void colsum_final_kernel(const float* __restrict__ partial, int chunks, int cols, float* __restrict__ out,
                                    int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int k = 0; k < chunks; ++k) s += partial[(long)k * cols + c];
  out[c] = accumulate ? out[c] + s : s;
}

// ---- f32 GEMM: classifier head of the bf16 step, and every projection of the fp32 (exact) forward.
// Exact f32 on the matrix core (v_mfma_f32_16x16x4_f32: f32 operands, f32 accumulation; no bf16
// rounding anywhere). 32 x 32 output tile per 256-thread workgroup; the four waves split the K loop
// (k-tiles of 16, wave w takes tiles w, w+4, ...) so narrow problems still fill the chip (the head:
// 256 x 1000 x 768 = 256 workgroups), and their partial tiles are summed through LDS at the end.
// Each wave stages its own k-tile (A 32x16, B 16x32) through a private LDS image with coalesced
// loads in either operand layout; rows padded to 48 floats so the fragment reads are conflict-free.
constexpr int GF_LD = 48;
__global__ void __launch_bounds__(256) gemm_f32_kernel(int M, int N, int K, const float* __restrict__ A, long lda,
                                                       int at, const float* __restrict__ B, long ldb, int bt,
                                                       float* __restrict__ C, long ldc, const float* __restrict__ bias,
                                                       int accumulate) {
  __shared__ float smem[4 * 2 * 16 * GF_LD];  // per wave: As[k][m], Bs[k][n]; reused for the reduction
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  float* As = smem + wave * 2 * 16 * GF_LD;
  float* Bs = As + 16 * GF_LD;
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const int nkt = (K + 15) / 16;
  // the wave's next k-tile is loaded into registers while the current one is multiplied
  auto load = [&](int kt, float* av, float* bv) {
    const int k0 = kt * 16;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = lane + e * 64;
      int m, k;
      if (at) { k = idx >> 5; m = idx & 31; } else { m = idx >> 4; k = idx & 15; }
      const int gm = m0 + m, gk = k0 + k;
      av[e] = (kt < nkt && gm < M && gk < K) ? (at ? A[(long)gk * lda + gm] : A[(long)gm * lda + gk]) : 0.f;
      int n, kb;
      if (bt) { n = idx >> 4; kb = idx & 15; } else { kb = idx >> 5; n = idx & 31; }
      const int gn = n0 + n, gkb = k0 + kb;
      bv[e] = (kt < nkt && gn < N && gkb < K) ? (bt ? B[(long)gn * ldb + gkb] : B[(long)gkb * ldb + gn]) : 0.f;
    }
  };
  float av[8], bv[8];
  load(wave, av, bv);
  for (int kt = wave; kt < nkt; kt += 4) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int idx = lane + e * 64;
      if (at) As[(idx >> 5) * GF_LD + (idx & 31)] = av[e]; else As[(idx & 15) * GF_LD + (idx >> 4)] = av[e];
      if (bt) Bs[(idx & 15) * GF_LD + (idx >> 4)] = bv[e]; else Bs[(idx >> 5) * GF_LD + (idx & 31)] = bv[e];
    }
    load(kt + 4, av, bv);
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k = ks * 4 + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = As[k * GF_LD + t * 16 + (lane & 15)];
        b[t] = Bs[k * GF_LD + t * 16 + (lane & 15)];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  // sum the four waves' partial tiles: red[w][row][col], row stride 33
  __syncthreads();
  float* red = smem;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[wave * 32 * 33 + (i * 16 + 4 * (lane >> 4) + r) * 33 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int idx = threadIdx.x + e * 256, row = idx >> 5, col = idx & 31;
    const int m = m0 + row, n = n0 + col;
    if (m >= M || n >= N) continue;
    float v = red[row * 33 + col] + red[32 * 33 + row * 33 + col] + red[2 * 32 * 33 + row * 33 + col] +
              red[3 * 32 * 33 + row * 33 + col];
    if (bias) v += bias[n];
    float* dst = C + (long)m * ldc + n;
    *dst = accumulate ? *dst + v : v;
  }
}

// ---- cross entropy + top-1/top-5 (src/train.py:22, src/utils.py:28-41) -------------------------
__global__ void __launch_bounds__(256) ce_kernel(const float* __restrict__ logits, const int64_t* __restrict__ labels,
                                                 int C, float* __restrict__ dlogits, float grad_scale,
                                                 float* __restrict__ row_stats) {
  __shared__ float red[4];
  __shared__ float red2[4];
  const int b = blockIdx.x;
  const float* x = logits + (long)b * C;
  const int64_t y64 = labels[b];
  // a label outside [0, C) (torch's CrossEntropyLoss raises) is never dereferenced: the row's loss and
  // gradient become NaN instead
  const bool ok = y64 >= 0 && y64 < C;
  const int y = ok ? (int)y64 : 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float mx = -INFINITY;
  for (int c = threadIdx.x; c < C; c += 256) mx = fmaxf(mx, x[c]);
  mx = wave_max(mx);
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  const float xy = ok ? x[y] : __builtin_nanf("");
  float s = 0.f, gt = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) {
    s += __expf(x[c] - mx);
    gt += x[c] > xy ? 1.f : 0.f;
  }
  s = wave_sum(s);
  gt = wave_sum(gt);
  if (lane == 0) {
    red[wave] = s;
    red2[wave] = gt;
  }
  __syncthreads();
  s = red[0] + red[1] + red[2] + red[3];
  gt = red2[0] + red2[1] + red2[2] + red2[3];
  const float lse = mx + logf(s);
  if (dlogits) {
    for (int c = threadIdx.x; c < C; c += 256) {
      const float p = __expf(x[c] - lse);
      dlogits[(long)b * C + c] = ok ? (p - (c == y ? 1.f : 0.f)) * grad_scale : __builtin_nanf("");
    }
  }
  if (threadIdx.x == 0 && row_stats) {
    row_stats[b * 3 + 0] = lse - xy;
    row_stats[b * 3 + 1] = gt < 1.f ? 1.f : 0.f;
    row_stats[b * 3 + 2] = gt < 5.f ? 1.f : 0.f;
  }
}

// ---- SGD momentum (torch.optim.SGD, dampening 0, no nesterov), src/train.py:154-158 -------------
// One body for both entry points: the scalars {lr, momentum, first} come either as kernel arguments (vit_sgd_step)
// or from three floats in device memory (vit_sgd_step_dev: the step can sit in a captured HIP graph while the
// schedule moves; the caller refreshes the floats before each launch).
struct SgdHostScalars {
  float lr, mom;
  int first;
  __device__ __forceinline__ void get(float& l, float& m, bool& f) const { l = lr; m = mom; f = first != 0; }
};
struct SgdDevScalars {
  const float* hyper;
  __device__ __forceinline__ void get(float& l, float& m, bool& f) const {
    l = hyper[0];
    m = hyper[1];
    f = hyper[2] != 0.0f;
  }
};
template <class S>
__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf,
                           bf16_t* __restrict__ pb, long n, const S sc, float wd) {
  float lr, mom;
  bool first;
  sc.get(lr, mom, first);
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 d = make_float4(gv.x + wd * pv.x, gv.y + wd * pv.y, gv.z + wd * pv.z, gv.w + wd * pv.w);
    if (!first) {
      const float4 bv = reinterpret_cast<float4*>(buf)[i];
      d = make_float4(mom * bv.x + d.x, mom * bv.y + d.y, mom * bv.z + d.z, mom * bv.w + d.w);
    }
    reinterpret_cast<float4*>(buf)[i] = d;
    pv = make_float4(pv.x - lr * d.x, pv.y - lr * d.y, pv.z - lr * d.z, pv.w - lr * d.w);
    reinterpret_cast<float4*>(p)[i] = pv;
    if (pb) {
      uint2 u;
      u.x = pack2bf(pv.x, pv.y);
      u.y = pack2bf(pv.z, pv.w);
      reinterpret_cast<uint2*>(pb)[i] = u;
    }
  }
  // tail
  const long t = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) {
    float d = g[t] + wd * p[t];
    if (!first) d = mom * buf[t] + d;
    buf[t] = d;
    p[t] -= lr * d;
    if (pb) pb[t] = f2bf(p[t]);
  }
}

__global__ void cast_kernel(const float* __restrict__ in, bf16_t* __restrict__ out, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) out[i] = f2bf(in[i]);
}
__global__ void cast_pad_kernel(const float* __restrict__ in, long rows, long cols, bf16_t* __restrict__ out, long ldo) {
  const long total = rows * ldo;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / ldo, c = i % ldo;
    out[i] = c < cols ? f2bf(in[r * cols + c]) : (bf16_t)0;
  }
}
__global__ void axpby_kernel(const float* __restrict__ x, float* __restrict__ y, long n, float a, float b) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = a * x[i] + (b == 0.f ? 0.f : b * y[i]);
}

unsigned grid_for(long n, int per_thread = 1) {
  long b = (n / per_thread + 255) / 256;
  if (b < 1) b = 1;
  if (b > 8192) b = 8192;
  return (unsigned)b;
}

}  // namespace

extern "C" int vit_im2col(const float* x, void* out, int64_t B, int64_t img, int64_t P, int64_t Kpad,
                          vit_stream_t stream) {
  VIT_CHECK_ARG(x && out && B > 0 && P > 0 && img >= P && Kpad >= 3 * P * P, "vit_im2col: bad args");
  const int64_t g = img / P, N = g * g + 1;
  if (P % 8 == 0 && img % 4 == 0 && Kpad == 3 * P * P && (uintptr_t)x % 16 == 0 && (uintptr_t)out % 16 == 0)
    hipLaunchKernelGGL(im2col8_kernel<bf16_t>, dim3(grid_for(B * N * Kpad / 8)), dim3(256), 0, (hipStream_t)stream, x,
                       (bf16_t*)out, (int)B, (int)img, (int)P);
  else
    hipLaunchKernelGGL(im2col_kernel<bf16_t>, dim3(grid_for(B * N * Kpad)), dim3(256), 0, (hipStream_t)stream, x,
                       (bf16_t*)out, (int)B, (int)img, (int)P, (int)Kpad);
  VIT_LAUNCH_CHECK("vit_im2col");
}

extern "C" int vit_embed_grad(const float* dh0, int64_t B, int64_t N, int64_t D, float* dpos, float* dcls,
                              float* dconv_bias, const vit_dropout* dropout, vit_stream_t stream) {
  VIT_CHECK_ARG(dh0 && dpos && dcls && dconv_bias && B > 0 && N > 0 && D > 0, "vit_embed_grad: bad args");
  hipStream_t s = (hipStream_t)stream;
  int ys = 0;
  if (D % 4 == 0 && ((uintptr_t)dh0 % 16) == 0 && ((uintptr_t)dpos % 16) == 0) {
    // column slices of at most 96 float4 columns, at least 2 when the rows alone leave CUs idle
    const int d4 = (int)(D / 4);
    for (int y = (d4 + 95) / 96; y <= d4; ++y)
      if (d4 % y == 0) { ys = y; break; }
    if (ys == 1 && N < 256 && d4 % 2 == 0) ys = 2;
  }
  if (ys > 0)
    hipLaunchKernelGGL(pos_grad4_kernel, dim3((unsigned)N, (unsigned)ys), dim3((unsigned)(8 * (D / 4 / ys))), 0, s, dh0,
                       (int)B, (int)N, (int)D, dpos, make_drop(dropout));
  else
    hipLaunchKernelGGL(pos_grad_kernel, dim3((unsigned)((D + 255) / 256), (unsigned)N), dim3(256), 0, s, dh0, (int)B,
                       (int)N, (int)D, dpos, make_drop(dropout));
  hipLaunchKernelGGL(cls_bias_grad16_kernel, dim3((unsigned)((D + 15) / 16)), dim3(256), 0, s, dpos, (int)N, (int)D,
                     dcls, dconv_bias);
  VIT_LAUNCH_CHECK("vit_embed_grad");
}

extern "C" int64_t vit_colsum_partial_rows(int64_t rows) {
  int64_t c = rows / COLSUM_MIN_ROWS_PER_CHUNK;
  if (c > COLSUM_MAX_CHUNKS) c = COLSUM_MAX_CHUNKS;
  return c < 1 ? 1 : c;
}

extern "C" int vit_colsum3(const void* in, int32_t in_bf16, int64_t rows, int64_t seg, int64_t ld, float* partial,
                           float* out0, float* out1, float* out2, int32_t accumulate, vit_stream_t stream) {
  const int64_t cols = 3 * seg;
  VIT_CHECK_ARG(in && partial && seg > 0 && ld >= cols, "vit_colsum3: bad args");
  const int chunks = (int)vit_colsum_partial_rows(rows);
  const bool vec = cols % 8 == 0 && ld % 8 == 0 && ((uintptr_t)in % 32) == 0 && ((uintptr_t)partial % 16) == 0;
  VIT_CHECK_ARG(vec, "vit_colsum3: needs 8-column aligned rows");
  hipStream_t s = (hipStream_t)stream;
  const unsigned gx = (unsigned)((cols / 8 + 31) / 32);
  if (chunks == 1) {
    if (in_bf16)
      hipLaunchKernelGGL(colsum8_kernel<true>, dim3(gx, 1), dim3(256), 0, s, in, (long)rows, (int)cols, (long)ld, 1,
                         out0, (int)accumulate, (long)seg, out1, out2);
    else
      hipLaunchKernelGGL(colsum8_kernel<false>, dim3(gx, 1), dim3(256), 0, s, in, (long)rows, (int)cols, (long)ld, 1,
                         out0, (int)accumulate, (long)seg, out1, out2);
    VIT_LAUNCH_CHECK("vit_colsum3");
  }
  if (in_bf16)
    hipLaunchKernelGGL(colsum8_kernel<true>, dim3(gx, chunks), dim3(256), 0, s, in, (long)rows, (int)cols, (long)ld,
                       chunks, partial, 0, 0L, (float*)nullptr, (float*)nullptr);
  else
    hipLaunchKernelGGL(colsum8_kernel<false>, dim3(gx, chunks), dim3(256), 0, s, in, (long)rows, (int)cols, (long)ld,
                       chunks, partial, 0, 0L, (float*)nullptr, (float*)nullptr);
  hipLaunchKernelGGL(colsum8_kernel<false>, dim3(gx, 1), dim3(256), 0, s, (const void*)partial, (long)chunks,
                     (int)cols, (long)cols, 1, out0, (int)accumulate, (long)seg, out1, out2);
  VIT_LAUNCH_CHECK("vit_colsum3");
}

extern "C" int vit_colsum(const void* in, int32_t in_bf16, int64_t rows, int64_t cols, int64_t ld, float* partial,
                          float* out, int32_t accumulate, vit_stream_t stream) {
  VIT_CHECK_ARG(in && partial && out && cols > 0 && ld >= cols, "vit_colsum: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int chunks = (int)vit_colsum_partial_rows(rows);
  const bool vec = cols % 8 == 0 && ld % 8 == 0 && ((uintptr_t)in % 32) == 0 && ((uintptr_t)partial % 16) == 0 &&
                   ((uintptr_t)out % 4) == 0;
  if (vec) {
    const unsigned gx = (unsigned)((cols / 8 + 31) / 32);
    float* dst1 = chunks == 1 ? out : partial;
    if (in_bf16)
      hipLaunchKernelGGL(colsum8_kernel<true>, dim3(gx, chunks), dim3(256), 0, s, in, (long)rows, (int)cols, (long)ld,
                         chunks, dst1, chunks == 1 ? (int)accumulate : 0);
    else
      hipLaunchKernelGGL(colsum8_kernel<false>, dim3(gx, chunks), dim3(256), 0, s, in, (long)rows, (int)cols,
                         (long)ld, chunks, dst1, chunks == 1 ? (int)accumulate : 0);
    if (chunks > 1)
      hipLaunchKernelGGL(colsum8_kernel<false>, dim3(gx, 1), dim3(256), 0, s, (const void*)partial, (long)chunks,
                         (int)cols, (long)cols, 1, out, (int)accumulate);
    VIT_LAUNCH_CHECK("vit_colsum");
  }
  const unsigned gx = (unsigned)((cols + 255) / 256);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(gx, chunks), dim3(256), 0, s, in, (int)in_bf16, (long)rows, (int)cols,
                     (long)ld, chunks, partial);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(gx), dim3(256), 0, s, partial, chunks, (int)cols, out, (int)accumulate);
  VIT_LAUNCH_CHECK("vit_colsum");
}

// ---- batched column sums: every bias-gradient reduction of one encoder layer in one launch ----------
// A workgroup owns 64 columns of one job: 16 column groups of 4 (one 16-B load per row) x 16 row lanes,
// eight rows in flight per lane, then a fixed-order sum of the 16 lanes through LDS (deterministic).
// The jobs ride in the kernel argument (no descriptor upload); workgroups [blk0_j, blk0_{j+1}) are job j's.
namespace {
struct ColsumJobDev {
  const float* in;
  float* out[3];
  long ld;
  int rows, cols, seg, acc, blk0;
  int pad;  // 1: cols % 4 == 0, ld % 4 == 0 and 16-B aligned rows (vector loads)
};
struct ColsumBatchDev {
  ColsumJobDev j[VIT_COLSUM_BATCH_MAX];
  int n;
};

__global__ void __launch_bounds__(256) colsum_batch_kernel(const ColsumBatchDev bt) {
  __shared__ float4 red[16][17];
  const int bid = blockIdx.x;
  int jx = 0;
#pragma unroll
  for (int k = 1; k < VIT_COLSUM_BATCH_MAX; ++k)
    if (k < bt.n && bid >= bt.j[k].blk0) jx = k;
  const ColsumJobDev& J = bt.j[jx];
  const int c0 = (bid - J.blk0) * 64;
  const int cg = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int c = c0 + cg * 4;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  if (J.pad && c < J.cols) {  // 16-B rows: one float4 per row, eight rows in flight
    const float* p = J.in + c;
    const long ld = J.ld;
    int r = rl;
    for (; r + 112 < J.rows; r += 128) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(p + (long)(r + 16 * u) * ld);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
    for (; r < J.rows; r += 16) {
      const float4 v = *reinterpret_cast<const float4*>(p + (long)r * ld);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  } else if (c < J.cols) {  // any width / stride (e.g. a 10-class head): scalar loads, same order
    const float* p = J.in + c;
    const int nc = J.cols - c < 4 ? J.cols - c : 4;
    for (int r = rl; r < J.rows; r += 16) {
      const float* q = p + (long)r * J.ld;
      acc.x += q[0];
      if (nc > 1) acc.y += q[1];
      if (nc > 2) acc.z += q[2];
      if (nc > 3) acc.w += q[3];
    }
  }
  red[rl][cg] = acc;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int g = threadIdx.x >> 2, k = threadIdx.x & 3;
    const int col = c0 + threadIdx.x;
    if (col < J.cols) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) s += reinterpret_cast<const float*>(&red[q][g])[k];
      const int sg = J.seg > 0 ? col / J.seg : 0;
      float* base = J.out[sg];
      if (base) {
        float* dst = base + (col - sg * J.seg);
        *dst = J.acc ? *dst + s : s;
      }
    }
  }
}
}  // namespace

extern "C" int vit_colsum_batch(const vit_colsum_job* jobs, int32_t njobs, vit_stream_t stream) {
  VIT_CHECK_ARG(jobs && njobs >= 1 && njobs <= VIT_COLSUM_BATCH_MAX, "vit_colsum_batch: njobs=%d outside [1, %d]",
                (int)njobs, VIT_COLSUM_BATCH_MAX);
  ColsumBatchDev bt{};
  int blk = 0;
  for (int k = 0; k < njobs; ++k) {
    const vit_colsum_job& s = jobs[k];
    VIT_CHECK_ARG(s.in && s.rows >= 1 && s.cols >= 1 && s.ld >= s.cols && s.rows <= 0x7fffffff &&
                      s.cols <= 0x7fffffff,
                  "vit_colsum_batch: job %d: bad shape (rows %lld, cols %lld, ld %lld)", k, (long long)s.rows,
                  (long long)s.cols, (long long)s.ld);
    VIT_CHECK_ARG(s.seg >= 0 && (s.seg == 0 || s.cols <= 3 * s.seg), "vit_colsum_batch: job %d: seg %lld", k,
                  (long long)s.seg);
    VIT_CHECK_ARG(s.out0 || s.out1 || s.out2, "vit_colsum_batch: job %d has no output", k);
    ColsumJobDev& d = bt.j[k];
    d.in = s.in;
    d.out[0] = s.out0;
    d.out[1] = s.out1;
    d.out[2] = s.out2;
    d.ld = (long)s.ld;
    d.rows = (int)s.rows;
    d.cols = (int)s.cols;
    d.seg = (int)s.seg;
    d.acc = s.accumulate ? 1 : 0;
    d.blk0 = blk;
    d.pad = (s.cols % 4 == 0 && s.ld % 4 == 0 && ((uintptr_t)s.in % 16) == 0) ? 1 : 0;
    blk += (int)((s.cols + 63) / 64);
  }
  bt.n = njobs;
  hipLaunchKernelGGL(colsum_batch_kernel, dim3(blk), dim3(256), 0, (hipStream_t)stream, bt);
  return vit::check_hip(hipGetLastError(), "vit_colsum_batch");
}

extern "C" int vit_gemm_f32(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int32_t a_trans,
                            const float* B, int64_t ldb, int32_t b_trans, float* C, int64_t ldc, const float* bias,
                            int32_t accumulate, vit_stream_t stream) {
  VIT_CHECK_ARG(A && B && C && M >= 0 && N >= 0 && K >= 0, "vit_gemm_f32: bad args");
  if (M == 0 || N == 0) return VIT_OK;
  dim3 grid((unsigned)((N + 31) / 32), (unsigned)((M + 31) / 32)), block(256);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, block, 0, (hipStream_t)stream, (int)M, (int)N, (int)K, A, (long)lda,
                     (int)a_trans, B, (long)ldb, (int)b_trans, C, (long)ldc, bias, (int)accumulate);
  VIT_LAUNCH_CHECK("vit_gemm_f32");
}

extern "C" int vit_cross_entropy(const float* logits, const int64_t* labels, int64_t B, int64_t C, float* dlogits,
                                 float grad_scale, float* row_stats, vit_stream_t stream) {
  VIT_CHECK_ARG(logits && labels && B > 0 && C > 0, "vit_cross_entropy: bad args");
  hipLaunchKernelGGL(ce_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, logits, labels, (int)C, dlogits,
                     grad_scale, row_stats);
  VIT_LAUNCH_CHECK("vit_cross_entropy");
}

extern "C" int vit_sgd_step_dev(float* p, const float* g, float* buf, void* p_bf16, int64_t n, const float* hyper,
                                float weight_decay, vit_stream_t stream) {
  VIT_CHECK_ARG(p && g && buf && hyper && n >= 0, "vit_sgd_step_dev: bad args");
  VIT_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)buf) % 16 == 0 && ((uintptr_t)p_bf16 % 8 == 0),
                "vit_sgd_step_dev: buffers must be 16-B aligned (bf16 mirror 8-B)");
  if (n == 0) return VIT_OK;
  hipLaunchKernelGGL(sgd_kernel<SgdDevScalars>, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, p, g, buf,
                     (bf16_t*)p_bf16, (long)n, SgdDevScalars{hyper}, weight_decay);
  VIT_LAUNCH_CHECK("vit_sgd_step_dev");
}

extern "C" int vit_sgd_step(float* p, const float* g, float* buf, void* p_bf16, int64_t n, float lr, float momentum,
                            float weight_decay, int32_t first, vit_stream_t stream) {
  VIT_CHECK_ARG(p && g && buf && n >= 0, "vit_sgd_step: bad args");
  VIT_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)buf) % 16 == 0 && ((uintptr_t)p_bf16 % 8 == 0),
                "vit_sgd_step: buffers must be 16-B aligned (bf16 mirror 8-B)");
  if (n == 0) return VIT_OK;
  hipLaunchKernelGGL(sgd_kernel<SgdHostScalars>, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, p, g, buf,
                     (bf16_t*)p_bf16, (long)n, SgdHostScalars{lr, momentum, (int)first}, weight_decay);
  VIT_LAUNCH_CHECK("vit_sgd_step");
}

extern "C" int vit_cast_f32_bf16(const float* in, void* out, int64_t n, vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && n >= 0, "vit_cast_f32_bf16: bad args");
  if (n == 0) return VIT_OK;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, in, (bf16_t*)out, (long)n);
  VIT_LAUNCH_CHECK("vit_cast_f32_bf16");
}

extern "C" int vit_cast_pad_rows(const float* in, int64_t rows, int64_t cols, void* out, int64_t ldo,
                                 vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && ldo >= cols, "vit_cast_pad_rows: bad args");
  if (rows * ldo == 0) return VIT_OK;
  hipLaunchKernelGGL(cast_pad_kernel, dim3(grid_for(rows * ldo)), dim3(256), 0, (hipStream_t)stream, in, (long)rows,
                     (long)cols, (bf16_t*)out, (long)ldo);
  VIT_LAUNCH_CHECK("vit_cast_pad_rows");
}

// ---- batched f32 -> bf16 casts into zero-padded operands: several small weight / operand casts in one launch -----
namespace {
struct CastJobDev {
  const float* in;
  bf16_t* out;
  long rows, cols, ldi, ldo, rows_pad, cols_pad;
  int blk0, nb;
  int vec;  // 4-column pieces (float4 in, 8-B out): every width / leading dimension a multiple of 4, aligned rows
};
struct CastBatchDev {
  CastJobDev j[VIT_CAST_BATCH_MAX];
  int n;
};
__global__ void __launch_bounds__(256) cast_pad_batch_kernel(const CastBatchDev bt) {
  int jx = 0;
#pragma unroll
  for (int k = 1; k < VIT_CAST_BATCH_MAX; ++k)
    if (k < bt.n && (int)blockIdx.x >= bt.j[k].blk0) jx = k;
  const CastJobDev& J = bt.j[jx];
  if (J.vec) {  // (the big operand casts: 32-bit index math, 16 B read and 8 B written per thread and step)
    const unsigned cq = (unsigned)(J.cols_pad >> 2), tq = (unsigned)(J.rows_pad * cq);
    for (unsigned q = (blockIdx.x - J.blk0) * 256u + threadIdx.x; q < tq; q += (unsigned)J.nb * 256u) {
      const unsigned r = q / cq, c = (q - r * cq) << 2;
      uint2 o = {0u, 0u};
      if (r < J.rows && c < J.cols) {
        const float4 v = *reinterpret_cast<const float4*>(J.in + r * J.ldi + c);
        o.x = pack2bf(v.x, v.y);
        o.y = pack2bf(v.z, v.w);
      }
      *reinterpret_cast<uint2*>(J.out + r * J.ldo + c) = o;
    }
    return;
  }
  const long total = J.rows_pad * J.cols_pad;
  for (long i = (long)(blockIdx.x - J.blk0) * 256 + threadIdx.x; i < total; i += (long)J.nb * 256) {
    const long r = i / J.cols_pad, c = i - r * J.cols_pad;
    J.out[r * J.ldo + c] = r < J.rows && c < J.cols ? f2bf(J.in[r * J.ldi + c]) : (bf16_t)0;
  }
}
}  // namespace

extern "C" int vit_cast_pad_batch(const vit_cast_job* jobs, int32_t njobs, vit_stream_t stream) {
  VIT_CHECK_ARG(jobs && njobs >= 1 && njobs <= VIT_CAST_BATCH_MAX, "vit_cast_pad_batch: 1..%d jobs, got %d",
                VIT_CAST_BATCH_MAX, (int)njobs);
  CastBatchDev bt{};
  long blk = 0;
  for (int k = 0; k < njobs; ++k) {
    const vit_cast_job& j = jobs[k];
    VIT_CHECK_ARG(j.in && j.out && j.rows >= 0 && j.cols >= 0 && j.ldi >= j.cols && j.rows_pad >= j.rows &&
                      j.cols_pad >= j.cols && j.ldo >= j.cols_pad,
                  "vit_cast_pad_batch: job %d: bad shape", k);
    const int vec = (j.cols | j.cols_pad | j.ldi | j.ldo) % 4 == 0 && (uintptr_t)j.in % 16 == 0 &&
                    (uintptr_t)j.out % 8 == 0 && j.rows_pad * j.cols_pad / 4 < (1L << 31) ? 1 : 0;
    long nb = (j.rows_pad * j.cols_pad / (vec ? 4 : 1) + 255) / 256;
    if (nb > 2048) nb = 2048;
    if (nb < 1) nb = 1;
    CastJobDev& d = bt.j[k];
    d.in = j.in; d.out = (bf16_t*)j.out; d.rows = j.rows; d.cols = j.cols; d.ldi = j.ldi; d.ldo = j.ldo;
    d.rows_pad = j.rows_pad; d.cols_pad = j.cols_pad; d.blk0 = (int)blk; d.nb = (int)nb;
    d.vec = vec;
    blk += nb;
  }
  bt.n = njobs;
  hipLaunchKernelGGL(cast_pad_batch_kernel, dim3((unsigned)blk), dim3(256), 0, (hipStream_t)stream, bt);
  VIT_LAUNCH_CHECK("vit_cast_pad_batch");
}

extern "C" int vit_axpby(const float* x, float* y, int64_t n, float a, float b, vit_stream_t stream) {
  VIT_CHECK_ARG(x && y && n >= 0, "vit_axpby: bad args");
  if (n == 0) return VIT_OK;
  hipLaunchKernelGGL(axpby_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, y, (long)n, a, b);
  VIT_LAUNCH_CHECK("vit_axpby");
}

// ---- column-block gather/cast: out[r][z*cols + c] = in[z*zstride + r*ldi + c] ------------------
// Packs the q/k/v LinearGeneral weights [D][H,hd] x 3 into one [D][3D] bf16 operand (and the
// biases into [3D] f32) so the fused QKV projection is a single GEMM.
namespace {
template <bool BF16OUT>
__global__ void pack_cols_kernel(const float* __restrict__ in, long zstride, long ldi, int rows, int cols, int Z,
                                 void* __restrict__ out, long ldo, long in_bs = 0, long out_bs = 0) {
  in += (long)blockIdx.y * in_bs;  // batch (blockIdx.y): one matrix set per encoder layer
  out = (char*)out + (long)blockIdx.y * out_bs * (BF16OUT ? 2 : 4);
  const long total = (long)rows * Z * cols;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / ((long)Z * cols);
    const int zc = (int)(i % ((long)Z * cols));
    const int z = zc / cols, c = zc % cols;
    const float v = in[z * zstride + r * ldi + c];
    if constexpr (BF16OUT)
      ((bf16_t*)out)[r * ldo + zc] = f2bf(v);
    else
      ((float*)out)[r * ldo + zc] = v;
  }
}
}  // namespace

extern "C" int vit_pack_cols(const float* in, int64_t zstride, int64_t ldi, int64_t rows, int64_t cols, int64_t Z,
                             void* out, int64_t ldo, int32_t out_bf16, vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && rows >= 0 && cols >= 0 && Z >= 1 && ldo >= Z * cols, "vit_pack_cols: bad args");
  const long total = rows * Z * cols;
  if (total == 0) return VIT_OK;
  if (out_bf16)
    hipLaunchKernelGGL(pack_cols_kernel<true>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, in,
                       (long)zstride, (long)ldi, (int)rows, (int)cols, (int)Z, out, (long)ldo);
  else
    hipLaunchKernelGGL(pack_cols_kernel<false>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, in,
                       (long)zstride, (long)ldi, (int)rows, (int)cols, (int)Z, out, (long)ldo);
  VIT_LAUNCH_CHECK("vit_pack_cols");
}

extern "C" int vit_pack_cols_batched(const float* in, int64_t in_batch_stride, int64_t zstride, int64_t ldi,
                                     int64_t rows, int64_t cols, int64_t Z, void* out, int64_t out_batch_stride,
                                     int64_t ldo, int32_t out_bf16, int64_t batch, vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && rows >= 0 && cols >= 0 && Z >= 1 && ldo >= Z * cols && batch >= 1 && batch < 65536,
                "vit_pack_cols_batched: bad args");
  const long total = rows * Z * cols;
  if (total == 0) return VIT_OK;
  long gx = (total + 255) / 256;
  if (gx > 1024) gx = 1024;
  const dim3 grid((unsigned)gx, (unsigned)batch);
  if (out_bf16)
    hipLaunchKernelGGL(pack_cols_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, in, (long)zstride, (long)ldi,
                       (int)rows, (int)cols, (int)Z, out, (long)ldo, (long)in_batch_stride, (long)out_batch_stride);
  else
    hipLaunchKernelGGL(pack_cols_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, in, (long)zstride, (long)ldi,
                       (int)rows, (int)cols, (int)Z, out, (long)ldo, (long)in_batch_stride, (long)out_batch_stride);
  VIT_LAUNCH_CHECK("vit_pack_cols_batched");
}

// ---- transposed bf16 weight copies: out[c*ldo + r] = bf16(in[r*ldi + c]) ---------------------------
// Keeps a K-contiguous copy of every weight whose natural layout would make a GEMM operand
// M/N-contiguous (fc1 / fc2 dgrad, out-proj and fused-QKV forward), so every forward and dgrad GEMM
// runs on the both-K-contiguous ping-pong kernel. 64 x 64 tiles through LDS, coalesced both ways.
namespace {
__global__ void __launch_bounds__(256) transpose_f32_bf16_kernel(const float* __restrict__ in, long ldi, int rows,
                                                                 int cols, bf16_t* __restrict__ out, long ldo,
                                                                 long in_bs, long out_bs, int vec) {
  __shared__ float tile[64][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  in += blockIdx.z * in_bs;
  out += blockIdx.z * out_bs;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int r = r0 + ty + 4 * k, c = c0 + tx;
    tile[ty + 4 * k][tx] = (r < rows && c < cols) ? in[(long)r * ldi + c] : 0.f;
  }
  __syncthreads();
  // each thread: 16 consecutive outputs of one output row (two 16-B stores; 2-B stores per lane made
  // this kernel store-instruction-bound)
  const int oc = threadIdx.x >> 2, seg = (threadIdx.x & 3) * 16;
  const int c = c0 + oc;
  if (c >= cols) return;
  bf16_t* o = out + (long)c * ldo + r0 + seg;
  if (vec && r0 + seg + 16 <= rows) {
    unsigned w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = pack2bf(tile[seg + 2 * j][oc], tile[seg + 2 * j + 1][oc]);
    *reinterpret_cast<uint4*>(o) = make_uint4(w[0], w[1], w[2], w[3]);
    *reinterpret_cast<uint4*>(o + 8) = make_uint4(w[4], w[5], w[6], w[7]);
  } else {
    for (int j = 0; j < 16 && r0 + seg + j < rows; ++j) o[j] = f2bf(tile[seg + j][oc]);
  }
}
}  // namespace

extern "C" int vit_transpose_f32_bf16(const float* in, int64_t rows, int64_t cols, int64_t ldi, void* out,
                                      int64_t ldo, int64_t batch, int64_t in_batch_stride, int64_t out_batch_stride,
                                      vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && rows >= 0 && cols >= 0 && ldi >= cols && ldo >= rows && batch >= 1,
                "vit_transpose_f32_bf16: bad args");
  if (rows == 0 || cols == 0) return VIT_OK;
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64), (unsigned)batch);
  const int vec = ldo % 8 == 0 && out_batch_stride % 8 == 0 && (uintptr_t)out % 16 == 0;
  hipLaunchKernelGGL(transpose_f32_bf16_kernel, grid, dim3(256), 0, (hipStream_t)stream, in, (long)ldi, (int)rows,
                     (int)cols, (bf16_t*)out, (long)ldo, (long)in_batch_stride, (long)out_batch_stride, vec);
  VIT_LAUNCH_CHECK("vit_transpose_f32_bf16");
}


// ---- fp32 (exact) forward helpers -----------------------------------------------------------------
namespace {
// h[b*N + t] = (t == 0 ? cls : h[b*N + t]) + pos[t]  (src/model.py:203-204, PositionEmbs :16-17)
__global__ void embed_fwd_kernel(float* __restrict__ h, int B, int N, int D, const float* __restrict__ pos,
                                 const float* __restrict__ cls) {
  const long total = (long)B * N * D;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const int t = (int)((i / D) % N);
    h[i] = (t == 0 ? cls[d] : h[i]) + pos[(long)t * D + d];
  }
}
// exact-erf GELU, nn.GELU() (src/model.py:33)
__global__ void gelu_f32_kernel(const float* __restrict__ in, float* __restrict__ out, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float u = in[i];
    out[i] = 0.5f * u * (1.0f + erff(u * 0.70710678118654752f));
  }
}
}  // namespace

extern "C" int vit_im2col_f32(const float* x, float* out, int64_t B, int64_t img, int64_t P, int64_t Kpad,
                              vit_stream_t stream) {
  VIT_CHECK_ARG(x && out && B > 0 && P > 0 && img >= P && Kpad >= 3 * P * P, "vit_im2col_f32: bad args");
  const int64_t g = img / P, N = g * g + 1;
  if (P % 8 == 0 && img % 4 == 0 && Kpad == 3 * P * P && (uintptr_t)x % 16 == 0 && (uintptr_t)out % 16 == 0)
    hipLaunchKernelGGL(im2col8_kernel<float>, dim3(grid_for(B * N * Kpad / 8)), dim3(256), 0, (hipStream_t)stream, x,
                       out, (int)B, (int)img, (int)P);
  else
    hipLaunchKernelGGL(im2col_kernel<float>, dim3(grid_for(B * N * Kpad)), dim3(256), 0, (hipStream_t)stream, x, out,
                       (int)B, (int)img, (int)P, (int)Kpad);
  VIT_LAUNCH_CHECK("vit_im2col_f32");
}

extern "C" int vit_embed_fwd_f32(float* h, int64_t B, int64_t N, int64_t D, const float* pos, const float* cls,
                                 vit_stream_t stream) {
  VIT_CHECK_ARG(h && pos && cls && B > 0 && N > 0 && D > 0, "vit_embed_fwd_f32: bad args");
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(grid_for(B * N * D)), dim3(256), 0, (hipStream_t)stream, h, (int)B,
                     (int)N, (int)D, pos, cls);
  VIT_LAUNCH_CHECK("vit_embed_fwd_f32");
}

extern "C" int vit_gelu_f32(const float* in, float* out, int64_t n, vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && n >= 0, "vit_gelu_f32: bad args");
  if (n == 0) return VIT_OK;
  hipLaunchKernelGGL(gelu_f32_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, in, out, (long)n);
  VIT_LAUNCH_CHECK("vit_gelu_f32");
}

extern "C" int vit_dropout_mask(const vit_dropout* d, int64_t row0, int64_t rows, int64_t cols, float* mult,
                                int64_t ld, vit_stream_t stream) {
  VIT_CHECK_ARG(mult && rows >= 0 && rows <= 65535 && cols > 0 && ld >= cols, "vit_dropout_mask: bad args");
  if (rows == 0) return VIT_OK;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3((unsigned)((cols + 255) / 256), (unsigned)rows), dim3(256), 0,
                     (hipStream_t)stream, make_drop(d), (long)row0, (long)rows, (int)cols, mult, (long)ld);
  VIT_LAUNCH_CHECK("vit_dropout_mask");
}

// ---- standalone sub-module path (vitmi.model Encoder / EncoderBlock / MlpBlock / ... .forward) ----
namespace {
// dx = dy * GELU'(u), exact erf (nn.GELU backward, src/model.py:33)
__global__ void gelu_bwd_f32_kernel(const float* __restrict__ u, const float* __restrict__ dy, float* __restrict__ dx,
                                    long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = u[i];
    const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
    const float pdf = 0.39894228040143268f * expf(-0.5f * x * x);
    dx[i] = dy[i] * (cdf + x * pdf);
  }
}
// out[r][c] = in[r][c] * dropout multiplier of (r, c)  (nn.Dropout, src/model.py:19-20,46-51,124-125)
__global__ void dropout_apply_kernel(DropDev drop, const float* __restrict__ in, float* __restrict__ out, long rows,
                                     int cols) {
  const long total = rows * cols;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols;
    const int c = (int)(i % cols);
    out[i] = in[i] * drop_mult1(drop, r, c);
  }
}
// out[o*inner + i] = x[o*inner + i] + y[i]   (broadcast add: PositionEmbs, src/model.py:17)
__global__ void add_bcast_kernel(const float* __restrict__ x, const float* __restrict__ y, float* __restrict__ out,
                                 long outer, long inner) {
  const long total = outer * inner;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x)
    out[i] = x[i] + y[i % inner];
}
}  // namespace

extern "C" int vit_gelu_bwd_f32(const float* u, const float* dy, float* dx, int64_t n, vit_stream_t stream) {
  VIT_CHECK_ARG(u && dy && dx && n >= 0, "vit_gelu_bwd_f32: bad args");
  if (n == 0) return VIT_OK;
  hipLaunchKernelGGL(gelu_bwd_f32_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, u, dy, dx, (long)n);
  VIT_LAUNCH_CHECK("vit_gelu_bwd_f32");
}

extern "C" int vit_dropout_apply_f32(const vit_dropout* d, const float* in, float* out, int64_t rows, int64_t cols,
                                     vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && rows >= 0 && cols > 0, "vit_dropout_apply_f32: bad args");
  if (rows == 0) return VIT_OK;
  hipLaunchKernelGGL(dropout_apply_kernel, dim3(grid_for(rows * cols)), dim3(256), 0, (hipStream_t)stream,
                     make_drop(d), in, out, (long)rows, (int)cols);
  VIT_LAUNCH_CHECK("vit_dropout_apply_f32");
}

extern "C" int vit_add_bcast_f32(const float* x, const float* y, float* out, int64_t outer, int64_t inner,
                                 vit_stream_t stream) {
  VIT_CHECK_ARG(x && y && out && outer >= 0 && inner > 0, "vit_add_bcast_f32: bad args");
  if (outer == 0) return VIT_OK;
  hipLaunchKernelGGL(add_bcast_kernel, dim3(grid_for(outer * inner)), dim3(256), 0, (hipStream_t)stream, x, y, out,
                     (long)outer, (long)inner);
  VIT_LAUNCH_CHECK("vit_add_bcast_f32");
}

// ---- Res-ViT router backward helpers (res-vit/model.py:186-190 RouterModule: the global half of out_conv's
// input and in_conv's GELU) ------------------------------------------------------------------------------------
namespace {
// out[s][c] = scale * sum over rows [s * seg_stride + row0, + seg_rows) of in[row][c]. Workgroup = (segment, 128
// columns): 4 row lanes x 64 column pairs, each lane sums every 4th row (four rows in flight), the lanes are added
// in order through LDS (deterministic)
template <bool BF16>
__global__ void __launch_bounds__(256) segment_colsum_kernel(const void* __restrict__ in, long ld, long seg_stride,
                                                             long row0, long seg_rows, int cols, float scale,
                                                             float* __restrict__ out, long ldo,
                                                             bf16_t* __restrict__ bc, long ldbc, long bc_rows) {
  __shared__ float2 red[4][64];
  const int cp = threadIdx.x & 63, lane_r = threadIdx.x >> 6;
  const int c = blockIdx.y * 128 + cp * 2;
  const long base = (long)blockIdx.x * seg_stride + row0;
  float2 acc = {0.f, 0.f};
  auto ld2 = [&](long r) -> float2 {
    const long i = (base + r) * ld + c;
    if constexpr (BF16) {
      if (c + 1 < cols) {
        const unsigned u = *reinterpret_cast<const unsigned*>((const bf16_t*)in + i);
        return float2{bf2f((bf16_t)(u & 0xffff)), bf2f((bf16_t)(u >> 16))};
      }
      return float2{bf2f(((const bf16_t*)in)[i]), 0.f};
    } else {
      if (c + 1 < cols) return *reinterpret_cast<const float2*>((const float*)in + i);
      return float2{((const float*)in)[i], 0.f};
    }
  };
  if (c < cols) {
    long r = lane_r;
    for (; r + 12 < seg_rows; r += 16) {
      const float2 a = ld2(r), b = ld2(r + 4), d = ld2(r + 8), e = ld2(r + 12);
      acc.x += a.x; acc.y += a.y; acc.x += b.x; acc.y += b.y;
      acc.x += d.x; acc.y += d.y; acc.x += e.x; acc.y += e.y;
    }
    for (; r < seg_rows; r += 4) {
      const float2 a = ld2(r);
      acc.x += a.x; acc.y += a.y;
    }
  }
  red[lane_r][cp] = acc;
  __syncthreads();
  if (lane_r == 0 && c < cols) {
    float2 t = red[0][cp];
#pragma unroll
    for (int q = 1; q < 4; ++q) { t.x += red[q][cp].x; t.y += red[q][cp].y; }
    float* o = out + (long)blockIdx.x * ldo + c;
    o[0] = scale * t.x;
    if (c + 1 < cols) o[1] = scale * t.y;
    red[0][cp] = float2{scale * t.x, scale * t.y};
  }
  if (bc) {  // the segment's result, rounded to bf16, into rows [s * seg_stride, + bc_rows) of bc
    __syncthreads();
    if (c < cols) {
      const float2 v = red[0][cp];
      const bf16_t b0 = f2bf(v.x), b1 = f2bf(v.y);
      bf16_t* row = bc + (long)blockIdx.x * seg_stride * ldbc + c;
      for (long r = lane_r; r < bc_rows; r += 4) {
        if (c + 1 < cols)
          *reinterpret_cast<unsigned*>(row + r * ldbc) = (unsigned)b0 | ((unsigned)b1 << 16);
        else
          row[r * ldbc] = b0;
      }
    }
  }
}

// out (bf16 [rows_pad][cols_pad]) = (dx[t][c] + [t % N >= reserve] * g_scale * g[t / N][c]) * gp[t][c] on the T x cols
// block, rounded once to bf16, zero elsewhere; col_partial[blockIdx.y][c] = the column sums of the rounded values of
// the block's RB rows. A thread owns a column pair (cols_pad, ldx, ldgp, ldo even) and walks the block's rows RDG_U at
// a time, every load of the group issued before any use (one row at a time left the kernel waiting on HBM latency:
// 72 us for 25 216 x 512), with the image / position counters stepped, not divided, per row
constexpr int RDG_RB = 32;
constexpr int RDG_U = 8;  // rows whose loads are in flight together
__global__ void __launch_bounds__(256) router_dx_gate_kernel(const float* __restrict__ dx, long ldx,
                                                             const float* __restrict__ g, long ldg, float g_scale,
                                                             const bf16_t* __restrict__ gp, long ldgp, long T, long N,
                                                             long reserve, int cols, bf16_t* __restrict__ out,
                                                             long ldo, long rows_pad, int cols_pad,
                                                             float* __restrict__ col_partial, long ldp) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 2;
  if (c >= cols_pad) return;
  const long r0 = (long)blockIdx.y * RDG_RB;
  const long r1 = r0 + RDG_RB < rows_pad ? r0 + RDG_RB : rows_pad;
  const long tv = r1 < T ? r1 : T;  // rows [r0, tv) hold data
  const bool c0v = c < cols, c1v = c + 1 < cols;
  long img = r0 / N, pos = r0 - img * N;
  float a0 = 0.f, a1 = 0.f;
  for (long t = r0; t < r1; t += RDG_U) {
    float2 dv[RDG_U], gv[RDG_U];
    unsigned gu[RDG_U];
    bool ok[RDG_U];
#pragma unroll
    for (int k = 0; k < RDG_U; ++k) {
      ok[k] = c0v && t + k < tv;
      dv[k] = float2{0.f, 0.f};
      gv[k] = float2{0.f, 0.f};
      gu[k] = 0u;
      if (ok[k]) {
        const float* d = dx + (t + k) * ldx + c;
        const float* gr = g + img * ldg + c;
        if (c1v) {  // (dx and g rows 8-B aligned: checked by the launcher)
          dv[k] = *reinterpret_cast<const float2*>(d);
          if (pos >= reserve) {
            const float2 gg = *reinterpret_cast<const float2*>(gr);
            gv[k] = float2{__fmul_rn(g_scale, gg.x), __fmul_rn(g_scale, gg.y)};
          }
        } else {
          dv[k].x = d[0];
          if (pos >= reserve) gv[k].x = __fmul_rn(g_scale, gr[0]);
        }
        gu[k] = *reinterpret_cast<const unsigned*>(gp + (t + k) * ldgp + c);
      }
      if (++pos == N) {
        pos = 0;
        ++img;
      }
    }
#pragma unroll
    for (int k = 0; k < RDG_U; ++k) {
      if (t + k >= r1) break;
      unsigned o = 0u;
      if (ok[k]) {
        const bf16_t o0 = f2bf(__fmul_rn(__fadd_rn(dv[k].x, gv[k].x), bf2f((bf16_t)(gu[k] & 0xffff))));
        const bf16_t o1 = c1v ? f2bf(__fmul_rn(__fadd_rn(dv[k].y, gv[k].y), bf2f((bf16_t)(gu[k] >> 16)))) : (bf16_t)0;
        a0 += bf2f(o0);
        a1 += bf2f(o1);
        o = (unsigned)o0 | ((unsigned)o1 << 16);
      }
      *reinterpret_cast<unsigned*>(out + (t + k) * ldo + c) = o;
    }
  }
  if (col_partial) {
    if (c0v) col_partial[blockIdx.y * ldp + c] = a0;
    if (c1v) col_partial[blockIdx.y * ldp + c + 1] = a1;
  }
}

// the common case of router_dx_gate_kernel (cols even and equal to cols_pad, T >= 1): no per-row branch, every load of
// a group of RDG_U rows issued unconditionally (rows past T clamped to row T - 1 and their results discarded), so the
// loads of a group are in flight together
__global__ void __launch_bounds__(256) router_dx_gate_pair_kernel(const float* __restrict__ dx, long ldx,
                                                                  const float* __restrict__ g, long ldg,
                                                                  float g_scale, const bf16_t* __restrict__ gp,
                                                                  long ldgp, long T, long N, long reserve, int cols,
                                                                  bf16_t* __restrict__ out, long ldo, long rows_pad,
                                                                  float* __restrict__ col_partial, long ldp) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 2;
  if (c >= cols) return;
  const long r0 = (long)blockIdx.y * RDG_RB;
  const long r1 = r0 + RDG_RB < rows_pad ? r0 + RDG_RB : rows_pad;
  const long tlast = T - 1, ilast = (T - 1) / N;
  long img = r0 / N, pos = r0 - img * N;
  float a0 = 0.f, a1 = 0.f;
  for (long t = r0; t < r1; t += RDG_U) {
    float2 dv[RDG_U], gg[RDG_U];
    unsigned gu[RDG_U];
    float gs[RDG_U];
#pragma unroll
    for (int k = 0; k < RDG_U; ++k) {
      const long rr = t + k < tlast ? t + k : tlast;
      const long ii = img < ilast ? img : ilast;
      dv[k] = *reinterpret_cast<const float2*>(dx + rr * ldx + c);
      gg[k] = *reinterpret_cast<const float2*>(g + ii * ldg + c);
      gu[k] = *reinterpret_cast<const unsigned*>(gp + rr * ldgp + c);
      gs[k] = pos >= reserve ? g_scale : 0.f;
      if (++pos == N) {
        pos = 0;
        ++img;
      }
    }
#pragma unroll
    for (int k = 0; k < RDG_U; ++k) {
      if (t + k >= r1) break;
      const bool ok = t + k < T;
      // (no fma contraction: the same two roundings as (dx + s * g) * gp in f32 elsewhere)
      const bf16_t o0 = f2bf(__fmul_rn(__fadd_rn(dv[k].x, __fmul_rn(gs[k], gg[k].x)), bf2f((bf16_t)(gu[k] & 0xffff))));
      const bf16_t o1 = f2bf(__fmul_rn(__fadd_rn(dv[k].y, __fmul_rn(gs[k], gg[k].y)), bf2f((bf16_t)(gu[k] >> 16))));
      const unsigned o = ok ? ((unsigned)o0 | ((unsigned)o1 << 16)) : 0u;
      if (ok) {
        a0 += bf2f(o0);
        a1 += bf2f(o1);
      }
      *reinterpret_cast<unsigned*>(out + (t + k) * ldo + c) = o;
    }
  }
  if (col_partial) {
    col_partial[blockIdx.y * ldp + c] = a0;
    col_partial[blockIdx.y * ldp + c + 1] = a1;
  }
}
}  // namespace

extern "C" int vit_segment_colsum(const void* in, int32_t in_bf16, int64_t ld, int64_t segs, int64_t seg_stride,
                                  int64_t row0, int64_t seg_rows, int64_t cols, float scale, float* out, int64_t ldo,
                                  vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && segs >= 0 && seg_rows >= 0 && row0 >= 0 && seg_stride >= 0 && cols > 0 && ld >= cols &&
                    ldo >= cols && cols < (1L << 30) && ld % 2 == 0 && ((uintptr_t)in % (in_bf16 ? 4 : 8)) == 0,
                "vit_segment_colsum: bad args (even ld, 2-element aligned rows)");
  if (segs == 0) return VIT_OK;
  const dim3 grid((unsigned)segs, (unsigned)((cols + 127) / 128));
  if (in_bf16)
    hipLaunchKernelGGL(segment_colsum_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, in, (long)ld,
                       (long)seg_stride, (long)row0, (long)seg_rows, (int)cols, scale, out, (long)ldo, nullptr, 0L, 0L);
  else
    hipLaunchKernelGGL(segment_colsum_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, in, (long)ld,
                       (long)seg_stride, (long)row0, (long)seg_rows, (int)cols, scale, out, (long)ldo, nullptr, 0L,
                       0L);
  VIT_LAUNCH_CHECK("vit_segment_colsum");
}

extern "C" int vit_segment_colsum_bcast(const void* in, int32_t in_bf16, int64_t ld, int64_t segs, int64_t seg_stride,
                                        int64_t row0, int64_t seg_rows, int64_t cols, float scale, float* out,
                                        int64_t ldo, void* bc, int64_t ldbc, int64_t bc_rows, vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && bc && segs >= 0 && seg_rows >= 0 && row0 >= 0 && seg_stride >= 0 && cols > 0 &&
                    ld >= cols && ldo >= cols && ldbc >= cols && bc_rows >= 0 && bc_rows <= seg_stride &&
                    cols < (1L << 30) && ld % 2 == 0 && ldbc % 2 == 0 && ((uintptr_t)bc % 4) == 0 &&
                    ((uintptr_t)in % (in_bf16 ? 4 : 8)) == 0,
                "vit_segment_colsum_bcast: bad args (even ld / ldbc, 2-element aligned rows, bc_rows <= seg_stride)");
  if (segs == 0) return VIT_OK;
  const dim3 grid((unsigned)segs, (unsigned)((cols + 127) / 128));
  if (in_bf16)
    hipLaunchKernelGGL(segment_colsum_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, in, (long)ld,
                       (long)seg_stride, (long)row0, (long)seg_rows, (int)cols, scale, out, (long)ldo, (bf16_t*)bc,
                       (long)ldbc, (long)bc_rows);
  else
    hipLaunchKernelGGL(segment_colsum_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, in, (long)ld,
                       (long)seg_stride, (long)row0, (long)seg_rows, (int)cols, scale, out, (long)ldo, (bf16_t*)bc,
                       (long)ldbc, (long)bc_rows);
  VIT_LAUNCH_CHECK("vit_segment_colsum_bcast");
}

extern "C" int64_t vit_router_dx_gate_partial_rows(int64_t rows_pad) { return (rows_pad + RDG_RB - 1) / RDG_RB; }

extern "C" int vit_router_dx_gate(const float* dx, int64_t ldx, const float* g, int64_t ldg, float g_scale,
                                  const void* gp, int64_t ldgp, int64_t T, int64_t N, int64_t reserve, int64_t cols,
                                  void* out, int64_t ldo, int64_t rows_pad, int64_t cols_pad, float* col_partial,
                                  int64_t ldp, vit_stream_t stream) {
  VIT_CHECK_ARG(dx && g && gp && out && T >= 0 && N > 0 && reserve >= 0 && cols > 0 && cols_pad >= cols &&
                    rows_pad >= T && ldx >= cols && ldg >= cols && ldgp >= cols_pad && ldo >= cols_pad &&
                    (!col_partial || ldp >= cols) && cols_pad < (1L << 30) && cols_pad % 2 == 0 && ldgp % 2 == 0 &&
                    ldo % 2 == 0 && ((uintptr_t)gp % 4) == 0 && ((uintptr_t)out % 4) == 0 && ldx % 2 == 0 &&
                    ldg % 2 == 0 && ((uintptr_t)dx % 8) == 0 && ((uintptr_t)g % 8) == 0,
                "vit_router_dx_gate: bad args (even leading dimensions, 8-B aligned f32 / 4-B aligned bf16 rows; gp as "
                "wide as the padded output)");
  if (rows_pad == 0) return VIT_OK;
  const dim3 grid((unsigned)((cols_pad / 2 + 255) / 256), (unsigned)vit_router_dx_gate_partial_rows(rows_pad));
  if (cols % 2 == 0 && cols == cols_pad && T >= 1) {
    hipLaunchKernelGGL(router_dx_gate_pair_kernel, grid, dim3(256), 0, (hipStream_t)stream, dx, (long)ldx, g,
                       (long)ldg, g_scale, (const bf16_t*)gp, (long)ldgp, (long)T, (long)N, (long)reserve, (int)cols,
                       (bf16_t*)out, (long)ldo, (long)rows_pad, col_partial, (long)ldp);
    VIT_LAUNCH_CHECK("vit_router_dx_gate");
  }
  hipLaunchKernelGGL(router_dx_gate_kernel, grid, dim3(256), 0, (hipStream_t)stream, dx, (long)ldx, g, (long)ldg,
                     g_scale, (const bf16_t*)gp, (long)ldgp, (long)T, (long)N, (long)reserve, (int)cols, (bf16_t*)out,
                     (long)ldo, (long)rows_pad, (int)cols_pad, col_partial, (long)ldp);
  VIT_LAUNCH_CHECK("vit_router_dx_gate");
}

namespace {
__global__ void unpack_bf16_f32_kernel(const bf16_t* __restrict__ in, long ldi, long rows, int cols,
                                       float* __restrict__ out, long ldo) {
  const long total = rows * cols;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols;
    const int c = (int)(i % cols);
    out[r * ldo + c] = bf2f(in[r * ldi + c]);
  }
}
}  // namespace

extern "C" int vit_unpack_bf16_f32(const void* in, int64_t ldi, int64_t rows, int64_t cols, float* out, int64_t ldo,
                                   vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && rows >= 0 && cols > 0 && ldi >= cols && ldo >= cols, "vit_unpack_bf16_f32: bad args");
  if (rows == 0) return VIT_OK;
  hipLaunchKernelGGL(unpack_bf16_f32_kernel, dim3(grid_for(rows * cols)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)in, (long)ldi, (long)rows, (int)cols, out, (long)ldo);
  VIT_LAUNCH_CHECK("vit_unpack_bf16_f32");
}

// ---- Res-ViT router head (res-vit/model.py:191-211: RouterModule.forward after out_conv) ----------------------------
// Per token t and block position i (logits [T][bs][2], T = B * N rows): soft = softmax(logits) in the arithmetic of
// torch's two-element warp softmax (max, exp(x - max), sum, x / sum); the entropy term p log(p + 1e-8) summed over the
// non-reserved tokens (block partials, then one fixed-order sum); in training y_soft = softmax(logits + g) with the
// Gumbel noise g given (noise_mode 1) or as -log of the exponential draws (noise_mode 2), the one-hot of its argmax (or
// the caller's y_hard) and the straight-through value (y_hard - y_soft) + y_soft; in evaluation the one-hot of argmax
// soft; reserved tokens' rows set to (0, 1); the pattern index sum_i hard[t][i][1] 2^(bs-1-i). Replaces ~25 ATen launches
// per routed layer.
namespace {
constexpr int RH_THREADS = 256;
constexpr int RH_BS_MAX = 8;

__device__ __forceinline__ void softmax2(float a, float b, float& p0, float& p1) {
  const float m = a >= b ? a : b;
  const float e0 = expf(a - m), e1 = expf(b - m);
  const float s = e0 + e1;
  p0 = e0 / s;
  p1 = e1 / s;
}

__global__ void __launch_bounds__(RH_THREADS) router_head_fwd_kernel(const float* __restrict__ logits,
                                                                     const float* __restrict__ noise, int noise_mode,
                                                                     const float* __restrict__ yhard_in, long T, int N,
                                                                     int bs, int reserve, int training,
                                                                     float* __restrict__ soft, float* __restrict__ ysoft,
                                                                     float* __restrict__ hard,
                                                                     float* __restrict__ indices,
                                                                     float* __restrict__ ent_part) {
  __shared__ float red[RH_THREADS];
  const long t = (long)blockIdx.x * RH_THREADS + threadIdx.x;
  float ent = 0.f;
  if (t < T) {
    const bool res = (int)(t % N) < reserve;
    float idx = 0.f;
    for (int i = 0; i < bs; ++i) {
      const long q = (t * bs + i) * 2;
      const float l0 = logits[q], l1 = logits[q + 1];
      float p0, p1;
      softmax2(l0, l1, p0, p1);
      soft[q] = p0;
      soft[q + 1] = p1;
      if (!res) ent += p0 * logf(p0 + 1e-8f) + p1 * logf(p1 + 1e-8f);
      float h0, h1;
      if (training) {
        float g0 = 0.f, g1 = 0.f;
        if (noise_mode == 1) {
          g0 = noise[q];
          g1 = noise[q + 1];
        } else if (noise_mode == 2) {
          g0 = -logf(noise[q]);
          g1 = -logf(noise[q + 1]);
        }
        float y0, y1;
        softmax2(l0 + g0, l1 + g1, y0, y1);
        ysoft[q] = y0;
        ysoft[q + 1] = y1;
        float yh0, yh1;
        if (yhard_in) {
          yh0 = yhard_in[q];
          yh1 = yhard_in[q + 1];
        } else {
          yh1 = y1 > y0 ? 1.f : 0.f;  // (the first index on a tie, as torch's max)
          yh0 = 1.f - yh1;
        }
        h0 = (yh0 - y0) + y0;
        h1 = (yh1 - y1) + y1;
      } else if (yhard_in) {
        h0 = yhard_in[q];
        h1 = yhard_in[q + 1];
      } else {
        h1 = p1 > p0 ? 1.f : 0.f;
        h0 = 1.f - h1;
      }
      if (res) {
        h0 = 0.f;
        h1 = 1.f;
      }
      hard[q] = h0;
      hard[q + 1] = h1;
      idx = fmaf(h1, (float)(1 << (bs - 1 - i)), idx);
    }
    indices[t] = idx;
  }
  red[threadIdx.x] = ent;
  __syncthreads();
  for (int s = RH_THREADS / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) ent_part[blockIdx.x] = red[0];
}

// entropy[0] = -(sum of the block partials, fixed order) / norm
__global__ void __launch_bounds__(RH_THREADS) router_head_ent_kernel(const float* __restrict__ part, int n, float norm,
                                                                     float* __restrict__ entropy) {
  __shared__ float red[RH_THREADS];
  float s = 0.f;
  for (int k = threadIdx.x; k < n; k += RH_THREADS) s += part[k];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = RH_THREADS / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) entropy[0] = -red[0] / norm;
}

// dlogits: the softmax backward of (dsoft + the entropy term's gradient) and, in training, of the straight-through
// path (dhard, and dindices through the pattern index) on y_soft; reserved tokens' hard rows take no gradient
__global__ void __launch_bounds__(RH_THREADS) router_head_bwd_kernel(const float* __restrict__ soft,
                                                                     const float* __restrict__ ysoft,
                                                                     const float* __restrict__ dsoft,
                                                                     const float* __restrict__ dhard,
                                                                     const float* __restrict__ dind,
                                                                     const float* __restrict__ dent, float norm, long T,
                                                                     int N, int bs, int reserve, int training,
                                                                     float* __restrict__ dlogits) {
  const long t = (long)blockIdx.x * RH_THREADS + threadIdx.x;
  if (t >= T) return;
  const bool res = (int)(t % N) < reserve;
  const float ge = dent && !res ? -dent[0] / norm : 0.f;  // d entropy / d (sum of p log(p + 1e-8))
  for (int i = 0; i < bs; ++i) {
    const long q = (t * bs + i) * 2;
    const float p0 = soft[q], p1 = soft[q + 1];
    float d0 = dsoft ? dsoft[q] : 0.f, d1 = dsoft ? dsoft[q + 1] : 0.f;
    if (ge != 0.f) {
      d0 += ge * (logf(p0 + 1e-8f) + p0 / (p0 + 1e-8f));
      d1 += ge * (logf(p1 + 1e-8f) + p1 / (p1 + 1e-8f));
    }
    const float sd = d0 * p0 + d1 * p1;
    float o0 = p0 * (d0 - sd), o1 = p1 * (d1 - sd);
    if (training && ysoft && !res && (dhard || dind)) {
      float h0 = dhard ? dhard[q] : 0.f, h1 = dhard ? dhard[q + 1] : 0.f;
      if (dind) h1 += dind[t] * (float)(1 << (bs - 1 - i));
      const float y0 = ysoft[q], y1 = ysoft[q + 1];
      const float sy = h0 * y0 + h1 * y1;
      o0 += y0 * (h0 - sy);
      o1 += y1 * (h1 - sy);
    }
    dlogits[q] = o0;
    dlogits[q + 1] = o1;
  }
}
}  // namespace

extern "C" int64_t vit_router_head_partials(int64_t T) { return (T + RH_THREADS - 1) / RH_THREADS; }

extern "C" int vit_router_head_fwd(const float* logits, const float* noise, int32_t noise_mode, const float* yhard_in,
                                   int64_t T, int64_t N, int32_t bs, int64_t reserve, int32_t training, float norm,
                                   float* soft, float* ysoft, float* hard, float* indices, float* ent_part,
                                   float* entropy, vit_stream_t stream) {
  VIT_CHECK_ARG(logits && soft && hard && indices && ent_part && entropy && T >= 0 && N > 0 && reserve >= 0 &&
                    bs >= 1 && bs <= RH_BS_MAX && noise_mode >= 0 && noise_mode <= 2 && (noise_mode == 0 || noise) &&
                    (!training || ysoft) && norm > 0.f && T < (1L << 40),
                "vit_router_head_fwd: bad args (bs 1..%d, noise_mode 0..2 with noise, ysoft in training, norm > 0)",
                RH_BS_MAX);
  const long nb = (long)vit_router_head_partials(T);
  if (nb > 0)
    hipLaunchKernelGGL(router_head_fwd_kernel, dim3((unsigned)nb), dim3(RH_THREADS), 0, (hipStream_t)stream, logits,
                       noise, (int)noise_mode, yhard_in, (long)T, (int)N, (int)bs, (int)reserve, (int)training, soft,
                       ysoft, hard, indices, ent_part);
  hipLaunchKernelGGL(router_head_ent_kernel, dim3(1), dim3(RH_THREADS), 0, (hipStream_t)stream, ent_part, (int)nb, norm,
                     entropy);
  VIT_LAUNCH_CHECK("vit_router_head_fwd");
}

extern "C" int vit_router_head_bwd(const float* soft, const float* ysoft, const float* dsoft, const float* dhard,
                                   const float* dind, const float* dent, float norm, int64_t T, int64_t N, int32_t bs,
                                   int64_t reserve, int32_t training, float* dlogits, vit_stream_t stream) {
  VIT_CHECK_ARG(soft && dlogits && T >= 0 && N > 0 && reserve >= 0 && bs >= 1 && bs <= RH_BS_MAX && norm > 0.f &&
                    (!training || ysoft),
                "vit_router_head_bwd: bad args");
  if (T == 0) return VIT_OK;
  hipLaunchKernelGGL(router_head_bwd_kernel, dim3((unsigned)vit_router_head_partials(T)), dim3(RH_THREADS), 0,
                     (hipStream_t)stream, soft, ysoft, dsoft, dhard, dind, dent, norm, (long)T, (int)N, (int)bs,
                     (int)reserve, (int)training, dlogits);
  VIT_LAUNCH_CHECK("vit_router_head_bwd");
}

// ---- Res-ViT distillation loss on the cls rows (res-vit/model.py:40-59, DistillLoss = mse_loss(student[:, 0],
// teacher[:, 0].detach()), applied after every routed layer) ------------------------------------------------------------
// forward: e[b][d] = x[b*ldx + d] - t[b*ldt + d] (kept for the backward), per-row sums of e*e, then loss = sum / (B D)
// in a fixed order; backward: dx[b*lddx + d] += ((2 / (B D)) e) g, torch's mse_loss_backward arithmetic, added in place
// into the student's incoming gradient (no zero-filled slice gradient, no separate add)
namespace {
__global__ void __launch_bounds__(256) cls_mse_rows_kernel(const float* __restrict__ x, long ldx,
                                                           const float* __restrict__ t, long ldt, int D,
                                                           float* __restrict__ e, float* __restrict__ part) {
  __shared__ float red[256];
  const int b = blockIdx.x;
  float s = 0.f;
  for (int d = threadIdx.x; d < D; d += 256) {
    const float v = x[b * ldx + d] - t[b * ldt + d];
    e[(long)b * D + d] = v;
    s += v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[b] = red[0];
}

__global__ void __launch_bounds__(256) cls_mse_final_kernel(const float* __restrict__ part, int B, float n,
                                                            float* __restrict__ loss) {
  __shared__ float red[256];
  float s = 0.f;
  for (int k = threadIdx.x; k < B; k += 256) s += part[k];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] / n;
}

__global__ void __launch_bounds__(256) cls_mse_bwd_kernel(float* __restrict__ dx, long lddx,
                                                          const float* __restrict__ e, int D,
                                                          const float* __restrict__ g, float norm) {
  const int b = blockIdx.x;
  const float gv = g[0];
  for (int d = threadIdx.x; d < D; d += 256) dx[b * lddx + d] += (norm * e[(long)b * D + d]) * gv;
}
}  // namespace

extern "C" int vit_cls_mse(const float* x, int64_t ldx, const float* t, int64_t ldt, int64_t B, int64_t D, float* e,
                           float* part, float* loss, vit_stream_t stream) {
  VIT_CHECK_ARG(x && t && e && part && loss && B > 0 && D > 0 && ldx >= D && ldt >= D && B < (1L << 31) &&
                    D < (1L << 30),
                "vit_cls_mse: bad args");
  hipLaunchKernelGGL(cls_mse_rows_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, x, (long)ldx, t,
                     (long)ldt, (int)D, e, part);
  hipLaunchKernelGGL(cls_mse_final_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, part, (int)B,
                     (float)((double)B * (double)D), loss);
  VIT_LAUNCH_CHECK("vit_cls_mse");
}

extern "C" int vit_cls_mse_bwd(float* dx, int64_t lddx, const float* e, int64_t B, int64_t D, const float* g,
                               vit_stream_t stream) {
  VIT_CHECK_ARG(dx && e && g && B > 0 && D > 0 && lddx >= D && B < (1L << 31) && D < (1L << 30),
                "vit_cls_mse_bwd: bad args");
  hipLaunchKernelGGL(cls_mse_bwd_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, dx, (long)lddx, e,
                     (int)D, g, (float)(2.0 / ((double)B * (double)D)));
  VIT_LAUNCH_CHECK("vit_cls_mse_bwd");
}

// ---- Res-ViT routing masks (res-vit/model.py:486-512, 336-368): from the pattern index of every token, which tokens run
// each block position's full layer (isin(index.long(), that position's transformer set)) and which tokens each
// approximator takes (index == key, exact float compare as the reference's), plus whether any token took it. One
// workgroup (T is one batch of tokens); replaces the cast / compare / reduce launches per routed layer and per
// approximator --------------------------------------------------------------------------------------------------------
namespace {
constexpr int RS_POS_MAX = 8, RS_KEYS_MAX = 32;
struct RouterSelectArgs {
  unsigned mask[RS_POS_MAX];
};
__global__ void __launch_bounds__(1024) router_select_kernel(const float* __restrict__ idx, long T, int npos,
                                                             const RouterSelectArgs a, int nkeys,
                                                             unsigned char* __restrict__ active,
                                                             unsigned char* __restrict__ sel,
                                                             unsigned char* __restrict__ any) {
  __shared__ int anyf[RS_KEYS_MAX];
  if ((int)threadIdx.x < RS_KEYS_MAX) anyf[threadIdx.x] = 0;
  __syncthreads();
  // four tokens per thread and step (one 16-B load, one 4-B store per output row; T % 4 == 0 and 16-B aligned
  // indices, else one token at a time): the loop is latency-bound in a single workgroup
  const bool vec = T % 4 == 0 && ((uintptr_t)idx % 16) == 0 && ((uintptr_t)active % 4) == 0 &&
                   ((uintptr_t)sel % 4) == 0;
  const long step = vec ? 4 : 1;
  for (long t = (long)threadIdx.x * step; t < T; t += 1024 * step) {
    float v[4];
    int n = 1;
    if (vec) {
      const float4 q = *reinterpret_cast<const float4*>(idx + t);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
      n = 4;
    } else {
      v[0] = idx[t];
    }
    for (int j = 0; j < npos; ++j) {
      unsigned w = 0;
      for (int e = 0; e < n; ++e) {
        // torch's .long(): truncation toward zero (so (-1, 0) -> 0); values whose truncation is outside [0, 32) (and
        // NaN) are in no set, and are not converted (an out-of-range float -> integer conversion is undefined)
        const bool in_range = v[e] > -1.f && v[e] < 32.f;
        const int lv = in_range ? (int)v[e] : 0;
        if (in_range && ((a.mask[j] >> lv) & 1u)) w |= 1u << (8 * e);
      }
      if (vec) *reinterpret_cast<unsigned*>(active + j * T + t) = w;
      else active[j * T + t] = (unsigned char)w;
    }
    for (int k = 0; k < nkeys; ++k) {
      unsigned w = 0;
      for (int e = 0; e < n; ++e)
        if (v[e] == (float)k) w |= 1u << (8 * e);
      if (vec) *reinterpret_cast<unsigned*>(sel + k * T + t) = w;
      else sel[k * T + t] = (unsigned char)w;
      if (w) anyf[k] = 1;  // (every writer stores the same 1)
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < nkeys) any[threadIdx.x] = anyf[threadIdx.x] ? 1 : 0;
}
}  // namespace

extern "C" int vit_router_select(const float* indices, int64_t T, int32_t npos, const uint32_t* active_masks,
                                 int32_t nkeys, void* active, void* sel, void* any, vit_stream_t stream) {
  VIT_CHECK_ARG(indices && T >= 0 && T < (1L << 40) && npos >= 0 && npos <= RS_POS_MAX && nkeys >= 0 &&
                    nkeys <= RS_KEYS_MAX && (npos == 0 || (active && active_masks)) && (nkeys == 0 || (sel && any)),
                "vit_router_select: bad args (npos <= %d, nkeys <= %d)", RS_POS_MAX, RS_KEYS_MAX);
  RouterSelectArgs a{};
  for (int j = 0; j < npos; ++j) a.mask[j] = active_masks[j];
  hipLaunchKernelGGL(router_select_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, indices, (long)T, (int)npos, a,
                     (int)nkeys, (unsigned char*)active, (unsigned char*)sel, (unsigned char*)any);
  VIT_LAUNCH_CHECK("vit_router_select");
}

// ---- f32 rows -> bf16 rows, rows whose mask byte is 0 written as zeros without reading them (Res-ViT's routed layer:
// its output gradient enters the layer's backward as the bf16 operand of the fc2 data gradient on the active rows
// only, res-vit/model.py:507-512) --------------------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(256) cast_rows_masked_kernel(const float* __restrict__ in, long ldi, long rows,
                                                               int cols, const unsigned char* __restrict__ mask,
                                                               bf16_t* __restrict__ out, long ldo) {
  const int cq = cols >> 2;
  const long total = rows * cq;
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < total; q += (long)gridDim.x * 256) {
    const long r = q / cq;
    const int c = (int)(q - r * cq) << 2;
    uint2 o = {0u, 0u};
    if (!mask || mask[r]) {
      const float4 v = *reinterpret_cast<const float4*>(in + r * ldi + c);
      o.x = pack2bf(v.x, v.y);
      o.y = pack2bf(v.z, v.w);
    }
    *reinterpret_cast<uint2*>(out + r * ldo + c) = o;
  }
}
}  // namespace

extern "C" int vit_cast_rows_masked(const float* in, int64_t ldi, int64_t rows, int64_t cols, const void* mask,
                                    void* out, int64_t ldo, vit_stream_t stream) {
  VIT_CHECK_ARG(in && out && rows >= 0 && cols > 0 && cols % 4 == 0 && ldi % 4 == 0 && ldo % 4 == 0 && ldi >= cols &&
                    ldo >= cols && (uintptr_t)in % 16 == 0 && (uintptr_t)out % 8 == 0 && cols < (1L << 30),
                "vit_cast_rows_masked: bad args (cols, ldi, ldo multiples of 4; 16-B aligned in, 8-B aligned out)");
  if (rows == 0) return VIT_OK;
  hipLaunchKernelGGL(cast_rows_masked_kernel, dim3(grid_for(rows * (cols / 4), 4)), dim3(256), 0,
                     (hipStream_t)stream, in, (long)ldi, (long)rows, (int)cols, (const unsigned char*)mask,
                     (bf16_t*)out, (long)ldo);
  VIT_LAUNCH_CHECK("vit_cast_rows_masked");
}
