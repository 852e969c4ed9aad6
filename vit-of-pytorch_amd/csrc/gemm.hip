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
#include "common.h"
#include <stdlib.h>

namespace {

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
};

// blockIdx (after the XCD remap) -> output tile. Grouping tile rows keeps the weight panels a
// group's concurrent workgroups share hot in the XCD's L2.
__device__ __forceinline__ void tile_coords(int wg, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  if (gm <= 1) {
    tm = wg / tiles_n;
    tn = wg % tiles_n;
    return;
  }
  const int per = gm * tiles_n;
  const int first = (wg / per) * gm;
  const int rows = tiles_m - first < gm ? tiles_m - first : gm;
  const int r = wg % per;
  tm = first + r % rows;
  tn = r / rows;
}

// K-contiguous image [rows][BK]: XOR of the 16-B chunk index, conflict-free for the 16x16x32
// fragment read (16 rows x 16 B per ds_read_b128 lane group).
template <int BK>
__device__ __forceinline__ int swz_k(int row) {
  if constexpr (BK == 64) return (row >> 1) & 7;
  return (-(row >> 2)) & 3;  // BK == 32: 64-B rows
}
// M/N-contiguous image [BK][rows]: XOR of the 32-B granule, conflict-free for ds_read_b64_tr_b16.
__device__ __forceinline__ int swz_mn(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }

// Issue the LDS-DMA of one operand k-tile (ROWS rows of the M/N dim x BK k) to byte offset lds_off.
// Instruction i of a wave covers image rows advanced by a multiple of the swizzle period (16) from
// instruction 0, so its per-lane source offset is instruction 0's plus a wave-uniform step: one
// lane-offset VGPR per call instead of one per instruction (the per-instruction offsets of the four
// half-image loads of gemm_pp2_kernel spilled to scratch, and hipcc waited vmcnt(0) on every reload).
template <int ROWS, int BK, bool KC, int NWAVE>
__device__ __forceinline__ void stage_tile(char* smem, int lds_off, __amdgpu_buffer_rsrc_t rs, long ld, int kt,
                                           int wave, int lane, int vbase = 0) {
  constexpr int BYTES = ROWS * BK * 2;
  constexpr int INSTR = BYTES / 1024 / NWAVE;
  static_assert(INSTR * 1024 * NWAVE == BYTES, "tile must split evenly over waves");
  constexpr int CPR = KC ? BK / 8 : ROWS * 2 / 16;  // 16-B chunks per image row
  constexpr int RSTEP = NWAVE * 64 / CPR;             // image rows between a wave's instructions
  static_assert(RSTEP % 16 == 0, "swizzle must repeat between a wave's instructions");
  const int c = wave * 64 + lane;  // chunk of instruction 0
  const int r = c / CPR, pc = c % CPR;
  int lane_off, step, base;
  if constexpr (KC) {
    const int lc = pc ^ swz_k<BK>(r);
    lane_off = (int)(r * ld * 2) + lc * 16;
    step = (int)(RSTEP * ld * 2);
    base = kt * BK * 2 + vbase;
  } else {
    lane_off = (int)(r * ld * 2) + ((pc * 16) ^ (swz_mn(r) << 5));
    step = (int)(RSTEP * ld * 2);
    base = (int)((long)kt * BK * ld * 2) + vbase;
  }
  base = __builtin_amdgcn_readfirstlane(base);
  step = __builtin_amdgcn_readfirstlane(step);
#pragma unroll
  for (int i = 0; i < INSTR; ++i) {
    const int piece = i * NWAVE + wave;  // 1 KiB piece of the LDS image
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, smem + lds_off + piece * 1024), 16,
                                             lane_off + (base + i * step), 0, 0, 0);
  }
}

// 16 rows (r0..r0+15) x 32 k (kk*32..) MFMA fragment of this lane.
template <int ROWS, int BK, bool KC>
__device__ __forceinline__ v8s read_frag(const char* smem, int lds_off, int r0, int kk, int lane) {
  if constexpr (KC) {
    const int row = r0 + (lane & 15);
    const int lc = kk * 4 + (lane >> 4);
    const int pc = lc ^ swz_k<BK>(row);
    return *reinterpret_cast<const v8s*>(smem + lds_off + row * BK * 2 + pc * 16);
  } else {
    constexpr int RB = ROWS * 2;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int col_b = (r0 + 4 * p) * 2;
    const int ra = kk * 32 + 8 * g + q;
    const int rb = ra + 4;
    v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        LDS_PTR(v4s, smem + lds_off + ra * RB + (col_b ^ (swz_mn(ra) << 5))));
    v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        LDS_PTR(v4s, smem + lds_off + rb * RB + (col_b ^ (swz_mn(rb) << 5))));
    v8s r;
    r.lo = lo;
    r.hi = hi;
    return r;
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Internal epilogue flag: the dropout variant of PATCH / BIAS_RESID_F32 / BIAS_GELU_DGELU (its own
// instantiation, so the dropout-free kernels carry none of the Philox code)
constexpr int EPI_DROP = 16;

template <int EPI>
__device__ __forceinline__ void epi_store(const GemmDev& p, int z, int split_idx, int m, int n, float v) {
  constexpr int E = EPI & 15;                  // base epilogue
  constexpr bool DROP = (EPI & EPI_DROP) != 0;  // dropout variant
  if (m >= p.M || n >= p.N) return;
  if constexpr (E == VIT_EPI_F32) {
    float* C = (float*)p.C + z * p.c_bs;
    C[(long)m * p.ldc + n] = v;
  } else if constexpr (E == VIT_EPI_BF16) {
    bf16_t* C = (bf16_t*)p.C + z * p.c_bs;
    C[(long)m * p.ldc + n] = f2bf(v);
  } else if constexpr (E == VIT_EPI_BIAS_BF16) {
    bf16_t* C = (bf16_t*)p.C + z * p.c_bs;
    const float b = p.bias ? p.bias[z * p.bias_bs + n] : 0.f;
    C[(long)m * p.ldc + n] = f2bf(v + b);
  } else if constexpr (E == VIT_EPI_BIAS_GELU) {
    bf16_t* C = (bf16_t*)p.C + z * p.c_bs;
    bf16_t* C2 = (bf16_t*)p.C2 + z * p.c_bs;
    const float u = v + (p.bias ? p.bias[z * p.bias_bs + n] : 0.f);
    C[(long)m * p.ldc + n] = f2bf(u);
    C2[(long)m * p.ldc2 + n] = f2bf(gelu_f(u));
  } else if constexpr (E == VIT_EPI_BIAS_RESID_F32) {
    float* C = (float*)p.C + z * p.c_bs;
    const float* R = (const float*)p.aux;
    const float b = p.bias ? p.bias[z * p.bias_bs + n] : 0.f;
    const float dm = DROP ? drop_mult1(p.drop, m, n) : 1.0f;
    C[(long)m * p.ldc + n] = (v + b) * dm + R[(long)m * p.ldaux + n];
  } else if constexpr (E == VIT_EPI_GELU_BWD) {
    bf16_t* C = (bf16_t*)p.C + z * p.c_bs;
    const bf16_t* U = (const bf16_t*)p.aux;
    C[(long)m * p.ldc + n] = f2bf(v * gelu_grad_f(bf2f(U[(long)m * p.ldaux + n])));
  } else if constexpr (E == VIT_EPI_BIAS_GELU_DGELU) {
    bf16_t* C = (bf16_t*)p.C + z * p.c_bs;
    bf16_t* C2 = (bf16_t*)p.C2 + z * p.c_bs;
    const float u = v + (p.bias ? p.bias[z * p.bias_bs + n] : 0.f);
    float pdf;
    const float cdf = phi_and_pdf(u, &pdf);
    const float dm = DROP ? drop_mult1(p.drop, m, n) : 1.0f;
    C[(long)m * p.ldc + n] = f2bf((cdf + u * pdf) * dm);
    C2[(long)m * p.ldc2 + n] = f2bf(u * cdf * dm);
  } else if constexpr (E == VIT_EPI_MUL_BF16) {
    bf16_t* C = (bf16_t*)p.C + z * p.c_bs;
    const bf16_t* U = (const bf16_t*)p.aux;
    C[(long)m * p.ldc + n] = f2bf(v * bf2f(U[(long)m * p.ldaux + n]));
  } else if constexpr (E == VIT_EPI_PATCH) {
    float* C = (float*)p.C;
    const float* pos = (const float*)p.aux;
    const int t = m % p.tokens;
    float o;
    if (t == 0)
      o = p.aux2[n] + pos[n];
    else
      o = v + p.bias[n] + pos[(long)t * p.ldaux + n];
    if constexpr (DROP) o *= drop_mult1(p.drop, m, n);
    C[(long)m * p.ldc + n] = o;
  } else if constexpr (E == VIT_EPI_SPLITK) {
    float* C = (float*)p.C + ((long)z * p.split_k + split_idx) * (long)p.M * p.N;
    C[(long)m * p.N + n] = v;
  }
}

__device__ __forceinline__ void ld8f(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
typedef float v4f_t __attribute__((ext_vector_type(4)));
typedef unsigned v4u_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st8f(float* p, const float* v, bool nt = false) {
  const v4f_t a = {v[0], v[1], v[2], v[3]}, b = {v[4], v[5], v[6], v[7]};
  if (nt) {
    __builtin_nontemporal_store(a, reinterpret_cast<v4f_t*>(p));
    __builtin_nontemporal_store(b, reinterpret_cast<v4f_t*>(p + 4));
  } else {
    *reinterpret_cast<v4f_t*>(p) = a;
    *reinterpret_cast<v4f_t*>(p + 4) = b;
  }
}
__device__ __forceinline__ void st8bf(bf16_t* p, const float* v, bool nt = false) {
  const v4u_t u = {pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
  if (nt)
    __builtin_nontemporal_store(u, reinterpret_cast<v4u_t*>(p));
  else
    *reinterpret_cast<v4u_t*>(p) = u;
}
__device__ __forceinline__ void ld8bf(const bf16_t* p, float* v) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  v[0] = bf2f(u.x & 0xffff); v[1] = bf2f(u.x >> 16); v[2] = bf2f(u.y & 0xffff); v[3] = bf2f(u.y >> 16);
  v[4] = bf2f(u.z & 0xffff); v[5] = bf2f(u.z >> 16); v[6] = bf2f(u.w & 0xffff); v[7] = bf2f(u.w >> 16);
}

// 8 consecutive columns n..n+7 of row m (all in range, aligned: p.vec).
// GELU(u) and GELU'(u) of two values on packed f32 math (v_pk_fma/mul/add_f32: two lanes' worth per
// instruction; the two transcendentals per value stay scalar). erf from Abramowitz & Stegun 7.1.25,
// |error| <= 2.5e-5 — two orders below the bf16 rounding of both outputs. This is the fc1 forward
// epilogue, whose VALU (not its stores) was the largest cost of that GEMM after its main loop.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gelu_dgelu2(f2v u, f2v& gelu, f2v& dgelu) {
  const f2v one = {1.f, 1.f}, half = {0.5f, 0.5f};
  const f2v x2 = u * u;
  const f2v e = {__builtin_amdgcn_exp2f(x2.x * -0.72134752044448170f),  // exp(-u^2/2) = 2^(-u^2 log2(e)/2)
                 __builtin_amdgcn_exp2f(x2.y * -0.72134752044448170f)};
  const f2v au = __builtin_elementwise_abs(u);
  const f2v a = __builtin_elementwise_fma(au, f2v{0.47047f * 0.70710678118654752f, 0.47047f * 0.70710678118654752f}, one);
  const f2v t = {__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)};
  f2v q = __builtin_elementwise_fma(t, f2v{0.7478556f, 0.7478556f}, f2v{-0.0958798f, -0.0958798f});
  q = __builtin_elementwise_fma(q, t, f2v{0.3480242f, 0.3480242f});
  q = q * t;
  const f2v erfa = __builtin_elementwise_fma(-q, e, one);  // erf(|u| / sqrt 2)
  const f2v sg = {__builtin_copysignf(erfa.x, u.x), __builtin_copysignf(erfa.y, u.y)};
  const f2v cdf = __builtin_elementwise_fma(sg, half, half);
  const f2v pdf = e * f2v{0.39894228040143268f, 0.39894228040143268f};
  gelu = u * cdf;
  dgelu = __builtin_elementwise_fma(u, pdf, cdf);
}

// pre: the 8 aux values of (m, n..n+7) already loaded by the caller (GELU_BWD / MUL / RESID), or null.
template <int EPI>
__device__ __forceinline__ void epi_store8(const GemmDev& p, int z, int split_idx, int m, int n, float* v,
                                           const float* pre = nullptr) {
  constexpr int E = EPI & 15;
  constexpr bool DROP = (EPI & EPI_DROP) != 0;
  float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (E == VIT_EPI_BIAS_BF16 || E == VIT_EPI_BIAS_GELU || E == VIT_EPI_BIAS_RESID_F32 ||
                E == VIT_EPI_BIAS_GELU_DGELU) {
    if (p.bias) ld8f(p.bias + z * p.bias_bs + n, b);
  }
  if constexpr (E == VIT_EPI_F32) {
    st8f((float*)p.C + z * p.c_bs + (long)m * p.ldc + n, v, p.nt);
  } else if constexpr (E == VIT_EPI_BF16) {
    st8bf((bf16_t*)p.C + z * p.c_bs + (long)m * p.ldc + n, v, p.nt);
  } else if constexpr (E == VIT_EPI_BIAS_BF16) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += b[k];
    st8bf((bf16_t*)p.C + z * p.c_bs + (long)m * p.ldc + n, v, p.nt);
  } else if constexpr (E == VIT_EPI_BIAS_GELU) {
    float gl[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] += b[k];
      gl[k] = gelu_f(v[k]);
    }
    st8bf((bf16_t*)p.C + z * p.c_bs + (long)m * p.ldc + n, v, p.nt);
    st8bf((bf16_t*)p.C2 + z * p.c_bs + (long)m * p.ldc2 + n, gl, p.nt);
  } else if constexpr (E == VIT_EPI_BIAS_RESID_F32) {
    float r[8];
    if (pre) {
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = pre[k];
    } else {
      ld8f((const float*)p.aux + (long)m * p.ldaux + n, r);
    }
    if constexpr (DROP) {
      float dm[8];
      drop_mult8(p.drop, m, n >> 3, dm);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (v[k] + b[k]) * dm[k] + r[k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += b[k] + r[k];
    }
    st8f((float*)p.C + z * p.c_bs + (long)m * p.ldc + n, v, p.nt);
  } else if constexpr (E == VIT_EPI_GELU_BWD) {
    float u[8];
    if (pre) {
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = pre[k];
    } else {
      ld8bf((const bf16_t*)p.aux + (long)m * p.ldaux + n, u);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= gelu_grad_f(u[k]);
    st8bf((bf16_t*)p.C + z * p.c_bs + (long)m * p.ldc + n, v, p.nt);
  } else if constexpr (E == VIT_EPI_BIAS_GELU_DGELU) {
    float gl[8];
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
      f2v g2, d2;
      gelu_dgelu2(f2v{v[k] + b[k], v[k + 1] + b[k + 1]}, g2, d2);
      gl[k] = g2.x;
      gl[k + 1] = g2.y;
      v[k] = d2.x;
      v[k + 1] = d2.y;
    }
    if constexpr (DROP) {
      float dm[8];
      drop_mult8(p.drop, m, n >> 3, dm);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        gl[k] *= dm[k];
        v[k] *= dm[k];
      }
    }
    st8bf((bf16_t*)p.C + z * p.c_bs + (long)m * p.ldc + n, v, p.nt);
    st8bf((bf16_t*)p.C2 + z * p.c_bs + (long)m * p.ldc2 + n, gl, p.nt);
  } else if constexpr (E == VIT_EPI_MUL_BF16) {
    float u[8];
    if (pre) {
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = pre[k];
    } else {
      ld8bf((const bf16_t*)p.aux + (long)m * p.ldaux + n, u);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= u[k];
    st8bf((bf16_t*)p.C + z * p.c_bs + (long)m * p.ldc + n, v, p.nt);
  } else if constexpr (E == VIT_EPI_PATCH) {
    const int t = m % p.tokens;
    float ps[8];
    ld8f((const float*)p.aux + (long)t * p.ldaux + n, ps);
    if (t == 0) {
      ld8f(p.aux2 + n, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = b[k] + ps[k];
    } else {
      ld8f(p.bias + n, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += b[k] + ps[k];
    }
    if constexpr (DROP) {
      float dm[8];
      drop_mult8(p.drop, m, n >> 3, dm);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= dm[k];
    }
    st8f((float*)p.C + (long)m * p.ldc + n, v, p.nt);
  } else if constexpr (E == VIT_EPI_SPLITK) {
    st8f((float*)p.C + ((long)z * p.split_k + split_idx) * (long)p.M * p.N + (long)m * p.N + n, v, p.nt);
  }
}

// Epilogue operand prefetch: the aux values (bf16 GELU input / multiplier, f32 residual) of 8-column
// chunks are requested a whole staging pass ahead, so the HBM latency of the lock-step epilogue is
// paid once per tile instead of once per chunk. AuxPre<EPI>::W uint4 per chunk (0: no aux).
template <int EPI>
struct AuxPre {
  static constexpr int E = EPI & 15;
  static constexpr int W = (E == VIT_EPI_GELU_BWD || E == VIT_EPI_MUL_BF16) ? 1
                           : E == VIT_EPI_BIAS_RESID_F32                      ? 2
                                                                                : 0;
  __device__ __forceinline__ static void fetch(const GemmDev& p, int m, int n, uint4* d) {
    if constexpr (W == 1) {
      d[0] = *reinterpret_cast<const uint4*>((const bf16_t*)p.aux + (long)m * p.ldaux + n);
    } else if constexpr (W == 2) {
      const float* a = (const float*)p.aux + (long)m * p.ldaux + n;
      d[0] = *reinterpret_cast<const uint4*>(a);
      d[1] = *reinterpret_cast<const uint4*>(a + 4);
    }
  }
  __device__ __forceinline__ static void unpack(const uint4* d, float* u) {
    if constexpr (W == 1) {
      const uint4 x = d[0];
      u[0] = bf2f(x.x & 0xffff); u[1] = bf2f(x.x >> 16); u[2] = bf2f(x.y & 0xffff); u[3] = bf2f(x.y >> 16);
      u[4] = bf2f(x.z & 0xffff); u[5] = bf2f(x.z >> 16); u[6] = bf2f(x.w & 0xffff); u[7] = bf2f(x.w >> 16);
    } else if constexpr (W == 2) {
      u[0] = __uint_as_float(d[0].x); u[1] = __uint_as_float(d[0].y); u[2] = __uint_as_float(d[0].z);
      u[3] = __uint_as_float(d[0].w); u[4] = __uint_as_float(d[1].x); u[5] = __uint_as_float(d[1].y);
      u[6] = __uint_as_float(d[1].z); u[7] = __uint_as_float(d[1].w);
    }
  }
};

// Multi-stage LDS-DMA pipeline: STAGES k-tile buffers; at step t the DMA of step t+STAGES-1 is
// issued into the buffer read at step t-1, so STAGES-2 k-tiles stay in flight across every
// barrier (counted vmcnt, raw s_barrier: no vmcnt(0) drain inside the loop).
// waves per SIMD the register allocation must allow: 2 resident workgroups when the LDS fits twice
template <int BM, int BN, int BK, int STAGES, int WM, int WN>
constexpr int gemm_min_waves() {
  return (STAGES * (BM + BN) * BK * 2 <= 80 * 1024) ? (2 * WM * WN) / 4 : (WM * WN) / 4;
}

template <int BM, int BN, int BK, int STAGES, int WM, int WN, bool AK, bool BKC, int EPI>
__global__ void __launch_bounds__(WM* WN * 64, (gemm_min_waves<BM, BN, BK, STAGES, WM, WN>()))
    gemm_bf16_kernel(const GemmDev p) {
  constexpr int NWAVE = WM * WN;
  constexpr int NT = NWAVE * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int KK = BK / 32;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int PIPE = STAGES * STAGE;
  constexpr int LPS = (A_BYTES + B_BYTES) / 1024 / NWAVE;  // DMA instructions per wave per k-step
  constexpr int LDC = BN + 4;                               // fp32 staging row stride (floats)
  // stage the epilogue in 2 passes when one pass would not fit, or would cost the 2nd resident WG
  constexpr int NPASS = (BM * LDC * 4 > 160 * 1024 || (PIPE <= 80 * 1024 && BM * LDC * 4 > 80 * 1024)) ? 2 : 1;
  constexpr int PASS_ROWS = BM / NPASS;
  constexpr int STG = PASS_ROWS * LDC * 4;
  constexpr int SMEM = PIPE > STG ? PIPE : STG;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(NPASS == 1 || WM % 2 == 0, "two-pass epilogue splits the wave rows");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // ---- tile scheduling: XCD-aware bijective remap of blockIdx.x ----
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn, z, split_idx;
  if (p.split_k > 1 && p.split_xcd) {
    // split-K weight gradients: the dispatcher deals the linear workgroup id (x fastest, then the
    // split, then the batch) round-robin over the 8 XCDs. Remap the whole (tile, split, batch) space
    // XCD-major so an XCD's ~32 concurrent workgroups cover one or two K-chunks: they walk the same
    // token rows in step and read each row panel from HBM once per XCD instead of once per XCD
    // per chunk (fc1 wgrad fetch 2.3x -> ~1.2x the operand bytes).
    const int total = nwg * p.split_k * (int)gridDim.z;
    const int lin = blockIdx.x + nwg * (blockIdx.y + p.split_k * blockIdx.z);
    const int xcd = lin & 7, q8 = total >> 3, r8 = total & 7;
    const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (lin >> 3);
    const int zs = w / nwg;
    z = zs / p.split_k;
    split_idx = zs % p.split_k;
    tile_coords(w % nwg, tiles_m, tiles_n, p.group_m, tm, tn);
  } else {
    const int orig = blockIdx.x;
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    tile_coords(wg, tiles_m, tiles_n, p.group_m, tm, tn);
    z = blockIdx.z;
    split_idx = blockIdx.y;
  }
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- operand descriptors (base moved to the block's first row/col) ----
  const char* Ab = p.A + (long)z * p.a_bs * 2;
  const char* Bb = p.B + (long)z * p.b_bs * 2;
  const long a_shift = AK ? (long)m0 * p.lda * 2 : (long)m0 * 2;
  const long b_shift = BKC ? (long)n0 * p.ldb * 2 : (long)n0 * 2;
  const uint32_t a_rec = (long)p.a_bytes > a_shift ? (uint32_t)(p.a_bytes - a_shift) : 0u;
  const uint32_t b_rec = (long)p.b_bytes > b_shift ? (uint32_t)(p.b_bytes - b_shift) : 0u;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(Ab + a_shift, a_rec);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(Bb + b_shift, b_rec);

  // ---- k range of this split ----
  const int nkt = p.K / BK;
  const int kt0 = (int)((long)nkt * split_idx / p.split_k);
  const int kt1 = (int)((long)nkt * (split_idx + 1) / p.split_k);
  const int nk = kt1 - kt0;

  v4f acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const int wm0 = wm * TM, wn0 = wn * TN;

  auto issue = [&](int step) {
    const int buf = (step % STAGES) * STAGE;
    stage_tile<BM, BK, AK, NWAVE>(smem, buf, rsA, p.lda, kt0 + step, wave, lane);
    stage_tile<BN, BK, BKC, NWAVE>(smem, buf + A_BYTES, rsB, p.ldb, kt0 + step, wave, lane);
  };
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);

  for (int t = 0; t < nk; ++t) {
    // step t's DMA must have landed (own wave), leaving the younger steps in flight
    const int younger = nk - 1 - t;
    if (younger >= STAGES - 2) {
      wait_vm<LPS * (STAGES - 2)>();
    } else if constexpr (STAGES > 3) {
      if (younger == 1) wait_vm<LPS>(); else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();  // every wave's share landed; every wave done reading step t-1
    asm volatile("" ::: "memory");
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
    const int cur = (t % STAGES) * STAGE;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      v8s bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = read_frag<BN, BK, BKC>(smem, cur + A_BYTES, wn0 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const v8s af = read_frag<BM, BK, AK>(smem, cur, wm0 + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, af),
                                                              __builtin_bit_cast(v8bf, bfr[j]), acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("" ::: "memory");
  }

  // ---- epilogue: stage the fp32 tile in LDS (1 or 2 passes of rows), then each thread finishes
  //      8-column row chunks (coalesced 16/32-B stores, vector loads of bias / residual / GELU input)
  const int g = lane >> 4, c = lane & 15;
  wait_vm<0>();
  __syncthreads();
  float* cs = reinterpret_cast<float*>(smem);
  constexpr int CPR = BN / 8;
  static_assert(NT % CPR == 0, "a thread keeps one 8-column chunk across the epilogue loop");
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    if (NPASS == 1 || wm / (WM / NPASS) == pass) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            cs[(wm0 - pass * PASS_ROWS + i * 16 + 4 * g + r) * LDC + wn0 + j * 16 + c] = acc[i][j][r];
    }
    __syncthreads();
#pragma unroll 2
    for (int e = threadIdx.x; e < PASS_ROWS * CPR; e += NT) {
      const int row = e / CPR, ch = e % CPR;
      const int m = m0 + pass * PASS_ROWS + row, n = n0 + ch * 8;
      if (m >= p.M || n >= p.N) continue;
      float v[8];
      ld8f(cs + row * LDC + ch * 8, v);
      if (p.vec && n + 8 <= p.N) {
        epi_store8<EPI>(p, z, split_idx, m, n, v);  // v becomes the stored values
        if (p.col_partial) {
#pragma unroll
          for (int k = 0; k < 8; ++k) csum[k] += v[k];
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) epi_store<EPI>(p, z, split_idx, m, n + k, v[k]);
      }
    }
    if (NPASS > 1) __syncthreads();
  }
  if (p.col_partial) {
    // per-tile column sums of the written values (e.g. the bias gradient of the next layer down)
    __syncthreads();
    float* red = cs;
    constexpr int RL = NT / CPR;  // threads sharing one 8-column chunk
    const int ch = threadIdx.x % CPR;
#pragma unroll
    for (int k = 0; k < 8; ++k) red[(threadIdx.x / CPR) * BN + ch * 8 + k] = csum[k];
    __syncthreads();
    for (int c = threadIdx.x; c < BN; c += NT) {
      float sum = 0.f;
#pragma unroll 8
      for (int r = 0; r < RL; ++r) sum += red[r * BN + c];
      if (n0 + c < p.N) p.col_partial[(long)tm * p.N + n0 + c] = sum;
    }
  }
}

// ---- ping-pong kernel ---------------------------------------------------------------------------
// 256 x BN x 64 workgroup tile, 8 waves in two groups of 4: group g owns output rows 128g..128g+127,
// wave w of a group owns columns w*BN/4 .. +BN/4 (8 x BN/64 accumulator fragments). Time is cut into
// slots separated by workgroup barriers. In every slot one group reads the fragments of a 64-deep
// k-tile from LDS while the other group multiplies the fragments it read in the previous slot, so on
// each SIMD (one wave of each group) LDS reads and MFMA chains of the two waves alternate instead of
// serialising. Two LDS k-tile buffers: the LDS-DMA of k-tile u+1 is issued at the start of the slot
// in which group 0 starts on k-tile u (both groups are done reading k-tile u-1 from that buffer) and
// is waited for at the end of the following slot, before group 0 first reads it: two slots of flight,
// raw s_barrier (no vmcnt(0) drain at the barriers in between).
// Epilogue: wave-private fp32 staging in the then idle LDS (32 rows per pass), 8-column chunks.
// Outstanding-DMA wait with a runtime count of younger k-tiles (0 .. L-1) and compile-time vmcnt.
template <int LPT, int L>
__device__ __forceinline__ void wait_tiles(int younger) {
  if constexpr (L >= 4) {
    if (younger >= 3) { wait_vm<3 * LPT>(); return; }
  }
  if constexpr (L >= 3) {
    if (younger == 2) { wait_vm<2 * LPT>(); return; }
  }
  if constexpr (L >= 2) {
    if (younger == 1) { wait_vm<LPT>(); return; }
  }
  wait_vm<0>();
}

#ifdef VIT_GEMM_STAMPS
// Diagnostic build only (tools/gemm_diag.hip): s_memtime stamps of waves 0 and 4 of one workgroup,
// kept in spare LDS (no vmcnt traffic inside the loop) and copied out at the end.
__device__ int g_stamp_wg = -1;
__device__ unsigned long long g_stamps[2][1024];
#define PP_STAMP()                                                                        \
  do {                                                                                    \
    if (stamp_on && si < 1024) st_lds[si] = __builtin_amdgcn_s_memtime();                 \
    ++si;                                                                                 \
  } while (0)
constexpr int PP_STAMP_LDS = 16 * 1024;  // dropped (no stamps) where the pipeline leaves no room
#else
#define PP_STAMP() \
  do {             \
  } while (0)
constexpr int PP_STAMP_LDS = 0;
#endif

template <int BN, int BK, int NBUF, bool AK, bool BKC, int EPI>
__global__ void __launch_bounds__(512) gemm_pp_kernel(const GemmDev p) {
  constexpr int BM = 256, NWAVE = 8, KK = BK / 32;
  constexpr int TN = BN / 4, FM = 8, FN = TN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int LPT = STAGE / 1024 / NWAVE;  // DMA instructions per wave per k-tile
  constexpr int LDW = TN + 4;                // staging row stride (floats): conflict-free ds_write_b32
  constexpr int PR = 32;                     // staged rows per pass (4 passes over the wave's 128 rows)
  constexpr int WST = PR * LDW * 4;          // staging bytes per wave
  static_assert(NWAVE * WST <= NBUF * STAGE, "staging must fit in the pipeline buffers");
  static_assert(NBUF >= 2 && NBUF <= 5, "k-tile buffers");
  static_assert(BK == 32 || BK == 64, "k-tile depth");
  constexpr int STL = NBUF * STAGE + PP_STAMP_LDS <= 160 * 1024 ? PP_STAMP_LDS : 0;
  static_assert(NBUF * STAGE <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[NBUF * STAGE + STL];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2, wn = wave & 3;
#ifdef VIT_GEMM_STAMPS
  const bool stamp_on = STL > 0 && (int)blockIdx.x == g_stamp_wg && blockIdx.y == 0 && wn == 0 && lane == 0;
  unsigned long long* st_lds = reinterpret_cast<unsigned long long*>(smem + NBUF * STAGE) + grp * 1024;
  int si = 0;
  PP_STAMP();
#endif

  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn, z, split_idx;
  if (p.split_k > 1 && p.split_xcd) {
    // split-K weight gradients: the dispatcher deals the linear workgroup id (x fastest, then the
    // split, then the batch) round-robin over the 8 XCDs. Remap the whole (tile, split, batch) space
    // XCD-major so an XCD's ~32 concurrent workgroups cover one or two K-chunks: they walk the same
    // token rows in step and read each row panel from HBM once per XCD instead of once per XCD
    // per chunk (fc1 wgrad fetch 2.3x -> ~1.2x the operand bytes).
    const int total = nwg * p.split_k * (int)gridDim.z;
    const int lin = blockIdx.x + nwg * (blockIdx.y + p.split_k * blockIdx.z);
    const int xcd = lin & 7, q8 = total >> 3, r8 = total & 7;
    const int w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (lin >> 3);
    const int zs = w / nwg;
    z = zs / p.split_k;
    split_idx = zs % p.split_k;
    tile_coords(w % nwg, tiles_m, tiles_n, p.group_m, tm, tn);
  } else {
    const int orig = blockIdx.x;
    const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    tile_coords(wg, tiles_m, tiles_n, p.group_m, tm, tn);
    z = blockIdx.z;
    split_idx = blockIdx.y;
  }
  const int m0 = tm * BM, n0 = tn * BN;

  const char* Ab = p.A + (long)z * p.a_bs * 2;
  const char* Bb = p.B + (long)z * p.b_bs * 2;
  const long a_shift = AK ? (long)m0 * p.lda * 2 : (long)m0 * 2;
  const long b_shift = BKC ? (long)n0 * p.ldb * 2 : (long)n0 * 2;
  const uint32_t a_rec = (long)p.a_bytes > a_shift ? (uint32_t)(p.a_bytes - a_shift) : 0u;
  const uint32_t b_rec = (long)p.b_bytes > b_shift ? (uint32_t)(p.b_bytes - b_shift) : 0u;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(Ab + a_shift, a_rec);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(Bb + b_shift, b_rec);

  const int nkt = p.K / BK;
  const int kt0 = (int)((long)nkt * split_idx / p.split_k);
  const int kt1 = (int)((long)nkt * (split_idx + 1) / p.split_k);
  const int nk = kt1 - kt0;

  v4f acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s af[KK][FM], bfr[KK][FN];
  const int wm0 = grp * 128, wn0 = wn * TN;

  auto issue = [&](int t) {
    const int buf = (t % NBUF) * STAGE;
    stage_tile<BM, BK, AK, NWAVE>(smem, buf, rsA, p.lda, kt0 + t, wave, lane);
    stage_tile<BN, BK, BKC, NWAVE>(smem, buf + A_BYTES, rsB, p.ldb, kt0 + t, wave, lane);
  };
  auto mem = [&](int j) {
    const int cur = (j % NBUF) * STAGE;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
      for (int jn = 0; jn < FN; ++jn) bfr[kk][jn] = read_frag<BN, BK, BKC>(smem, cur + A_BYTES, wn0 + jn * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[kk][i] = read_frag<BM, BK, AK>(smem, cur, wm0 + i * 16, kk, lane);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto compute = [&]() {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jn = 0; jn < FN; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, af[kk][i]),
                                                               __builtin_bit_cast(v8bf, bfr[kk][jn]), acc[i][jn], 0, 0, 0);
  };

  // prologue: k-tiles 0 .. L-1 in flight, k-tile 0 landed
  constexpr int L = NBUF - 1;
#pragma unroll
  for (int t = 0; t < L; ++t)
    if (t < nk) issue(t);
  wait_tiles<LPT, L>((nk < L ? nk : L) - 1);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // slot s: group g reads k-tile j in slot 2j+g and multiplies it in slot 2j+g+1. At the start of
  // slot 2u, k-tile u+L goes into the buffer k-tile u-1 used (read by group 1 in slot 2u-1); at the
  // end of slot 2u+1 k-tile u+1 has landed (group 0 reads it in slot 2u+2). The two groups run
  // separate straight-line loops (a slot-role branch inside one loop makes the compiler copy the
  // accumulators at every join).
  auto end_odd = [&](int u) {  // end of slot 2u+1
    const int issued = u + L < nk ? u + L : nk - 1;
    __builtin_amdgcn_sched_barrier(0);
    wait_tiles<LPT, L>(issued - u - 1);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto end_even = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  PP_STAMP();
  if (grp == 0) {
    for (int j = 0; j < nk; ++j) {
      if (j + L < nk) issue(j + L);  // slot 2j
      mem(j);
      PP_STAMP();
      end_even();
      PP_STAMP();
      compute();  // slot 2j+1
      end_odd(j);
      PP_STAMP();
    }
  } else if (nk > 0) {
    if (L < nk) issue(L);  // slot 0
    end_even();
    PP_STAMP();
    for (int j = 0; j < nk - 1; ++j) {
      mem(j);  // slot 2j+1
      PP_STAMP();
      end_odd(j);
      PP_STAMP();
      if (j + 1 + L < nk) issue(j + 1 + L);  // slot 2j+2
      compute();
      end_even();
      PP_STAMP();
    }
    mem(nk - 1);  // slot 2nk-1
    end_odd(nk - 1);
    compute();  // slot 2nk: LDS is free from here on
  }
  PP_STAMP();

  // ---- epilogue ----
  const int g = lane >> 4, c = lane & 15;
  float* ws = reinterpret_cast<float*>(smem + wave * WST);
  constexpr int CPR = TN / 8;  // 8-column chunks per staged row
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int pass = 0; pass < 128 / PR; ++pass) {
#pragma unroll
    for (int i = 0; i < PR / 16; ++i)
#pragma unroll
      for (int jn = 0; jn < FN; ++jn)
#pragma unroll
        for (int r = 0; r < 4; ++r) ws[(i * 16 + 4 * g + r) * LDW + jn * 16 + c] = acc[pass * (PR / 16) + i][jn][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll 2
    for (int e = lane; e < PR * CPR; e += 64) {
      const int row = e / CPR, ch = e % CPR;
      const int m = m0 + wm0 + pass * PR + row, n = n0 + wn0 + ch * 8;
      float v[8];
      ld8f(ws + row * LDW + ch * 8, v);
      if (m >= p.M || n >= p.N) continue;
      if (p.vec && n + 8 <= p.N) {
        epi_store8<EPI>(p, z, split_idx, m, n, v);
        if (p.col_partial) {
#pragma unroll
          for (int k = 0; k < 8; ++k) csum[k] += v[k];
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) epi_store<EPI>(p, z, split_idx, m, n + k, v[k]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  if (p.col_partial) {
    // lanes with equal (lane % CPR) hold the same 8 columns: reduce over the rest of the wave
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) csum[k] += __shfl_xor(csum[k], o, 64);
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [group][BN]
    if (lane < CPR) {
#pragma unroll
      for (int k = 0; k < 8; ++k) red[grp * BN + wn0 + lane * 8 + k] = csum[k];
    }
    __syncthreads();
    for (int col = threadIdx.x; col < BN; col += 512)
      if (n0 + col < p.N) p.col_partial[(long)tm * p.N + n0 + col] = red[col] + red[BN + col];
  }
#ifdef VIT_GEMM_STAMPS
  PP_STAMP();
  if (stamp_on) {
    for (int k = 0; k < si && k < 1024; ++k) g_stamps[grp][k] = st_lds[k];
    if (si < 1024) g_stamps[grp][si] = 0;
  }
#endif
}

#include "gemm_pp2.inc"

template <int BN, int BK, int NBUF, bool AK, bool BKC, int EPI>
hipError_t launch_pp(const GemmDev& d, int batch, int split, hipStream_t s) {
  const int tiles = ((d.M + 255) / 256) * ((d.N + BN - 1) / BN);
  dim3 grid(tiles, split, batch);
  hipLaunchKernelGGL((gemm_pp_kernel<BN, BK, NBUF, AK, BKC, EPI>), grid, dim3(512), 0, s, d);
  return hipGetLastError();
}

template <int BM, int BN, int BK, int STAGES, int WM, int WN, bool AK, bool BKC, int EPI>
hipError_t launch_t(const GemmDev& d, int batch, int split, hipStream_t s) {
  const int tiles = ((d.M + BM - 1) / BM) * ((d.N + BN - 1) / BN);
  dim3 grid(tiles, split, batch);
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, BK, STAGES, WM, WN, AK, BKC, EPI>), grid, dim3(WM * WN * 64), 0, s, d);
  return hipGetLastError();
}

// Tile configurations:
//   0: 128x128x64, 2 stages, 4 waves (2x2)   — small problems
//   1: 256x256x32, 4 stages, 8 waves (2x4)   — large M and N >= 1536, and the split-K wgrads
//   2: 256x128x64, 3 stages, 8 waves (4x2)   — large M, narrow N (768)
//   3: 256x128x32, 3 stages, 8 waves (4x2)   — 2 workgroups per CU (epilogue overlaps MFMA)
//   4: 128x128x32, 4 stages, 4 waves (2x2)   — 2 workgroups per CU
template <int EPI, bool AK, bool BKC>
hipError_t launch_cfg(int cfg, const GemmDev& d, int batch, int split, hipStream_t s) {
  switch (cfg) {
    case 1: return launch_t<256, 256, 32, 4, 2, 4, AK, BKC, EPI>(d, batch, split, s);
    case 2: return launch_t<256, 128, 64, 3, 4, 2, AK, BKC, EPI>(d, batch, split, s);
    case 3: return launch_t<256, 128, 32, 3, 4, 2, AK, BKC, EPI>(d, batch, split, s);
    case 4: return launch_t<128, 128, 32, 4, 2, 2, AK, BKC, EPI>(d, batch, split, s);
    case 5: return launch_pp<256, 64, 2, AK, BKC, EPI>(d, batch, split, s);
    case 6: return launch_pp<128, 64, 3, AK, BKC, EPI>(d, batch, split, s);
    case 7: return launch_pp<256, 32, 4, AK, BKC, EPI>(d, batch, split, s);
    case 8: return launch_pp<256, 32, 5, AK, BKC, EPI>(d, batch, split, s);
    case 9: return launch_pp2<AK, BKC, EPI>(d, batch, split, s);
    default: return launch_t<128, 128, 64, 2, 2, 2, AK, BKC, EPI>(d, batch, split, s);
  }
}

template <int EPI>
hipError_t launch_layout(int cfg, const GemmDev& d, bool ak, bool bk, int batch, int split, hipStream_t s) {
  if (ak && bk) return launch_cfg<EPI, true, true>(cfg, d, batch, split, s);
  if (ak && !bk) return launch_cfg<EPI, true, false>(cfg, d, batch, split, s);
  if (!ak && !bk) return launch_cfg<EPI, false, false>(cfg, d, batch, split, s);
  return launch_cfg<EPI, false, true>(cfg, d, batch, split, s);
}

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
    static const int env_sk = [] {  // tuning override for the split-K weight gradients (5 .. 8)
      const char* e = getenv("VIT_GEMM_SPLITK_CFG");
      return e ? atoi(e) : 5;
    }();
    return env_sk == 6 || env_sk == 7 || env_sk == 8 ? env_sk : 5;
  }
  if (a->M >= 1024 && a->N >= 256) {
    // (short-K f32 residual outputs keep 2 workgroups per CU; the aux-reading epilogues run on the
    // half-tile kernel since their operand is prefetched a staging pass ahead: fc2 dgrad x GELU'
    // 286 us vs 356 us on 256x128)
    // (short-K f32 residual outputs — the out-projection — also run here: 7418 vs 7385 img/s over
    // the 256x128 two-workgroup kernel, profiles/r02/gemm_epilogue_diag.txt; VIT_GEMM_RESID_PP2=0
    // restores that)
    static const int env_rs = [] {
      const char* e = getenv("VIT_GEMM_RESID_PP2");
      return e ? atoi(e) : 1;
    }();
    if (ak && bk && (env_rs || !(a->epilogue == VIT_EPI_BIAS_RESID_F32 && a->K < 2048))) return 9;
    if (a->N >= 2048 && a->epilogue != VIT_EPI_GELU_BWD && a->epilogue != VIT_EPI_MUL_BF16) return 5;
    if (!bk && a->K >= 3072) return 5;
    return 3;
  }
  return 0;
}

}  // namespace

extern "C" int64_t vit_gemm_tile_rows(const vit_gemm_args* a) {
  if (!a) return 0;
  switch (pick_tile(a)) {
    case 1: case 2: case 3: case 5: case 6: case 7: case 8: case 9: return 256;
    default: return 128;
  }
}

extern "C" int vit_gemm_bf16(const vit_gemm_args* a, vit_stream_t stream) {
  VIT_CHECK_ARG(a != nullptr, "vit_gemm_bf16: null args");
  VIT_CHECK_ARG(a->M >= 0 && a->N >= 0 && a->K >= 0, "vit_gemm_bf16: negative size");
  VIT_CHECK_ARG(a->K % 64 == 0, "vit_gemm_bf16: K=%lld must be a multiple of 64", (long long)a->K);
  VIT_CHECK_ARG(a->M < (1 << 30) && a->N < (1 << 30), "vit_gemm_bf16: M/N too large");
  VIT_CHECK_ARG(a->A && a->B && a->C, "vit_gemm_bf16: null operand");
  VIT_CHECK_ARG(a->batch >= 1 && a->split_k >= 1, "vit_gemm_bf16: batch/split_k must be >= 1");
  VIT_CHECK_ARG(a->split_k == 1 || a->epilogue == VIT_EPI_SPLITK, "vit_gemm_bf16: split_k>1 needs VIT_EPI_SPLITK");
  VIT_CHECK_ARG(a->a_layout == VIT_K_CONTIG || a->a_layout == VIT_MN_CONTIG, "vit_gemm_bf16: bad a_layout");
  VIT_CHECK_ARG(a->b_layout == VIT_K_CONTIG || a->b_layout == VIT_MN_CONTIG, "vit_gemm_bf16: bad b_layout");
  if (a->M == 0 || a->N == 0) return VIT_OK;
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
  GemmDev d;
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
  VIT_CHECK_ARG(!d.drop.thr || (a->a_layout == VIT_K_CONTIG && a->b_layout == VIT_K_CONTIG),
                "vit_gemm_bf16: dropout epilogues need K-contiguous A and B");
  {
    // tile order: groups of 8 tile rows, column-major inside, so the workgroups resident at once
    // share A row panels and B column panels in L2 (fc1 fwd 326 -> 306 us; VIT_GEMM_GROUP_M=1:
    // row-major)
    static const int env_gm = [] {
      const char* e = getenv("VIT_GEMM_GROUP_M");
      return e ? atoi(e) : 8;
    }();
    static const int env_nt = [] {
      const char* e = getenv("VIT_GEMM_NT");
      return e ? atoi(e) : 0;
    }();
    d.group_m = env_gm;
    d.nt = env_nt;
    static const int env_diag = [] {
      const char* e = getenv("VIT_GEMM_DIAG");
      return e ? atoi(e) : 0;
    }();
    d.diag = env_diag;
    static const int env_sx = [] {
      const char* e = getenv("VIT_GEMM_SPLIT_XCD");
      return e ? atoi(e) : 1;
    }();
    d.split_xcd = env_sx;
  }
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
  VIT_CHECK_ARG(cfg >= 0 && cfg <= 9, "vit_gemm_bf16: bad tile config %d", cfg);
  VIT_CHECK_ARG(cfg != 1 || a->K % 32 == 0, "vit_gemm_bf16: K");
  auto run = [&](int c, const GemmDev& g) -> hipError_t {
    switch (a->epilogue) {
      case VIT_EPI_F32: return launch_layout<VIT_EPI_F32>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BF16: return launch_layout<VIT_EPI_BF16>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BIAS_BF16: return launch_layout<VIT_EPI_BIAS_BF16>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BIAS_GELU: return launch_layout<VIT_EPI_BIAS_GELU>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BIAS_RESID_F32:
        if (g.drop.thr) return launch_cfg<VIT_EPI_BIAS_RESID_F32 | EPI_DROP, true, true>(c, g, batch, split, s);
        return launch_layout<VIT_EPI_BIAS_RESID_F32>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_GELU_BWD: return launch_layout<VIT_EPI_GELU_BWD>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_BIAS_GELU_DGELU:
        if (g.drop.thr) return launch_cfg<VIT_EPI_BIAS_GELU_DGELU | EPI_DROP, true, true>(c, g, batch, split, s);
        return launch_layout<VIT_EPI_BIAS_GELU_DGELU>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_MUL_BF16: return launch_layout<VIT_EPI_MUL_BF16>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_PATCH:
        if (g.drop.thr) return launch_cfg<VIT_EPI_PATCH | EPI_DROP, true, true>(c, g, batch, split, s);
        return launch_layout<VIT_EPI_PATCH>(c, g, ak, bk, batch, split, s);
      case VIT_EPI_SPLITK: return launch_layout<VIT_EPI_SPLITK>(c, g, ak, bk, batch, split, s);
      default: return hipErrorInvalidValue;
    }
  };
  if (a->epilogue < 0 || a->epilogue > VIT_EPI_MUL_BF16) {
    vit::set_error("vit_gemm_bf16: unknown epilogue %d", a->epilogue);
    return VIT_ERR_INVALID_ARG;
  }
  // Wave quantisation of the one-workgroup-per-CU 256 x 256 kernels: when the last wave of tiles
  // would run less than half full (M = 50 432, N = 768: 591 tiles = 2.3 waves on 256 CUs), the
  // rows that fill whole waves run on them and the remaining rows on 128 x 128 tiles (several
  // workgroups per CU), ~2.4 instead of 3 wave-times. Row-local epilogues only.
  if ((cfg == 5 || cfg == 9) && batch == 1 && split == 1 && !a->col_partial && a->epilogue != VIT_EPI_PATCH &&
      a->tile == 0) {
    static const int ncu = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess)
        return 0;
      return n;
    }();
    const long tiles_n = (a->N + 255) / 256, tiles = ((a->M + 255) / 256) * tiles_n;
    if (ncu > 0) {
      const long full = tiles / ncu, rem = tiles - full * ncu;
      const long main_rows = (full * ncu / tiles_n) * 256;
      if (full >= 1 && rem > 0 && 2 * rem <= ncu && main_rows > 0 && main_rows < a->M) {
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
        g2.drop.row0 = (int)r0;  // dropout masks are indexed by the absolute row
        hipError_t e = run(cfg, g1);
        static const int rem_cfg = [] {
          const char* e = getenv("VIT_GEMM_REM_CFG");
          return e ? atoi(e) : 0;
        }();
        if (e == hipSuccess) e = run(rem_cfg >= 0 && rem_cfg <= 4 ? rem_cfg : 0, g2);
        return vit::check_hip(e, "vit_gemm_bf16 launch");
      }
    }
  }
  return vit::check_hip(run(cfg, d), "vit_gemm_bf16 launch");
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
}  // namespace

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
