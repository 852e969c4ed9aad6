// Kernel bodies of the bf16 MFMA GEMM (see gemm_decl.h); included only by the gemm_e*.hip units.
#pragma once
#include "gemm_decl.h"

namespace {
using vitg::GemmDev;
using vitg::GemmGroup;
using vitg::GEMM_GROUP_MAX;

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
// piece i (0 <= i < INSTR) of stage_tile's image alone (gemm_pp2's interleaved read slot). Same addressing as
// stage_tile, which keeps its own loop so that the lane offset and the row step are computed once per image.
template <int ROWS, int BK, bool KC, int NWAVE>
__device__ __forceinline__ void stage_piece(char* smem, int lds_off, __amdgpu_buffer_rsrc_t rs, long ld, int kt,
                                            int wave, int lane, int vbase, int i) {
  constexpr int CPR = KC ? BK / 8 : ROWS * 2 / 16;
  constexpr int RSTEP = NWAVE * 64 / CPR;
  static_assert(RSTEP % 16 == 0, "swizzle must repeat between a wave's instructions");
  const int c = wave * 64 + lane;
  const int r = c / CPR, pc = c % CPR;
  int lane_off, base;
  if constexpr (KC) {
    lane_off = (int)(r * ld * 2) + (pc ^ swz_k<BK>(r)) * 16;
    base = kt * BK * 2 + vbase;
  } else {
    lane_off = (int)(r * ld * 2) + ((pc * 16) ^ (swz_mn(r) << 5));
    base = (int)((long)kt * BK * ld * 2) + vbase;
  }
  base = __builtin_amdgcn_readfirstlane(base + i * (int)(RSTEP * ld * 2));
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, smem + lds_off + (i * NWAVE + wave) * 1024), 16,
                                           lane_off + base, 0, 0, 0);
}

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

// M/N-contiguous fragment reads of gemm_pp_kernel by inline asm. With the k-tile buffers in one LDS
// array indexed at run time, hipcc cannot tell a ds_read_b64_tr_b16 of k-tile j from the LDS-DMA of
// k-tile j+1 just issued into the other buffer, and its waitcnt pass put an s_waitcnt vmcnt(0) in
// front of the reads: every read slot waited for the DMA it had just issued to land (tools/gemm_diag
// stamps of the split-K weight gradient: ~2 550 of ~3 900 cycles per k-tile). The asm reads are not
// tracked by that pass; the caller ends its read phase with an explicit lgkmcnt(0) and a
// sched_barrier before any use. `a` = the fragment's lane address without the k offset (swz_mn of
// rows 8g + q and 8g + q + 4 + 32 kk is the same for every kk, so kk and the hi half are immediates).
template <int ROWS>
__device__ __forceinline__ uint32_t frag_tr_lane_off(int r0, int lane) {
  constexpr int RB = ROWS * 2;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int ra = 8 * g + q;
  return (uint32_t)(ra * RB + (((r0 + 4 * p) * 2) ^ (swz_mn(ra) << 5)));
}
template <int ROWS, int KKI>
__device__ __forceinline__ v8s read_frag_tr_asm(uint32_t a) {
  constexpr int RB = ROWS * 2;
  v4s lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(a), "i"(KKI * 32 * RB));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a), "i"(KKI * 32 * RB + 4 * RB));
  v8s r;
  r.lo = lo;
  r.hi = hi;
  return r;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

using vitg::EPI_DROP;

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

// ---- register-resident epilogue (whole in-range tiles) ----------------------------------------
// hipcc protects the data VGPRs of an outstanding global store: a register that is overwritten while
// a store still reads it gets an `s_waitcnt vmcnt` in front of the overwrite, and vmcnt retires in
// order, so a store loop whose iterations reuse the same registers waits for every store to be
// acknowledged before the next chunk (16 serialized store round trips per 256x256 tile; the fc1
// forward spent 38% of its time there). The fast epilogue therefore computes a whole staging pass
// into registers (epi_prep8), issues its stores (epi_put8), and keeps every pass's store registers
// live to the end of the tile (keep_live), so no store source is ever overwritten.
template <int EPI>
struct EpiOut {  // 16-B words per 8-column chunk: one bf16 output, or f32 / two bf16 outputs
  static constexpr int E = EPI & 15;
  static constexpr int W = (E == VIT_EPI_BF16 || E == VIT_EPI_BIAS_BF16 || E == VIT_EPI_GELU_BWD || E == VIT_EPI_MUL_BF16)
                               ? 1
                               : 2;
  static constexpr bool BIAS = E == VIT_EPI_BIAS_BF16 || E == VIT_EPI_BIAS_GELU || E == VIT_EPI_BIAS_RESID_F32 ||
                               E == VIT_EPI_BIAS_GELU_DGELU;
  static constexpr bool FAST = E != VIT_EPI_PATCH;  // PATCH reads per-row operands: generic path only
};

__device__ __forceinline__ uint4 pack8bf(const float* v) {
  return make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
}
__device__ __forceinline__ void keep_live(const uint4& x) {
  asm volatile("" ::"v"(x.x), "v"(x.y), "v"(x.z), "v"(x.w));
}

// the arithmetic of epi_store8 for chunk (m, n..n+7) with the bias `b` and aux values `pre` already in
// registers; v becomes the values written (col_partial sums them), o the packed store words
template <int EPI>
__device__ __forceinline__ void epi_prep8(const GemmDev& p, int m, int n, float* v, const float* pre, const float* b,
                                          uint4* o) {
  constexpr int E = EPI & 15;
  constexpr bool DROP = (EPI & EPI_DROP) != 0;
  if constexpr (E == VIT_EPI_F32 || E == VIT_EPI_SPLITK) {
    o[0] = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
    o[1] = make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7]));
  } else if constexpr (E == VIT_EPI_BF16) {
    o[0] = pack8bf(v);
  } else if constexpr (E == VIT_EPI_BIAS_BF16) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += b[k];
    o[0] = pack8bf(v);
  } else if constexpr (E == VIT_EPI_BIAS_GELU) {
    float gl[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] += b[k];
      gl[k] = gelu_f(v[k]);
    }
    o[0] = pack8bf(v);
    o[1] = pack8bf(gl);
  } else if constexpr (E == VIT_EPI_BIAS_RESID_F32) {
    if constexpr (DROP) {
      float dm[8];
      drop_mult8(p.drop, m, n >> 3, dm);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (v[k] + b[k]) * dm[k] + pre[k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += b[k] + pre[k];
    }
    o[0] = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
    o[1] = make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7]));
  } else if constexpr (E == VIT_EPI_GELU_BWD) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= gelu_grad_f(pre[k]);
    o[0] = pack8bf(v);
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
    o[0] = pack8bf(v);
    o[1] = pack8bf(gl);
  } else if constexpr (E == VIT_EPI_MUL_BF16) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= pre[k];
    o[0] = pack8bf(v);
  }
}

__device__ __forceinline__ void st16(void* q, const uint4& x, bool nt) {
  const v4u_t u = {x.x, x.y, x.z, x.w};
  if (nt)
    __builtin_nontemporal_store(u, reinterpret_cast<v4u_t*>(q));
  else
    *reinterpret_cast<v4u_t*>(q) = u;
}

template <int EPI>
__device__ __forceinline__ void epi_put8(const GemmDev& p, int z, int split_idx, int m, int n, const uint4* o) {
  constexpr int E = EPI & 15;
  if constexpr (E == VIT_EPI_SPLITK) {
    float* q = (float*)p.C + ((long)z * p.split_k + split_idx) * (long)p.M * p.N + (long)m * p.N + n;
    st16(q, o[0], p.nt);
    st16(q + 4, o[1], p.nt);
  } else if constexpr (EpiOut<EPI>::W == 1) {
    st16((bf16_t*)p.C + z * p.c_bs + (long)m * p.ldc + n, o[0], p.nt);
  } else if constexpr (E == VIT_EPI_BIAS_GELU || E == VIT_EPI_BIAS_GELU_DGELU) {
    st16((bf16_t*)p.C + z * p.c_bs + (long)m * p.ldc + n, o[0], p.nt);
    st16((bf16_t*)p.C2 + z * p.c_bs + (long)m * p.ldc2 + n, o[1], p.nt);
  } else {  // f32 output
    float* q = (float*)p.C + z * p.c_bs + (long)m * p.ldc + n;
    st16(q, o[0], p.nt);
    st16(q + 4, o[1], p.nt);
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

// Register-resident epilogue of a wave that owns 128 rows (8 fragments of 16) x FN*16 columns of a
// whole in-range tile (the ping-pong kernels): 16-row passes through the wave's LDS strip `ws`. This
// lane's 8-column chunk is the same in every pass (64 % CPR == 0), so the bias is read once, before
// any store; the aux operand is requested one pass ahead; the packed store words of the last NSET
// passes stay live (keep_live), so no store's source register is overwritten (see epi_prep8).
template <int EPI, int FN, int LDW, int CPR>
__device__ __forceinline__ void epilogue_fast(const GemmDev& p, v4f (&acc)[8][FN], float* ws, int lane, int mw0,
                                              int nw0, int z, int split_idx, float* csum) {
  static_assert(64 % CPR == 0 && CPR == FN * 2, "one fixed 8-column chunk per lane");
  constexpr int W = EpiOut<EPI>::W;
  constexpr int AW = AuxPre<EPI>::W > 0 ? AuxPre<EPI>::W : 1;
  constexpr int PF = 16, ITF = PF * CPR / 64, NPF = 8;
  constexpr int NSET = W == 2 ? 4 : NPF;  // output register sets (ring of passes)
  const int g = lane >> 4, c = lane & 15;
  const int ch = lane % CPR;
  const int n = nw0 + ch * 8;
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (EpiOut<EPI>::BIAS) {
    if (p.bias) ld8f(p.bias + z * p.bias_bs + n, bv);
  }
  uint4 fc[ITF][AW], fn_[ITF][AW];
  auto fetch_f = [&](uint4 (*ax)[AW], int pass) {
    if constexpr (AuxPre<EPI>::W > 0) {
#pragma unroll
      for (int it = 0; it < ITF; ++it) AuxPre<EPI>::fetch(p, mw0 + pass * PF + (lane + it * 64) / CPR, n, ax[it]);
    }
  };
  fetch_f(fc, 0);
  uint4 ob[NSET][ITF][W];
#pragma unroll
  for (int pass = 0; pass < NPF; ++pass) {
    if (pass + 1 < NPF) fetch_f(fn_, pass + 1);
#pragma unroll
    for (int jn = 0; jn < FN; ++jn)
#pragma unroll
      for (int r = 0; r < 4; ++r) ws[(4 * g + r) * LDW + jn * 16 + c] = acc[pass][jn][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    uint4(*os)[W] = ob[pass % NSET];
#pragma unroll
    for (int it = 0; it < ITF; ++it) {
      const int row = (lane + it * 64) / CPR;
      float v[8], u[8];
      ld8f(ws + row * LDW + ch * 8, v);
      if constexpr (AuxPre<EPI>::W > 0) AuxPre<EPI>::unpack(fc[it], u);
      epi_prep8<EPI>(p, mw0 + pass * PF + row, n, v, u, bv, os[it]);
      if (p.col_partial) {
#pragma unroll
        for (int k = 0; k < 8; ++k) csum[k] += v[k];
      }
    }
#pragma unroll
    for (int it = 0; it < ITF; ++it) epi_put8<EPI>(p, z, split_idx, mw0 + pass * PF + (lane + it * 64) / CPR, n, os[it]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if constexpr (AuxPre<EPI>::W > 0) {
#pragma unroll
      for (int it = 0; it < ITF; ++it)
#pragma unroll
        for (int w = 0; w < AW; ++w) fc[it][w] = fn_[it][w];
    }
  }
#pragma unroll
  for (int s = 0; s < NSET; ++s)
#pragma unroll
    for (int it = 0; it < ITF; ++it)
#pragma unroll
      for (int w = 0; w < W; ++w) keep_live(ob[s][it][w]);
}

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
    if (p.diag >= 100 && (orig >> 3) >= 32 && (orig >> 3) < 64) {
      // diagnostic (VIT_GEMM_DIAG = 100 + us): start the second resident workgroup of every CU late
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)(p.diag - 100) * 100ull)
        __builtin_amdgcn_s_sleep(8);
    }
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
    if constexpr (AK && BKC) {
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
    } else {
      // an M/N-contiguous operand: its transposed fragment reads by inline asm (hipcc puts a vmcnt(0) in front of
      // a ds_read_b64_tr_b16 of this array while the DMA just issued into another stage is in flight: the
      // round-3 gemm_pp_kernel finding; 60 vs 27 us for the fc1 data gradient's wave-split remainder with W1 read
      // in place), every read of a k-step issued before an explicit lgkmcnt(0), then the MFMAs
      const uint32_t sb = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)LDS_PTR(char, smem) + cur);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        v8s bfr[FN], af[FM];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (BKC)
            bfr[j] = read_frag<BN, BK, BKC>(smem, cur + A_BYTES, wn0 + j * 16, kk, lane);
          else
            bfr[j] = kk == 0 ? read_frag_tr_asm<BN, 0>(sb + A_BYTES + frag_tr_lane_off<BN>(wn0 + j * 16, lane))
                             : read_frag_tr_asm<BN, 1>(sb + A_BYTES + frag_tr_lane_off<BN>(wn0 + j * 16, lane));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          if constexpr (AK)
            af[i] = read_frag<BM, BK, AK>(smem, cur, wm0 + i * 16, kk, lane);
          else
            af[i] = kk == 0 ? read_frag_tr_asm<BM, 0>(sb + frag_tr_lane_off<BM>(wm0 + i * 16, lane))
                            : read_frag_tr_asm<BM, 1>(sb + frag_tr_lane_off<BM>(wm0 + i * 16, lane));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, af[i]),
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
  constexpr int AWB = AuxPre<EPI>::W > 0 ? AuxPre<EPI>::W : 1;
  const bool fast = EpiOut<EPI>::FAST && p.vec && m0 + BM <= p.M && n0 + BN <= p.N;
  float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (EpiOut<EPI>::BIAS) {
    if (fast && p.bias) ld8f(p.bias + z * p.bias_bs + n0 + (threadIdx.x % CPR) * 8, bv);
  }
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
    if (fast) {
      // whole in-range tile: this thread's 8-column chunk is fixed (NT % CPR == 0); every aux chunk
      // of the pass is requested before the first store and the store words stay live (epi_prep8)
      constexpr int ITB = PASS_ROWS * CPR / NT;
      static_assert(ITB * NT == PASS_ROWS * CPR, "whole chunks per thread");
      const int ch = threadIdx.x % CPR, n = n0 + ch * 8;
      uint4 ax[ITB][AWB], ob[ITB][EpiOut<EPI>::W];
      if constexpr (AuxPre<EPI>::W > 0) {
#pragma unroll
        for (int it = 0; it < ITB; ++it)
          AuxPre<EPI>::fetch(p, m0 + pass * PASS_ROWS + (threadIdx.x + it * NT) / CPR, n, ax[it]);
      }
#pragma unroll
      for (int it = 0; it < ITB; ++it) {
        const int row = (threadIdx.x + it * NT) / CPR;
        float v[8], u[8];
        ld8f(cs + row * LDC + ch * 8, v);
        if constexpr (AuxPre<EPI>::W > 0) AuxPre<EPI>::unpack(ax[it], u);
        epi_prep8<EPI>(p, m0 + pass * PASS_ROWS + row, n, v, u, bv, ob[it]);
        if (p.col_partial) {
#pragma unroll
          for (int k = 0; k < 8; ++k) csum[k] += v[k];
        }
      }
#pragma unroll
      for (int it = 0; it < ITB; ++it)
        epi_put8<EPI>(p, z, split_idx, m0 + pass * PASS_ROWS + (threadIdx.x + it * NT) / CPR, n, ob[it]);
#pragma unroll
      for (int it = 0; it < ITB; ++it)
#pragma unroll
        for (int w = 0; w < EpiOut<EPI>::W; ++w) keep_live(ob[it][w]);
    } else
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
// serialising. Two LDS k-tile buffers: each group issues its half of the LDS-DMA of k-tile u+1 at
// the end of its read slot of k-tile u (group 0 in slot 2u, group 1 in slot 2u-1 ... k-tile u-1's
// buffer, which both groups have finished reading), and it is waited for at the end of slot 2u+1,
// before group 0 first reads it; raw s_barrier (no vmcnt(0) drain at the barriers in between).
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
  // both operands M/N-contiguous (the weight gradients): asm transpose reads (frag_tr_lane_off)
  constexpr bool TR_ASM = !AK && !BKC;
  uint32_t a_lane[FM], b_lane[FN];
  if constexpr (TR_ASM) {
    const uint32_t s0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
#pragma unroll
    for (int i = 0; i < FM; ++i) a_lane[i] = s0 + frag_tr_lane_off<BM>(wm0 + i * 16, lane);
#pragma unroll
    for (int jn = 0; jn < FN; ++jn) b_lane[jn] = s0 + A_BYTES + frag_tr_lane_off<BN>(wn0 + jn * 16, lane);
  }
  auto mem = [&](int j) {
    const int cur = (j % NBUF) * STAGE;
    if constexpr (TR_ASM) {
      const uint32_t c = __builtin_amdgcn_readfirstlane(cur);
#pragma unroll
      for (int jn = 0; jn < FN; ++jn) {
        bfr[0][jn] = read_frag_tr_asm<BN, 0>(b_lane[jn] + c);
        if constexpr (KK > 1) bfr[KK - 1][jn] = read_frag_tr_asm<BN, 1>(b_lane[jn] + c);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        af[0][i] = read_frag_tr_asm<BM, 0>(a_lane[i] + c);
        if constexpr (KK > 1) af[KK - 1][i] = read_frag_tr_asm<BM, 1>(a_lane[i] + c);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
        for (int jn = 0; jn < FN; ++jn)
          bfr[kk][jn] = read_frag<BN, BK, BKC>(smem, cur + A_BYTES, wn0 + jn * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < FM; ++i) af[kk][i] = read_frag<BM, BK, AK>(smem, cur, wm0 + i * 16, kk, lane);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };
  auto compute = [&]() {
    if (p.prio) __builtin_amdgcn_s_setprio(1);  // the MFMA cluster ahead of the partner group's issue
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jn = 0; jn < FN; ++jn)
          acc[i][jn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, af[kk][i]),
                                                               __builtin_bit_cast(v8bf, bfr[kk][jn]), acc[i][jn], 0, 0, 0);
    if (p.prio) __builtin_amdgcn_s_setprio(0);
  };

  // prologue: k-tiles 0 .. L-1 in flight, k-tile 0 landed
  constexpr int L = NBUF - 1;
#pragma unroll
  for (int t = 0; t < L; ++t)
    if (t < nk) issue(t);
  wait_tiles<LPT, L>((nk < L ? nk : L) - 1);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // slot s: group g reads k-tile j in slot 2j+g and multiplies it in slot 2j+g+1. After its reads of
  // k-tile j, a group issues its half of k-tile j+L into the buffer of k-tile j+L-NBUF (group 1: of
  // k-tile j+1+L into k-tile j's buffer, which group 0 read in slot 2j); at the end of slot 2u+1
  // k-tile u+1 has landed (group 0 reads it in slot 2u+2). The two groups run
  // separate straight-line loops (a slot-role branch inside one loop makes the compiler copy the
  // accumulators at every join).
  auto end_odd = [&](int u, int ahead) {  // end of slot 2u+1; this wave has issued k-tiles up to u + ahead
    const int issued = u + ahead < nk ? u + ahead : nk - 1;
    __builtin_amdgcn_sched_barrier(0);
    wait_tiles<LPT, L + 1>(issued - u - 1);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto end_even = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  PP_STAMP();
  // Both groups issue their DMA half at the END of their read slot (after the fragment reads): the
  // buffer they refill held the k-tile both groups have finished reading. Issued at the start of a
  // slot instead, group 1's half queued behind group 0's in the same slot and held group 1's MFMAs
  // back ~1 200 cycles per k-tile (tools/gemm_diag stamps, profiles/r03/wgrad_slots_summary.txt:
  // split-K fc1 weight gradient 3 780 -> 3 130 cycles per k-tile, step +3.5%).
  if (grp == 0) {
    for (int j = 0; j < nk; ++j) {
      mem(j);  // slot 2j
      if (j + L < nk) issue(j + L);
      PP_STAMP();
      end_even();
      PP_STAMP();
      compute();  // slot 2j+1
      end_odd(j, L);
      PP_STAMP();
    }
  } else if (nk > 0) {
    if (L < nk) issue(L);  // slot 0
    end_even();
    PP_STAMP();
    for (int j = 0; j < nk - 1; ++j) {
      mem(j);  // slot 2j+1
      if (j + 1 + L < nk) issue(j + 1 + L);
      PP_STAMP();
      end_odd(j, L + 1);
      PP_STAMP();
      compute();  // slot 2j+2
      end_even();
      PP_STAMP();
    }
    mem(nk - 1);  // slot 2nk-1
    end_odd(nk - 1, L);
    compute();  // slot 2nk: LDS is free from here on
  }
  PP_STAMP();

  // ---- epilogue ----
  const int g = lane >> 4, c = lane & 15;
  float* ws = reinterpret_cast<float*>(smem + wave * WST);
  constexpr int CPR = TN / 8;  // 8-column chunks per staged row
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (EpiOut<EPI>::FAST && p.vec && m0 + BM <= p.M && n0 + BN <= p.N) {
    epilogue_fast<EPI, FN, LDW, CPR>(p, acc, ws, lane, m0 + wm0, n0 + wn0, z, split_idx, csum);
  } else {
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
#ifdef VIT_DIAG_KNOBS
    case 10: return launch_pp2<AK, BKC, EPI, 32, 2>(d, batch, split, s);  // diagnostic: 32-deep k-tiles
    case 11: return launch_pp2<AK, BKC, EPI, 32, 4>(d, batch, split, s);  // ... with a 3-k-tile-deep ring
#endif
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

}  // namespace
