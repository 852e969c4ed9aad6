// Shared device helpers for the gfx950 (CDNA4) ViT training kernels.
#pragma once
#include <stdlib.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <string>

#include "../../include/vit_hip.h"

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef unsigned short bf16_t;  // storage type for bf16 in HBM

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ bf16_t f2bf(float x) {
  __bf16 b = (__bf16)x;  // RNE, lowers to v_cvt_pk_bf16_f32 (NaN-preserving)
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((unsigned)u) << 16); }

__device__ __forceinline__ unsigned pack2bf(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Erf GELU (nn.GELU() default approximate='none', reference src/model.py:33) and its derivative.
// erf(x) = 1 - poly(t) exp(-x^2), t = 1/(1 + p|x|) (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7,
// i.e. fp32-erff class; GELU abs error <= 2.2e-7): one v_rcp and one v_exp instead of the ~40-op
// libm erff, and the derivative reuses the same exp(-u^2/2) for the normal pdf.
__device__ __forceinline__ float phi_and_pdf(float u, float* pdf) {
  const float e = __expf(-0.5f * u * u);  // exp(-x^2), x = u/sqrt(2)
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, fabsf(u), 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float erfa = 1.0f - p * t * e;  // erf(|x|)
  *pdf = 0.39894228040143268f * e;
  return 0.5f + 0.5f * copysignf(erfa, u);
}
__device__ __forceinline__ float gelu_f(float u) {
  float pdf;
  return u * phi_and_pdf(u, &pdf);
}
__device__ __forceinline__ float gelu_grad_f(float u) {
  float pdf;
  const float cdf = phi_and_pdf(u, &pdf);
  return cdf + u * pdf;
}

// Buffer resource descriptor for raw buffer loads (out-of-range lanes read 0).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// ---- dropout: Philox4x32-10 counter-based masks (see vit_dropout in vit_hip.h) ----
struct DropDev {
  uint32_t thr;    // keep iff the 16-bit draw >= thr; 0 = dropout off
  uint32_t site, k0, k1, off;
  float scale;     // 1 / (1 - p)
  int row0;        // added to the launch's row index (a GEMM launched on a row sub-range)
  int row_mul;     // mask row = row * row_mul + row0
};
static inline DropDev make_drop(const vit_dropout* d) {
  DropDev r = {0u, 0u, 0u, 0u, 0u, 1.0f, 0, 1};
  if (!d || !(d->p > 0.0f)) return r;
  const double t = (double)d->p * 65536.0 + 0.5;
  r.thr = t >= 65536.0 ? 65536u : (uint32_t)t;
  if (r.thr == 0) return r;
  r.site = d->site;
  r.k0 = (uint32_t)d->seed;
  r.k1 = (uint32_t)(d->seed >> 32) ^ (uint32_t)(d->offset >> 32);
  r.off = (uint32_t)d->offset;
  r.scale = d->p < 1.0f ? 1.0f / (1.0f - d->p) : 0.0f;
  r.row_mul = d->row_stride > 1 ? (int)d->row_stride : 1;
  return r;
}
// Random123 Philox4x32 with 10 rounds
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1, uint32_t* r) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  r[0] = c0; r[1] = c1; r[2] = c2; r[3] = c3;
}
// multipliers (0 or 1/(1-p)) of columns 8*col8 .. 8*col8+7 of `row`
__device__ __forceinline__ void drop_mult8(const DropDev& d, long row, int col8, float* m) {
  uint32_t r[4];
  philox4x32_10((uint32_t)col8, (uint32_t)(row * d.row_mul + d.row0), d.site, d.off, d.k0, d.k1, r);
#pragma unroll
  for (int k = 0; k < 8; ++k) m[k] = ((r[k >> 1] >> (16 * (k & 1))) & 0xffffu) >= d.thr ? d.scale : 0.0f;
}
__device__ __forceinline__ float drop_mult1(const DropDev& d, long row, int col) {
  uint32_t r[4];
  philox4x32_10((uint32_t)(col >> 3), (uint32_t)(row * d.row_mul + d.row0), d.site, d.off, d.k0, d.k1, r);
  const int k = col & 7;
  return ((r[k >> 1] >> (16 * (k & 1))) & 0xffffu) >= d.thr ? d.scale : 0.0f;
}

// ---- host-side error plumbing (thread-local last error, int status returns) ----
namespace vit {
void set_error(const char* fmt, ...);
int check_hip(hipError_t e, const char* what);
// Tuning / diagnostic knobs: the shipped library always takes the default; a build with
// -DVIT_DIAG_KNOBS (tools/, never the product) reads them from the environment instead.
inline int knob(const char* name, int dflt) {
#ifdef VIT_DIAG_KNOBS
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
#else
  (void)name;
  return dflt;
#endif
}
}  // namespace vit

#define VIT_CHECK_ARG(cond, ...)                 \
  do {                                           \
    if (!(cond)) {                               \
      vit::set_error(__VA_ARGS__);               \
      return VIT_ERR_INVALID_ARG;                \
    }                                            \
  } while (0)

#define VIT_LAUNCH_CHECK(what) return vit::check_hip(hipGetLastError(), what)
