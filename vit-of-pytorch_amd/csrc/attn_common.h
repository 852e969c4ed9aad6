// Shared device helpers of the attention kernels (attention.hip: LDS-resident exact softmax for
// N <= 320; attention_tiled.hip: K/V-tiled online softmax for longer sequences).
#pragma once
#include "common.h"

namespace vit_attn {

constexpr float LOG2E = 1.4426950408889634f;
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

template <int HD>
__device__ __forceinline__ int aswz(int row) {
  if constexpr (HD == 64) return ((row >> 1) & 3) << 1;
  return 0;
}

template <int HD>
__device__ __forceinline__ int img_off(int row, int chunk) {
  return row * HD * 2 + ((chunk ^ aswz<HD>(row)) << 4);
}

// Load rows [0, NP) x [0, HD) of two strided bf16 matrices into swizzled LDS images (zero padded).
// Every load of the thread is issued before the first LDS write (one HBM latency per image pair
// instead of one per 16-B chunk): buffer loads against a descriptor that covers the valid rows, so
// padding rows / columns >= hd read as zero without a branch around the load.
template <int HD, int NP, int NT>
__device__ __forceinline__ void load_images(char* imgA, const bf16_t* srcA, long strideA, char* imgB,
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
    if (c < TOTAL) {
      const int row = c / CPR, ch = c % CPR;
      *reinterpret_cast<v4u*>(imgA + img_off<HD>(row, ch)) = a[k];
      *reinterpret_cast<v4u*>(imgB + img_off<HD>(row, ch)) = b[k];
    }
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

// ---- 80-wide images (ViT-H/14's hd 80): two 32-k fragments + one 16-k tail ----
// A row of 160 B needs no swizzle: the row read (16 rows x one 16-B chunk, two lane groups) and the
// transposed read (8 rows x 32 B) both land on distinct banks (row r starts at bank 40r mod 64). The
// k tail (k = 64 + 4g .. + 3) goes to v_mfma_f32_16x16x16_bf16, whose operand lane (g, i) holds row i,
// k = 4g .. 4g + 3: an 8-B read per lane.
template <int HD>
constexpr bool k_tail = HD % 32 != 0;  // HD = 80 (16 trailing k columns)
template <int HD>
constexpr int k_full = HD / 32;  // whole 32-k fragments

template <int HD>
__device__ __forceinline__ v4s rd_row16(const char* img, int r0, int lane) {
  static_assert(HD % 32 == 16, "16-k tail fragments exist for HD = 32m + 16");
  const int row = r0 + (lane & 15);
  return *reinterpret_cast<const v4s*>(img + row * HD * 2 + (k_full<HD> * 32 + 4 * (lane >> 4)) * 2);
}

// tail fragment straight from global memory: row r0 + i, columns 32 k_full + 4g .. + 3 (zero past N / hd)
template <int HD>
__device__ __forceinline__ v4s gl_row16(const bf16_t* __restrict__ src, long row_stride, int r0, int N, int hd,
                                        int lane) {
  const int row = r0 + (lane & 15), col = k_full<HD> * 32 + 4 * (lane >> 4);
  v4s v = {0, 0, 0, 0};
  if (row < N && col < hd) v = *reinterpret_cast<const v4s*>(src + (long)row * row_stride + col);
  return v;
}

// one tile of rd_tr: lane (g, i) gets column d0 + i of image rows 16t + 4g + 0..3 (16x16x16 operand)
template <int HD>
__device__ __forceinline__ v4s rd_tr1(const char* img, int t, int d0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int colb = (d0 + 4 * p) * 2;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      LDS_PTR(v4s, img + img_off<HD>(16 * t + 4 * g + q, colb >> 4) + (colb & 15)));
}

__device__ __forceinline__ v8bf pack8(const v4f& a, const v4f& b) {
  v8s r;
  r[0] = (short)f2bf(a[0]); r[1] = (short)f2bf(a[1]); r[2] = (short)f2bf(a[2]); r[3] = (short)f2bf(a[3]);
  r[4] = (short)f2bf(b[0]); r[5] = (short)f2bf(b[1]); r[6] = (short)f2bf(b[2]); r[7] = (short)f2bf(b[3]);
  return __builtin_bit_cast(v8bf, r);
}

// 2^x on the transcendental unit (bare v_exp_f32). Arguments are s*log2e - lse <= ~0, so results
// only underflow (to 0) for keys whose softmax weight is below f32 resolution anyway.
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ v4f mfma(const v8bf& a, const v8bf& b, const v4f& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void store4(bf16_t* dst, const v4f& v, float s) {
  uint2 u;
  u.x = pack2bf(v[0] * s, v[1] * s);
  u.y = pack2bf(v[2] * s, v[3] * s);
  *reinterpret_cast<uint2*>(dst) = u;
}

// A row of HD/16 accumulator fragments (columns 16dt + 4g .. +3), packed to bf16 before any of its
// stores is issued. hipcc protects the source registers of an outstanding store with an
// `s_waitcnt vmcnt` before they are overwritten (and vmcnt retires in order), so store4 calls that
// reuse one temporary serialize on the store round trip; packing every fragment first, storing them,
// and keeping the packed words live (keep_live2) lets the stores of a row overlap.
__device__ __forceinline__ uint2 pack4bf(const v4f& v, float s) {
  uint2 u;
  u.x = pack2bf(v[0] * s, v[1] * s);
  u.y = pack2bf(v[2] * s, v[3] * s);
  return u;
}
__device__ __forceinline__ void keep_live2(const uint2& u) { asm volatile("" ::"v"(u.x), "v"(u.y)); }

// Global row fragment (16 rows x 32 k, MFMA operand layout) straight to registers: lane (g, i) gets
// row r0 + i, columns kk*32 + 8g .. +7; rows >= N and columns >= hd read as zero.
template <int HD>
__device__ __forceinline__ v8bf gl_row(const bf16_t* __restrict__ src, long row_stride, int r0, int kk, int N, int hd,
                                       int lane) {
  const int row = r0 + (lane & 15), col = kk * 32 + 8 * (lane >> 4);
  v8s v = {0, 0, 0, 0, 0, 0, 0, 0};
  if (row < N && col < hd) v = *reinterpret_cast<const v8s*>(src + (long)row * row_stride + col);
  return __builtin_bit_cast(v8bf, v);
}

// sum of the 16 lanes that share (lane >> 4): reduction over the MFMA column (key / query) index
__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

// Column sums over the 16 lanes of a DPP row for 16 values at once: v[k] of every lane of the row summed, the
// total of v[k] landing in lane k of the row (a fixed-order butterfly, deterministic). Each step halves the
// values a lane holds: the lane keeps the half selected by one bit of its row index and adds what its
// partner (ror 8, half-mirror, xor 2, xor 1: partners differ in that bit and agree on the bits already
// used) sends of the same half: 8 + 4 + 2 + 1 DPP moves instead of 16 x 4 row-sum steps.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
template <int NV, int CTRL>
__device__ __forceinline__ void butterfly_step(float* v, bool upper) {
#pragma unroll
  for (int k = 0; k < NV / 2; ++k) {
    const float keep = upper ? v[k + NV / 2] : v[k];
    const float send = upper ? v[k] : v[k + NV / 2];
    v[k] = keep + dpp_mov<CTRL>(send);
  }
}
__device__ __forceinline__ float reduce16(float (&v)[16], int i) {
  butterfly_step<16, 0x128>(v, (i & 8) != 0);  // row_ror:8 (lane ^ 8)
  butterfly_step<8, 0x141>(v, (i & 4) != 0);   // row_half_mirror (j <-> 7 - j within 8 lanes)
  butterfly_step<4, 0x4E>(v, (i & 2) != 0);    // quad_perm [2,3,0,1] (lane ^ 2)
  butterfly_step<2, 0xB1>(v, (i & 1) != 0);    // quad_perm [1,0,3,2] (lane ^ 1)
  return v[0];
}

// reduce16 for 4 or 8 values: the butterfly over row bits 3, 2 (, 1), then plain DPP sums over the bits left.
// The total of value k lands in the lanes i with k = i >> (4 - log2 NV) (every lane for 16 values, even lanes
// for 8, lanes 4m for 4).
template <int NV>
__device__ __forceinline__ float reduce_row(float (&v)[NV], int i) {
  static_assert(NV == 4 || NV == 8 || NV == 16, "4, 8 or 16 values");
  butterfly_step<NV, 0x128>(v, (i & 8) != 0);
  butterfly_step<NV / 2, 0x141>(v, (i & 4) != 0);
  if constexpr (NV >= 8) butterfly_step<NV / 4, 0x4E>(v, (i & 2) != 0);
  else v[0] += dpp_mov<0x4E>(v[0]);
  if constexpr (NV == 16) butterfly_step<2, 0xB1>(v, (i & 1) != 0);
  else v[0] += dpp_mov<0xB1>(v[0]);
  return v[0];
}

// dst[16dt + 4g + r] += s * (sum over the 16 lanes i of acc[dt][r]), dt in [D0, HD / 16): column sums of a
// 16 x HD accumulator strip (lane i = row) added to one wave's LDS row, four dt (16 values) per butterfly
template <int HD, int D0 = 0>
__device__ __forceinline__ void add_colsums(float* dst, const v4f* acc, float s, int lane) {
  constexpr int ND = HD / 16 - D0 < 4 ? HD / 16 - D0 : 4;
  constexpr int NV = 4 * ND;
  constexpr int SH = NV == 16 ? 0 : NV == 8 ? 1 : 2;
  const int g = lane >> 4, i = lane & 15;
  float v[NV];
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[4 * d + r] = acc[D0 + d][r];
  const float t = reduce_row<NV>(v, i);
  const int k = i >> SH;
  if ((i & ((1 << SH) - 1)) == 0) dst[(D0 + (k >> 2)) * 16 + 4 * g + (k & 3)] += t * s;
  if constexpr (D0 + ND < HD / 16) add_colsums<HD, D0 + ND>(dst, acc, s, lane);
}

// ---- explicit LDS address space (byte offsets from the dynamic LDS base) ----
typedef __attribute__((address_space(3))) char lds_t;
template <class T>
__device__ __forceinline__ T lds_ld(const lds_t* p) {
  return *reinterpret_cast<const __attribute__((address_space(3))) T*>(p);
}
template <class T>
__device__ __forceinline__ void lds_st(lds_t* p, const T& v) {
  *reinterpret_cast<__attribute__((address_space(3))) T*>(p) = v;
}
__device__ __forceinline__ v4s lds_tr(const lds_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(reinterpret_cast<__attribute__((address_space(3))) v4s*>(
      const_cast<lds_t*>(p)));
}
__device__ __forceinline__ v4f mfma16(const v4s& a, const v4s& b, const v4f& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
// c + A B over 16 k on its own zero accumulator, added by VALU. A v_mfma_f32_16x16x16_bf16 that takes
// as its accumulator the exact result registers of a v_mfma_f32_16x16x32_bf16 issued just before it
// (hipcc pads that pair with no wait states: an exactly overlapped accumulator is forwarded between
// MFMAs) read stale values on gfx950: the 16-k tail of hd-80 scores came out wrong in whole strips at
// some schedules. Every 16-k step that extends a 32-k chain goes through here.
__device__ __forceinline__ v4f mfma16_add(const v4s& a, const v4s& b, const v4f& c) {
  const v4f t = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, v4f{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  return c + t;
}
// x - x computed by the hardware: 0 for finite x, NaN for NaN / inf (the attention objects are built with
// -fno-honor-nans, under which the compiler would fold x - x to 0)
__device__ __forceinline__ float nan_of(float x) {
  float r;
  asm("v_sub_f32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
}
// max(a, b, c): plain fmaxf, which hipcc folds into v_max3_f32 under -mno-amdgpu-ieee -fno-honor-nans (the
// attention objects' flags). Not inline asm: the operands are MFMA results, and hipcc's hazard recognizer
// does not pad an asm statement that reads an MFMA's destination registers with the wait states the
// MFMA -> VALU read needs, so an asm v_max3_f32 placed a few instructions after the MFMA read the
// register's previous contents (a partial score): a wrong row max, which the shift-invariant softmax
// turned into last-bit differences between runs (and which could overflow exp2 for a large gap).
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
__device__ __forceinline__ v4s pack4(const v4f& a) {
  v4s r;
  r[0] = (short)f2bf(a[0]); r[1] = (short)f2bf(a[1]); r[2] = (short)f2bf(a[2]); r[3] = (short)f2bf(a[3]);
  return r;
}

// Per-lane byte offsets into a [rows][HD] swizzled image (img_off), for
//   row reads (16 rows x 32 k MFMA fragment, ds_read_b128):  row 16t + (lane & 15), chunk 4kk + (lane >> 4)
//   transposed reads (ds_read_b64_tr_b16, rd_tr): rows 16t + 4g + q, columns 16dt + 4p .. (+ 8 B within the chunk)
// A tile index t adds t * 16 * HD * 2 bytes (an immediate): the swizzle depends only on row bits 1..2.
template <int HD>
struct ImgLane {
  int row[HD / 32 > 0 ? HD / 32 : 1];
  int row16;  // the 16-k tail fragment (HD = 80; 8-B reads)
  int tr[HD / 16];
  __device__ __forceinline__ explicit ImgLane(int lane) {
    const int g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) row[kk] = i * HD * 2 + (((kk * 4 + g) ^ aswz<HD>(i)) << 4);
    row16 = i * HD * 2 + (HD / 32 * 32 + 4 * g) * 2;
    const int q = i >> 2, p = i & 3, rr = 4 * g + q;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) tr[dt] = rr * HD * 2 + (((dt * 2 + (p >> 1)) ^ aswz<HD>(rr)) << 4) + 8 * (p & 1);
  }
  static constexpr int TILE = 16 * HD * 2;
};

// ---- epilogue: a wave's 16-row x HD output strip, written as whole rows ----
// The O^T / dQ^T / dK^T accumulators hold 4 consecutive columns (16dt + 4g ..) of one row (lane i) per
// register quad, i.e. 8-B pieces of 16 rows per store instruction. Staging the strip through a
// wave-private LDS tile ([16][HD] bf16, rows padded to HD*2 + 16 bytes: the 8-B writes of a 16-lane
// group land on distinct banks) lets every lane store 16 contiguous bytes, each instruction covering
// whole 2*HD-byte rows.
template <int HD>
struct StripOut {
  static constexpr int LD = HD * 2 + 16;  // bytes per staged row
  static constexpr int BYTES = 16 * LD;
  // stage: acc[dt] * s (bf16) at row i, columns 16dt + 4g .. + 3
  __device__ __forceinline__ static void stage(lds_t* buf, const v4f* acc, float s, int lane) {
    const int g = lane >> 4, i = lane & 15;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      v2u u;
      u[0] = pack2bf(acc[dt][0] * s, acc[dt][1] * s);
      u[1] = pack2bf(acc[dt][2] * s, acc[dt][3] * s);
      lds_st(buf + i * LD + (dt * 16 + 4 * g) * 2, u);
    }
  }
  // store rows [0, 16) of the staged strip to dst + r * ld (elements), rows < nrows, columns < hd
  __device__ __forceinline__ static void store(const lds_t* buf, bf16_t* dst, long ld, int nrows, int hd, int lane) {
    constexpr int CPR = HD / 8;              // 16-B chunks per row
    constexpr int ROWS_PER = 64 / CPR;       // rows per wave-instruction
    // HD = 80: 10 chunks a row, 6 rows an instruction; lanes 60..63 idle and the last pass stops at row 16
    constexpr bool EXACT = ROWS_PER * CPR == 64 && 16 % ROWS_PER == 0;
    // the staged 8-B writes and these 16-B reads have different types: keep the compiler from moving
    // the reads above the writes (one wave's LDS operations then execute in order)
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r0 = 0; r0 < 16; r0 += ROWS_PER) {
      const int r = r0 + lane / CPR, ch = lane % CPR;
      const bool in = EXACT || (lane < ROWS_PER * CPR && r < 16);
      const v4u v = lds_ld<v4u>(buf + (in ? r : 0) * LD + ch * 16);
      if (in && r < nrows && ch * 8 < hd) *reinterpret_cast<v4u*>(dst + (long)r * ld + ch * 8) = v;
    }
  }
};

}  // namespace vit_attn
