// Prototype (diagnostic tool, not product code): a 4-wave 256 x 256 x 64 bf16 GEMM main loop with one wave per
// SIMD and a 128 x 128 output tile per wave (256 f32 accumulators per lane, in AGPRs), the geometry hipBLASLt
// picks for the B/16 shapes (profiles/r06/blas_geometry.txt: MT256x256x64, MIWT8_8, WG32_8_1). Operands go
// HBM -> VGPR (buffer_load_dwordx4, one k-tile ahead) -> LDS (ds_write_b128, XOR-swizzled image) -> fragments
// (ds_read_b128); one s_barrier per k-tile; the k-tile's two 32-deep MFMA halves each hide one half of the LDS
// traffic (half 0: the next k-tile's image writes, the global loads of the one after, half 1's fragments; half 1:
// the next k-tile's half-0 fragments).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/w4_proto tools/w4_proto.hip && tools/w4_proto
//
// C = A B^T with A [M][K], B [N][K] (both K-contiguous, the NT layout of the data-gradient GEMMs on K-contiguous
// weights), bf16 in, f32 accumulation, bf16 out.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <algorithm>
#include <vector>
#include <type_traits>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned short bf16_t;
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))
#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ unsigned pack2(float a, float b) {
  __bf16 x = (__bf16)a, y = (__bf16)b;
  return (unsigned)__builtin_bit_cast(unsigned short, x) | ((unsigned)__builtin_bit_cast(unsigned short, y) << 16);
}
__device__ __forceinline__ int xcd_major(int lin, int total) {
  const int xcd = lin & 7, q8 = total >> 3, r8 = total & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (lin >> 3);
}

// MFMA with its accumulator tied in place in AGPRs (hipcc otherwise renames the 64 accumulators of a 128 x 128 wave
// tile every k-tile and shuffles them through v_accvgpr moves). The A / B operands are compiler-visible ds_read
// results, so hipcc's waitcnt pass still waits for them; no hazard inside the chain (accumulate: 0 states).
template <int AM>
__device__ __forceinline__ void mfma_acc(v4f& c, const v8s& a, const v8s& b) {
  if constexpr (AM == 1)
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b), c, 0, 0, 0);
}

struct Args {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  int M, N, K, lda, ldb, ldc;
  int tiles_m, tiles_n;
  int ntiles;  // tiles_m * tiles_n
};

// SG: sched_group_barrier interleave in the main loop (0 = compiler's order)
// PERS: 0 = one tile per workgroup (grid = tiles, XCD-major), 1 = persistent: workgroup w takes tiles
// w*per .. (the grid divides the tiles), 2 = persistent strided
template <int SG, int PERS, int AM, int DG = 0, int PA = 1>
__global__ void __launch_bounds__(256, 1) w4_kernel(const Args p) {
  constexpr int BK = 64, STAGE = 64 * 1024;  // A 32 KiB + B 32 KiB per k-tile image
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nk = p.K / BK;

  // staging: thread t moves chunks t + 256 i (i < 8) of each operand image: row (t >> 3) + 32 i, 16-B chunk t & 7
  const int srow = tid >> 3, skc = tid & 7;
  const int ssw = (srow >> 1) & 7;                            // swizzle of rows srow + 32 i (constant over i)
  const uint32_t st_lds = srow * 128 + ((skc ^ ssw) << 4);    // + i * 4096 (+ stage, + 32 KiB for B)
  const uint32_t a_vo = srow * p.lda * 2 + skc * 16, b_vo = srow * p.ldb * 2 + skc * 16;
  // fragment reads: row r0 + (lane & 15), chunk (kk * 4 + (lane >> 4)) ^ s, s = ((lane & 15) >> 1) & 7
  const int fr = lane & 15, fg = lane >> 4, fs = (fr >> 1) & 7;
  const uint32_t fa0 = (wr * 128 + fr) * 128 + (((0 + fg) ^ fs) << 4);
  const uint32_t fa1 = (wr * 128 + fr) * 128 + (((4 + fg) ^ fs) << 4);
  const uint32_t fb0 = 32768 + (wc * 128 + fr) * 128 + (((0 + fg) ^ fs) << 4);
  const uint32_t fb1 = 32768 + (wc * 128 + fr) * 128 + (((4 + fg) ^ fs) << 4);

  const int per = PERS == 1 ? p.ntiles / gridDim.x : 1;
  const int wg = PERS == 0 ? xcd_major(blockIdx.x, gridDim.x) : xcd_major(blockIdx.x, gridDim.x);
  const int nt_mine = PERS == 0 ? 1 : (PERS == 1 ? per : (p.ntiles - wg + (int)gridDim.x - 1) / (int)gridDim.x);

  for (int s = 0; s < nt_mine; ++s) {
    const int tile = PERS == 0 ? wg : (PERS == 1 ? wg * per + s : wg + s * (int)gridDim.x);
    const int tm = tile / p.tiles_n, tn = tile % p.tiles_n;
    const int m0 = tm * 256, n0 = tn * 256;
    const long a_sh = (long)m0 * p.lda * 2, b_sh = (long)n0 * p.ldb * 2;
    const long a_tot = (long)p.M * p.lda * 2, b_tot = (long)p.N * p.ldb * 2;
    const __amdgpu_buffer_rsrc_t rA = mk_rsrc((const char*)p.A + a_sh, (uint32_t)(a_tot - a_sh));
    const __amdgpu_buffer_rsrc_t rB = mk_rsrc((const char*)p.B + b_sh, (uint32_t)(b_tot - b_sh));
    const int a_st = __builtin_amdgcn_readfirstlane(32 * p.lda * 2), b_st = __builtin_amdgcn_readfirstlane(32 * p.ldb * 2);

    v4u st[16];
    v4u sa2[8];  // PA = 2: the second A staging buffer (A of k-tile k lives in buffer k & 1: 0 = st[0..7], 1 = sa2)
    auto gload = [&](int kt) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        st[i] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rA, a_vo, kt * 128 + i * a_st, 0));
#pragma unroll
      for (int i = 0; i < 8; ++i)
        st[8 + i] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rB, b_vo, kt * 128 + i * b_st, 0));
    };
    auto swrite = [&](int stage) {
      char* base = smem + stage * STAGE;
#pragma unroll
      for (int i = 0; i < 8; ++i) *LDS_PTR(v4u, base + st_lds + i * 4096) = st[i];
#pragma unroll
      for (int i = 0; i < 8; ++i) *LDS_PTR(v4u, base + 32768 + st_lds + i * 4096) = st[8 + i];
    };
    v8s a0[8], b0[8], a1[8], b1[8];
    auto fread0 = [&](int stage) {
      const char* base = smem + stage * STAGE;
#pragma unroll
      for (int i = 0; i < 8; ++i) a0[i] = *LDS_PTR(const v8s, base + fa0 + i * 2048);
#pragma unroll
      for (int j = 0; j < 8; ++j) b0[j] = *LDS_PTR(const v8s, base + fb0 + j * 2048);
    };
    auto fread1 = [&](int stage) {
      const char* base = smem + stage * STAGE;
#pragma unroll
      for (int i = 0; i < 8; ++i) a1[i] = *LDS_PTR(const v8s, base + fa1 + i * 2048);
#pragma unroll
      for (int j = 0; j < 8; ++j) b1[j] = *LDS_PTR(const v8s, base + fb1 + j * 2048);
    };
    v4f acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

    if constexpr (AM == 1) asm volatile("s_nop 4" ::: "memory");  // accumulator writes -> first MFMA reading them as C
    // prologue: k-tile 0 into stage 0, k-tile 1 into registers, half-0 fragments of k-tile 0
    if (s > 0) __syncthreads();  // the previous tile's epilogue staging is done with the LDS
    gload(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    swrite(0);
    if constexpr (PA == 2) {  // A1 -> buffer 1, B1, A2 -> buffer 0 (nk >= 4, even: host-checked)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        sa2[i] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rA, a_vo, 128 + i * a_st, 0));
#pragma unroll
      for (int i = 0; i < 8; ++i)
        st[8 + i] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rB, b_vo, 128 + i * b_st, 0));
#pragma unroll
      for (int i = 0; i < 8; ++i)
        st[i] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rA, a_vo, 256 + i * a_st, 0));
    } else {
      if (nk > 1) gload(1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    fread0(0);

    // one k-tile: MORE1 = a k-tile t+1 exists (write its image, read its half-0 fragments), MORE2 = t+2 exists (load it).
    // Each 32-deep half is 16 groups of 4 MFMAs (row i = q / 2, columns 4 (q & 1) ..), every group followed by its
    // share of the memory work, pinned by sched_barrier so hipcc issues the MFMAs first and waits by count.
    // Fragment order R: the order the groups consume them (b0..3, a0, b4..7, a1..7).
    auto rd = [&](auto& av, auto& bv, const char* base, uint32_t fa, uint32_t fb, int r) {
      if (r < 4) bv[r] = *LDS_PTR(const v8s, base + fb + r * 2048);
      else if (r == 4) av[0] = *LDS_PTR(const v8s, base + fa);
      else if (r < 9) bv[r - 1] = *LDS_PTR(const v8s, base + fb + (r - 1) * 2048);
      else av[r - 8] = *LDS_PTR(const v8s, base + fa + (r - 8) * 2048);
    };
    auto step = [&](int t, auto more1_c, auto more2_c, auto more3_c, auto par_c) {
      constexpr bool MORE1 = decltype(more1_c)::value, MORE2 = decltype(more2_c)::value;
      constexpr bool MORE3 = decltype(more3_c)::value;  // PA = 2: A of k-tile t+3 exists
      constexpr int PB = decltype(par_c)::value;         // PA = 2: the A buffer of k-tile t+1 (= (t + 1) & 1)
      const int cur = t & 1, nxt = cur ^ 1;
      const char* bcur = smem + cur * STAGE;
      const char* bnxt = smem + nxt * STAGE;
      char* wnxt = smem + nxt * STAGE;
      // half 0: MFMAs on a0/b0; per group: image chunk q of k-tile t+1, its global load for k-tile t+2, one half-1 fragment
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = q >> 1, j0 = (q & 1) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) mfma_acc<AM>(acc[i][j0 + j], a0[i], b0[j0 + j]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (PA == 2) {
          if constexpr (MORE1 && !(DG & 2)) {
            if (q < 8) *LDS_PTR(v4u, wnxt + st_lds + q * 4096) = PB ? sa2[q] : st[q];
            else *LDS_PTR(v4u, wnxt + 32768 + st_lds + (q - 8) * 4096) = st[q];
          }
          if (q < 8) {
            if constexpr (MORE3 && !(DG & 1)) {
              const v4u v = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rA, a_vo, (t + 3) * 128 + q * a_st, 0));
              if constexpr (PB) sa2[q] = v; else st[q] = v;
            }
          } else {
            if constexpr (MORE2 && !(DG & 1))
              st[q] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rB, b_vo, (t + 2) * 128 + (q - 8) * b_st, 0));
          }
        } else {
          if constexpr (MORE1 && !(DG & 2)) {
            if (q < 8) *LDS_PTR(v4u, wnxt + st_lds + q * 4096) = st[q];
            else *LDS_PTR(v4u, wnxt + 32768 + st_lds + (q - 8) * 4096) = st[q];
          }
          if constexpr (MORE2 && !(DG & 1)) {
            if (q < 8)
              st[q] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rA, a_vo, (t + 2) * 128 + q * a_st, 0));
            else
              st[q] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rB, b_vo, (t + 2) * 128 + (q - 8) * b_st, 0));
          }
        }
        if constexpr (!(DG & 4)) rd(a1, b1, bcur, fa1, fb1, q);
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DG & 8)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // half 1: MFMAs on a1/b1; the half-0 fragments of k-tile t+1, two per group in the first eight groups
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = q >> 1, j0 = (q & 1) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) mfma_acc<AM>(acc[i][j0 + j], a1[i], b1[j0 + j]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (MORE1 && !(DG & 4)) {
          if (q < 8) {
            rd(a0, b0, bnxt, fa0, fb0, 2 * q);
            rd(a0, b0, bnxt, fa0, fb0, 2 * q + 1);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    if constexpr (PA == 2) {
      using P0 = std::integral_constant<int, 0>;
      using P1 = std::integral_constant<int, 1>;
      for (int t = 0; t + 4 < nk; t += 2) {
        step(t, T_{}, T_{}, T_{}, P1{});
        step(t + 1, T_{}, T_{}, T_{}, P0{});
      }
      step(nk - 4, T_{}, T_{}, T_{}, P1{});
      step(nk - 3, T_{}, T_{}, F_{}, P0{});
      step(nk - 2, T_{}, F_{}, F_{}, P1{});
      step(nk - 1, F_{}, F_{}, F_{}, P0{});
    } else {
      using Q0 = std::integral_constant<int, 0>;
      for (int t = 0; t + 2 < nk; ++t) step(t, T_{}, T_{}, F_{}, Q0{});
      if (nk >= 2) step(nk - 2, T_{}, F_{}, F_{}, Q0{});
      step(nk - 1, F_{}, F_{}, F_{}, Q0{});
    }

    if constexpr (AM == 1) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA's D -> epilogue reads
    // epilogue: bf16 C through a wave-private f32 staging image of 32 rows x 128 columns (+4 pad)
    __syncthreads();
    constexpr int LDW = 132;
    float* ws = reinterpret_cast<float*>(smem + wave * (32 * LDW * 4));
    const int g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) ws[(ii * 16 + 4 * g + r) * LDW + j * 16 + c] = acc[pass * 2 + ii][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int e = lane + it * 64, row = e >> 4, ch = e & 15;
        const float* src = ws + row * LDW + ch * 8;
        const v4f x = *reinterpret_cast<const v4f*>(src), y = *reinterpret_cast<const v4f*>(src + 4);
        const int m = m0 + wr * 128 + pass * 32 + row, n = n0 + wc * 128 + ch * 8;
        if (m < p.M && n + 8 <= p.N) {
          uint4 o = make_uint4(pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(y[0], y[1]), pack2(y[2], y[3]));
          *reinterpret_cast<uint4*>(p.C + (long)m * p.ldc + n) = o;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// LDS-DMA variant: operands HBM -> LDS by buffer_load ... lds (two 64 KiB k-tile stages, the DMA of k-tile t+2 issued
// in the second half of k-tile t, once every wave has read its stage), fragments by inline-asm ds_read_b128 (hipcc
// would otherwise put a vmcnt(0) in front of every LDS read while a DMA is in flight) with explicit lgkmcnt waits.
template <int OFF>
__device__ __forceinline__ v8s lds_rd(uint32_t addr) {
  v8s r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int PERS, int DG = 0>
__global__ void __launch_bounds__(256, 1) w4d_kernel(const Args p) {
  constexpr int BK = 64, STAGE = 64 * 1024;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nk = p.K / BK;
  // DMA piece i (< 8) of an operand image: LDS bytes (4 i + wave) KiB, rows 32 i + r, r = (64 wave + lane) / 8
  const int dr = (wave * 64 + lane) >> 3, dpc = lane & 7;
  const int dsw = (dr >> 1) & 7;
  const uint32_t a_lo = dr * p.lda * 2 + ((dpc ^ dsw) << 4), b_lo = dr * p.ldb * 2 + ((dpc ^ dsw) << 4);
  const int fr = lane & 15, fg = lane >> 4, fs = (fr >> 1) & 7;
  const uint32_t sbase = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
  const uint32_t fa0 = sbase + (wr * 128 + fr) * 128 + (((0 + fg) ^ fs) << 4);
  const uint32_t fa1 = sbase + (wr * 128 + fr) * 128 + (((4 + fg) ^ fs) << 4);
  const uint32_t fb0 = sbase + 32768 + (wc * 128 + fr) * 128 + (((0 + fg) ^ fs) << 4);
  const uint32_t fb1 = sbase + 32768 + (wc * 128 + fr) * 128 + (((4 + fg) ^ fs) << 4);

  const int per = PERS == 1 ? p.ntiles / gridDim.x : 1;
  const int wg = xcd_major(blockIdx.x, gridDim.x);
  const int nt_mine = PERS == 0 ? 1 : (PERS == 1 ? per : (p.ntiles - wg + (int)gridDim.x - 1) / (int)gridDim.x);

  for (int s = 0; s < nt_mine; ++s) {
    const int tile = PERS == 0 ? wg : (PERS == 1 ? wg * per + s : wg + s * (int)gridDim.x);
    const int tm = tile / p.tiles_n, tn = tile % p.tiles_n;
    const int m0 = tm * 256, n0 = tn * 256;
    const long a_sh = (long)m0 * p.lda * 2, b_sh = (long)n0 * p.ldb * 2;
    const long a_tot = (long)p.M * p.lda * 2, b_tot = (long)p.N * p.ldb * 2;
    const __amdgpu_buffer_rsrc_t rA = mk_rsrc((const char*)p.A + a_sh, (uint32_t)(a_tot - a_sh));
    const __amdgpu_buffer_rsrc_t rB = mk_rsrc((const char*)p.B + b_sh, (uint32_t)(b_tot - b_sh));
    const int a_st = __builtin_amdgcn_readfirstlane(32 * p.lda * 2), b_st = __builtin_amdgcn_readfirstlane(32 * p.ldb * 2);
    // DMA piece q (< 16: A pieces 0..7, B pieces 8..15) of k-tile kt into stage st
    auto dma = [&](int q, int kt, int st) {
      if (q < 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, LDS_PTR(void, smem + st * STAGE + (q * 4 + wave) * 1024), 16, a_lo,
                                                 __builtin_amdgcn_readfirstlane(kt * 128 + q * a_st), 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, LDS_PTR(void, smem + st * STAGE + 32768 + ((q - 8) * 4 + wave) * 1024),
                                                 16, b_lo, __builtin_amdgcn_readfirstlane(kt * 128 + (q - 8) * b_st), 0, 0);
    };
    v8s a0[8], b0[8], a1[8], b1[8];
    v4f acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_nop 4" ::: "memory");
    if (s > 0) __syncthreads();
    // prologue: k-tiles 0 and 1 into stages 0 and 1; half-0 fragments of k-tile 0
#pragma unroll
    for (int q = 0; q < 16; ++q) dma(q, 0, 0);
    if (nk > 1) {
#pragma unroll
      for (int q = 0; q < 16; ++q) dma(q, 1, 1);
      wait_vm<16>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    // reads in the order the groups consume them: b0..3, a0, b4..7, a1..7 (compile-time offsets)
#define W4_RD(AV, BV, FA, FB, ST, R)                                                          \
  do {                                                                                        \
    if constexpr ((R) < 4) BV[(R)] = lds_rd<(R) * 2048>((FB) + (ST) * STAGE);                 \
    else if constexpr ((R) == 4) AV[0] = lds_rd<0>((FA) + (ST) * STAGE);                      \
    else if constexpr ((R) < 9) BV[(R) - 1] = lds_rd<((R) - 1) * 2048>((FB) + (ST) * STAGE);  \
    else AV[(R) - 8] = lds_rd<((R) - 8) * 2048>((FA) + (ST) * STAGE);                         \
  } while (0)
    auto rd_all0 = [&](auto st_c) {
      constexpr int ST = decltype(st_c)::value;
      W4_RD(a0, b0, fa0, fb0, ST, 0); W4_RD(a0, b0, fa0, fb0, ST, 1); W4_RD(a0, b0, fa0, fb0, ST, 2);
      W4_RD(a0, b0, fa0, fb0, ST, 3); W4_RD(a0, b0, fa0, fb0, ST, 4); W4_RD(a0, b0, fa0, fb0, ST, 5);
      W4_RD(a0, b0, fa0, fb0, ST, 6); W4_RD(a0, b0, fa0, fb0, ST, 7); W4_RD(a0, b0, fa0, fb0, ST, 8);
      W4_RD(a0, b0, fa0, fb0, ST, 9); W4_RD(a0, b0, fa0, fb0, ST, 10); W4_RD(a0, b0, fa0, fb0, ST, 11);
      W4_RD(a0, b0, fa0, fb0, ST, 12); W4_RD(a0, b0, fa0, fb0, ST, 13); W4_RD(a0, b0, fa0, fb0, ST, 14);
      W4_RD(a0, b0, fa0, fb0, ST, 15);
    };
    rd_all0(std::integral_constant<int, 0>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    // k-tile t in stage CUR: half 0 = MFMAs on a0/b0 + the half-1 fragments (two per group, groups 0..7);
    // vmcnt(0) (k-tile t+1 landed) + barrier; half 1 = MFMAs on a1/b1 + the half-0 fragments of k-tile t+1 (stage
    // CUR ^ 1) + the DMA of k-tile t+2 into stage CUR (one piece per group)
    auto step = [&](int t, auto more1_c, auto more2_c) {
      const int CUR = t & 1, NXT = CUR ^ 1;
      constexpr bool MORE1 = decltype(more1_c)::value, MORE2 = decltype(more2_c)::value;
#define W4_GROUP_MF(AV, BV, Q)                                                         \
  do {                                                                                 \
    constexpr int i_ = (Q) >> 1, j0_ = ((Q) & 1) * 4;                                  \
    mfma_acc<1>(acc[i_][j0_ + 0], AV[i_], BV[j0_ + 0]);                                \
    mfma_acc<1>(acc[i_][j0_ + 1], AV[i_], BV[j0_ + 1]);                                \
    mfma_acc<1>(acc[i_][j0_ + 2], AV[i_], BV[j0_ + 2]);                                \
    mfma_acc<1>(acc[i_][j0_ + 3], AV[i_], BV[j0_ + 3]);                                \
  } while (0)
#define W4_H0(Q)                                                                         \
  do {                                                                                   \
    W4_GROUP_MF(a0, b0, Q);                                                              \
    if constexpr ((Q) < 8 && !(DG & 4)) {                                                \
      W4_RD(a1, b1, fa1, fb1, CUR, 2 * (Q));                                             \
      W4_RD(a1, b1, fa1, fb1, CUR, 2 * (Q) + 1);                                         \
    }                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                   \
  } while (0)
#define W4_H1(Q)                                                                         \
  do {                                                                                   \
    W4_GROUP_MF(a1, b1, Q);                                                              \
    if constexpr (MORE1 && (Q) < 8 && !(DG & 4)) {                                       \
      W4_RD(a0, b0, fa0, fb0, NXT, 2 * (Q));                                             \
      W4_RD(a0, b0, fa0, fb0, NXT, 2 * (Q) + 1);                                         \
    }                                                                                    \
    if constexpr (MORE2 && !(DG & 1)) dma((Q), t + 2, CUR);                              \
    __builtin_amdgcn_sched_barrier(0);                                                   \
  } while (0)
      W4_H0(0); W4_H0(1); W4_H0(2); W4_H0(3); W4_H0(4); W4_H0(5); W4_H0(6); W4_H0(7);
      W4_H0(8); W4_H0(9); W4_H0(10); W4_H0(11); W4_H0(12); W4_H0(13); W4_H0(14); W4_H0(15);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (MORE1) wait_vm<0>();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(DG & 8)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      W4_H1(0); W4_H1(1); W4_H1(2); W4_H1(3); W4_H1(4); W4_H1(5); W4_H1(6); W4_H1(7);
      W4_H1(8); W4_H1(9); W4_H1(10); W4_H1(11); W4_H1(12); W4_H1(13); W4_H1(14); W4_H1(15);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    for (int t = 0; t + 2 < nk; ++t) step(t, T_{}, T_{});  // nk >= 2 (K >= 128) checked by the host
    step(nk - 2, T_{}, F_{});
    step(nk - 1, F_{}, F_{});
#undef W4_H0
#undef W4_H1
#undef W4_GROUP_MF
#undef W4_RD
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    __syncthreads();
    constexpr int LDW = 132;
    float* ws = reinterpret_cast<float*>(smem + wave * (32 * LDW * 4));
    const int g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) ws[(ii * 16 + 4 * g + r) * LDW + j * 16 + c] = acc[pass * 2 + ii][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int e = lane + it * 64, row = e >> 4, ch = e & 15;
        const float* src = ws + row * LDW + ch * 8;
        const v4f x = *reinterpret_cast<const v4f*>(src), y = *reinterpret_cast<const v4f*>(src + 4);
        const int m = m0 + wr * 128 + pass * 32 + row, n = n0 + wc * 128 + ch * 8;
        if (m < p.M && n + 8 <= p.N) {
          uint4 o = make_uint4(pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(y[0], y[1]), pack2(y[2], y[3]));
          *reinterpret_cast<uint4*>(p.C + (long)m * p.ldc + n) = o;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// reference: one thread per output, f32 accumulation
__global__ void ref_kernel(const bf16_t* A, const bf16_t* B, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += __uint_as_float((unsigned)A[(long)m * K + k] << 16) * __uint_as_float((unsigned)B[(long)n * K + k] << 16);
  C[(long)m * N + n] = s;
}

static unsigned short f2bf_host(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}
static float bf2f_host(unsigned short b) {
  unsigned u = (unsigned)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

struct Variant {
  const char* name;
  void (*fn)(const Args&, hipStream_t, int);
  int grid;
};

template <int SG, int PERS, int AM = 1, int DG = 0, int PA = 1>
static void launch(const Args& a, hipStream_t s, int grid) {
  hipLaunchKernelGGL((w4_kernel<SG, PERS, AM, DG, PA>), dim3(grid), dim3(256), 0, s, a);
}

template <int PERS, int DG = 0>
static void launchd(const Args& a, hipStream_t s, int grid) {
  hipLaunchKernelGGL((w4d_kernel<PERS, DG>), dim3(grid), dim3(256), 0, s, a);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 50432, N = argc > 2 ? atoi(argv[2]) : 768, K = argc > 3 ? atoi(argv[3]) : 2304;
  const int iters = 20, rounds = 5;
  printf("M=%d N=%d K=%d\n", M, N, K);
  std::vector<unsigned short> hA((size_t)M * K), hB((size_t)N * K);
  uint32_t x = 12345;
  auto rnd = [&]() {
    x = x * 1664525u + 1013904223u;
    return ((x >> 8) & 0xffff) / 32768.0f - 1.0f;
  };
  for (auto& v : hA) v = f2bf_host(rnd());
  for (auto& v : hB) v = f2bf_host(rnd());
  bf16_t *dA, *dB, *dC;
  float* dR;
  CHECK(hipMalloc(&dA, hA.size() * 2));
  CHECK(hipMalloc(&dB, hB.size() * 2));
  CHECK(hipMalloc(&dC, (size_t)M * N * 2));
  CHECK(hipMalloc(&dR, (size_t)M * N * 4));
  CHECK(hipMemcpy(dA, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dB, hB.data(), hB.size() * 2, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, M), dim3(256), 0, 0, dA, dB, dR, M, N, K);
  CHECK(hipDeviceSynchronize());
  std::vector<float> hR((size_t)M * N);
  CHECK(hipMemcpy(hR.data(), dR, hR.size() * 4, hipMemcpyDeviceToHost));

  Args a{dA, dB, dC, M, N, K, K, K, N, (M + 255) / 256, (N + 255) / 256, 0};
  a.ntiles = a.tiles_m * a.tiles_n;
  std::vector<Variant> vs;
  vs.push_back({"w4 one-shot", launch<0, 0>, a.ntiles});
  if (a.ntiles % 3 == 0) vs.push_back({"w4 pers tiles/3 (3 each)", launch<0, 1>, a.ntiles / 3});
  vs.push_back({"w4 pers 256 strided", launch<0, 2>, 256});
  if ((K / 64) % 2 == 0 && K / 64 >= 4) {
    vs.push_back({"w4p A 2-ahead one-shot", launch<0, 0, 1, 0, 2>, a.ntiles});
    if (a.ntiles % 3 == 0) vs.push_back({"w4p A 2-ahead pers /3", launch<0, 1, 1, 0, 2>, a.ntiles / 3});
    vs.push_back({"w4p A 2-ahead pers 256", launch<0, 2, 1, 0, 2>, 256});
  }
  vs.push_back({"w4d dma one-shot", launchd<0>, a.ntiles});
  if (a.ntiles % 3 == 0) vs.push_back({"w4d dma pers tiles/3", launchd<1>, a.ntiles / 3});
  vs.push_back({"w4d dma pers 256 strided", launchd<2>, 256});
  if (getenv("W4_DIAG")) {
    vs.push_back({"w4d diag no dma", launchd<0, 1>, a.ntiles});
    vs.push_back({"w4d diag no dma/reads", launchd<0, 5>, a.ntiles});
    vs.push_back({"w4d diag no reads", launchd<0, 4>, a.ntiles});
    vs.push_back({"diag no gload", launch<0, 0, 1, 1>, a.ntiles});
    vs.push_back({"diag no gload/dswrite", launch<0, 0, 1, 3>, a.ntiles});
    vs.push_back({"diag no gload/dsw/dsread", launch<0, 0, 1, 7>, a.ntiles});
    vs.push_back({"diag mfma only (no barrier)", launch<0, 0, 1, 15>, a.ntiles});
    vs.push_back({"diag no dsread", launch<0, 0, 1, 4>, a.ntiles});
    vs.push_back({"diag no dswrite", launch<0, 0, 1, 2>, a.ntiles});
  }
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> times(vs.size());
  std::vector<unsigned short> hC((size_t)M * N);
  for (size_t v = 0; v < vs.size(); ++v) {
    CHECK(hipMemset(dC, 0, (size_t)M * N * 2));
    vs[v].fn(a, s, vs[v].grid);
    CHECK(hipStreamSynchronize(s));
    CHECK(hipMemcpy(hC.data(), dC, hC.size() * 2, hipMemcpyDeviceToHost));
    double num = 0, den = 0, maxe = 0;
    for (size_t i = 0; i < hC.size(); ++i) {
      const double d = bf2f_host(hC[i]) - hR[i];
      num += d * d;
      den += (double)hR[i] * hR[i];
      maxe = std::max(maxe, fabs(d) / (fabs(hR[i]) + 1.0));
    }
    printf("%-28s rel fro err %.3e  max rel %.3e %s\n", vs[v].name, sqrt(num / den), maxe, sqrt(num / den) < 5e-3 ? "OK" : "BAD");
  }
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      for (int w = 0; w < 3; ++w) vs[v].fn(a, s, vs[v].grid);
      CHECK(hipEventRecord(e0, s));
      for (int it = 0; it < iters; ++it) vs[v].fn(a, s, vs[v].grid);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      times[v].push_back(ms * 1000.f / iters);
    }
  const double flop = 2.0 * M * N * K;
  for (size_t v = 0; v < vs.size(); ++v) {
    std::vector<float> t = times[v];
    std::sort(t.begin(), t.end());
    printf("%-28s grid %5d: median %8.1f us  min %8.1f us  %7.1f TF/s\n", vs[v].name, vs[v].grid, t[t.size() / 2], t[0],
           flop / t[t.size() / 2] / 1e6);
  }
  return 0;
}
