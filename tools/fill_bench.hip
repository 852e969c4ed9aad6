// Per-CU LDS-DMA fill-rate microbenchmark (diagnostic tool, not product code).
//
// One 512-thread workgroup per CU (160 KiB LDS). Every iteration each of the 8 waves issues P
// buffer_load_dwordx4 ... lds pieces (1 KiB each) into a ring slot, optionally issues R ds_read_b128
// fragment reads of an older slot and M v_mfma_f32_16x16x32_bf16 on register operands, then waits
// for the DMA issued DEPTH iterations ago (counted vmcnt) and joins a raw s_barrier. Reported: bytes
// landed per CU per second and per cycle at the measured clock, for sources that sit in the XCD's
// L2 (every workgroup of an XCD reads one small region), in the Infinity Cache, or stream from HBM.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/fill_bench tools/fill_bench.hip && tools/fill_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))
#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// MODE 0: LDS-DMA pieces; 1: the same bytes by buffer_load_dwordx4 into VGPRs (no LDS); S: 1 KiB stores per
// wave per iteration (buffer_store_dwordx4) into a per-workgroup 2 MiB region of dst
template <int P, int DEPTH, int R, int M, int MODE = 0, int S = 0>
__global__ void __launch_bounds__(512, 1) fill_kernel(const char* __restrict__ src, long region, long wg_stride,
                                                       int iters, float* sink, char* dst = nullptr) {
  constexpr int NW = 8;
  constexpr int SLOT = NW * (P > 0 ? P : 1) * 1024;
  constexpr int NSLOT = (160 * 1024) / SLOT;
  static_assert(NSLOT >= DEPTH + 2, "ring too small");
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const char* base = src + (long)blockIdx.x * wg_stride;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)(region + 4096), 0x00020000);
  v4f acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s a = v8s{1, 2, 3, 4, 5, 6, 7, 8}, b = v8s{8, 7, 6, 5, 4, 3, 2, 1};
  unsigned x = 0;
  int off = 0;
  const int rmask = (int)region - 1;  // region: a power of two
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
      dst ? dst + (long)blockIdx.x * (2L << 20) : const_cast<char*>(src), (short)0, 2 << 20, 0x00020000);
  uint4 keep[P > 0 ? P : 1];
  for (int t = 0; t < iters; ++t) {
    const int slot = t % NSLOT;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int piece = p * NW + wave;
      const int o = (off + piece * 1024) & rmask;
      if constexpr (MODE == 0) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, smem + slot * SLOT + piece * 1024), 16,
                                                 lane * 16 + __builtin_amdgcn_readfirstlane(o), 0, 0, 0);
      } else {
        keep[p] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                rs, lane * 16 + __builtin_amdgcn_readfirstlane(o), 0, 0));
      }
    }
#pragma unroll
    for (int q = 0; q < S; ++q) {
      const int o = ((t * NW * S + q * NW + wave) * 1024) & ((2 << 20) - 1);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, make_uint4(t, q, wave, lane)), rd,
                                             lane * 16 + __builtin_amdgcn_readfirstlane(o), 0, 0);
    }
    off += SLOT;
    if constexpr (R > 0) {
      const int rslot = (t + NSLOT - DEPTH - 1) % NSLOT;  // landed and behind a barrier
#pragma unroll
      for (int r = 0; r < R; ++r) {
        // asm read (hipcc would put vmcnt(0) in front of a C++ LDS read while a DMA is in flight)
        const unsigned a_ = (unsigned)(uintptr_t)LDS_PTR(char, smem) + rslot * SLOT +
                            ((r * 1024 + lane * 16 + wave * 4096) & (SLOT - 1));
        v4u v;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a_));
        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        asm volatile("" ::"v"(v));
      }
    }
    if constexpr (M > 0) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        acc[m & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b),
                                                             acc[m & 7], 0, 0, 0);
    }
    if (t >= DEPTH) wait_vm<(P + S) * DEPTH>();
    if constexpr (MODE == 1) {
#pragma unroll
      for (int p = 0; p < P; ++p) asm volatile("" ::"v"(keep[p].x));
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  wait_vm<0>();
  float s = (float)x;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 1234.5f) sink[threadIdx.x] = s;
}

template <int P, int DEPTH, int R, int M, int MODE = 0, int S = 0>
void run(const char* name, const char* src, long region, long wg_stride, int cus, char* dst = nullptr) {
  float* sink;
  CHECK(hipMalloc(&sink, 4096));
  const int iters = 4000 / (P + S);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((fill_kernel<P, DEPTH, R, M, MODE, S>), dim3(cus), dim3(512), 0, 0, src, region, wg_stride,
                       iters / 4, sink, dst);
  CHECK(hipEventRecord(e0));
  const int reps = 5;
  for (int w = 0; w < reps; ++w)
    hipLaunchKernelGGL((fill_kernel<P, DEPTH, R, M, MODE, S>), dim3(cus), dim3(512), 0, 0, src, region, wg_stride,
                       iters, sink, dst);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)reps * iters * 8 * (P + S) * 1024;  // per CU, loaded + stored
  const double us = ms * 1e3;
  const double gbs = bytes / (us * 1e-6) / 1e9;
  const double mfma_cyc = (double)reps * iters * 2 * M * 16;  // per SIMD (2 waves per SIMD)
  printf("%-26s mode=%d P=%d S=%d depth=%d reads=%2d mfma=%2d: %7.1f GB/s per CU (%5.1f B/clk @2.1GHz), %6.2f us/iter, "
         "mfma floor %.2f us/iter\n",
         name, MODE, P, S, DEPTH, R, M, gbs, gbs / 2.1, us / (reps * iters), mfma_cyc / 2.1e3 / (reps * iters));
  CHECK(hipFree(sink));
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const long big = 3L << 30;
  char *src, *dst;
  CHECK(hipMalloc(&src, big));
  CHECK(hipMemset(src, 0x3c, big));
  CHECK(hipMalloc(&dst, (long)cus * (2L << 20)));
  // L2-distinct: workgroup b reads its own 64 KiB (32 x 64 KiB = 2 MiB per XCD under round-robin placement)
  // L2-shared: every workgroup reads the same 1 MiB; MALL: 512 KiB per workgroup; HBM: 12 MiB per workgroup
  struct Src {
    const char* name;
    long region, stride;
  } srcs[4] = {{"L2-distinct (64 KiB/WG)", 64L << 10, 64L << 10}, {"L2-shared (1 MiB)", 1L << 20, 0},
               {"MALL (512 KiB per WG)", 512L << 10, 512L << 10}, {"HBM (8 MiB per WG)", 8L << 20, 8L << 20}};
  for (auto& s : srcs) {
    run<4, 2, 0, 0, 0>(s.name, src, s.region, s.stride, cus);
    run<4, 2, 0, 0, 1>(s.name, src, s.region, s.stride, cus);
    run<4, 2, 0, 32, 0>(s.name, src, s.region, s.stride, cus);
    run<4, 2, 24, 32, 0>(s.name, src, s.region, s.stride, cus);
    run<2, 2, 0, 0, 0>(s.name, src, s.region, s.stride, cus);
  }
  // stores: alone, and beside LDS-DMA fills from L2 / beyond
  run<0, 2, 0, 0, 0, 4>("stores only", src, 64L << 10, 64L << 10, cus, dst);
  run<0, 2, 0, 0, 0, 1>("stores only", src, 64L << 10, 64L << 10, cus, dst);
  run<4, 2, 0, 0, 0, 1>("L2-distinct + stores", src, 64L << 10, 64L << 10, cus, dst);
  run<4, 2, 0, 0, 0, 2>("L2-distinct + stores", src, 64L << 10, 64L << 10, cus, dst);
  run<4, 2, 0, 0, 0, 1>("MALL + stores", src, 512L << 10, 512L << 10, cus, dst);
  CHECK(hipFree(src));
  CHECK(hipFree(dst));
  return 0;
}
