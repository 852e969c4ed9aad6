// Can a GEMM main loop absorb its epilogue's stores? (diagnostic tool, not product code)
//
// One 512-thread workgroup per CU (160 KiB LDS ring), 8 waves, two per SIMD. One iteration models half a 256 x 256 x
// 64 k-tile of the ping-pong GEMM: each wave issues P LDS-DMA pieces (buffer_load_dwordx4 ... lds, 1 KiB; P = 4 is
// half the tile's 64 KiB per CU), S global stores of 1 KiB (buffer_store_dwordx4) AFTER its DMA, R ds_read_b128
// fragment reads of a landed slot, M v_mfma_f32_16x16x32_bf16 (M = 32 per wave = 64 per SIMD = half a k-tile),
// then waits for the DMA issued DEPTH iterations earlier with a counted vmcnt that leaves every younger DMA and
// store in flight (vmcnt retires in issue order: a store issued after iteration u's DMA only has to complete by
// the wait for iteration u + 1's DMA, DEPTH - 1 iterations later), and joins an s_barrier.
// S = 0 is the main loop alone; fc1's epilogue writes 256 KiB per tile over 24 half k-tiles, i.e. S ~ 1.33 per wave
// and iteration, a bf16 output ~0.67. Reported: us per iteration and the MFMA floor at the measured clock is not known, so
// compare rows of one run.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/overlap_bench tools/overlap_bench.hip && tools/overlap_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))
#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// SEVERY: the S stores are issued every SEVERY-th iteration (S * SEVERY pieces per wave ... rate S / SEVERY)
template <int P, int S, int SEVERY, int R, int M, int DEPTH>
__global__ void __launch_bounds__(512, 1) overlap_kernel(const char* __restrict__ src, long region, long wg_stride,
                                                          int iters, float* sink, char* dst) {
  constexpr int NW = 8;
  constexpr int SLOT = NW * P * 1024;
  constexpr int NSLOT = (160 * 1024) / SLOT;
  static_assert(NSLOT >= DEPTH + 1, "ring too small");
  static_assert((P + S) * DEPTH + S < 64, "vmcnt is 6 bits");
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * SLOT];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const char* base = src + (long)blockIdx.x * wg_stride;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)(region + 4096), 0x00020000);
  const __amdgpu_buffer_rsrc_t rd =
      __builtin_amdgcn_make_buffer_rsrc(dst + (long)blockIdx.x * (4L << 20), (short)0, 4 << 20, 0x00020000);
  v4f acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s a = v8s{1, 2, 3, 4, 5, 6, 7, 8}, b = v8s{8, 7, 6, 5, 4, 3, 2, 1};
  int off = 0, soff = 0;
  const int rmask = (int)region - 1;  // region: a power of two
  for (int t = 0; t < iters; ++t) {
    const int slot = t % NSLOT;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int piece = p * NW + wave;
      const int o = (off + piece * 1024) & rmask;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(void, smem + slot * SLOT + piece * 1024), 16,
                                               lane * 16 + __builtin_amdgcn_readfirstlane(o), 0, 0, 0);
    }
    off += SLOT;
    const bool st = S > 0 && (t % SEVERY) == 0;
#pragma unroll
    for (int q = 0; q < S; ++q) {
      // a store every SEVERY-th iteration; otherwise an out-of-range (dropped) store keeps the vmcnt count static
      const int o = st ? ((soff + (q * NW + wave) * 1024) & ((4 << 20) - 1)) : (8 << 20);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, make_uint4(t, q, wave, lane)), rd,
                                             lane * 16 + __builtin_amdgcn_readfirstlane(o), 0, 0);
    }
    if (st) soff += S * NW * 1024;
    if constexpr (R > 0) {
      const int rslot = (t + NSLOT - DEPTH) % NSLOT;  // landed and behind a barrier
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const unsigned a_ = (unsigned)(uintptr_t)LDS_PTR(char, smem) + rslot * SLOT +
                            ((r * 1024 + lane * 16 + wave * 4096) & (SLOT - 1));
        v4u v;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a_));
        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        asm volatile("" ::"v"(v));
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m)
      acc[m & 7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(v8bf, a), __builtin_bit_cast(v8bf, b),
                                                           acc[m & 7], 0, 0, 0);
    // the DMA of iteration t - DEPTH + 1 landed: younger ones are its own S stores and DEPTH - 1 whole iterations
    if (t >= DEPTH - 1) wait_vm<S + (P + S) * (DEPTH - 1)>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  wait_vm<0>();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 1234.5f) sink[threadIdx.x] = s;
}

template <int P, int S, int SEVERY, int R, int M, int DEPTH>
void run(const char* name, const char* src, long region, long wg_stride, int cus, char* dst) {
  float* sink;
  CHECK(hipMalloc(&sink, 4096));
  const int iters = 600;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w)
    hipLaunchKernelGGL((overlap_kernel<P, S, SEVERY, R, M, DEPTH>), dim3(cus), dim3(512), 0, 0, src, region, wg_stride,
                       iters / 4, sink, dst);
  CHECK(hipEventRecord(e0));
  const int reps = 5;
  for (int w = 0; w < reps; ++w)
    hipLaunchKernelGGL((overlap_kernel<P, S, SEVERY, R, M, DEPTH>), dim3(cus), dim3(512), 0, 0, src, region, wg_stride,
                       iters, sink, dst);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / (reps * iters);
  const double st_gbs = (double)S * 8 * 1024 / SEVERY / (us * 1e-6) / 1e9;
  printf("%-24s P=%d S=%d/%d R=%2d M=%2d depth=%d: %6.3f us/iter  (stores %5.1f GB/s per CU, %5.2f TB/s chip)\n", name, P,
         S, SEVERY, R, M, DEPTH, us, st_gbs, st_gbs * cus / 1e3);
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
  CHECK(hipMalloc(&dst, (long)cus * (4L << 20)));
  struct Src {
    const char* name;
    long region, stride;
  } srcs[2] = {{"L2-shared (1 MiB)", 1L << 20, 0}, {"MALL (512 KiB per WG)", 512L << 10, 512L << 10}};
  for (int rep = 0; rep < 2; ++rep)
    for (auto& s : srcs) {
      run<4, 0, 1, 12, 32, 3>(s.name, src, s.region, s.stride, cus, dst);  // main loop alone
      run<4, 1, 2, 12, 32, 3>(s.name, src, s.region, s.stride, cus, dst);  // ~ a bf16 output's rate
      run<4, 1, 1, 12, 32, 3>(s.name, src, s.region, s.stride, cus, dst);  // ~ 0.75 x fc1's two outputs
      run<4, 3, 2, 12, 32, 3>(s.name, src, s.region, s.stride, cus, dst);  // ~ 1.1 x fc1's rate, pairs of iterations
      run<4, 2, 1, 12, 32, 3>(s.name, src, s.region, s.stride, cus, dst);  // 1.5 x fc1's rate
      run<4, 1, 1, 12, 0, 3>(s.name, src, s.region, s.stride, cus, dst);   // no MFMA: the memory side alone
      run<4, 0, 1, 12, 0, 3>(s.name, src, s.region, s.stride, cus, dst);
    }
  CHECK(hipFree(src));
  CHECK(hipFree(dst));
  return 0;
}
