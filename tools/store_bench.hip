// Store-throughput probe for the GEMM epilogue design (not part of the product library).
//   hipcc -O3 --offload-arch=gfx950 tools/store_bench.hip -o tools/store_bench && tools/store_bench
// Every workgroup (512 threads) writes BYTES_PER_WG bytes of 16-B-per-lane dwordx4 stores in one of
// three address patterns, on `wgs` workgroups (one per CU when wgs <= 256):
//   rows128: an instruction covers 8 rows x 128 B (row stride `stride`), like a 64-column bf16 strip
//   rows512: 2 rows x 512 B
//   contig : 1 KiB contiguous
// and prints the kernel time and the per-CU / chip store rate.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// per wave: `instr` store instructions; wave w of workgroup b owns a disjoint region
template <int PAT>
__global__ void __launch_bounds__(512) store_kernel(char* out, long stride, int instr, int waves_storing) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave >= waves_storing) return;
  const v4u val = {(unsigned)lane, (unsigned)wave, (unsigned)blockIdx.x, 7u};
  // region of this (block, wave): `instr` instructions worth of rows
  if (PAT == 0) {  // 8 rows x 128 B per instruction; a wave owns a 128-B-wide column strip
    const long row0 = ((long)blockIdx.x * instr) * 8;
    char* base = out + row0 * stride + wave * 128 + (lane & 7) * 16;
#pragma unroll 8
    for (int i = 0; i < instr; ++i)
      *reinterpret_cast<v4u*>(base + (long)(i * 8 + (lane >> 3)) * stride) = val;
  } else if (PAT == 1) {  // 2 rows x 512 B
    const long row0 = ((long)blockIdx.x * instr) * 2;
    char* base = out + row0 * stride + wave * 512 + (lane & 31) * 16;
#pragma unroll 8
    for (int i = 0; i < instr; ++i)
      *reinterpret_cast<v4u*>(base + (long)(i * 2 + (lane >> 5)) * stride) = val;
  } else {  // 1 KiB contiguous
    char* base = out + (((long)blockIdx.x * 8 + wave) * instr) * 1024 + lane * 16;
#pragma unroll 8
    for (int i = 0; i < instr; ++i) *reinterpret_cast<v4u*>(base + (long)i * 1024) = val;
  }
}

int main() {
  const long stride = 6144;  // fc1 output row (3072 bf16)
  const int instr = 32;      // per wave: 32 KiB; 8 waves: 256 KiB per workgroup (one fc1 tile)
  char* out;
  const size_t cap = (size_t)2 << 30;
  CK(hipMalloc(&out, cap));
  CK(hipMemset(out, 0, cap));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[3] = {"rows128", "rows512", "contig"};
  for (int pat = 0; pat < 3; ++pat)
    for (int wgs : {256, 128, 64, 512, 1024})
      for (int ws : {8, 4}) {
        auto launch = [&]() {
          if (pat == 0) hipLaunchKernelGGL(store_kernel<0>, dim3(wgs), dim3(512), 0, 0, out, stride, instr, ws);
          if (pat == 1) hipLaunchKernelGGL(store_kernel<1>, dim3(wgs), dim3(512), 0, 0, out, stride * 4, instr, ws);
          if (pat == 2) hipLaunchKernelGGL(store_kernel<2>, dim3(wgs), dim3(512), 0, 0, out, stride, instr, ws);
        };
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(e0));
        for (int r = 0; r < it; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / it;
        const double bytes = (double)wgs * ws * instr * 1024;
        printf("%-8s wgs=%4d waves=%d  %8.2f us  %6.2f MB  chip %6.2f TB/s  per-WG %6.1f GB/s\n", names[pat], wgs, ws, us,
               bytes / 1e6, bytes / us / 1e6, bytes / wgs / us / 1e3);
      }
  CK(hipFree(out));
  return 0;
}
