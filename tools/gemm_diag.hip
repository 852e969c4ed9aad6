// Standalone GEMM diagnostic (not part of the product library): times vit_gemm_bf16 on one shape
// and, in the stamped build, prints the per-slot timeline of one ping-pong workgroup.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DVIT_GEMM_STAMPS tools/gemm_diag.hip -o tools/gemm_diag
//   tools/gemm_diag M N K tile [epi] [wg] [a_layout b_layout] [split]
#include "../vit-of-pytorch_amd/csrc/capi.hip"
#include "../vit-of-pytorch_amd/csrc/gemm.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e0.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e1.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e2.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e3.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e4.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e5.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e6.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e7.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e8.hip"
#include "../vit-of-pytorch_amd/csrc/gemm_e9.hip"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void fill_kernel(unsigned short* p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u + seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    const float f = ((x & 0xffffff) / 16777216.0f) * 2.f - 1.f;
    p[i] = (unsigned short)(__float_as_uint(f) >> 16);
  }
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s M N K tile [epi=1] [wg=-1] [a_layout=0] [b_layout=0] [split=1]\n", argv[0]);
    return 2;
  }
  const long M = atol(argv[1]), N = atol(argv[2]), K = atol(argv[3]);
  const int tile = atoi(argv[4]);
  const int epi = argc > 5 ? atoi(argv[5]) : VIT_EPI_BF16;
  const int wg = argc > 6 ? atoi(argv[6]) : -1;
  const int al = argc > 7 ? atoi(argv[7]) : VIT_K_CONTIG, bl = argc > 8 ? atoi(argv[8]) : VIT_K_CONTIG;
  const int split = argc > 9 ? atoi(argv[9]) : 1;
  unsigned short *A, *B, *C, *C2;
  float* bias;
  CK(hipMalloc(&A, M * K * 2));
  CK(hipMalloc(&B, N * K * 2));
  CK(hipMalloc(&C, M * N * 4 * (long)split));
  CK(hipMalloc(&C2, M * N * 2));
  CK(hipMalloc(&bias, N * 4));
  CK(hipMemset(bias, 0, N * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, A, M * K, 1u);
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, B, N * K, 7u);
  vit_gemm_args a;
  memset(&a, 0, sizeof(a));
  a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda = al == VIT_K_CONTIG ? K : M; a.a_layout = al;
  a.B = B; a.ldb = bl == VIT_K_CONTIG ? K : N; a.b_layout = bl;
  a.C = C; a.ldc = N; a.C2 = C2; a.ldc2 = N; a.bias = bias;
  a.batch = 1; a.split_k = split; a.epilogue = epi; a.tile = tile;
  for (int i = 0; i < 5; ++i)
    if (vit_gemm_bf16(&a, 0)) { fprintf(stderr, "gemm: %s\n", vit_last_error()); return 1; }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 20;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) vit_gemm_bf16(&a, 0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / iters;
  printf("M=%ld N=%ld K=%ld tile=%d epi=%d: %.1f us  %.1f TF/s\n", M, N, K, tile, epi, us, 2.0 * M * N * K / us / 1e6);
#ifdef VIT_GEMM_STAMPS
  if (wg >= 0) {
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_wg), &wg, sizeof(int)));
    vit_gemm_bf16(&a, 0);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> st(2 * 1024);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8));
    const unsigned long long t0 = st[0] < st[1024] ? st[0] : st[1024];
    for (int g = 0; g < 2; ++g) {
      printf("group %d stamps (cycles since first):", g);
      for (int k = 0; k < 1024 && st[g * 1024 + k]; ++k) printf(" %llu", st[g * 1024 + k] - t0);
      printf("\n");
    }
  }
#endif
  return 0;
}
