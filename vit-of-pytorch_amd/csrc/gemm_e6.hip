// Instantiation unit: every tile config and operand layout of GEMM epilogue 6 (and its dropout variant 22).
#include "gemm_kernels.h"

template <> hipError_t vitg::launch_layout_x<6>(int cfg, const GemmDev& d, bool ak, bool bk, int batch, int split, hipStream_t s) {
  return launch_layout<6>(cfg, d, ak, bk, batch, split, s);
}
template <> hipError_t vitg::launch_kk_x<22>(int cfg, const GemmDev& d, bool bk, int batch, int split, hipStream_t s) {
  if (!bk) return hipErrorInvalidValue;  // (vit_gemm_bf16 checks: K-contiguous B only)
  return launch_cfg<22, true, true>(cfg, d, batch, split, s);
}
