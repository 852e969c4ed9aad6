// Instantiation unit: every tile config and operand layout of GEMM epilogue 8 (and its dropout variant 24).
#include "gemm_kernels.h"

template <> hipError_t vitg::launch_layout_x<8>(int cfg, const GemmDev& d, bool ak, bool bk, int batch, int split, hipStream_t s) {
  return launch_layout<8>(cfg, d, ak, bk, batch, split, s);
}
template <> hipError_t vitg::launch_kk_x<24>(int cfg, const GemmDev& d, bool bk, int batch, int split, hipStream_t s) {
  if (!bk) return hipErrorInvalidValue;  // (vit_gemm_bf16 checks: K-contiguous B only)
  return launch_cfg<24, true, true>(cfg, d, batch, split, s);
}
