// Instantiation unit: every tile config and operand layout of GEMM epilogue 4 (and its dropout variant 20).
#include "gemm_kernels.h"

template <> hipError_t vitg::launch_layout_x<4>(int cfg, const GemmDev& d, bool ak, bool bk, int batch, int split, hipStream_t s) {
  return launch_layout<4>(cfg, d, ak, bk, batch, split, s);
}
template <> hipError_t vitg::launch_kk_x<20>(int cfg, const GemmDev& d, bool bk, int batch, int split, hipStream_t s) {
  // (the out-projection reads the LinearGeneral weight [in][out] as it is: B M/N-contiguous)
  return bk ? launch_cfg<20, true, true>(cfg, d, batch, split, s) : launch_cfg<20, true, false>(cfg, d, batch, split, s);
}
