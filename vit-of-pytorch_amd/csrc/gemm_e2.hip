// Instantiation unit: every tile config and operand layout of GEMM epilogue 2.
#include "gemm_kernels.h"

template <> hipError_t vitg::launch_layout_x<2>(int cfg, const GemmDev& d, bool ak, bool bk, int batch, int split, hipStream_t s) {
  return launch_layout<2>(cfg, d, ak, bk, batch, split, s);
}
