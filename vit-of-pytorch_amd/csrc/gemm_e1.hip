// Instantiation unit: every tile config and operand layout of GEMM epilogue 1.
#include "gemm_kernels.h"

template <> hipError_t vitg::launch_layout_x<1>(int cfg, const GemmDev& d, bool ak, bool bk, int batch, int split, hipStream_t s) {
  return launch_layout<1>(cfg, d, ak, bk, batch, split, s);
}
