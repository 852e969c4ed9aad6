// Instantiation unit: every tile config and operand layout of GEMM epilogue 9.
#include "gemm_kernels.h"

template <> hipError_t vitg::launch_layout_x<9>(int cfg, const GemmDev& d, bool ak, bool bk, int batch, int split, hipStream_t s) {
  return launch_layout<9>(cfg, d, ak, bk, batch, split, s);
}
