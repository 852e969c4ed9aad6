// Instantiation unit: every tile config and operand layout of GEMM epilogue 7.
#include "gemm_kernels.h"

template <> hipError_t vitg::launch_layout_x<7>(int cfg, const GemmDev& d, bool ak, bool bk, int batch, int split, hipStream_t s) {
  return launch_layout<7>(cfg, d, ak, bk, batch, split, s);
}

hipError_t vitg::launch_splitk_group(const GemmGroup& g, hipStream_t s) { return launch_pp2_group(g, s); }
