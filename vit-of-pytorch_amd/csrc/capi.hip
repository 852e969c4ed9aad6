// C-ABI plumbing: thread-local error strings and HIP status translation.
#include <stdarg.h>

#include "common.h"
// VIT_BUILD_ID: the source fingerprint the Makefile generates (vitmi/buildid.py)
#include "build_id.h"

namespace vit {
static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

int check_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return VIT_OK;
  set_error("%s: %s", what, hipGetErrorString(e));
  return VIT_ERR_HIP;
}
}  // namespace vit

extern "C" const char* vit_last_error(void) { return vit::g_last_error; }
extern "C" int vit_abi_version(void) { return 18; }
extern "C" const char* vit_build_id(void) { return VIT_BUILD_ID; }
