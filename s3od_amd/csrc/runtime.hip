// Error reporting + misc runtime entry points of the C ABI.
#include "common.hpp"
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

static thread_local char g_err[1024] = "";

void s3od_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int s3od_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    s3od_set_error("%s: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

extern "C" {

const char* s3od_last_error(void) { return g_err; }

// ABI version 2 (round 5) changed these signatures against version 1:
//   s3od_colsum         + float* ws, long ws_bytes   (caller-owned partial-sum buffer; new query s3od_colsum_ws)
//   s3od_avgpool        + float* ws                  (per-block partials, deterministic two-pass sum)
//   s3od_linear_wgrad   + float* slab, long slab_bytes (split-K slabs; new query s3od_linear_wgrad_ws)
//   s3od_conv_wgrad     + float* slab, long slab_bytes (split-K slabs; new query s3od_conv_wgrad_ws)
int s3od_abi_version(void) { return 2; }

}  // extern "C"
