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

int s3od_abi_version(void) { return 2; }   // 2: s3od_colsum takes a partial-sum workspace (+ s3od_colsum_ws)

}  // extern "C"
