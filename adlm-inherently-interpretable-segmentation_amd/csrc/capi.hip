// capi.hip — library-wide C ABI entry points: version and error reporting.
#include <cstdarg>
#include <cstdio>

#include "protoseg_host.h"

namespace protoseg {

namespace {
thread_local char g_last_error[512] = "";
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(PROTOSEG_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
  return PROTOSEG_OK;
}

}  // namespace protoseg

extern "C" int protoseg_version(void) { return 1 * 10000 + 0 * 100 + 0; }

extern "C" const char* protoseg_last_error(void) { return protoseg::g_last_error; }

