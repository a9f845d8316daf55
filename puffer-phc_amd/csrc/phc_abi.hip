// phc_abi.hip — error reporting and version of the C ABI (include/phc.h).
#include <cstdarg>

#include "phc_common.h"

namespace phc {

static thread_local std::string g_last_error;

void set_error(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

int check_launch(const char *what) {
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(err));
    return PHC_ELAUNCH;
  }
  return PHC_OK;
}

}  // namespace phc

extern "C" int phc_version(void) { return 1; }

extern "C" const char *phc_last_error(void) { return phc::g_last_error.c_str(); }
