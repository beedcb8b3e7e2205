// Runtime helpers of the C-ABI: version, thread-local last error, device arch query.
#include <hip/hip_runtime.h>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include "common.h"

namespace zs {
static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}
}  // namespace zs

extern "C" int zs_version(void) { return 1; }

extern "C" int zs_last_error(char* buf, size_t len) {
  if (!buf || len == 0) return ZS_ERR_ARG;
  std::snprintf(buf, len, "%s", zs::g_last_error.c_str());
  return (int)zs::g_last_error.size();
}

extern "C" int zs_device_arch(char* buf, size_t len) {
  if (!buf || len == 0) return ZS_ERR_ARG;
  int dev = 0;
  ZS_CHECK_HIP(hipGetDevice(&dev));
  hipDeviceProp_t p;
  ZS_CHECK_HIP(hipGetDeviceProperties(&p, dev));
  std::snprintf(buf, len, "%s", p.gcnArchName);
  return 0;
}
