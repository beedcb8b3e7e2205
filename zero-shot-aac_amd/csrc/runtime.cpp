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

// A dedicated non-blocking stream, bound to its hardware queue now: ROCclr gives a stream its
// hardware queue (round-robin over GPU_MAX_HW_QUEUES) at its first dispatch, so streams that
// stay idle while other code creates and uses streams can end up sharing one queue — and two
// streams on one queue run strictly one after the other.  One 4-byte fill + sync right after
// creation makes streams created back to back take consecutive queues.
// priority < 0: the device's highest stream priority, > 0: its lowest, 0: the default (the caption
// runner puts the pipelines' begins and decode grids above the encoder that runs ahead).
extern "C" int zs_stream_create(void** stream, int priority) {
  if (!stream) return ZS_ERR_ARG;
  static int* scratch = nullptr;
  if (!scratch) ZS_CHECK_HIP(hipMalloc(&scratch, 256));
  hipStream_t s = nullptr;
  if (priority == 0) {
    ZS_CHECK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  } else {
    int least = 0, greatest = 0;
    ZS_CHECK_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    ZS_CHECK_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority < 0 ? greatest : least));
  }
  ZS_CHECK_HIP(hipMemsetAsync(scratch, 0, 4, s));
  ZS_CHECK_HIP(hipStreamSynchronize(s));
  *stream = (void*)s;
  return 0;
}

extern "C" int zs_stream_create_masked(void** stream, const unsigned* cu_mask, int mask_words) {
  if (!stream || !cu_mask || mask_words <= 0 || mask_words > 64) return ZS_ERR_ARG;
  static int* scratch = nullptr;
  if (!scratch) ZS_CHECK_HIP(hipMalloc(&scratch, 256));
  hipStream_t s = nullptr;
  ZS_CHECK_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, cu_mask));
  ZS_CHECK_HIP(hipMemsetAsync(scratch, 0, 4, s));
  ZS_CHECK_HIP(hipStreamSynchronize(s));
  *stream = (void*)s;
  return 0;
}

extern "C" int zs_stream_destroy(void* stream) {
  if (!stream) return ZS_ERR_ARG;
  ZS_CHECK_HIP(hipStreamDestroy((hipStream_t)stream));
  return 0;
}
