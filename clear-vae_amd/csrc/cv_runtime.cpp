// Host-side runtime pieces of libclearvae_hip.so: thread-local error string and version.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <hip/hip_runtime.h>
#include "../../include/clearvae.h"

namespace cv {
static thread_local char g_err[1024];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
void clear_error() { g_err[0] = 0; }
}  // namespace cv

extern "C" const char* cv_last_error(void) { return cv::g_err; }
extern "C" int cv_version(void) { return 1; }

extern "C" int cv_zero(void* ptr, size_t bytes, cv_stream_t stream) {
  cv::clear_error();
  if (!ptr) {
    cv::set_error("zero: null pointer");
    return 1;
  }
  hipError_t e = hipMemsetAsync(ptr, 0, bytes, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) {
    cv::set_error("zero: %s", hipGetErrorString(e));
    return 2;
  }
  return 0;
}
