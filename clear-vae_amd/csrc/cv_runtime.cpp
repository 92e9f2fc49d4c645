// Host-side runtime pieces of libclearvae_hip.so: thread-local error string and version.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <cxxabi.h>
#include <stdlib.h>
#include <hip/hip_runtime.h>
#include <string>
#include <vector>
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

// ---- launch log: which kernels a call really issued (bench.py checks that the PMC passes it quotes were taken on
// the kernels the timed call runs)
namespace cv {
static thread_local bool t_klog = false;
static thread_local std::vector<const void*> t_klaunch;
void note_launch(const void* kernel) {
  if (t_klog) t_klaunch.push_back(kernel);
}
}  // namespace cv

extern "C" int cv_debug_kernel_log(int on) {
  const int prev = cv::t_klog ? 1 : 0;
  cv::t_klog = on != 0;
  cv::t_klaunch.clear();
  return prev;
}

extern "C" int cv_debug_kernel_names(char* buf, size_t cap) {
  std::string all;
  for (const void* k : cv::t_klaunch) {
    const char* m = hipKernelNameRefByPtr(k, nullptr);
    std::string name = m ? m : "?";
    int st = 0;
    char* d = (m && m[0] == '_' && m[1] == 'Z') ? abi::__cxa_demangle(m, nullptr, nullptr, &st) : nullptr;
    if (d && st == 0) name = d;
    free(d);
    if (!all.empty()) all += '\n';
    all += name;
  }
  if (buf && cap) {
    const size_t n = all.size() < cap - 1 ? all.size() : cap - 1;
    memcpy(buf, all.data(), n);
    buf[n] = 0;
  }
  return (int)cv::t_klaunch.size();
}

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

// ---- step graphs: capture / replay without a framework in between ----
// PyTorch's CUDAGraph.replay() refreshes its RNG generators' seed / offset before every launch (two host-to-
// device copies on the stream, ~5 us each on this runtime); the step graphs use their own device counters, so
// they are captured and launched directly.
extern "C" int cv_graph_begin(cv_stream_t stream) {
  cv::clear_error();
  hipError_t e = hipStreamBeginCapture(reinterpret_cast<hipStream_t>(stream), hipStreamCaptureModeThreadLocal);
  if (e != hipSuccess) {
    cv::set_error("graph_begin: %s", hipGetErrorString(e));
    return 2;
  }
  return 0;
}

extern "C" int cv_graph_end(cv_stream_t stream, void** exec_out) {
  cv::clear_error();
  if (!exec_out) {
    cv::set_error("graph_end: null exec_out");
    return 1;
  }
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(reinterpret_cast<hipStream_t>(stream), &g);
  if (e != hipSuccess) {
    cv::set_error("graph_end: capture: %s", hipGetErrorString(e));
    return 2;
  }
  hipGraphExec_t x = nullptr;
  e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    cv::set_error("graph_end: instantiate: %s", hipGetErrorString(e));
    return 2;
  }
  *exec_out = reinterpret_cast<void*>(x);
  return 0;
}

extern "C" int cv_graph_launch(void* exec, cv_stream_t stream) {
  cv::clear_error();
  hipError_t e = hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(exec), reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) {
    cv::set_error("graph_launch: %s", hipGetErrorString(e));
    return 2;
  }
  return 0;
}

extern "C" int cv_graph_destroy(void* exec) {
  cv::clear_error();
  if (exec) (void)hipGraphExecDestroy(reinterpret_cast<hipGraphExec_t>(exec));
  return 0;
}
