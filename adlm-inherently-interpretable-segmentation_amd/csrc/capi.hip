// capi.hip — library-wide C ABI entry points: version and error reporting.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

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

namespace {
std::mutex g_timer_mu;
std::string g_timer_kernel;
std::string g_timer_last;  // full name of the last kernel the hook bracketed
hipEvent_t g_timer_start = nullptr, g_timer_stop = nullptr;
}  // namespace

namespace {
// Eager launches only: under graph capture the hook stays silent (a plain record there would only
// order streams), so capturing a call with the hook set is harmless.
hipError_t record(hipEvent_t e, hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return hipErrorNotReady;
  return hipEventRecord(e, s);
}
}  // namespace

namespace {
thread_local bool t_span_active = false;
// Exact kernel name, or a family prefix: "l2_fwd" matches l2_fwd_kernel and l2_fwd_bf16_kernel,
// whichever family serves the call. Caller holds g_timer_mu.
bool hook_matches(const char* kernel) {
  if (!g_timer_start) return false;
  const size_t n = g_timer_kernel.size();
  return g_timer_kernel == kernel || (std::strncmp(kernel, g_timer_kernel.c_str(), n) == 0 && kernel[n] == '_');
}
}  // namespace

KernelSpan::KernelSpan(const char* kernel_a, const char* kernel_b, hipStream_t s) {
  std::lock_guard<std::mutex> lock(g_timer_mu);
  if (t_span_active || !(hook_matches(kernel_a) || hook_matches(kernel_b))) return;
  if (record(g_timer_start, s) == hipSuccess) {
    t_span_active = true;
    stop_ = g_timer_stop;
    s_ = s;
  }
}

KernelSpan::~KernelSpan() {
  if (!stop_) return;
  (void)record(stop_, s_);
  t_span_active = false;
}

KernelTimer::KernelTimer(const char* kernel, hipStream_t s) {
  std::lock_guard<std::mutex> lock(g_timer_mu);
  if (!hook_matches(kernel)) return;
  if (t_span_active) {  // inside a matching span: name the kernel, leave the events to the span
    g_timer_last = kernel;
    return;
  }
  if (record(g_timer_start, s) == hipSuccess) {
    g_timer_last = kernel;
    stop_ = g_timer_stop;
    s_ = s;
  }
}

KernelTimer::~KernelTimer() {
  if (stop_) (void)record(stop_, s_);
}

}  // namespace protoseg

extern "C" const char* protoseg_timing_kernel(void) {
  std::lock_guard<std::mutex> lock(protoseg::g_timer_mu);
  return protoseg::g_timer_last.c_str();
}

extern "C" int protoseg_timing_events(const char* kernel, void* start_event, void* stop_event) {
  std::lock_guard<std::mutex> lock(protoseg::g_timer_mu);
  if (!kernel || !start_event || !stop_event) {
    protoseg::g_timer_kernel.clear();
    protoseg::g_timer_start = protoseg::g_timer_stop = nullptr;
    return PROTOSEG_OK;
  }
  protoseg::g_timer_kernel = kernel;
  protoseg::g_timer_start = static_cast<hipEvent_t>(start_event);
  protoseg::g_timer_stop = static_cast<hipEvent_t>(stop_event);
  return PROTOSEG_OK;
}

extern "C" int protoseg_version(void) { return 1 * 10000 + 0 * 100 + 0; }

extern "C" const char* protoseg_last_error(void) { return protoseg::g_last_error; }

