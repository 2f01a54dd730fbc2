// capi.hip — library-wide C ABI entry points: version and error reporting.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <string>
#include <vector>

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

int stream_scratch(ScratchKind kind, size_t need, size_t min_bytes, hipStream_t s, void** out) {
  static std::mutex mu;
  static std::map<std::tuple<int, hipStream_t, int>, std::pair<void*, size_t>> blocks;
  static std::vector<void*> retired;  // kept until the process exits (captured graphs may point there)
  int dev = 0;
  *out = nullptr;
  if (hipGetDevice(&dev) != hipSuccess) return check_launch("hipGetDevice");
  std::lock_guard<std::mutex> lock(mu);
  auto& b = blocks[{dev, s, static_cast<int>(kind)}];
  if (b.second < need) {
    // 1.5x geometric growth: a sequence of ever larger calls retires O(log) blocks whose total
    // stays within ~3x the largest, not the sum of every size seen
    size_t bytes = b.second + b.second / 2;
    if (bytes < need) bytes = need;
    if (bytes < min_bytes) bytes = min_bytes;
    bytes = (bytes + 4095) & ~static_cast<size_t>(4095);
    void* p = nullptr;
    const hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return fail(PROTOSEG_ERR_HIP, "hipMalloc (scratch kind %d, %zu B): %s", static_cast<int>(kind), bytes,
                  hipGetErrorString(e));
    }
    if (b.first) retired.push_back(b.first);
    b = {p, bytes};
  }
  *out = b.first;
  return PROTOSEG_OK;
}

namespace {
std::mutex g_timer_mu;
std::string g_timer_kernel;
std::string g_timer_last;  // full name of the last kernel the hook bracketed
hipEvent_t g_timer_start = nullptr, g_timer_stop = nullptr;
// Per-launch mode (protoseg_timing_events_n): launch i of the matching kernel records pair i;
// spans are off, so a chunked call's launches are timed one by one, as rocprofv3 sees them.
std::vector<hipEvent_t> g_starts, g_stops;
int g_launches = 0;
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
  if (!g_timer_start && g_starts.empty()) return false;
  const size_t n = g_timer_kernel.size();
  return g_timer_kernel == kernel || (std::strncmp(kernel, g_timer_kernel.c_str(), n) == 0 && kernel[n] == '_');
}
}  // namespace

KernelSpan::KernelSpan(const char* kernel_a, const char* kernel_b, hipStream_t s) {
  std::lock_guard<std::mutex> lock(g_timer_mu);
  if (t_span_active || !g_starts.empty() || !(hook_matches(kernel_a) || hook_matches(kernel_b))) return;
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
  if (!g_starts.empty()) {  // per-launch mode: the next free pair, silently none past the last
    g_timer_last = kernel;
    const size_t i = static_cast<size_t>(g_launches);
    if (i < g_starts.size() && record(g_starts[i], s) == hipSuccess) {
      ++g_launches;
      stop_ = g_stops[i];
      s_ = s;
    }
    return;
  }
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

extern "C" int protoseg_timing_events_n(const char* kernel, void* const* start_events, void* const* stop_events,
                                        int n) {
  std::lock_guard<std::mutex> lock(protoseg::g_timer_mu);
  protoseg::g_starts.clear();
  protoseg::g_stops.clear();
  protoseg::g_launches = 0;
  protoseg::g_timer_start = protoseg::g_timer_stop = nullptr;
  if (!kernel || !start_events || !stop_events || n <= 0) {
    protoseg::g_timer_kernel.clear();
    return PROTOSEG_OK;
  }
  for (int i = 0; i < n; ++i) {
    if (!start_events[i] || !stop_events[i]) return protoseg::fail(PROTOSEG_ERR_INVALID, "null timing event %d", i);
    protoseg::g_starts.push_back(static_cast<hipEvent_t>(start_events[i]));
    protoseg::g_stops.push_back(static_cast<hipEvent_t>(stop_events[i]));
  }
  protoseg::g_timer_kernel = kernel;
  return PROTOSEG_OK;
}

extern "C" int protoseg_timing_launches(void) {
  std::lock_guard<std::mutex> lock(protoseg::g_timer_mu);
  const int n = protoseg::g_launches;
  protoseg::g_launches = 0;
  return n;
}

extern "C" int protoseg_timing_events(const char* kernel, void* start_event, void* stop_event) {
  std::lock_guard<std::mutex> lock(protoseg::g_timer_mu);
  protoseg::g_starts.clear();
  protoseg::g_stops.clear();
  protoseg::g_launches = 0;
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

