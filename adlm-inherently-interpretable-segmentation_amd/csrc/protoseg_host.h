// protoseg_host.h — host-side helpers for the C ABI launchers (status, errors, LDS opt-in).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <mutex>
#include <type_traits>

#include "protoseg_hip.h"

namespace protoseg {

// Records a formatted message in the thread-local error slot and returns `code`.
int fail(int code, const char* fmt, ...);

// Maps a pending launch error to PROTOSEG_ERR_HIP (with text) or returns PROTOSEG_OK.
int check_launch(const char* what);

// Grow-only device scratch, one block per (device, stream, kind), allocated on first use and
// reused, so a call's launch sequence is kernel launches only (capturable in a HIP graph once the
// block exists). Kernels on one stream are ordered, so a call never overwrites scratch an earlier
// call's kernels still read. A call that needs more takes a new block (1.5x growth, at least
// `min_bytes`) and retires the old one without freeing it: a graph that captured an earlier call
// still points there, and a replay must not touch freed memory.
enum class ScratchKind : int { kImages = 0, kWideF16 = 1, kWideForward = 2, kWidePush = 3, kPush = 4, kPushUpdate = 5 };
int stream_scratch(ScratchKind kind, size_t need, size_t min_bytes, hipStream_t s, void** out);

// gfx950 has 160 KiB of LDS per CU; a kernel opts in once to dynamic LDS above 64 KiB.
constexpr size_t kMaxLds = 160 * 1024;

// One flag per kernel (the template parameter is the kernel itself). `bytes` is the largest
// dynamic LDS the kernel is launched with; static LDS plus `bytes` must fit the 160 KiB.
template <auto kernel, size_t bytes = kMaxLds>
int ensure_lds() {
  static std::once_flag once;
  static hipError_t status = hipSuccess;
  std::call_once(once, [] {
    status = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                 static_cast<int>(bytes));
  });
  if (status != hipSuccess) return fail(PROTOSEG_ERR_HIP, "hipFuncSetAttribute: %s", hipGetErrorString(status));
  return PROTOSEG_OK;
}

inline long long ceil_div(long long a, long long b) { return (a + b - 1) / b; }

// Measurement hook (protoseg_timing_events): when events are registered for `kernel`, its
// launcher records them on the launch stream around that one kernel, so a caller times the
// kernel alone (not the call's prep / reduce launches) with HIP events, the figure rocprofv3
// reports per dispatch. The scope is a no-op for every other kernel and when nothing is set.
class KernelTimer {
 public:
  KernelTimer(const char* kernel, hipStream_t s);
  ~KernelTimer();
  KernelTimer(const KernelTimer&) = delete;
  KernelTimer& operator=(const KernelTimer&) = delete;

 private:
  hipEvent_t stop_ = nullptr;
  hipStream_t s_ = nullptr;
};

// A call that runs a kernel several times (the prototype-chunked backward) brackets the whole
// sequence instead: while a KernelSpan that matched the hook is alive, the KernelTimers inside
// it record nothing, and the span's events cover everything launched in between (conservative:
// the chunks' prep and reduce launches are inside).
class KernelSpan {
 public:
  KernelSpan(const char* kernel_a, const char* kernel_b, hipStream_t s);
  ~KernelSpan();
  KernelSpan(const KernelSpan&) = delete;
  KernelSpan& operator=(const KernelSpan&) = delete;

 private:
  hipEvent_t stop_ = nullptr;
  hipStream_t s_ = nullptr;
};

// Compute units of the current device, queried once per device (launch shapes read it per call).
inline int device_cus() {
  constexpr int kMaxDev = 64;
  static std::atomic<int> cache[kMaxDev] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 256;
  int c = cache[dev].load(std::memory_order_relaxed);
  if (c > 0) return c;
  c = 256;
  if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) c = 256;
  cache[dev].store(c, std::memory_order_relaxed);
  return c;
}

// Workgroups of `kernel` resident on the whole device at (threads, lds): CUs x blocks per CU
// from the occupancy calculator (VGPRs and LDS), at least the CU count. Cached per
// (kernel, threads, lds) of the first call — the launchers use one configuration per shape.
template <auto kernel>
int resident_blocks(int threads, size_t lds) {
  static std::mutex mu;
  static int cached_threads = -1, cached = 0;
  static size_t cached_lds = 0;
  std::lock_guard<std::mutex> lock(mu);
  if (threads == cached_threads && lds == cached_lds) return cached;
  int dev = 0, cus = 256, per_cu = 1;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kernel), threads, lds) !=
          hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  cached_threads = threads;
  cached_lds = lds;
  cached = cus * per_cu;
  return cached;
}

}  // namespace protoseg
