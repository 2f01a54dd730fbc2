// protoseg_host.h — host-side helpers for the C ABI launchers (status, errors, LDS opt-in).
#pragma once
#include <hip/hip_runtime.h>
#include <mutex>
#include <type_traits>

#include "protoseg_hip.h"

namespace protoseg {

// Records a formatted message in the thread-local error slot and returns `code`.
int fail(int code, const char* fmt, ...);

// Maps a pending launch error to PROTOSEG_ERR_HIP (with text) or returns PROTOSEG_OK.
int check_launch(const char* what);

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
