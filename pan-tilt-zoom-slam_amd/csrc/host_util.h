// Host-side helpers shared by the C-ABI translation units: thread-local last-error string, HIP
// status checks, and an owning device buffer.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <string>
#include <vector>

namespace ptzba {

inline thread_local std::string g_err;

inline int fail(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return -1;
}

#define HIPCHK(expr)                                                                              \
  do {                                                                                            \
    hipError_t _e = (expr);                                                                       \
    if (_e != hipSuccess) return fail("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
  } while (0)

struct DBuf {
  void* p = nullptr;
  size_t bytes = 0;  // logical size (what the last alloc asked for)
  size_t cap = 0;    // allocated size
  DBuf() = default;
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
  ~DBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = cap = 0;
  }
  // n bytes of device memory, contents undefined; an allocation of at least n bytes is kept (a sliding-window map
  // calls set_problem per keyframe: ~40 hipFree / hipMalloc pairs per call otherwise), a smaller one replaced
  int alloc(size_t n) {
    if (n == 0) n = 16;
    if (p && cap >= n && cap <= 4 * n + (1u << 20)) {  // (a much larger old buffer is returned instead)
      bytes = n;
      return 0;
    }
    release();
    // a buffer below 256 MiB is allocated with a quarter of slack: a sliding window's problem grows by a few
    // percent per keyframe, and an exact fit would be replaced (hipFree + hipMalloc) at nearly every call
    const size_t c = n < ((size_t)256 << 20) ? ((n + n / 4 + 4095) & ~(size_t)4095) : n;
    hipError_t e = hipMalloc(&p, c);
    if (e != hipSuccess) return fail("hipMalloc(%zu) failed: %s", c, hipGetErrorString(e));
    bytes = n;
    cap = c;
    return 0;
  }
  // keep the allocation when it is already large enough (contents are not preserved otherwise)
  int reserve(size_t n) { return n <= cap && p ? 0 : alloc(n + n / 4); }
  template <typename T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// waits for a stream on scope exit (host buffers read by queued async copies must outlive them, also on
// error returns)
struct SyncOnExit {
  hipStream_t s;
  ~SyncOnExit() { (void)hipStreamSynchronize(s); }
};

// Device (hipSetDevice) check shared by the handle constructors.
inline int select_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail("no HIP device available");
  if (device < 0 || device >= n) return fail("device %d out of range (%d devices)", device, n);
  if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice(%d) failed", device);
  return 0;
}

// Per-device work buffers of a stateless entry point (front-end, SIFT), kept across calls (grown, never
// shrunk, deliberately not freed at exit): a stream calls them per frame / per pair.  They are shared by
// every caller on that device, so an entry point holds device_work_lock(device) for as long as it uses
// them (ctypes releases the GIL: two host threads may call the C-ABI at once).  One lock per device
// serialises all such entry points on it; they are synchronous on the null stream anyway.
inline std::mutex& device_work_mutex(int device) {
  static std::mutex mu[64];
  return mu[(unsigned)device % 64u];
}
inline std::unique_lock<std::mutex> device_work_lock(int device) {
  return std::unique_lock<std::mutex>(device_work_mutex(device));
}
// the caller holds device_work_lock(device)
template <typename Work>
Work& work_for(int device) {
  static std::mutex vec_mu;
  static std::vector<Work*> w;
  std::lock_guard<std::mutex> g(vec_mu);
  if ((int)w.size() <= device) w.resize(device + 1, nullptr);
  if (!w[device]) w[device] = new Work;
  return *w[device];
}

}  // namespace ptzba
