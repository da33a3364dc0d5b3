// Shared host-side plumbing for the algo-dsp MI355X engine: status codes that
// mirror the reference's sentinel errors, a thread-local last-error string,
// and HIP error propagation that never throws across the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/algodsp.h"

namespace adsp {

void set_last_error(const std::string& msg);

// Internal exception carrying an AD_* status; caught at the C-ABI boundary.
struct Status {
  int code;
  std::string msg;
};

#define AD_HIP(expr)                                                                          \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) {                                                                   \
      throw ::adsp::Status{AD_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)}; \
    }                                                                                         \
  } while (0)

#define AD_FAIL(code, msg) throw ::adsp::Status{(code), (msg)}

inline int64_t next_pow2(int64_t n) {
  // conv.go:250-261 nextPowerOf2
  if (n <= 1) return 1;
  int64_t p = 1;
  while (p < n) p <<= 1;
  return p;
}
inline bool is_pow2(int64_t n) { return n > 0 && (n & (n - 1)) == 0; }  // conv.go:264-266

// Runs fn, translating Status / std::exception into a return code + last error.
template <class Fn>
int guard(Fn&& fn) {
  try {
    fn();
    return AD_OK;
  } catch (const Status& s) {
    set_last_error(s.msg);
    return s.code;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return AD_ERR_INTERNAL;
  } catch (...) {
    set_last_error("unknown error");
    return AD_ERR_INTERNAL;
  }
}

// RAII device buffer.
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  void alloc(size_t count) {
    if (count == n && p) return;
    release();
    if (count == 0) return;
    AD_HIP(hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)));
    n = count;
  }
  // grow-only allocation (keeps the pointer if large enough)
  void reserve(size_t count) {
    if (count <= n && p) return;
    alloc(count);
  }
};

// Library-owned streams (non-blocking), counted process-wide for gate_acquire.
hipError_t lib_stream_create(hipStream_t* s);
hipError_t lib_stream_destroy(hipStream_t s);

// Pre-enqueued launches that wait in their stream for a host go word (the
// streaming chains' gated K1, the partitioned engine's gated emit) hold up
// every later launch that shares their hardware queue.  HIP maps streams onto
// GPU_MAX_HW_QUEUES hardware queues (4 on the MI355X boxes): with more
// streams than that, streams share queues.  So a handle arms such a launch
// only while no other handle has one armed (gate_acquire takes the one
// process-wide slot for `owner`; true if owner already holds it) and while
// the library owns at most kGateMaxStreams streams on the device of `s`, the
// stream the armed launch goes to (one queue left for the caller's; other
// devices' streams take other queues and do not count); gate_release(owner) frees the slot (no-op for another owner).
// Streams the library does not own (the caller's, torch's) take queues too, so
// the stream count alone cannot keep another handle's work off the armed
// launch's queue: gate_preempt(me), called by a low-latency or streaming call
// before it enqueues anything, aborts another owner's armed launch at once
// (kGateAbort into its go word, `abort_word` of gate_acquire).  The launch
// exits as skipped, and its owner's next call takes the path it takes after a
// timeout (rolls the block back, ordinary launches).
constexpr int kGateMaxStreams = 3;
bool gate_acquire(const void* owner, uint64_t* abort_word, hipStream_t s);
void gate_release(const void* owner);
void gate_preempt(const void* me);

// Validates a device index (no CPU fallback: no device is an error).
inline int pick_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) AD_FAIL(AD_ERR_NO_DEVICE, "no HIP device available");
  if (device < 0 || device >= n) AD_FAIL(AD_ERR_NO_DEVICE, "device index out of range");
  return device;
}

// Selects the device for the lifetime of a scope and restores the previous one.
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    AD_HIP(hipGetDevice(&prev));
    if (prev != dev) AD_HIP(hipSetDevice(dev));
  }
  ~DeviceScope() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev && prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace adsp
