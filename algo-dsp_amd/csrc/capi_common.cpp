// C-ABI plumbing shared by every module: last-error string, version, devices.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>

#include "ad_common.hpp"

namespace adsp {
namespace {
thread_local std::string g_last_error;
// library-owned streams per device: hardware queues are per device, so only
// the armed handle's own device counts (gate_acquire)
constexpr int kMaxDevices = 64;
std::atomic<int> g_lib_streams[kMaxDevices] = {};
int stream_device(hipStream_t s) {
  hipDevice_t d = -1;
  if (hipStreamGetDevice(s, &d) != hipSuccess || d < 0 || d >= kMaxDevices) return -1;
  return (int)d;
}
// the armed-launch slot: its owner and that owner's go word (gate_preempt)
std::mutex g_gate_mu;
const void* g_gate_owner = nullptr;
uint64_t* g_gate_abort = nullptr;
}  // namespace
void set_last_error(const std::string& msg) { g_last_error = msg; }

hipError_t lib_stream_create(hipStream_t* s) {
  const hipError_t e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  if (e == hipSuccess) {
    const int d = stream_device(*s);
    if (d >= 0) g_lib_streams[d].fetch_add(1);
  }
  return e;
}
hipError_t lib_stream_destroy(hipStream_t s) {
  const int d = stream_device(s);
  const hipError_t e = hipStreamDestroy(s);
  if (e == hipSuccess && d >= 0) g_lib_streams[d].fetch_sub(1);
  return e;
}

bool gate_acquire(const void* owner, uint64_t* abort_word, hipStream_t s) {
  const int d = stream_device(s);
  if (d < 0 || g_lib_streams[d].load() > kGateMaxStreams) return false;
  std::lock_guard<std::mutex> lk(g_gate_mu);
  if (g_gate_owner != nullptr && g_gate_owner != owner) return false;
  // a fresh acquisition: the owner has no launch armed, so any value in its go
  // word is stale (an abort that landed after its last launch took the block)
  if (g_gate_owner == nullptr) __atomic_store_n(abort_word, 0ull, __ATOMIC_RELEASE);
  g_gate_owner = owner;
  g_gate_abort = abort_word;
  return true;
}
void gate_release(const void* owner) {
  std::lock_guard<std::mutex> lk(g_gate_mu);
  if (g_gate_owner == owner) {
    g_gate_owner = nullptr;
    g_gate_abort = nullptr;
  }
}
void gate_preempt(const void* me) {
  std::lock_guard<std::mutex> lk(g_gate_mu);
  if (g_gate_owner != nullptr && g_gate_owner != me && g_gate_abort != nullptr) {
    __atomic_store_n(g_gate_abort, ~0ull, __ATOMIC_RELEASE);  // kGateAbort (conv_kernels.hpp)
  }
}
}  // namespace adsp

extern "C" {

const char* ad_last_error(void) { return adsp::g_last_error.c_str(); }

int ad_version(void) { return 1; }

int ad_device_count(int* count) {
  int n = 0;
  const hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  if (count) *count = n;
  return AD_OK;
}

}  // extern "C"
