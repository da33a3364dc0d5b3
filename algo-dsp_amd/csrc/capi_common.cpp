// C-ABI plumbing shared by every module: last-error string, version, devices.
#include <hip/hip_runtime.h>

#include <atomic>
#include <string>

#include "ad_common.hpp"

namespace adsp {
namespace {
thread_local std::string g_last_error;
std::atomic<int> g_lib_streams{0};
std::atomic<const void*> g_gate_owner{nullptr};
}  // namespace
void set_last_error(const std::string& msg) { g_last_error = msg; }

hipError_t lib_stream_create(hipStream_t* s) {
  const hipError_t e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  if (e == hipSuccess) g_lib_streams.fetch_add(1);
  return e;
}
hipError_t lib_stream_destroy(hipStream_t s) {
  const hipError_t e = hipStreamDestroy(s);
  if (e == hipSuccess) g_lib_streams.fetch_sub(1);
  return e;
}

bool gate_acquire(const void* owner) {
  if (g_lib_streams.load() > kGateMaxStreams) return false;
  const void* cur = nullptr;
  return g_gate_owner.compare_exchange_strong(cur, owner) || cur == owner;
}
void gate_release(const void* owner) {
  const void* cur = owner;
  g_gate_owner.compare_exchange_strong(cur, nullptr);
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
