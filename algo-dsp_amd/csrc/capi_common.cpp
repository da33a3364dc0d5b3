// C-ABI plumbing shared by every module: last-error string, version, devices.
#include <hip/hip_runtime.h>

#include <string>

#include "ad_common.hpp"

namespace adsp {
namespace {
thread_local std::string g_last_error;
}
void set_last_error(const std::string& msg) { g_last_error = msg; }
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
