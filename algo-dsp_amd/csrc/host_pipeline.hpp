// Host-buffer I/O for the offline convolution entry points (OverlapSave /
// OverlapAdd Process / ProcessTo on host memory, and the multichannel
// ad_conv_ols_process_multi): the signal crosses PCIe in chunks through
// page-locked double buffers so that three things overlap,
//
//   H2D of chunk i+1  ||  UPOLS segment of chunk i  ||  D2H of chunk i-1,
//
// each on its own HIP stream, ordered by events; the host copies between the
// caller's buffers and the pinned buffers with a small worker pool (one
// memcpy thread cannot keep up with PCIe Gen5).  The segment of chunk i
// computes every output block whose input window [(j-1)L, (j+1)L) is already
// on the device (Upols::run with a block range; the delay line carries from
// one segment to the next), so the result equals one whole-signal call bit
// for bit.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <vector>

#include "ad_common.hpp"
#include "upols_engine.hpp"

namespace adsp {

// Runs fn(i) for i in [0, n) on up to `workers` pool threads plus the caller.
void parallel_for(int64_t n, const std::function<void(int64_t)>& fn, int workers = 8);

// Page-locks a caller's host range for the scope of one call
// (hipHostRegister), so the DMA engines move it directly instead of staging
// pageable memory.  Ranges below `min_bytes` are left alone; `ok` is false
// when the runtime refuses or another call holds an overlapping range (the
// copies then stay pageable).  Registrations are reference-counted process-
// wide, so threads passing the same array share one.  The scope must end
// after every copy touching the range has completed.
struct HostPin {
  std::vector<uintptr_t> held;  // registry entries this scope keeps locked
  bool ok = false;              // the whole range is page-locked
  HostPin(const void* ptr, size_t bytes, size_t min_bytes = size_t(4) << 20);
  ~HostPin();
  HostPin(const HostPin&) = delete;
  HostPin& operator=(const HostPin&) = delete;
};

class HostPipeline {
 public:
  explicit HostPipeline(int device);
  ~HostPipeline();
  HostPipeline(const HostPipeline&) = delete;
  HostPipeline& operator=(const HostPipeline&) = delete;

  // Full linear convolution (out_len <= n + K - 1 samples per channel) of C
  // host channels in[c][0..n) into out[c][0..out_len) through `eng` (C must
  // equal eng.channels()).  Blocks until the output is on the host.
  void offline(Upols& eng, const double* const* in, int C, int64_t n, double* const* out, int64_t out_len,
               hipStream_t s_comp);

  // How host buffers cross PCIe (ad_conv_set_host_io): kAuto registers calls
  // of >= 64 MiB and stages smaller ones; kStage copies through pinned double
  // buffers with `workers` host threads; kRegister page-locks the caller's
  // buffers for the call (falling back to staging if the runtime refuses).
  enum Mode { kAuto = 0, kStage = 1, kRegister = 2 };
  void set_mode(int mode, int workers) {
    mode_ = mode;
    workers_ = workers > 0 ? workers : 8;
  }

  // Bytes of one pinned staging buffer (two for input, two for output).
  static constexpr int64_t kChunkBytes = int64_t(16) << 20;

  // Wall-time split of the last offline() call (ms): page-locking the
  // caller's buffers (hipHostRegister, 0 when staged), the transfers and
  // compute, and unlocking them again (hipHostUnregister).
  double last_register_ms() const { return last_reg_ms_; }
  double last_transfer_ms() const { return last_xfer_ms_; }
  double last_unregister_ms() const { return last_unreg_ms_; }

 private:
  hipStream_t s_in_ = nullptr, s_out_ = nullptr;
  double* pin_in_[2] = {nullptr, nullptr};
  double* pin_out_[2] = {nullptr, nullptr};
  int64_t pin_cap_ = 0;  // doubles per pinned buffer
  hipEvent_t ev_in_[2] = {nullptr, nullptr};    // H2D of slot done (pin_in free, input on device)
  hipEvent_t ev_comp_ = nullptr;                // compute of the latest segment done
  hipEvent_t ev_out_[2] = {nullptr, nullptr};   // D2H of slot done (pin_out filled)
  DevBuf<double> din_, dout_;
  double last_reg_ms_ = 0, last_xfer_ms_ = 0, last_unreg_ms_ = 0;
  int mode_ = kAuto;
  int workers_ = 8;
  void ensure_pinned(int64_t doubles);
  void offline_direct(Upols& eng, const double* const* in, int C, int64_t n, double* const* out, int64_t out_len,
                      hipStream_t s_comp);
};

}  // namespace adsp
