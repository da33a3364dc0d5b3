// Non-uniformly partitioned low-latency convolution engine: the MI355X form
// of conv.PartitionedConvolutionT's streaming mode (dsp/conv/partitioned.go:
// 212-436).
//
// Output contract (as the reference): y[t] = (h * x)[t - lambda], lambda =
// 2^minOrder, for any call length.  The taps are split into stages of
// doubling partition size p_s = lambda, 2 lambda, ..., p_max, each over its
// own tap segment [T_s, T_s + n_s p_s).  Stage s runs once per p_s input
// samples and its block output lands at output times offset by T_s;
// T_s + lambda >= p_s makes every contribution arrive before it is emitted.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <climits>
#include <cstdint>
#include <memory>
#include <vector>

#include "ad_common.hpp"
#include "upols_engine.hpp"

namespace adsp {

// Device-resident engine: `channels` copies of
// PartitionedConvolution sharing one IR (the batched effect-chain runtime's
// reverb-conv node, one instance per graph copy; ad_conv_pc_multi_*).  Every
// stage is ONE zero-latency UPOLS engine over all channels (one launch per
// engine kernel per stage per call, whatever the channel count), its K3 adds
// straight into a device accumulator [C][acap] at the stage's tap offset T_s,
// and an emit kernel reads y[t - lambda] (optionally mixed dry/wet as
// ConvolutionReverb.ProcessInPlace does).  Input and accumulator are linear
// device buffers compacted in place of a ring, so each stage reads its blocks
// and writes its outputs as contiguous runs.  All work is enqueued on the
// caller's stream; nothing synchronises the host.
class NupolsDev {
 public:
  NupolsDev(int device, const double* h, int64_t K, int64_t lambda, int64_t p_max, int channels, hipStream_t s);
  // out[c][0..n) = (h * x_c)[t - lambda] (mix: dry*in + wet*that) for the next
  // n samples of every channel; in == out (in place) allowed.
  void process(const double* d_in, int64_t in_stride, double* d_out, int64_t out_stride, int64_t n, bool mix,
               double wet, double dry, hipStream_t s);
  // Host buffers in[C][n] -> out[C][n] through mapped pinned memory; blocks
  // until out is written.  Emits before this call's stage work when the
  // accumulator is already complete for the emitted range (see .cpp).
  void process_host(const double* in, double* out, int64_t n, bool mix, double wet, double dry, hipStream_t s);
  void reset(hipStream_t s);
  int channels() const { return C_; }
  // host calls that took a pre-enqueued emit / whose pre-enqueued emit timed out
  void lowlat_stats(int64_t* hits, int64_t* timeouts) const {
    if (hits) *hits = ghits_;
    if (timeouts) *timeouts = gtimeouts_;
  }
  ~NupolsDev();

 private:
  int64_t complete_upto() const;  // accumulator complete for times below this
  void append(const double* d_in, int64_t in_stride, int64_t n, bool mapped_src, hipStream_t s);
  void run_stages(int64_t emit_hi, hipStream_t s);
  void emit(const double* d_in, int64_t in_stride, double* d_out, int64_t out_stride, int64_t n, bool mix,
            double wet, double dry, hipStream_t s);
  void ensure_mapped(int64_t n);
  double* in_h_[2] = {nullptr, nullptr};
  double* in_d_[2] = {nullptr, nullptr};
  double *out_h_ = nullptr, *out_d_ = nullptr;
  int64_t map_cap_ = 0;
  int in_slot_ = 0;
  bool in_used_[2] = {false, false};
  hipEvent_t ev_emit_ = nullptr;
  hipEvent_t ev_in_[2] = {nullptr, nullptr};
  // Pre-enqueued emit of the next host call (one channel, n <= 256, calls
  // back to back): k_pc_emit_gated waits in the stream for the go word, so
  // the launch leaves the next call's critical path.  ctl: coherent mapped
  // host memory {go, k1_state, done}, a line each.
  struct GateCtl {
    uint64_t go, pad0[15];
    uint64_t state, pad1[15];
    uint64_t done, pad2[15];
  };
  GateCtl* gctl_ = nullptr;
  GateCtl* gctl_dev_ = nullptr;
  uint64_t gseq_ = 0, gtimeout_ = 0;
  struct Pending {
    bool on = false;
    uint64_t seq = 0;
    int64_t n = 0;
    int slot = 0;
    bool mix = false;
    double wet = 0, dry = 0;
  } gp_;
  double gap_ms_ = 0;
  int gmiss_ = 0;
  uint64_t gkhz_ = 100000;               // the device's real-time counter, ticks per ms
  int64_t ghits_ = 0, gtimeouts_ = 0;    // pre-enqueued emits taken / timed out (lowlat_stats)
  std::chrono::steady_clock::time_point glast_{};
  void gate_arm(int64_t n, bool mix, double wet, double dry, hipStream_t s);
  void gate_cancel(hipStream_t s);

  struct Stage {
    int64_t p = 0, T = 0, taps = 0;
    bool fused = false;        // two partitions, p <= 1024: k_pc_small (stateless per block)
    std::unique_ptr<Upols> eng;  // otherwise: a zero-latency UPOLS engine over all channels
    std::unique_ptr<DevBuf<double2>> H;  // fused: [2][2p] partition spectra
    int64_t done = 0;          // input samples consumed
  };
  DevBuf<double2> tw2048_;     // W_2048^m, m < 2048 (fused stages)
  int C_;
  int64_t lambda_;
  std::vector<Stage> st_;
  DevBuf<double> xin_[2];  // [C][xcap], ping-pong for compaction
  int xcur_ = 0;
  int64_t xcap_ = 0, xin_base_ = 0;
  DevBuf<double> acc_[2];  // [C][acap], ping-pong for compaction
  int acur_ = 0;
  int64_t acap_ = 0, acc_base_ = 0;
  int64_t received_ = 0, emitted_ = 0;
  int64_t acc_hi_ = 0;  // highest accumulator time written + 1 (columns beyond are zero)
  void ensure_xin(int64_t need_hi, hipStream_t s);
  void ensure_acc(int64_t lo_keep, int64_t need_hi, hipStream_t s);
};

}  // namespace adsp
