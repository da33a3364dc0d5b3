// Uniformly partitioned overlap-save engine (host runtime around the HIP
// kernels of conv_kernels.hip).  One engine owns the IR spectra of n_ir
// impulse responses, the per-channel frequency-domain delay line (X ring),
// the per-chunk product spectra (Y).  The ring holds one spectrum per input
// block (K1's block spectra), so streaming needs no separate input history.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "ad_common.hpp"
#include "conv_kernels.hpp"

namespace adsp {

// Stereo mixdown fused into the engine's inverse transform (Upols::run):
// mix [2][stride] receives L = the sum of the channels whose global index
// (first_parity + c) is even, R = the odd ones, instead of per-channel outputs.
struct MixOut {
  double* p;
  int64_t stride;
  int first_parity;
};

class Upols {
 public:
  // kernels: host [n_ir][K].  L: hop (power of two, 16..4096).  C: channels.
  // ir_map: host [C] IR index per channel (nullable: c % n_ir).
  // jc_max: blocks per channel per internal chunk.
  Upols(int device, const double* kernels, int n_ir, int64_t K, int L, int C, const int32_t* ir_map, int jc_max,
        hipStream_t stream);
  ~Upols();

  int hop() const { return L_; }
  int partitions() const { return P_; }
  int channels() const { return C_; }
  int64_t kernel_len() const { return K_; }
  hipStream_t stream() const { return stream_; }

  // Streaming state: zero the delay line.
  void reset_stream(hipStream_t s);
  // Steps the block counter back by `blocks`: the next run re-transforms
  // those blocks into the same delay-line slots (a streaming call that ended
  // inside a block; its spectrum was provisional).
  void rewind(int64_t blocks) { g_next_ -= blocks; }
  // The next run() launches its K1 / K2 / K3 as a gated chain (StreamGate,
  // conv_kernels.hpp); applies to that one run only.
  void set_gate(const StreamGate& g) {
    gate_ = g;
    gate_on_ = true;
  }
  // Offline call start: only the delay-line slots preceding block 0 are zeroed.
  void begin_offline(hipStream_t s);

  // Runs ceil(out_len/L) blocks for all channels.  d_in: [C][in_stride],
  // n valid samples.  d_out: [C][out_stride], out_len samples written.
  // use_hist: the call continues the stream (the blocks before it are the
  // previous calls' blocks, already in the ring); offline calls that start a
  // signal call begin_offline first, so the blocks before it read as zeros.
  // [jb, je): the output blocks to run (je < 0: through the end of out_len).
  // Offline segments of one signal run in increasing order (the delay line
  // carries from one segment to the next).
  // accumulate: K3 adds into d_out instead of storing (partitioned stages).
  // mix (hop >= 2048 only): d_out / out_stride are ignored and K3 writes the
  // group's stereo mix (MixOut) with the per-channel outputs never stored.
  void run(const double* d_in, int64_t in_stride, int64_t n, double* d_out, int64_t out_stride, int64_t out_len,
           bool use_hist, hipStream_t s, int64_t jb = 0, int64_t je = -1, bool accumulate = false,
           const MixOut* mix = nullptr);
  bool can_mix() const { return M_ >= 2048; }

  // Offline schedule of the device entry points (ad_conv_multi_set_schedule).
  // SERIAL: each chunk's K1 -> K2 -> K3 on the caller's stream, chunks of up
  // to jc_max blocks.  PIPELINED (hop >= 2048): chunks of `chunk` blocks per
  // channel whose block spectra and Z rows live in small rings that the
  // Infinity Cache holds; K1 runs on the caller's stream, K2 and K3 on two
  // internal streams.  K1 of chunk k+1 overlaps K2 and K3 of chunk k; it does
  // not overlap K3 of chunk k-1, because the caller's stream waits on K3(k-1)
  // before K1(k+1) (the X-ring sizing 2*jc + P + 2*PC + 1 depends on that
  // wait).  The caller's stream waits for the last K3 before the call returns
  // (the ABI's ordering holds).  `run`: K2's run length in blocks (0: auto).
  // Takes effect at the next signal start (begin_offline copies the request):
  // the segments of one signal share a ring sized for the schedule it began with.
  static constexpr int kSchedSerial = 0;
  static constexpr int kSchedPipelined = 1;
  static constexpr int kSchedChunked = 2;  // the pipelined rings and chunks, every kernel on the caller's stream
  void set_schedule(int mode, int chunk, int run);
  int schedule() const { return req_mode_; }
  int pipe_chunk() const { return req_jc_; }
  // the device entry points opt in (the host-buffer pipeline and the
  // partitioned stages call run() with their own streams and stay serial)
  void set_pipeline_call(bool on) { pipe_call_ = on; }
  // Kept for API symmetry: the ring already holds the last block's spectrum
  // (checks that a streaming call covers at least one hop).
  void save_history(const double* d_in, int64_t in_stride, int64_t n, hipStream_t s);

  // Live kernel timing with HIP events on the launch stream (kernel k:
  // 0 window rFFT, 1 FDL MAC, 2 inverse rFFT + store).  read_profile
  // synchronises, accumulates and clears the recorded launches.
  static constexpr int kKernels = 3;
  void set_profiling(bool on);
  void set_profile_mask(int mask) { prof_mask_ = mask; }
  void read_profile(double* ms, int64_t* launches, double* alg_bytes);

 private:
  int64_t K_;
  int L_, M_, MS_, P_, PC_, NH_, C_, n_ir_, jc_max_, Q_, R_;
  int64_t g_next_ = 0;  // logical index of the next spectrum block
  StreamGate gate_{};
  bool gate_on_ = false;
  hipStream_t stream_;
  DevBuf<double2> tw_;   // [twM (M) | twN (M)]
  DevBuf<double2> H_;    // [n_ir][P][MS]
  DevBuf<double2> X_;    // [C][Q][MS]
  DevBuf<double2> Y_;    // [C][jc_max][MS]
  DevBuf<int> irmap_;    // [C]

  // One chunk of output blocks and the buffers its kernels use.
  struct Chunk {
    int64_t cs;     // first output block (call-relative)
    int jc;         // output blocks per channel
    int jin;        // K1 items per channel (blocks holding input)
    int64_t g0;     // logical block of chunk block 0
    int64_t gend;   // last logical block holding input
  };
  struct Rings {
    double2* X;     // block-spectrum ring [C][Q+1][MS] (row Q: zeros)
    int Q;
    double2* Z;     // Z rows [C][zrows][MS]
    int zrows;
  };
  struct Io {
    const double* in;
    int64_t in_stride, n;
    int in_aligned;
    double* out;
    int64_t out_stride, out_len;
    int out_aligned;
    bool accumulate;
    const MixOut* mix;
  };
  void k1(const Chunk& ck, const Rings& rg, const Io& io, const StreamGate& sg, bool ordered, int runR, int runNy,
          hipStream_t s);
  void k2(const Chunk& ck, const Rings& rg, const StreamGate& sg, int runR, hipStream_t s);
  void k3(const Chunk& ck, const Rings& rg, const Io& io, const StreamGate& sg, bool ordered, int runR, int runNy,
          hipStream_t s);
  void run_pipelined(const Io& io, hipStream_t s, int64_t jb, int64_t J, int64_t nb_in);

  int sched_mode_ = kSchedSerial, pipe_jc_ = 0, pipe_run_ = 0;  // in force for the current signal
  int req_mode_ = kSchedSerial, req_jc_ = 0, req_run_ = 0;        // requested, applied at begin_offline
  bool pipe_call_ = false;  // this call may pipeline (device entry points)
  bool sig_pipe_ = false;   // the current signal runs pipelined (fixed at begin_offline)
  int Qp_ = 0, zrows_p_ = 0;
  DevBuf<double2> Xp_;      // pipelined block-spectrum ring [C][Qp+1][MS]
  DevBuf<double2> Zp_;      // pipelined Z rows, two halves [2][C][zrows_p][MS]
  hipStream_t ps_[2] = {nullptr, nullptr};  // K2, K3 streams
  hipEvent_t pev_[3][4] = {};               // K1 / K2 / K3 done, per chunk mod 4
  void ensure_pipe();

  struct ProfRec {
    hipEvent_t start, stop;
    int kernel;
    double bytes;
  };
  bool prof_ = false;
  int prof_mask_ = 7;
  std::vector<ProfRec> prof_recs_;
  std::vector<hipEvent_t> event_pool_;
  double acc_ms_[kKernels] = {0, 0, 0};
  int64_t acc_n_[kKernels] = {0, 0, 0};
  double acc_bytes_[kKernels] = {0, 0, 0};
  hipEvent_t take_event();
  void prof_begin(hipStream_t s, hipEvent_t* e, int kernel);
  void prof_end(hipStream_t s, hipEvent_t e0, int kernel, double bytes);
};

}  // namespace adsp
