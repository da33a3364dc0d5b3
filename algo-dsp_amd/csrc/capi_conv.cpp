// C ABI of dsp/conv (include/algodsp.h) on top of the UPOLS engine and the
// time-domain kernels.  Host logic here mirrors the reference constructors'
// validation and size selection; all sample arithmetic runs on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <vector>

#include "ad_common.hpp"
#include "conv_kernels.hpp"
#include "host_pipeline.hpp"
#include "nupols_engine.hpp"
#include "upols_engine.hpp"

using namespace adsp;

namespace {

enum class Kind { StreamOLS, StreamOLA, BatchOLS, BatchOLA, Partitioned, Multi, MultiStream, PartitionedMulti };

struct StageDesc {
  int64_t part_size;
  int64_t count;
  int64_t start;
};

// partitionIR (dsp/conv/partitioned.go:269-332) restated: host-side stage
// planning that StageCount/StageInfo report.
int trunc_log2(int64_t n) {  // partitioned.go:186-199
  if (n <= 0) return 0;
  int r = 0;
  while (n > 1) {
    n >>= 1;
    ++r;
  }
  return r;
}
int64_t bit_count_to_bits(int n) { return (int64_t(2) << n) - 1; }  // partitioned.go:202-204

std::vector<StageDesc> partition_ir(int64_t kernel_len_padded, int min_order, int max_order) {
  const int64_t min_block = int64_t(1) << min_order;
  int max_ir = trunc_log2(kernel_len_padded + min_block) - 1;
  int64_t res = kernel_len_padded - (bit_count_to_bits(max_ir) - bit_count_to_bits(min_order - 1));
  if (res > 0 && ((res >> max_ir) & 1) == 0 && max_ir > min_order) --max_ir;
  if (max_ir > max_order) max_ir = max_order;
  res = kernel_len_padded - (bit_count_to_bits(max_ir) - bit_count_to_bits(min_order - 1));
  std::vector<StageDesc> st;
  int64_t start = 0;
  for (int order = min_order; order < max_ir; ++order) {
    const int64_t count = 1 + ((res >> order) & 1);
    st.push_back({int64_t(1) << order, count, start});
    start += count << order;
    res -= (count - 1) << order;
  }
  int64_t count = 1;
  if (max_ir > 0) count = std::max<int64_t>(1, 1 + res / (int64_t(1) << max_ir));
  st.push_back({int64_t(1) << max_ir, count, start});
  return st;
}

int64_t largest_pow2_divisor(int64_t v, int64_t cap) {
  int64_t l = 1;
  while ((v % (l * 2)) == 0 && l * 2 <= cap) l *= 2;
  return l;
}

}  // namespace

struct ad_conv {
  Kind kind;
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t K = 0;
  int64_t conv_len = 0;    // taps actually convolved (partitioned: stage coverage)
  int64_t block_size = 0;  // streaming block / OLA block
  int64_t fft_size = 0;    // reported FFTSize()
  int64_t step_size = 0;   // OverlapSave.StepSize()
  int64_t latency = 0;     // partitioned
  double wet = 1.0, dry = 1.0;  // ConvolutionReverb mix (reverb/convolution.go:45-58)
  std::vector<StageDesc> stages;

  std::unique_ptr<Upols> eng;  // FFT path
  std::unique_ptr<HostPipeline> pipe;  // overlapped host-buffer offline calls
  int channels = 1;
  bool f32 = false;                    // float32 boundary (the *32 constructors)
  std::vector<double> w_in, w_out;     // float32 calls: widened block
  int64_t hop = 0;
  int64_t seg_next = -1;  // next out_begin of a segmented offline call (-1: none open)
  DevBuf<double> mix_scratch;  // ad_conv_multi_process_device_mix at hop < 2048: per-channel outputs
  // multi-channel streaming with a block size that is not a whole number of
  // hops (ms_partial): [C][carry_w] device rows holding the unfinished block's
  // samples + the call's block (two, swapped per call), and the touched
  // blocks' outputs [C][ms_out_w]
  DevBuf<double> carry[2], ms_out;
  int carry_cur = 0;
  int64_t carry_w = 0, ms_out_w = 0;

  // streaming blocks that are not a whole number of hops: samples of the
  // unfinished block carried in pin_in (stream_convolve)
  bool partial = false;
  int64_t part_fill = 0;

  // pre-enqueued block chains (StreamGate, conv_kernels.hpp): one block of
  // hop >= 2048 per call.  ctl lives in coherent mapped host memory: go
  // (host -> K1), k1_state (K1 -> host), done (K3 -> host), a line each.
  struct GateCtl {
    uint64_t go, pad0[15];
    uint64_t k1_state, pad1[15];
    uint64_t done, pad2[15];
  };
  bool gated = false;
  GateCtl* ctl = nullptr;      // host view
  GateCtl* ctl_dev = nullptr;  // device view
  DevBuf<uint64_t> gate_word;
  uint64_t seq = 0;            // last block sequence number issued
  uint64_t chain_pending = 0;  // sequence number of the pre-enqueued chain (0: none)
  uint64_t gate_timeout = 0;   // K1's wait, ticks of the device's real-time counter
  // pre-enqueueing pays only for back-to-back calls: the call
  // interval (EMA, ms) and the pre-enqueued chains that timed out in a row
  double gate_gap_ms = 0;
  int gate_misses = 0;
  std::chrono::steady_clock::time_point gate_last{};
  uint64_t gate_khz = 100000;   // the device's real-time counter, ticks per ms
  int64_t gate_hits = 0, gate_timeouts = 0;  // ad_conv_lowlat_stats

  // time-domain streaming path (blocks of fewer than 64 samples)
  bool direct_stream = false;
  DevBuf<double> hdev;
  DevBuf<double> sbuf[2];
  int cur = 0;

  // staging
  DevBuf<double> din, dout;
  // pinned host staging for the per-block host-buffer calls: DMA straight
  // from/to page-locked memory instead of the runtime's pageable bounce path
  double* pin_in = nullptr;
  double* pin_out = nullptr;
  double* pin_in_dev = nullptr;   // device-side addresses of the mapped buffers
  double* pin_out_dev = nullptr;
  size_t pin_n = 0;

  // multi-channel device calls: the engine's delay line and scratch are
  // shared by every caller stream, so a call on a new stream waits for the
  // previous call's last launch (has_last: last may be the NULL stream)
  hipStream_t last = nullptr;
  bool has_last = false;
  hipEvent_t done = nullptr;

  // partitioned: non-uniform multi-stage engine (64 <= latency <= 8192)
  std::unique_ptr<NupolsDev> nupd;

  // partitioned FIFO state (latency < 64: time-domain streaming fallback shape)
  std::vector<double> pending;   // input samples not yet convolved (< hop)
  std::deque<double> ylin;       // convolved samples not yet emitted
  int64_t emitted = 0;           // output samples emitted so far
  int64_t ylin_base = 0;         // linear-conv index of ylin.front()

  ~ad_conv() {
    if (chain_pending && ctl) {  // release a pre-enqueued chain's K1 at once (gate_cancel without errors)
      __atomic_store_n(&ctl->go, kGateAbort, __ATOMIC_RELEASE);
      if (stream) (void)hipStreamSynchronize(stream);
    }
    gate_release(this);
    pipe.reset();
    if (done) {
      (void)hipEventSynchronize(done);
      (void)hipEventDestroy(done);
    }
    nupd.reset();
    eng.reset();
    if (stream) (void)hipStreamSynchronize(stream);
    if (pin_in) (void)hipHostFree(pin_in);
    if (pin_out) (void)hipHostFree(pin_out);
    if (ctl) (void)hipHostFree(ctl);
    if (stream) (void)lib_stream_destroy(stream);
  }
};

namespace {

ad_conv* new_handle(Kind k, int device) {
  auto* h = new ad_conv();
  h->kind = k;
  h->device = device;
  DeviceScope ds(device);
  if (lib_stream_create(&h->stream) != hipSuccess) {
    delete h;
    AD_FAIL(AD_ERR_DEVICE, "hipStreamCreate failed");
  }
  return h;
}

// Orders a device call on stream s after the handle's previous one.
void order_after_last(ad_conv* h, hipStream_t s) {
  if (!h->done) AD_HIP(hipEventCreateWithFlags(&h->done, hipEventDisableTiming));
  if (h->has_last && h->last != s) AD_HIP(hipStreamWaitEvent(s, h->done, 0));
}
void mark_last(ad_conv* h, hipStream_t s) {
  AD_HIP(hipEventRecord(h->done, s));
  h->last = s;
  h->has_last = true;
}

// Zero-latency streaming convolution state for blocks of B samples
// (StreamingOverlapSaveT / StreamingOverlapAddT, streaming_overlap_save.go:45-164):
//  - B with a power-of-two divisor >= 256 (or B itself a power of two >= 64):
//    the hop is that divisor and every call is B/hop whole engine blocks;
//  - any other B >= 64 (480, 960, 1000, 4800 ...): hop = nextPow2(B) (<= 8192)
//    and the partial block is carried: a call re-transforms the block it
//    ends in with the samples not yet received read as zeros.  The output
//    sample r of a block depends only on inputs <= r, so the zeros never
//    reach an emitted sample, and once the block is complete its spectrum in
//    the delay line is final.  A call costs one or two FFT blocks (at most
//    ceil((hop - 1 + B) / hop)), never an O(K) time-domain sum per sample;
//  - B < 64: the time-domain kernel.
void setup_stream_engine(ad_conv* h, const double* kernel, int64_t K, int64_t B, int64_t hop_cap) {
  int64_t hop = largest_pow2_divisor(B, hop_cap);
  if (hop < 256 && hop != B && B >= 64) {
    // nextPow2(B), and at least K/64 so that a call's K2 (one output block per
    // touched block, k_fdl_mac_row) keeps <= 64 partitions per wave: with
    // K = 131072 and B = 480 a hop of 512 would give each of only 8 waves
    // 256 partitions in series
    hop = std::min<int64_t>(hop_cap, std::max(next_pow2(B), next_pow2((K + 63) / 64)));
    h->partial = (B % hop) != 0;
  }
  h->hop = hop;
  h->conv_len = K;
  h->part_fill = 0;
  if (hop >= 64) {
    const int64_t blocks = h->partial ? (hop - 1 + B + hop - 1) / hop : B / hop;
    const int jc = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, 256));
    h->eng.reset(new Upols(h->device, kernel, 1, K, (int)hop, 1, nullptr, jc, h->stream));
  } else {
    h->direct_stream = true;
    h->hdev.alloc((size_t)K);
    AD_HIP(hipMemcpyAsync(h->hdev.p, kernel, K * sizeof(double), hipMemcpyHostToDevice, h->stream));
  }
}

// ---- pre-enqueued streaming chains (StreamGate) ----------------------------
// Host side of the protocol in conv_kernels.hpp.  A call publishes its block
// (go = seq), enqueues the next block's chain behind the running one, and
// spins on the done word; the launches of block i+1 thus overlap block i's
// kernels and the wait is a load of host memory, not a HIP call.
using Clock = std::chrono::steady_clock;

void gate_setup(ad_conv* h) {
  h->gated = !h->partial && !h->direct_stream && h->hop >= 2048 && h->block_size == h->hop;
  if (!h->gated) return;
  AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->ctl), sizeof(ad_conv::GateCtl),
                       hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(h->ctl, 0, sizeof(ad_conv::GateCtl));
  AD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->ctl_dev), h->ctl, 0));
  h->gate_word.alloc(1);
  AD_HIP(hipMemsetAsync(h->gate_word.p, 0, sizeof(uint64_t), h->stream));
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device) != hipSuccess || khz <= 0) khz = 100000;
  h->gate_khz = (uint64_t)khz;
  h->gate_timeout = (uint64_t)khz * 20;  // 20 ms: a later block runs through ordinary launches
}

// Spins until pred() holds (acquire loads of the ctl words); gives up after
// 2 s (then the stream is synchronised so that a device fault surfaces).
template <class Pred>
void gate_spin(ad_conv* h, Pred&& pred) {
  const auto t0 = Clock::now();
  for (uint32_t i = 0;; ++i) {
    if (pred()) return;
    if ((i & 1023) == 1023 && Clock::now() - t0 > std::chrono::seconds(2)) {
      AD_HIP(hipStreamSynchronize(h->stream));
      if (pred()) return;
      AD_FAIL(AD_ERR_INTERNAL, "streaming block: completion word never written");
    }
    __builtin_ia32_pause();
  }
}
uint64_t ctl_load(const uint64_t* w) { return __atomic_load_n(w, __ATOMIC_ACQUIRE); }

void gate_enqueue(ad_conv* h, uint64_t sq, bool wait_for_go, int64_t n) {
  StreamGate g{};
  g.seq = sq;
  g.done = &h->ctl_dev->done;
  if (wait_for_go) {
    g.go = &h->ctl_dev->go;
    g.k1_state = &h->ctl_dev->k1_state;
    g.gate = h->gate_word.p;
    // the waiting K1 gives up after 4 call intervals (1 .. 20 ms): whatever
    // shares its hardware queue waits behind it at most that long
    const double ms = std::clamp(4.0 * h->gate_gap_ms, 1.0, 20.0);
    g.timeout = (uint64_t)(ms * (double)h->gate_khz);
  }
  h->eng->set_gate(g);
  h->eng->run(h->pin_in_dev, n, n, h->pin_out_dev, n, n, /*use_hist=*/true, h->stream);
}

// Drops the pre-enqueued chain (its K1 exits at once, K2 / K3 skip) and
// steps the engine back over its block; the stream is idle afterwards.
void gate_cancel(ad_conv* h) {
  if (!h->chain_pending) return;
  const uint64_t p = h->chain_pending;
  __atomic_store_n(&h->ctl->go, kGateAbort, __ATOMIC_RELEASE);
  gate_spin(h, [&] {
    const uint64_t v = ctl_load(&h->ctl->k1_state);
    return v == (p | kGateSkipped) || v == p;
  });
  AD_HIP(hipStreamSynchronize(h->stream));
  if (ctl_load(&h->ctl->k1_state) != p) h->eng->rewind(1);
  // release the slot before clearing go: a gate_preempt from another thread
  // writes the abort only while this handle owns the slot, so no stale abort
  // can land in go after the clear
  gate_release(h);
  __atomic_store_n(&h->ctl->go, 0, __ATOMIC_RELEASE);
  h->chain_pending = 0;
}

// Whether the next block's chain is pre-enqueued: only while calls come
// back to back.  A caller paced in real time (hop 2048 at 48 kHz calls every
// 42.7 ms) would otherwise leave a K1 workgroup polling mapped memory for the
// whole 20-ms timeout and then pay the cancel-and-relaunch fallback on every
// block: with an interval (EMA) above a quarter of the timeout, or after 3
// chains in a row timed out, the blocks run through ordinary launches (still
// completing through the done word) until calls come fast again.
bool gate_pre_enqueue(ad_conv* h) {
  const auto now = Clock::now();
  if (h->gate_last.time_since_epoch().count() != 0) {
    const double gap = std::chrono::duration<double, std::milli>(now - h->gate_last).count();
    h->gate_gap_ms = h->gate_gap_ms == 0 ? gap : 0.75 * h->gate_gap_ms + 0.25 * gap;
  }
  h->gate_last = now;
  const double timeout_ms = 20.0;
  // one measured interval first; then the process-wide slot (gate_acquire:
  // one armed launch at a time, and none while the library's streams could
  // share the caller's hardware queues)
  return h->gate_misses < 3 && h->gate_gap_ms > 0 && h->gate_gap_ms < timeout_ms / 4 &&
         gate_acquire(h, &h->ctl->go, h->stream);
}

// One block of n = hop samples (already in pin_in) through the chains.
void gate_block(ad_conv* h, int64_t n) {
  gate_preempt(h);  // another handle's armed launch must not hold up this block
  const uint64_t sq = ++h->seq;
  const bool pre = gate_pre_enqueue(h);
  if (h->chain_pending == sq) {
    __atomic_store_n(&h->ctl->go, sq, __ATOMIC_RELEASE);  // the waiting K1 takes the block
    if (pre) {
      gate_enqueue(h, sq + 1, true, n);  // the next block's chain, behind this one
      h->chain_pending = sq + 1;
    } else {
      h->chain_pending = 0;
      gate_release(h);
    }
    // done, or this chain's K1 gave up before go (the caller came late)
    gate_spin(h, [&] { return ctl_load(&h->ctl->done) == sq || ctl_load(&h->ctl->k1_state) == (sq | kGateSkipped); });
    if (ctl_load(&h->ctl->done) == sq) {
      h->gate_misses = 0;
      ++h->gate_hits;
      return;
    }
    ++h->gate_misses;
    ++h->gate_timeouts;
    gate_cancel(h);       // the chain behind it
    h->eng->rewind(1);    // this block's skipped chain
    gate_enqueue(h, sq, false, n);
    gate_spin(h, [&] { return ctl_load(&h->ctl->done) == sq; });
    return;
  }
  gate_enqueue(h, sq, false, n);  // ordinary launches, completion through done
  if (pre) {
    gate_enqueue(h, sq + 1, true, n);
    h->chain_pending = sq + 1;
  }
  gate_spin(h, [&] { return ctl_load(&h->ctl->done) == sq; });
  if (!pre && h->gate_misses >= 3 && h->gate_gap_ms < 2.0) h->gate_misses = 0;  // fast again: retry
}

void stream_reset(ad_conv* h) {
  gate_cancel(h);
  if (h->eng) h->eng->reset_stream(h->stream);
  for (auto& b : h->sbuf)
    if (b.p) AD_HIP(hipMemsetAsync(b.p, 0, b.n * sizeof(double), h->stream));
  h->pending.clear();
  h->ylin.clear();
  h->emitted = 0;
  h->ylin_base = 0;
  h->part_fill = 0;
  AD_HIP(hipStreamSynchronize(h->stream));
}

// Convolves n new samples (host) with the running history; n must be a
// multiple of the hop on the FFT path.  Writes n linear-conv samples to out.
void stream_convolve(ad_conv* h, const double* in, int64_t n, double* out) {
  if (n == 0) return;
  gate_preempt(h);  // every streaming path, gated or not: no other handle's armed launch ahead of this block
  hipStream_t s = h->stream;
  if (h->direct_stream) {
    const int64_t K = h->conv_len;
    const size_t need = (size_t)(K - 1 + n);
    DevBuf<double>& curb = h->sbuf[h->cur];
    DevBuf<double>& nxt = h->sbuf[h->cur ^ 1];
    if (curb.n < need) {
      // grow, keeping the K-1 history at the front
      DevBuf<double> tmp;
      tmp.alloc(need);
      AD_HIP(hipMemsetAsync(tmp.p, 0, need * sizeof(double), s));
      if (curb.p && K > 1) AD_HIP(hipMemcpyAsync(tmp.p, curb.p, (K - 1) * sizeof(double), hipMemcpyDeviceToDevice, s));
      AD_HIP(hipStreamSynchronize(s));
      std::swap(curb.p, tmp.p);
      std::swap(curb.n, tmp.n);
    }
    nxt.reserve(need);
    AD_HIP(hipMemcpyAsync(curb.p + (K - 1), in, n * sizeof(double), hipMemcpyHostToDevice, s));
    h->dout.reserve((size_t)n);
    launch_stream_direct(h->hdev.p, K, curb.p, n, h->dout.p, s);
    AD_HIP(hipGetLastError());
    if (K > 1) AD_HIP(hipMemcpyAsync(nxt.p, curb.p + n, (K - 1) * sizeof(double), hipMemcpyDeviceToDevice, s));
    h->cur ^= 1;
    AD_HIP(hipMemcpyAsync(out, h->dout.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
    AD_HIP(hipStreamSynchronize(s));
    return;
  }
  // Zero-copy: the block goes through page-locked host buffers that the GPU
  // reads (K1) and writes (K3) directly over PCIe, so a block costs three
  // kernels and one synchronisation, no DMA round trips.  K1 transforms each
  // input block once and keeps no input history (the previous block's
  // spectrum is in the delay line), so nothing but the block itself crosses
  // PCIe (config 2 measured 37.8 us per block direct vs 42.4-43.7 staged
  // through HBM by two copy kernels).
  // Partial-block form (h->partial): pin_in holds the samples of the block the
  // last call ended in (part_fill of them) followed by this call's; K1
  // transforms every block they touch (zeros past the last sample), K3 writes
  // those blocks whole to pin_out, and the call's samples are the slice
  // [part_fill, part_fill + n).  An unfinished last block is not committed:
  // the engine's block counter steps back so the next call transforms it
  // again with more samples.
  const int64_t L = h->hop;
  const size_t need_in = h->partial ? (size_t)(L + n) : (size_t)n;
  const size_t need_out = h->partial ? (size_t)(((L - 1 + n + L - 1) / L) * L) : (size_t)n;
  const size_t need = std::max(need_in, need_out);
  if (h->pin_n < need) {
    std::vector<double> keep(h->pin_in, h->pin_in + (h->pin_in ? h->part_fill : 0));
    if (h->pin_in) AD_HIP(hipHostFree(h->pin_in));
    if (h->pin_out) AD_HIP(hipHostFree(h->pin_out));
    h->pin_in = h->pin_out = nullptr;
    h->pin_n = 0;
    AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->pin_in), need * sizeof(double), hipHostMallocMapped));
    AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->pin_out), need * sizeof(double), hipHostMallocMapped));
    AD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->pin_in_dev), h->pin_in, 0));
    AD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->pin_out_dev), h->pin_out, 0));
    h->pin_n = need;
    if (!keep.empty()) std::memcpy(h->pin_in, keep.data(), keep.size() * sizeof(double));
  }
  if (!h->partial) {
    std::memcpy(h->pin_in, in, n * sizeof(double));
    if (h->gated) {
      gate_block(h, n);
    } else {
      h->eng->run(h->pin_in_dev, n, n, h->pin_out_dev, n, n, /*use_hist=*/true, s);
      AD_HIP(hipStreamSynchronize(s));
    }
    std::memcpy(out, h->pin_out, n * sizeof(double));
    return;
  }
  const int64_t f0 = h->part_fill;
  const int64_t tot = f0 + n;
  const int64_t blocks = (tot + L - 1) / L;
  std::memcpy(h->pin_in + f0, in, n * sizeof(double));
  h->eng->run(h->pin_in_dev, tot, tot, h->pin_out_dev, blocks * L, blocks * L, /*use_hist=*/true, s);
  const int64_t full = (tot / L) * L;
  if (full < tot) h->eng->rewind(1);  // the last block is not complete yet
  AD_HIP(hipStreamSynchronize(s));
  std::memcpy(out, h->pin_out + f0, n * sizeof(double));
  if (full > 0 && full < tot) std::memmove(h->pin_in, h->pin_in + full, (size_t)(tot - full) * sizeof(double));
  h->part_fill = tot - full;
}

// Offline full convolution of host channels with the handle's kernel(s):
// chunked and overlapped across PCIe (host_pipeline.hpp).
void batch_convolve_multi(ad_conv* h, const double* const* in, int C, int64_t n, double* const* out,
                          int64_t out_len) {
  if (!h->pipe) h->pipe.reset(new HostPipeline(h->device));
  order_after_last(h, h->stream);
  h->pipe->offline(*h->eng, in, C, n, out, out_len, h->stream);
  mark_last(h, h->stream);
}
void batch_convolve(ad_conv* h, const double* in, int64_t n, double* out, int64_t out_len) {
  batch_convolve_multi(h, &in, 1, n, &out, out_len);
}

int64_t batch_hop(int64_t K) {
  int64_t l = next_pow2(std::max<int64_t>(K, 256));
  return std::min<int64_t>(l, 8192);
}

void make_batch_engine(ad_conv* h, const double* kernel, int64_t K) {
  h->hop = batch_hop(K);
  // up to 512 blocks per launch (a host pipeline segment is <= 2^21 samples):
  // a mono call then fills the chip with few launches; the delay line and
  // product rows cost ~2 x 512 x (hop + 8) x 16 B (134 MB at hop 8192)
  h->eng.reset(new Upols(h->device, kernel, 1, K, (int)h->hop, 1, nullptr, 512, h->stream));
}

template <class Fn>
int create_guarded(ad_conv** out, Fn&& fn) {
  if (out) *out = nullptr;
  ad_conv* h = nullptr;
  const int rc = guard([&] { h = fn(); });
  if (rc != AD_OK) {
    delete h;
    return rc;
  }
  if (out) *out = h;
  return AD_OK;
}

}  // namespace

extern "C" {

// --- streaming ------------------------------------------------------------

static int stream_create(Kind kind, const double* kernel, int64_t K, int64_t B, int device, ad_conv** out) {
  // NewStreamingOverlapSaveT streaming_overlap_save.go:45-84 /
  // NewStreamingOverlapAddT streaming_overlap_add.go:43-83
  return create_guarded(out, [&]() -> ad_conv* {
    if (K <= 0 || !kernel) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    if (B <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "conv: blockSize must be positive, got " + std::to_string(B));
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_conv> h(new_handle(kind, dev));
    h->K = K;
    h->block_size = B;
    h->fft_size = next_pow2(B + K - 1);
    setup_stream_engine(h.get(), kernel, K, B, 8192);
    gate_setup(h.get());
    stream_reset(h.get());
    return h.release();
  });
}

int ad_conv_stream_ols_create(const double* kernel, int64_t kernel_len, int64_t block_size, int device,
                              ad_conv** out) {
  return stream_create(Kind::StreamOLS, kernel, kernel_len, block_size, device, out);
}

int ad_conv_stream_ola_create(const double* kernel, int64_t kernel_len, int64_t block_size, int device,
                              ad_conv** out) {
  return stream_create(Kind::StreamOLA, kernel, kernel_len, block_size, device, out);
}

int ad_conv_process_block(ad_conv* h, const double* in, int64_t in_len, double* out, int64_t out_len) {
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil handle");
    if (h->kind != Kind::StreamOLS && h->kind != Kind::StreamOLA)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "ProcessBlockTo on a non-streaming convolver");
    if (in_len != h->block_size)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch: expected " + std::to_string(h->block_size) +
                                          " input samples, got " + std::to_string(in_len));
    if (out_len != h->block_size)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch: expected " + std::to_string(h->block_size) +
                                          " output samples, got " + std::to_string(out_len));
    DeviceScope ds(h->device);
    stream_convolve(h, in, in_len, out);
  });
}

// --- float32 instantiations ---------------------------------------------------
// NewStreamingOverlapSave32 (streaming_overlap_save.go:94), NewStreamingOverlapAdd32
// (streaming_overlap_add.go:93), NewPartitionedConvolution32 (partitioned.go:340):
// float32 kernels and blocks at the boundary.  The samples are widened to
// float64 (exactly) on the way in and rounded once to float32 on the way out;
// the convolution itself runs on the float64 engine, so the result is the
// correctly rounded float32 of a float64 convolution -- within the reference's
// own complex64 error (its float32 tests allow 1e-4, streaming_test.go:175-265).

}  // extern "C"

namespace {
std::vector<double> widen(const float* p, int64_t n) {
  std::vector<double> v((size_t)std::max<int64_t>(n, 0));
  for (int64_t i = 0; i < n; ++i) v[(size_t)i] = (double)p[i];
  return v;
}
// Per-block float32 calls: validate before touching the buffers, then widen
// into the handle's reused vector (no allocation on the streaming hot path).
void widen_block(ad_conv* h, const float* in, int64_t in_len, const float* out, int64_t out_len) {
  if (in_len < 0 || out_len < 0) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: negative buffer length");
  if ((in_len > 0 && !in) || (out_len > 0 && !out)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null sample buffer");
  h->w_in.resize((size_t)in_len);
  for (int64_t i = 0; i < in_len; ++i) h->w_in[(size_t)i] = (double)in[i];
  h->w_out.resize((size_t)out_len);
}
}  // namespace

extern "C" {

int ad_conv_stream_ols32_create(const float* kernel, int64_t kernel_len, int64_t block_size, int device,
                                ad_conv** out) {
  if (out) *out = nullptr;
  if (kernel_len <= 0 || !kernel) {
    set_last_error("conv: empty kernel");
    return AD_ERR_EMPTY_KERNEL;
  }
  const std::vector<double> k = widen(kernel, kernel_len);
  const int rc = stream_create(Kind::StreamOLS, k.data(), kernel_len, block_size, device, out);
  if (rc == AD_OK) (*out)->f32 = true;
  return rc;
}

int ad_conv_stream_ola32_create(const float* kernel, int64_t kernel_len, int64_t block_size, int device,
                                ad_conv** out) {
  if (out) *out = nullptr;
  if (kernel_len <= 0 || !kernel) {
    set_last_error("conv: empty kernel");
    return AD_ERR_EMPTY_KERNEL;
  }
  const std::vector<double> k = widen(kernel, kernel_len);
  const int rc = stream_create(Kind::StreamOLA, k.data(), kernel_len, block_size, device, out);
  if (rc == AD_OK) (*out)->f32 = true;
  return rc;
}

int ad_conv_process_block32(ad_conv* h, const float* in, int64_t in_len, float* out, int64_t out_len) {
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil handle");
    if (!h->f32) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a float32 convolver");
    if (in_len != h->block_size || out_len != h->block_size)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch: expected " + std::to_string(h->block_size) +
                                          " samples, got " + std::to_string(in_len) + " in / " +
                                          std::to_string(out_len) + " out");
    widen_block(h, in, in_len, out, out_len);
    const int rc = ad_conv_process_block(h, h->w_in.data(), in_len, h->w_out.data(), out_len);
    if (rc != AD_OK) throw Status{rc, ad_last_error()};
    for (int64_t i = 0; i < out_len; ++i) out[i] = (float)h->w_out[(size_t)i];
  });
}

int ad_conv_partitioned32_create(const float* kernel, int64_t kernel_len, int min_block_order, int max_block_order,
                                 int device, ad_conv** out) {
  if (out) *out = nullptr;
  if (kernel_len <= 0 || !kernel) {
    set_last_error("conv: empty impulse response");
    return AD_ERR_EMPTY_IMPULSE_RESPONSE;
  }
  const std::vector<double> k = widen(kernel, kernel_len);
  const int rc = ad_conv_partitioned_create(k.data(), kernel_len, min_block_order, max_block_order, device, out);
  if (rc == AD_OK) (*out)->f32 = true;
  return rc;
}

int ad_conv_partitioned_process_block32(ad_conv* h, const float* in, int64_t in_len, float* out, int64_t out_len) {
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil handle");
    if (!h->f32) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a float32 convolver");
    if (in_len != out_len)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch: input length " + std::to_string(in_len) +
                                          " != output length " + std::to_string(out_len));
    widen_block(h, in, in_len, out, out_len);
    const int rc = ad_conv_partitioned_process_block(h, h->w_in.data(), in_len, h->w_out.data(), out_len);
    if (rc != AD_OK) throw Status{rc, ad_last_error()};
    for (int64_t i = 0; i < out_len; ++i) out[i] = (float)h->w_out[(size_t)i];
  });
}

// --- batch ------------------------------------------------------------------

int ad_conv_ols_create(const double* kernel, int64_t K, int64_t fft_size, int device, ad_conv** out) {
  // NewOverlapSave overlap_save.go:53-107
  return create_guarded(out, [&]() -> ad_conv* {
    if (K <= 0 || !kernel) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    int64_t n = fft_size;
    if (n <= 0) n = std::max<int64_t>(next_pow2(2 * K), 256);
    if (!is_pow2(n))
      AD_FAIL(AD_ERR_INVALID_BLOCK_SIZE, "conv: invalid block size: fftSize must be power of 2, got " +
                                             std::to_string(n));
    if (n < 2 * K) n = next_pow2(2 * K);
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_conv> h(new_handle(Kind::BatchOLS, dev));
    h->K = K;
    h->fft_size = n;
    h->step_size = n - K + 1;
    make_batch_engine(h.get(), kernel, K);
    AD_HIP(hipStreamSynchronize(h->stream));
    return h.release();
  });
}

int ad_conv_ola_create(const double* kernel, int64_t K, int64_t block_size, int device, ad_conv** out) {
  // NewOverlapAdd overlap_add.go:44-89
  return create_guarded(out, [&]() -> ad_conv* {
    if (K <= 0 || !kernel) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    int64_t b = block_size;
    if (b <= 0) b = std::max<int64_t>(next_pow2(K), 256);
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_conv> h(new_handle(Kind::BatchOLA, dev));
    h->K = K;
    h->block_size = b;
    h->fft_size = next_pow2(b + K - 1);
    make_batch_engine(h.get(), kernel, K);
    AD_HIP(hipStreamSynchronize(h->stream));
    return h.release();
  });
}

int ad_conv_process(ad_conv* h, const double* in, int64_t in_len, double* out, int64_t out_len) {
  // OverlapSave.Process/ProcessTo overlap_save.go:126-272,
  // OverlapAdd.Process/ProcessTo overlap_add.go:108-182
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil handle");
    if (h->kind != Kind::BatchOLS && h->kind != Kind::BatchOLA)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "Process on a non-batch convolver");
    const int64_t expected = in_len + h->K - 1;
    if (out_len != expected)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch: expected " + std::to_string(expected) +
                                          ", got " + std::to_string(out_len));
    if (in_len <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    DeviceScope ds(h->device);
    batch_convolve(h, in, in_len, out, out_len);
  });
}

// --- partitioned ---------------------------------------------------------------

int ad_conv_partitioned_create(const double* kernel, int64_t K, int min_order, int max_order, int device,
                               ad_conv** out) {
  // NewPartitionedConvolutionT partitioned.go:212-266
  return create_guarded(out, [&]() -> ad_conv* {
    if (K <= 0 || !kernel) AD_FAIL(AD_ERR_EMPTY_IMPULSE_RESPONSE, "conv: empty impulse response");
    if (min_order < 1)
      AD_FAIL(AD_ERR_INVALID_BLOCK_ORDER,
              "conv: invalid block order: minBlockOrder must be >= 1, got " + std::to_string(min_order));
    if (max_order < min_order)
      AD_FAIL(AD_ERR_INVALID_BLOCK_ORDER, "conv: invalid block order: maxBlockOrder (" + std::to_string(max_order) +
                                              ") must be >= minBlockOrder (" + std::to_string(min_order) + ")");
    if (min_order > 30) AD_FAIL(AD_ERR_INVALID_BLOCK_ORDER, "conv: invalid block order: minBlockOrder too large");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_conv> h(new_handle(Kind::Partitioned, dev));
    const int64_t latency = int64_t(1) << min_order;
    const int64_t padded = ((K + latency - 1) / latency) * latency;
    h->K = K;
    h->latency = latency;
    h->block_size = latency;
    h->stages = partition_ir(padded, min_order, max_order);
    // Effective kernel: the taps the stage layout covers (the reference never
    // convolves taps beyond the last stage).
    int64_t cover = 0;
    for (const auto& s : h->stages) cover = std::max(cover, s.start + s.count * s.part_size);
    const int64_t keff = std::min<int64_t>(K, cover);
    h->fft_size = 2 * h->stages.back().part_size;
    if (latency >= 64 && latency <= 8192) {
      // Device-resident non-uniform stages (NupolsDev, one channel): hop lambda
      // for the head of the IR, doubling up to 2^maxBlockOrder (<= 8192) for
      // the tail; mapped pinned block I/O, the accumulator on the device,
      // emit-before-convolve.
      const int64_t pmax = std::min<int64_t>(8192, std::max<int64_t>(latency, int64_t(1) << std::min(max_order, 13)));
      h->conv_len = keff;
      h->nupd.reset(new NupolsDev(dev, kernel, keff, latency, pmax, 1, h->stream));
      AD_HIP(hipStreamSynchronize(h->stream));
    } else {
      // Zero-latency engine with hop = latency (<= 8192), output delayed by latency.
      setup_stream_engine(h.get(), kernel, keff, latency, 8192);
      stream_reset(h.get());
    }
    return h.release();
  });
}

int ad_conv_partitioned_process_block(ad_conv* h, const double* in, int64_t in_len, double* out, int64_t out_len) {
  // PartitionedConvolutionT.ProcessBlock partitioned.go:348-396
  return guard([&] {
    if (!h || h->kind != Kind::Partitioned) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a partitioned convolver");
    if (in_len != out_len)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch: input length " + std::to_string(in_len) +
                                          " != output length " + std::to_string(out_len));
    if (in_len == 0) return;
    DeviceScope ds(h->device);
    if (h->nupd) {
      h->nupd->process_host(in, out, in_len, /*mix=*/false, 1.0, 0.0, h->stream);
      h->emitted += in_len;
      return;
    }
    // Convolve every complete hop-sized block (all samples on the direct path).
    h->pending.insert(h->pending.end(), in, in + in_len);
    const int64_t hop = h->direct_stream ? 1 : h->hop;
    const int64_t nconv = ((int64_t)h->pending.size() / hop) * hop;
    if (nconv > 0) {
      std::vector<double> y((size_t)nconv);
      stream_convolve(h, h->pending.data(), nconv, y.data());
      h->ylin.insert(h->ylin.end(), y.begin(), y.end());
      h->pending.erase(h->pending.begin(), h->pending.begin() + nconv);
    }
    // Emit: output sample o is ylin[o - latency] (zero before the latency).
    for (int64_t i = 0; i < out_len; ++i) {
      const int64_t o = h->emitted + i;
      const int64_t src = o - h->latency;
      if (src < 0) {
        out[i] = 0.0;
        continue;
      }
      while (h->ylin_base < src) {
        h->ylin.pop_front();
        ++h->ylin_base;
      }
      out[i] = h->ylin.front();
    }
    h->emitted += out_len;
  });
}

// --- reverb.ConvolutionReverb (dsp/effects/reverb/convolution.go:16-95) ----------

int ad_conv_reverb_create(const double* kernel, int64_t K, int min_order, int device, ad_conv** out) {
  // NewConvolutionReverb: partitioned engine with maxBlockOrder 13, wet = dry = 1
  if (out) *out = nullptr;
  if (K <= 0 || !kernel) {
    set_last_error("reverb: empty impulse response kernel");
    return AD_ERR_EMPTY_IMPULSE_RESPONSE;
  }
  return ad_conv_partitioned_create(kernel, K, min_order, 13, device, out);
}

int ad_conv_reverb_set_wet_dry(ad_conv* h, double wet, double dry) {
  return guard([&] {
    if (!h || (h->kind != Kind::Partitioned && h->kind != Kind::PartitionedMulti))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a convolution reverb");
    h->wet = wet;
    h->dry = dry;
  });
}

int ad_conv_reverb_process_inplace(ad_conv* h, double* block, int64_t n) {
  // ProcessInPlace: block[i] = dry*block[i] + wet*reverb(block)[i]  (convolution.go:60-85)
  if (n <= 0) return AD_OK;
  std::vector<double> rev((size_t)n);
  const int rc = ad_conv_partitioned_process_block(h, block, n, rev.data(), n);
  if (rc != AD_OK) return rc;
  {
#pragma clang fp contract(off)
    for (int64_t i = 0; i < n; ++i) block[i] = h->dry * block[i] + h->wet * rev[(size_t)i];
  }
  return AD_OK;
}

int ad_conv_stage_count(const ad_conv* h) { return h ? (int)h->stages.size() : 0; }

int ad_conv_stage_info(const ad_conv* h, int index, int64_t* part_size, int64_t* block_count) {
  // StageInfo partitioned.go:427-436
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil handle");
    if (index < 0 || index >= (int)h->stages.size())
      AD_FAIL(AD_ERR_STAGE_INDEX_OUT_OF_RANGE, "conv: stage index out of range: index " + std::to_string(index) +
                                                   ", have " + std::to_string(h->stages.size()) + " stages");
    if (part_size) *part_size = h->stages[index].part_size;
    if (block_count) *block_count = h->stages[index].count;
  });
}

// --- common -------------------------------------------------------------------

int ad_conv_reset(ad_conv* h) {
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil handle");
    DeviceScope ds(h->device);
    if (h->has_last) AD_HIP(hipStreamWaitEvent(h->stream, h->done, 0));  // after the last device call
    if (h->nupd) h->nupd->reset(h->stream);
    stream_reset(h);
    h->has_last = false;
  });
}

int ad_conv_set_host_io(ad_conv* h, int mode, int workers) {
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil handle");
    if (mode < AD_HOST_IO_AUTO || mode > AD_HOST_IO_REGISTER) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "unknown host I/O mode");
    if (workers < 0 || workers > 64) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "copy workers must be in [0, 64]");
    if (h->kind != Kind::BatchOLS && h->kind != Kind::BatchOLA && h->kind != Kind::Multi)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "host I/O mode applies to batch / multi-channel convolvers");
    DeviceScope ds(h->device);
    if (!h->pipe) h->pipe.reset(new HostPipeline(h->device));
    h->pipe->set_mode(mode, workers);
  });
}

int ad_conv_host_io_profile(const ad_conv* h, double* register_ms, double* transfer_ms, double* unregister_ms) {
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil handle");
    const HostPipeline* p = h->pipe.get();
    if (register_ms) *register_ms = p ? p->last_register_ms() : 0.0;
    if (transfer_ms) *transfer_ms = p ? p->last_transfer_ms() : 0.0;
    if (unregister_ms) *unregister_ms = p ? p->last_unregister_ms() : 0.0;
  });
}

int64_t ad_conv_block_size(const ad_conv* h) { return h ? h->block_size : 0; }
int64_t ad_conv_kernel_len(const ad_conv* h) { return h ? h->K : 0; }
int64_t ad_conv_fft_size(const ad_conv* h) { return h ? h->fft_size : 0; }
int64_t ad_conv_step_size(const ad_conv* h) { return h ? h->step_size : 0; }
int64_t ad_conv_latency(const ad_conv* h) { return h ? h->latency : 0; }

void ad_conv_destroy(ad_conv* h) {
  if (!h) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(h->device);
  delete h;
  (void)hipSetDevice(cur);
}

// --- one-shot -----------------------------------------------------------------

static void direct_on_device(const double* a, int64_t n, const double* b, int64_t m, double* dst, int device) {
  const int dev = pick_device(device);
  DeviceScope ds(dev);
  DevBuf<double> da, db, dd;
  da.alloc((size_t)n);
  db.alloc((size_t)m);
  dd.alloc((size_t)(n + m - 1));
  AD_HIP(hipMemcpy(da.p, a, n * sizeof(double), hipMemcpyHostToDevice));
  AD_HIP(hipMemcpy(db.p, b, m * sizeof(double), hipMemcpyHostToDevice));
  launch_direct(da.p, n, db.p, m, dd.p, nullptr);
  AD_HIP(hipGetLastError());
  AD_HIP(hipMemcpy(dst, dd.p, (n + m - 1) * sizeof(double), hipMemcpyDeviceToHost));
}

int ad_conv_direct(const double* a, int64_t n, const double* b, int64_t m, double* dst, int device) {
  // conv.Direct conv.go:76-93
  return guard([&] {
    if (n <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (m <= 0) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    direct_on_device(a, n, b, m, dst, device);
  });
}

int ad_conv_direct_device(const double* d_a, int64_t n, const double* d_b, int64_t m, double* d_dst, void* stream) {
  // conv.DirectTo conv.go:97-154 on device-resident buffers (dst: n+m-1)
  return guard([&] {
    if (n <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (m <= 0) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    if (!d_a || !d_b || !d_dst) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "conv: null device buffer");
    launch_direct(d_a, n, d_b, m, d_dst, (hipStream_t)stream);
    AD_HIP(hipGetLastError());
  });
}

int ad_conv_direct_circular(const double* a, int64_t n, const double* b, int64_t m, double* dst, int device) {
  // conv.DirectCircular conv.go:158-173
  return guard([&] {
    if (n <= 0 || m <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (n != m) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    DevBuf<double> da, db, dd;
    da.alloc((size_t)n);
    db.alloc((size_t)n);
    dd.alloc((size_t)n);
    AD_HIP(hipMemcpy(da.p, a, n * sizeof(double), hipMemcpyHostToDevice));
    AD_HIP(hipMemcpy(db.p, b, n * sizeof(double), hipMemcpyHostToDevice));
    launch_direct_circular(da.p, db.p, n, dd.p, nullptr);
    AD_HIP(hipGetLastError());
    AD_HIP(hipMemcpy(dst, dd.p, n * sizeof(double), hipMemcpyDeviceToHost));
  });
}

int ad_conv_convolve(const double* a, int64_t n, const double* b, int64_t m, int mode, double* dst, int64_t dst_cap,
                     int64_t* dst_len, int device) {
  // conv.Convolve conv.go:194-216 and ConvolveMode/trimToMode :219-247
  return guard([&] {
    if (n <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (m <= 0) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    const double* la = a;
    const double* lb = b;
    int64_t ln = n, lm = m;
    if (lm > ln) {
      std::swap(la, lb);
      std::swap(ln, lm);
    }
    const int64_t full_len = ln + lm - 1;
    std::vector<double> full((size_t)full_len);
    if (lm <= 64) {
      direct_on_device(la, ln, lb, lm, full.data(), device);
    } else {
      // OverlapAddConvolve overlap_add.go:221-253
      const int dev = pick_device(device);
      DeviceScope ds(dev);
      std::unique_ptr<ad_conv> h(new_handle(Kind::BatchOLA, dev));
      h->K = lm;
      make_batch_engine(h.get(), lb, lm);
      batch_convolve(h.get(), la, ln, full.data(), full_len);
    }
    int64_t start = 0, len = full_len;
    if (mode == AD_MODE_SAME) {
      start = (m - 1) / 2;
      len = n;
    } else if (mode == AD_MODE_VALID) {
      if (n >= m) {
        start = m - 1;
        len = n - (m - 1);
      } else {
        start = n - 1;
        len = m - (n - 1);
      }
    }
    if (dst_len) *dst_len = len;
    if (dst_cap < len) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "dst capacity too small");
    std::memcpy(dst, full.data() + start, (size_t)len * sizeof(double));
  });
}

// --- multi-channel device path ---------------------------------------------------

namespace {
// The device entry points may run the pipelined schedule (Upols::set_schedule).
struct PipeCall {
  Upols* e;
  explicit PipeCall(Upols* eng) : e(eng) { e->set_pipeline_call(true); }
  ~PipeCall() { e->set_pipeline_call(false); }
};
}  // namespace

int ad_conv_multi_create(const double* kernels, int n_ir, int64_t K, int64_t hop, int channels,
                         const int32_t* ir_index, int64_t max_chunk_blocks, int device, ad_conv** out) {
  return create_guarded(out, [&]() -> ad_conv* {
    if (K <= 0 || !kernels || n_ir <= 0) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    if (channels <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "channels must be positive");
    if (hop <= 0) hop = batch_hop(K);
    if (hop < 64 || hop > 8192 || !is_pow2(hop))
      AD_FAIL(AD_ERR_INVALID_BLOCK_SIZE, "hop must be a power of two in [64, 8192]");
    if (max_chunk_blocks <= 0) {
      // X ring + Z scratch cost ~32 B per (channel, block, bin): give the
      // chunked offline path an ~8 GiB working set, 64..4096 blocks per chunk
      const int64_t budget = (int64_t)8 << 30;
      max_chunk_blocks = std::max<int64_t>(64, std::min<int64_t>(4096, budget / ((int64_t)channels * hop * 32)));
    }
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_conv> h(new_handle(Kind::Multi, dev));
    h->K = K;
    h->hop = hop;
    h->block_size = hop;
    h->fft_size = 2 * hop;
    h->channels = channels;
    h->eng.reset(new Upols(dev, kernels, n_ir, K, (int)hop, channels, ir_index, (int)max_chunk_blocks, h->stream));
    return h.release();
  });
}

int ad_conv_lowlat_stats(const ad_conv* h, int64_t* pre_enqueued, int64_t* timed_out) {
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null handle");
    int64_t a = 0, b = 0;
    if (h->nupd) {
      h->nupd->lowlat_stats(&a, &b);
    } else {
      a = h->gate_hits;
      b = h->gate_timeouts;
    }
    if (pre_enqueued) *pre_enqueued = a;
    if (timed_out) *timed_out = b;
  });
}

int ad_conv_multi_set_schedule(ad_conv* h, int mode, int64_t chunk_blocks, int64_t run_blocks) {
  return guard([&] {
    if (!h || h->kind != Kind::Multi) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a multi-channel convolver");
    if (chunk_blocks < 0 || chunk_blocks > (1 << 20) || run_blocks < 0 || run_blocks > (1 << 20))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "schedule: chunk / run length out of range");
    const int m = mode == AD_CONV_SCHED_PIPELINED ? Upols::kSchedPipelined
                  : mode == AD_CONV_SCHED_CHUNKED ? Upols::kSchedChunked
                  : mode == AD_CONV_SCHED_SERIAL  ? Upols::kSchedSerial
                                                  : -1;
    if (m < 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "schedule: unknown mode");
    DeviceScope ds(h->device);
    h->eng->set_schedule(m, (int)chunk_blocks, (int)run_blocks);
  });
}

int ad_conv_multi_get_schedule(const ad_conv* h, int* mode, int64_t* chunk_blocks) {
  return guard([&] {
    if (!h || h->kind != Kind::Multi) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a multi-channel convolver");
    const int sm = h->eng->schedule();
    const bool p = sm != Upols::kSchedSerial && h->eng->hop() >= 2048;
    if (mode) *mode = !p ? AD_CONV_SCHED_SERIAL : sm == Upols::kSchedChunked ? AD_CONV_SCHED_CHUNKED : AD_CONV_SCHED_PIPELINED;
    if (chunk_blocks) *chunk_blocks = p ? h->eng->pipe_chunk() : 0;
  });
}

int ad_conv_multi_process_device(ad_conv* h, const double* d_in, int64_t in_stride, int64_t in_len, double* d_out,
                                 int64_t out_stride, int64_t out_len, void* stream) {
  return guard([&] {
    if (!h || h->kind != Kind::Multi) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a multi-channel convolver");
    if (in_len <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (out_len > in_len + h->K - 1 || out_len <= 0)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch");
    DeviceScope ds(h->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);  // NULL = the default (null) stream
    order_after_last(h, s);
    h->eng->begin_offline(s);
    PipeCall pc(h->eng.get());
    h->eng->run(d_in, in_stride, in_len, d_out, out_stride, out_len, /*use_hist=*/false, s);
    mark_last(h, s);
    h->seg_next = -1;
  });
}

int ad_conv_multi_process_device_segment(ad_conv* h, const double* d_in, int64_t in_stride, int64_t in_len,
                                         double* d_out, int64_t out_stride, int64_t out_len, int64_t out_begin,
                                         int64_t out_end, void* stream) {
  return guard([&] {
    if (!h || h->kind != Kind::Multi) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a multi-channel convolver");
    if (in_len <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (out_len > in_len + h->K - 1 || out_len <= 0)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch");
    const int64_t L = h->eng->hop();
    out_end = std::min(out_end, out_len);
    if (out_begin < 0 || out_begin >= out_end || out_begin % L != 0 || (out_end % L != 0 && out_end != out_len))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "conv segment: bounds must be hop multiples within the output");
    if (out_begin != 0 && out_begin != h->seg_next)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "conv segment: segments must follow each other in order");
    DeviceScope ds(h->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    order_after_last(h, s);
    if (out_begin == 0) h->eng->begin_offline(s);
    PipeCall pc(h->eng.get());
    h->eng->run(d_in, in_stride, in_len, d_out, out_stride, out_len, /*use_hist=*/false, s, out_begin / L,
                (out_end + L - 1) / L);
    mark_last(h, s);
    h->seg_next = out_end < out_len ? out_end : -1;
  });
}

int ad_conv_multi_process_device_mix(ad_conv* h, const double* d_in, int64_t in_stride, int64_t in_len,
                                     double* d_mix, int64_t mix_stride, int64_t out_len, int first_parity,
                                     int64_t out_begin, int64_t out_end, void* stream) {
  return guard([&] {
    if (!h || h->kind != Kind::Multi) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a multi-channel convolver");
    if (in_len <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (out_len > in_len + h->K - 1 || out_len <= 0)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch");
    if (!d_mix) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "mixdown: null mix buffer");
    if (mix_stride < out_len) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "mixdown: mix stride shorter than the output");
    const int64_t L = h->eng->hop();
    if (out_end <= 0) out_end = out_len;
    out_end = std::min(out_end, out_len);
    if (out_begin < 0 || out_begin >= out_end || out_begin % L != 0 || (out_end % L != 0 && out_end != out_len))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "conv segment: bounds must be hop multiples within the output");
    if (out_begin != 0 && out_begin != h->seg_next)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "conv segment: segments must follow each other in order");
    DeviceScope ds(h->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    order_after_last(h, s);
    if (out_begin == 0) h->eng->begin_offline(s);
    const int64_t jb = out_begin / L, je = (out_end + L - 1) / L;
    PipeCall pc(h->eng.get());
    if (h->eng->can_mix()) {
      const MixOut mix{d_mix, mix_stride, first_parity & 1};
      h->eng->run(d_in, in_stride, in_len, nullptr, 0, out_len, /*use_hist=*/false, s, jb, je, false, &mix);
    } else {  // hop < 2048: per-channel outputs into scratch, then k_mixdown (same sums)
      const int C = h->eng->channels();
      h->mix_scratch.reserve((size_t)C * out_len);
      h->eng->run(d_in, in_stride, in_len, h->mix_scratch.p, out_len, out_len, false, s, jb, je);
      launch_mixdown(h->mix_scratch.p + out_begin, C, out_len, out_end - out_begin, d_mix + out_begin, mix_stride,
                     first_parity & 1, s);
      AD_HIP(hipGetLastError());
    }
    mark_last(h, s);
    h->seg_next = out_end < out_len ? out_end : -1;
  });
}

int ad_conv_ols_process_multi(ad_conv* h, const double* const* in, double* const* out, int channels, int64_t n) {
  // OverlapSave.Process (overlap_save.go:126-254) of every channel of a
  // multi-channel handle, host buffers in and out (n + K - 1 samples each)
  return guard([&] {
    if (!h || h->kind != Kind::Multi) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a multi-channel convolver");
    if (channels != h->channels)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: channel count mismatch: handle has " + std::to_string(h->channels) +
                                          ", got " + std::to_string(channels));
    if (n <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (!in || !out) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null channel pointer array");
    for (int c = 0; c < channels; ++c)
      if (!in[c] || !out[c]) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null channel buffer");
    DeviceScope ds(h->device);
    h->seg_next = -1;
    batch_convolve_multi(h, in, channels, n, out, n + h->K - 1);
  });
}

// --- multi-channel streaming (persistent frequency-domain delay line) --------

int ad_conv_multi_stream_create(const double* kernels, int n_ir, int64_t K, int64_t block_size, int channels,
                                const int32_t* ir_index, int device, ad_conv** out) {
  // NewStreamingOverlapSave (streaming_overlap_save.go:45-84) for `channels`
  // channels sharing n_ir kernels: one handle, one launch per kernel per block
  return create_guarded(out, [&]() -> ad_conv* {
    if (K <= 0 || !kernels || n_ir <= 0) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    if (block_size <= 0)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "conv: blockSize must be positive, got " + std::to_string(block_size));
    if (channels <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "channels must be positive");
    // The hop: the largest power-of-two divisor of the block when it is >= 256
    // (or the block itself, a power of two >= 64): every call is whole blocks.
    // Any other block size (480, 960, 1000, 4800, < 64 ...) carries the
    // unfinished block between calls as the single-channel handle does
    // (setup_stream_engine): hop = nextPow2(B), at least K/64 (<= 64
    // partitions per K2 row wave) and 64, at most 8192; a call transforms the
    // <= ceil((hop - 1 + B) / hop) blocks it touches, so it costs FFT blocks
    // and never a hop below 256 on a long IR (B = 4800 used to run at hop 64:
    // 2048 partitions at K = 131072).
    int64_t hop = largest_pow2_divisor(block_size, 8192);
    bool partial = false;
    if (hop < 256 && hop != block_size) {
      hop = std::min<int64_t>(8192, std::max<int64_t>(64, std::max(next_pow2(block_size), next_pow2((K + 63) / 64))));
      partial = (block_size % hop) != 0;
    }
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_conv> h(new_handle(Kind::MultiStream, dev));
    h->K = K;
    h->hop = hop;
    h->block_size = block_size;
    h->fft_size = next_pow2(block_size + K - 1);  // FFTSize() of the reference streaming convolver
    h->channels = channels;
    h->partial = partial;
    h->part_fill = 0;
    const int64_t blocks = partial ? (hop - 1 + block_size + hop - 1) / hop : block_size / hop;
    const int jc = (int)std::max<int64_t>(1, std::min<int64_t>(blocks, 4096));
    h->eng.reset(new Upols(dev, kernels, n_ir, K, (int)hop, channels, ir_index, jc, h->stream));
    h->eng->reset_stream(h->stream);
    if (partial) {
      h->carry_w = (hop + block_size + 1) / 2 * 2;  // even: 16-byte aligned rows
      h->ms_out_w = blocks * hop;
      for (auto& b : h->carry) {
        b.alloc((size_t)channels * h->carry_w);
        AD_HIP(hipMemsetAsync(b.p, 0, b.n * sizeof(double), h->stream));
      }
      h->ms_out.alloc((size_t)channels * h->ms_out_w);
    }
    AD_HIP(hipStreamSynchronize(h->stream));
    return h.release();
  });
}

namespace {
// One block of every channel of a multi-channel streaming handle (device
// buffers).  Partial form: the call's block is appended after the carried
// samples of the unfinished block (part_fill of them) in carry[cur], the
// engine transforms every block they touch (zeros past the last sample; an
// output sample depends only on inputs up to it, so the zeros never reach an
// emitted one), the call's outputs are the slice [part_fill, part_fill + B)
// of those blocks, and the samples of a still unfinished block move to the
// front of the other carry buffer; the engine steps back over that block so
// the next call transforms it again with more samples.
void multi_stream_run(ad_conv* h, const double* d_in, int64_t in_stride, double* d_out, int64_t out_stride,
                      hipStream_t s) {
  const int64_t B = h->block_size;
  if (!h->partial) {
    h->eng->run(d_in, in_stride, B, d_out, out_stride, B, /*use_hist=*/true, s);
    return;
  }
  const int C = h->channels;
  const int64_t L = h->hop, f0 = h->part_fill, tot = f0 + B, blocks = (tot + L - 1) / L, full = (tot / L) * L;
  DevBuf<double>& cur = h->carry[h->carry_cur];
  const size_t cw = (size_t)h->carry_w * sizeof(double);
  AD_HIP(hipMemcpy2DAsync(cur.p + f0, cw, d_in, (size_t)in_stride * sizeof(double), (size_t)B * sizeof(double), C,
                          hipMemcpyDeviceToDevice, s));
  h->eng->run(cur.p, h->carry_w, tot, h->ms_out.p, h->ms_out_w, blocks * L, /*use_hist=*/true, s);
  if (full < tot) h->eng->rewind(1);  // the last block is not complete yet
  AD_HIP(hipMemcpy2DAsync(d_out, (size_t)out_stride * sizeof(double), h->ms_out.p + f0,
                          (size_t)h->ms_out_w * sizeof(double), (size_t)B * sizeof(double), C,
                          hipMemcpyDeviceToDevice, s));
  if (tot > full) {
    DevBuf<double>& nxt = h->carry[h->carry_cur ^ 1];
    AD_HIP(hipMemcpy2DAsync(nxt.p, cw, cur.p + full, cw, (size_t)(tot - full) * sizeof(double), C,
                            hipMemcpyDeviceToDevice, s));
    h->carry_cur ^= 1;
  }
  h->part_fill = tot - full;
}
}  // namespace

int ad_conv_multi_stream_process_block_device(ad_conv* h, const double* d_in, int64_t in_stride, double* d_out,
                                              int64_t out_stride, void* stream) {
  // ProcessBlockTo (streaming_overlap_save.go:152-164) for every channel;
  // device buffers [channels][stride], block_size samples each
  return guard([&] {
    if (!h || h->kind != Kind::MultiStream)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a multi-channel streaming convolver");
    if (!d_in || !d_out) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null device buffer");
    const int64_t B = h->block_size;
    if (in_stride < B || out_stride < B) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: stride shorter than the block");
    DeviceScope ds(h->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    order_after_last(h, s);
    multi_stream_run(h, d_in, in_stride, d_out, out_stride, s);
    mark_last(h, s);
  });
}

int ad_conv_multi_stream_process_block(ad_conv* h, const double* const* in, double* const* out, int channels,
                                       int64_t n) {
  // ProcessBlockTo for every channel, host buffers (copied through pinned
  // staging inside the call; returns when the output is on the host)
  return guard([&] {
    if (!h || h->kind != Kind::MultiStream)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a multi-channel streaming convolver");
    if (channels != h->channels)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: channel count mismatch: handle has " + std::to_string(h->channels) +
                                          ", got " + std::to_string(channels));
    if (n != h->block_size)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: buffer length mismatch: expected " + std::to_string(h->block_size) +
                                          " input samples, got " + std::to_string(n));
    if (!in || !out) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null channel pointer array");
    for (int c = 0; c < channels; ++c)
      if (!in[c] || !out[c]) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null channel buffer");
    DeviceScope ds(h->device);
    const size_t cnt = (size_t)channels * n;
    if (h->pin_n < cnt) {
      if (h->pin_in) AD_HIP(hipHostFree(h->pin_in));
      if (h->pin_out) AD_HIP(hipHostFree(h->pin_out));
      h->pin_in = h->pin_out = nullptr;
      h->pin_n = 0;
      AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->pin_in), cnt * sizeof(double), hipHostMallocDefault));
      AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&h->pin_out), cnt * sizeof(double), hipHostMallocDefault));
      h->pin_n = cnt;
    }
    h->din.reserve(cnt);
    h->dout.reserve(cnt);
    hipStream_t s = h->stream;
    order_after_last(h, s);
    const int workers = cnt >= ((size_t)1 << 16) ? 8 : 0;
    parallel_for(channels, [&](int64_t c) { std::memcpy(h->pin_in + c * n, in[c], (size_t)n * sizeof(double)); },
                 workers);
    AD_HIP(hipMemcpyAsync(h->din.p, h->pin_in, cnt * sizeof(double), hipMemcpyHostToDevice, s));
    multi_stream_run(h, h->din.p, n, h->dout.p, n, s);
    AD_HIP(hipMemcpyAsync(h->pin_out, h->dout.p, cnt * sizeof(double), hipMemcpyDeviceToHost, s));
    mark_last(h, s);
    AD_HIP(hipStreamSynchronize(s));
    parallel_for(channels, [&](int64_t c) { std::memcpy(out[c], h->pin_out + c * n, (size_t)n * sizeof(double)); },
                 workers);
  });
}

// --- many-channel partitioned convolution / convolution reverb (device) --------

int ad_conv_pc_multi_create(const double* kernel, int64_t K, int min_order, int max_order, int channels, int device,
                            ad_conv** out) {
  // `channels` NewPartitionedConvolution(kernel, minOrder, maxOrder)
  // instances (partitioned.go:212-266) sharing one IR, run together
  return create_guarded(out, [&]() -> ad_conv* {
    if (K <= 0 || !kernel) AD_FAIL(AD_ERR_EMPTY_IMPULSE_RESPONSE, "conv: empty impulse response");
    if (min_order < 1)
      AD_FAIL(AD_ERR_INVALID_BLOCK_ORDER,
              "conv: invalid block order: minBlockOrder must be >= 1, got " + std::to_string(min_order));
    if (max_order < min_order)
      AD_FAIL(AD_ERR_INVALID_BLOCK_ORDER, "conv: invalid block order: maxBlockOrder (" + std::to_string(max_order) +
                                              ") must be >= minBlockOrder (" + std::to_string(min_order) + ")");
    if (min_order < 6 || min_order > 13)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "many-channel partitioned engine: latency 2^minBlockOrder must be 64..8192");
    if (channels <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "channels must be positive");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_conv> h(new_handle(Kind::PartitionedMulti, dev));
    const int64_t latency = int64_t(1) << min_order;
    const int64_t padded = ((K + latency - 1) / latency) * latency;
    h->K = K;
    h->latency = latency;
    h->block_size = latency;
    h->channels = channels;
    h->stages = partition_ir(padded, min_order, max_order);
    int64_t cover = 0;
    for (const auto& st : h->stages) cover = std::max(cover, st.start + st.count * st.part_size);
    const int64_t keff = std::min<int64_t>(K, cover);
    h->conv_len = keff;
    h->fft_size = 2 * h->stages.back().part_size;
    const int64_t pmax = std::min<int64_t>(8192, std::max<int64_t>(latency, int64_t(1) << std::min(max_order, 13)));
    h->nupd.reset(new NupolsDev(dev, kernel, keff, latency, pmax, channels, h->stream));
    AD_HIP(hipStreamSynchronize(h->stream));
    return h.release();
  });
}

int ad_conv_reverb_multi_create(const double* kernel, int64_t K, int min_order, int channels, int device,
                                ad_conv** out) {
  // NewConvolutionReverb (reverb/convolution.go:28-44) x channels: maxBlockOrder 13, wet = dry = 1
  if (out) *out = nullptr;
  if (K <= 0 || !kernel) {
    set_last_error("reverb: empty impulse response kernel");
    return AD_ERR_EMPTY_IMPULSE_RESPONSE;
  }
  return ad_conv_pc_multi_create(kernel, K, min_order, 13, channels, device, out);
}

int ad_conv_pc_multi_process_device(ad_conv* h, const double* d_in, int64_t in_stride, double* d_out,
                                    int64_t out_stride, int64_t n, void* stream) {
  // PartitionedConvolutionT.ProcessBlock (partitioned.go:348-396) of every channel
  return guard([&] {
    if (!h || h->kind != Kind::PartitionedMulti) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a many-channel partitioned convolver");
    if (n == 0) return;
    if (n < 0 || in_stride < n || out_stride < n || !d_in || !d_out)
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: bad buffer geometry");
    DeviceScope ds(h->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    order_after_last(h, s);
    h->nupd->process(d_in, in_stride, d_out, out_stride, n, /*mix=*/false, 1.0, 0.0, s);
    mark_last(h, s);
  });
}

int ad_conv_reverb_multi_process_device(ad_conv* h, double* d_buf, int64_t stride, int64_t n, void* stream) {
  // ConvolutionReverb.ProcessInPlace (convolution.go:60-85) of every channel:
  // buf = dry*buf + wet*PartitionedConvolution(buf)
  return guard([&] {
    if (!h || h->kind != Kind::PartitionedMulti) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a many-channel convolution reverb");
    if (n == 0) return;
    if (n < 0 || stride < n || !d_buf) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "conv: bad buffer geometry");
    DeviceScope ds(h->device);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    order_after_last(h, s);
    h->nupd->process(d_buf, stride, d_buf, stride, n, /*mix=*/true, h->wet, h->dry, s);
    mark_last(h, s);
  });
}

int ad_conv_reverb_multi_process(ad_conv* h, double* buf, int64_t n) {
  // host buffer [channels][n], in place; returns when the block is back on the host
  return guard([&] {
    if (!h || h->kind != Kind::PartitionedMulti) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "not a many-channel convolution reverb");
    if (n == 0) return;
    if (n < 0 || !buf) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad buffer");
    DeviceScope ds(h->device);
    const size_t cnt = (size_t)h->channels * n;
    h->din.reserve(cnt);
    hipStream_t s = h->stream;
    order_after_last(h, s);
    AD_HIP(hipMemcpyAsync(h->din.p, buf, cnt * sizeof(double), hipMemcpyHostToDevice, s));
    h->nupd->process(h->din.p, n, h->din.p, n, n, /*mix=*/true, h->wet, h->dry, s);
    AD_HIP(hipMemcpyAsync(buf, h->din.p, cnt * sizeof(double), hipMemcpyDeviceToHost, s));
    mark_last(h, s);
    AD_HIP(hipStreamSynchronize(s));
  });
}

int ad_conv_profile_enable(ad_conv* h, int enable) {
  return guard([&] {
    if (!h || !h->eng) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "handle has no FFT engine");
    h->eng->set_profiling(enable != 0);
  });
}

int ad_conv_profile_kernels(ad_conv* h, int mask) {
  return guard([&] {
    if (!h || !h->eng) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "handle has no FFT engine");
    if (mask < 0 || mask > 7) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "kernel mask: bits 0..2");
    h->eng->set_profile_mask(mask);
  });
}

int ad_conv_profile_read(ad_conv* h, double* total_ms, int64_t* launches, double* alg_bytes) {
  return guard([&] {
    if (!h || !h->eng) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "handle has no FFT engine");
    DeviceScope ds(h->device);
    h->eng->read_profile(total_ms, launches, alg_bytes);
  });
}

int ad_conv_mixdown_device(const double* d_chan, int channels, int64_t stride, int64_t len, double* d_mix,
                           int64_t mix_stride, int first_parity, void* stream) {
  return guard([&] {
    if (channels <= 0 || len <= 0) AD_FAIL(AD_ERR_EMPTY_INPUT, "empty mixdown");
    if (!d_chan || !d_mix) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "mixdown: null device buffer");
    if (mix_stride < len || (channels > 1 && stride < len))
      AD_FAIL(AD_ERR_LENGTH_MISMATCH, "mixdown: strides shorter than the mixed length");
    launch_mixdown(d_chan, channels, stride, len, d_mix, mix_stride, first_parity, reinterpret_cast<hipStream_t>(stream));
    AD_HIP(hipGetLastError());
  });
}

}  // extern "C"
