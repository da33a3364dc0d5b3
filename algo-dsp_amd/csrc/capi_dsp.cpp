// C ABI of the per-sample processors (biquad chains, Compressor, Freeverb and
// their fused effect chain) and of the FIR block filter.  Host calls copy in
// and out inside the call (cgo rule); *_device calls run asynchronously on a
// caller stream.  See include/algodsp.h for the reference API each replaces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "ad_common.hpp"
#include "dsp_kernels.hpp"

using namespace adsp;

namespace {

constexpr double kLog2Of10Div20 = 0.166096404744;  // compressor.go:27 (truncated literal, kept)
constexpr double kLn2 = 0.693147180559945309417232121458176568;
constexpr double kPi = 3.14159265358979323846264338327950288;

// dynamicsCore recalculation (core.go:480-540, 600-617), host side.
CompParams comp_params(const ad_compressor_config& g) {
  CompParams p{};
  const double fs = g.sample_rate;
  double attack = 1.0 - std::exp(-kLn2 / (g.attack_ms * 0.001 * fs));
  double release = std::exp(-kLn2 / (g.release_ms * 0.001 * fs));
  if (g.topology == 1 && g.feedback_ratio_scale) {
    attack = 1.0 - std::exp(-kLn2 / (g.attack_ms * 0.001 * fs * g.ratio));
    release = std::exp(-kLn2 / (g.release_ms * 0.001 * fs * g.ratio));
  }
  p.attack = attack;
  p.release = release;
  {
    const double b = 1.0 - release;
    p.env_c1 = 0.5 * (attack + b);
    p.env_c2 = 0.5 * (attack - b);
    p.env_k1 = 1.0 - p.env_c1;
  }
  p.threshold_log2 = g.threshold_db * kLog2Of10Div20;
  p.knee_width_log2 = g.knee_db * kLog2Of10Div20;
  p.inv_knee_width_log2 = g.knee_db > 0 ? 1.0 / p.knee_width_log2 : 0.0;
  p.half_knee = p.knee_width_log2 * 0.5;
  p.knee_on = g.knee_db > 0;
  p.cf = 1.0 - 1.0 / g.ratio;
  if (g.topology == 1 && g.feedback_ratio_scale) p.cf = g.ratio - 1.0;
  const double makeup_db = g.auto_makeup ? -(g.threshold_db * (1.0 - 1.0 / g.ratio)) : g.makeup_db;
  p.makeup_lin = std::pow(10.0, makeup_db / 20.0);
  p.lp_on = g.sidechain_high_cut_hz > 0;
  p.lp_alpha = p.lp_on ? 1.0 - std::exp(-2.0 * kPi * g.sidechain_high_cut_hz / fs) : 0.0;
  p.hp_on = g.sidechain_low_cut_hz > 0;
  p.hp_alpha = p.hp_on ? 1.0 - std::exp(-2.0 * kPi * g.sidechain_low_cut_hz / fs) : 0.0;
  p.topology_fb = g.topology == 1;
  p.detector_rms = g.detector_mode == 1;
  p.rms_n = std::max(1, (int)std::llround(g.rms_window_ms * 0.001 * fs));
  return p;
}

void check_comp_config(const ad_compressor_config& g) {
  // the setters' validation: SetRatio / SetKnee / SetAttack / SetRelease /
  // SetRMSWindow / SetThreshold / SetManualMakeupGain (core.go:131-198,
  // ranges compressor.go:16-23, core.go:10-12), SetMakeupGain, SetTopology /
  // SetDetectorMode (core.go:106-124) and recalculatePrefilter's side-chain
  // cut rules (core.go:542-564); a config any setter would reject is rejected
  // whole, before anything changes
  auto fin = [](double v) { return std::isfinite(v); };
  if (!(g.sample_rate > 0) || !fin(g.sample_rate))
    AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: sample rate must be positive and finite");
  if (!fin(g.threshold_db)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: threshold must be finite");
  if (!(g.ratio >= 1.0 && g.ratio <= 100.0)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: ratio must be in [1, 100]");
  if (!(g.knee_db >= 0.0 && g.knee_db <= 24.0)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: knee must be in [0, 24] dB");
  if (!(g.attack_ms >= 0.1 && g.attack_ms <= 1000.0))
    AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: attack must be in [0.1, 1000] ms");
  if (!(g.release_ms >= 1.0 && g.release_ms <= 5000.0))
    AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: release must be in [1, 5000] ms");
  if (!(g.rms_window_ms >= 1.0 && g.rms_window_ms <= 1000.0))
    AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: rms window must be in [1, 1000] ms");
  if (!fin(g.makeup_db)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: makeup gain must be finite");
  if (g.topology != 0 && g.topology != 1) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: invalid topology");
  if (g.detector_mode != 0 && g.detector_mode != 1) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: invalid detector mode");
  // side-chain cuts: <= 0 is off (the setters reject negatives; the ABI's
  // "<= 0: off" keeps 0 and maps nothing else), on: [1 Hz, Nyquist), low < high
  const double lo = g.sidechain_low_cut_hz, hi = g.sidechain_high_cut_hz, nyq = g.sample_rate * 0.5;
  if (!fin(lo) || !fin(hi) || lo < 0 || hi < 0)
    AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: side-chain cuts must be non-negative and finite");
  if (lo > 0 && !(lo >= 1.0 && lo < nyq)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: side-chain low-cut must be in [1, nyquist)");
  if (hi > 0 && !(hi >= 1.0 && hi < nyq)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: side-chain high-cut must be in [1, nyquist)");
  if (lo > 0 && hi > 0 && lo >= hi) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: side-chain low-cut must be below high-cut");
}

// EQ state on the device is kept per pass of <= kMaxSecPerPass sections,
// each pass a slab [C][ns][2]; the ABI's layout is [C][nsec][2].
void eq_state_from_slabs(const double* raw, int C, int nsec, double* state) {
  for (int s0 = 0; s0 < nsec; s0 += kMaxSecPerPass) {
    const int ns = std::min(kMaxSecPerPass, nsec - s0);
    for (int c = 0; c < C; ++c)
      for (int i = 0; i < ns; ++i)
        for (int k = 0; k < 2; ++k)
          state[((int64_t)c * nsec + s0 + i) * 2 + k] = raw[(size_t)C * s0 * 2 + ((size_t)c * ns + i) * 2 + k];
  }
}
void eq_state_to_slabs(const double* state, int C, int nsec, double* raw) {
  for (int s0 = 0; s0 < nsec; s0 += kMaxSecPerPass) {
    const int ns = std::min(kMaxSecPerPass, nsec - s0);
    for (int c = 0; c < C; ++c)
      for (int i = 0; i < ns; ++i)
        for (int k = 0; k < 2; ++k)
          raw[(size_t)C * s0 * 2 + ((size_t)c * ns + i) * 2 + k] = state[((int64_t)c * nsec + s0 + i) * 2 + k];
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// effect chain handle
// ---------------------------------------------------------------------------
constexpr int kFxSlots = 4;  // chunk buffers in flight (staged engine; the split EQ stage lags one chunk)
struct ad_fx_chain {
  int device = 0, channels = 0, cpad = 0;
  hipStream_t stream = nullptr;
  // EQ
  int nsec = 0;
  bool eq_uniform = true;
  DevBuf<double> sec_dev;  // uniform: [nsec][6]; per-channel: [C][nsec][6]
  DevBuf<double> eq_state;       // [C][nsec][2]
  // compressor
  bool comp_on = false;
  CompParams cp{};
  DevBuf<CompChState> cs;
  DevBuf<double> ring;
  // Freeverb
  bool verb_on = false;
  VerbParams vp{};
  DevBuf<VerbChState> vs;
  DevBuf<double> vbuf;
  // host-call staging
  DevBuf<double> work;
  // staged engine (fx_staged.hip): stage streams eq / gain / comb / allpass,
  // per-slot events, double-buffered time-major chunk buffers
  bool staged_ok = true;  // the graph runtime turns the staged engine off when it runs branches concurrently
  hipStream_t st[2] = {};
  hipEvent_t ev_last = nullptr;  // end of the last call on its caller stream (quiesce waits for it)
  hipEvent_t ev_in = nullptr;
  hipEvent_t ev[3][kFxSlots] = {};
  DevBuf<double> xT[kFxSlots], vT[kFxSlots], envT[kFxSlots], inT[kFxSlots], coT[kFxSlots];
  DevBuf<double> midT[kFxSlots];  // split K_eq: the first part's output rows
  // EQ-only chains, one K_eq part per section (fx_run_staged): section k's
  // output rows of chunk c in secT[k][c & 1], read by section k + 1 one launch later
  DevBuf<double> secT[kMaxSecPerPass][2];
  DevBuf<double> lane_dump;  // K_lanes: the stores outside the signal (kFxEqLaneDump doubles)
  // time-parallel engine (fx_tp.hip): K_eq segment states
  DevBuf<double> tp_zs, tp_carry;
  // K_carry's segment maps per (seg, nseg): M = A^seg and M^Q per section and
  // coefficient set, double-double [nsec][sets][2][4][2] (fx_tp_mats)
  std::vector<double> sec_host;
  std::map<int, std::unique_ptr<DevBuf<double>>> tp_mats;  // by segment length
  DevBuf<double> inC[kFxSlots];  // reverb input, channel-major [cpad][tmax]
  DevBuf<double> vbufC;          // Freeverb lines channel-major [channels][kVerbLen] (K_verb)
  DevBuf<double> coC;            // K_verb comb outputs [channels][2][8][kFxVerbSB] (scratch, stream st[1] only)
  bool verb_cm = false;          // vbufC (not vbuf) holds the current delay lines
  int64_t tmax = 0;
  // engine selection (ad_fx_chain_set_engine) and per-wave clock counters of
  // the first chunk of each call (ad_fx_chain_set_profiling)
  int engine = AD_FX_ENGINE_AUTO;
  int64_t chunk = 0;  // staged chunk length (0: kFxChunk)
  int last_engine = -1;  // the engine that ran the last call (ad_fx_chain_last_engine)
  // the EQ's round-off noise estimate (fx_eq_noise) and whether it is small
  // enough for the time-parallel engine to stay within the chain's 1e-12 bar
  double eq_noise = 0.0;
  bool tp_cond_ok = true;
  bool prof_on = false;
  DevBuf<unsigned long long> prof;

  ~ad_fx_chain() {
    for (hipStream_t x : st)
      if (x) {
        (void)hipStreamSynchronize(x);
        (void)lib_stream_destroy(x);
      }
    for (auto& e2 : ev)
      for (hipEvent_t e : e2)
        if (e) (void)hipEventDestroy(e);
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_last) (void)hipEventDestroy(ev_last);
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)lib_stream_destroy(stream);
    }
  }
};

namespace {

// wait for everything enqueued on the handle's own and stage streams
void fx_quiesce(ad_fx_chain* h) {
  for (hipStream_t x : h->st)
    if (x) AD_HIP(hipStreamSynchronize(x));
  if (h->ev_last) AD_HIP(hipEventSynchronize(h->ev_last));
  AD_HIP(hipStreamSynchronize(h->stream));
}

void fx_reset_comp(ad_fx_chain* h) {
  if (!h->comp_on) return;
  std::vector<CompChState> init(h->channels);
  for (auto& s : init) {  // dynamicsCore.Reset + metrics reset (core.go:572-586)
    s = CompChState{};
    s.prev_gain = 1.0;
    s.gr = 1.0;
  }
  AD_HIP(hipMemcpyAsync(h->cs.p, init.data(), init.size() * sizeof(CompChState), hipMemcpyHostToDevice, h->stream));
  AD_HIP(hipMemsetAsync(h->ring.p, 0, h->ring.n * sizeof(double), h->stream));
}

void fx_reset_verb(ad_fx_chain* h) {
  if (!h->verb_on) return;
  AD_HIP(hipMemsetAsync(h->vs.p, 0, h->vs.n * sizeof(VerbChState), h->stream));
  AD_HIP(hipMemsetAsync(h->vbuf.p, 0, h->vbuf.n * sizeof(double), h->stream));
  if (h->vbufC.p) AD_HIP(hipMemsetAsync(h->vbufC.p, 0, h->vbufC.n * sizeof(double), h->stream));
}

// The staged engine runs the chain as stage kernels over time chunks of T
// samples on three streams: chunk i's EQ/detector + gain (the caller's
// stream), combs and allpasses overlap chunk i-1's and i-2's later stages.
// Three queues in all, so the stages keep their own hardware queues
// (GPU_MAX_HW_QUEUES is 4, and streams sharing a queue serialise at every
// cross-stream wait).  Chunk buffers come in kFxSlots slots; chunk i reuses
// slot i % kFxSlots only after chunk i - kFxSlots's allpasses (the last
// reader) are done: that slot's event, recorded for chunk i - kFxSlots, is
// its latest record when chunk i is enqueued.  Feed-forward compressor only
// (the feedback topology's gain feeds its own detector).
bool fx_staged_ok(const ad_fx_chain* h) {
  // With Freeverb, beyond ~8k channels the fused kernels fill the chip on
  // their own and win (tools/fx_crossover.py: 16384 ch config 5 fused 22.2
  // vs staged 11.6 Gsamples/s; 4096 ch staged 9.7 vs fused 8.3).
  if (h->engine == AD_FX_ENGINE_FUSED) return false;
  if (h->verb_on && h->channels > 8192) return false;
  if (h->comp_on && h->cp.mode == 2) return false;  // the gate's hold counter is serial in its gain
  return h->staged_ok && (!h->comp_on || !h->cp.topology_fb) && h->nsec <= kMaxSecPerPass &&
         (h->nsec > 0 || h->comp_on || h->verb_on);
}

// Split K_eq (sections 0 .. s1-1 of chunk i beside the rest + the detector of
// chunk i - 1, one launch): the EQ recurrences of a channel group run on two
// CUs, every wave on a SIMD of its own.  Returns s1, or 0 for one pipeline.
int fx_eq_split(const ad_fx_chain* h) {
  if (h->engine == AD_FX_ENGINE_STAGED_NOSPLIT) return 0;
  if (!h->comp_on || h->nsec < 3) return 0;
  return (h->nsec + 2) / 2;  // part waves (s1 + loader) vs (ns - s1 + detector + loader)
}

// EQ-only chains (no compressor) run one K_eq part per section (see
// fx_run_staged); STAGED_NOSPLIT keeps the one-workgroup pipeline.
#ifndef AD_FX_EQ_PER_SECTION  // tools/ A/B builds
#define AD_FX_EQ_PER_SECTION 1
#endif
#ifndef AD_FX_EQ_PER_SECTION_MAXCH
// above this many channels the one-workgroup-per-group kernel fills the chip and
// wins (tools/eq_cross.py, profiles/r05_eq_cross.txt: per-section / whole-chain
// Msamples/s at 4096 ch 39.4 / 38.2, 8192 ch 44.9 / 60.7, 16384 ch 47.9 / 85.2)
#define AD_FX_EQ_PER_SECTION_MAXCH 4096
#endif
// EQ-only chains without Freeverb run K_lanes (fx_eq_lanes.hip): the sections
// across the lanes of a DPP row, one launch over the whole call, in place on
// the user buffer (no transposes, no chunks).
#ifndef AD_FX_EQ_LANES  // tools/ A/B builds
#define AD_FX_EQ_LANES 1
#endif
#ifndef AD_FX_EQ_LANES_MAXCH
// above this many channels the one-workgroup-per-channel-group kernel fills
// the chip and wins (tools/eq_lanes_bench.py: 8192 ch 69.6 / 60.2, 16384 ch
// 79.1 / 84.8 Gsamples/s, lanes / one workgroup per group)
#define AD_FX_EQ_LANES_MAXCH 8192
#endif
bool fx_eq_lanes(const ad_fx_chain* h) {
  return AD_FX_EQ_LANES && h->engine != AD_FX_ENGINE_STAGED_NOSPLIT && !h->comp_on && !h->verb_on && h->nsec >= 1 &&
         h->nsec <= kMaxSecPerPass && h->channels <= AD_FX_EQ_LANES_MAXCH;
}

bool fx_eq_per_section(const ad_fx_chain* h) {
  return AD_FX_EQ_PER_SECTION && h->engine != AD_FX_ENGINE_STAGED_NOSPLIT && !h->comp_on && h->nsec >= 2 &&
         h->nsec <= kMaxSecPerPass && h->cpad <= AD_FX_EQ_PER_SECTION_MAXCH;
}

constexpr int64_t kFxChunk = 16384;  // staged engine: samples per stage chunk
constexpr int kFxProfWords = 32;

// The profile counters of this call's first chunk (or nullptr).
unsigned long long* fx_prof_begin(ad_fx_chain* h, size_t words, hipStream_t s) {
  if (!h->prof_on) return nullptr;
  h->prof.reserve(words);
  AD_HIP(hipMemsetAsync(h->prof.p, 0, h->prof.n * sizeof(unsigned long long), s));
  return h->prof.p;
}

// Raise the chunk row stride tmax shared by both engines.  A buffer of either
// engine that a raised stride would overrun is released here, so the engine
// that next uses it reallocates it at cpad * tmax (alternating
// engines with growing calls wrote past the other engine's buffers).
void fx_grow_tmax(ad_fx_chain* h, int64_t t) {
  if (t <= h->tmax) return;
  const size_t r = (size_t)h->cpad * t;
  for (int k = 0; k < kFxSlots; ++k) {
    for (DevBuf<double>* b : {&h->xT[k], &h->vT[k], &h->envT[k], &h->inT[k], &h->midT[k], &h->inC[k]})
      if (b->p && b->n < r) b->release();
    if (h->coT[k].p && h->coT[k].n < r * kVerbCombs) h->coT[k].release();
  }
  for (auto& sk : h->secT)
    for (auto& b : sk)
      if (b.p && b.n < r) b.release();
  h->tmax = t;
}

void fx_run_staged(ad_fx_chain* h, double* d_buf, int64_t stride, int64_t n, hipStream_t s) {
  const bool eq = h->nsec > 0, comp = h->comp_on, verb = h->verb_on;
  if (fx_eq_lanes(h)) {
    if (!h->lane_dump.p) h->lane_dump.alloc(kFxEqLaneDump);
    FxEqLaneArgs a{};
    a.buf = d_buf;
    a.stride = stride;
    a.n = n;
    a.channels = h->channels;
    a.eq.nsec = h->nsec;
    a.eq.sec = h->sec_dev.p;
    a.eq.sec_ch_stride = h->eq_uniform ? 0 : (int64_t)h->nsec * kSecStride;
    a.eq.state = h->eq_state.p;
    a.dump = h->lane_dump.p;
    // g1: every section after the first has pre-gain 1.0 in every table, so
    // the kernel multiplies only the input by section 0's pre-gain
    bool g1 = true;
    const size_t sets = h->sec_host.size() / ((size_t)h->nsec * kSecStride);
    for (size_t t = 0; t < sets && g1; ++t)
      for (int k = 1; k < h->nsec; ++k)
        if (h->sec_host[(t * h->nsec + k) * kSecStride] != 1.0) g1 = false;
    launch_fx_eq_lanes(a, g1, s);
    AD_HIP(hipGetLastError());
    return;
  }
  const int64_t T = std::min(h->chunk > 0 ? h->chunk : kFxChunk, n);
  if (!h->st[0]) {
    for (auto& x : h->st) AD_HIP(lib_stream_create(&x));
    for (auto& e2 : h->ev)
      for (auto& e : e2) AD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    AD_HIP(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
  }
  const bool need_x = eq || comp, need_v = comp || (eq && !verb);
  const int s1 = fx_eq_split(h);
  {
    // Every buffer a kernel indexes at row stride tmax must hold cpad * tmax
    // rows: tmax is shared with the time-parallel engine, which may have
    // raised it without sizing this engine's buffers (each buffer's own
    // capacity is checked, not tmax).
    const size_t r = (size_t)h->cpad * std::max(T, h->tmax);
    auto shortb = [](const DevBuf<double>& b, size_t want) { return !b.p || b.n < want; };
    bool grow = false;
    for (int k = 0; k < kFxSlots; ++k)
      grow = grow || (need_x && shortb(h->xT[k], r)) || (need_v && shortb(h->vT[k], r)) ||
             (comp && shortb(h->envT[k], r)) || (verb && (shortb(h->inT[k], r) || shortb(h->coT[k], r * kVerbCombs))) ||
             (s1 && shortb(h->midT[k], r));
    if (grow || T > h->tmax) {  // (re)size the chunk buffers once no stage is running
      for (hipStream_t x : h->st) AD_HIP(hipStreamSynchronize(x));
      AD_HIP(hipStreamSynchronize(s));
      fx_grow_tmax(h, std::max(T, h->tmax));
      for (int k = 0; k < kFxSlots; ++k) {
        if (need_x) h->xT[k].reserve(r);
        if (need_v) h->vT[k].reserve(r);
        if (comp) h->envT[k].reserve(r);
        if (verb) {
          h->inT[k].reserve(r);
          h->coT[k].reserve(r * kVerbCombs);
        }
        if (s1) h->midT[k].reserve(r);
      }
    }
  }
  // stage streams: the caller's stream runs input transpose + EQ/detector +
  // gain; st[0] the combs, st[1] the allpasses (three queues in all)
  hipStream_t sc = h->st[0], sa = h->st[1];
  enum { EE = 0, EC = 1, EA = 2 };
  if (verb) {
    AD_HIP(hipEventRecord(h->ev_in, s));
    AD_HIP(hipStreamWaitEvent(sc, h->ev_in, 0));
    AD_HIP(hipStreamWaitEvent(sa, h->ev_in, 0));
  }
  // chunk i's stage arguments (slot i % kFxSlots)
  auto chunk_args = [&](int64_t ci) {
    const int ks = (int)(ci % kFxSlots);
    const int64_t t0 = ci * T;
    FxStageArgs a{};
    a.channels = h->channels;
    a.cpad = h->cpad;
    a.len = std::min(T, n - t0);
    a.buf = d_buf + t0;
    a.stride = stride;
    a.xT = h->xT[ks].p;
    a.vT = h->vT[ks].p;
    a.envT = h->envT[ks].p;
    a.inT = h->inT[ks].p;
    a.coT = h->coT[ks].p;
    a.tmax = h->tmax;
    a.eq.nsec = h->nsec;
    a.eq.sec = h->sec_dev.p;
    a.eq.sec_ch_stride = h->eq_uniform ? 0 : (int64_t)h->nsec * kSecStride;
    a.eq.state = h->eq_state.p;
    a.cp = h->cp;
    a.cs = h->cs.p;
    a.rms_ring = h->ring.p;
    a.vp = h->vp;
    a.vs = h->vs.p;
    a.vbuf = h->vbuf.p;
    return a;
  };
  if (fx_eq_per_section(h)) {
    // EQ-only chain (a12-a14), one K_eq part per section: launch i runs section
    // k of chunk i - k for every k, each part a workgroup of its own (one
    // section wave and a loader: the section has a SIMD and a CU to itself),
    // reading section k - 1's rows of that chunk, which the previous launch
    // wrote into secT[k - 1][chunk & 1]; the last section writes vT (inT with
    // Freeverb), and that chunk's later stages follow the launch.  The bits
    // are the single-part kernel's: every section runs the reference
    // operations on the same samples, its state carried across chunks.
    const int ns = h->nsec;
    const size_t r = (size_t)h->cpad * std::max(T, h->tmax);
    for (int k = 0; k + 1 < ns; ++k)
      for (auto& b : h->secT[k]) b.reserve(r);
    const int64_t nch = (n + T - 1) / T;
    int kl = 0;
    for (int64_t li = 0; li < nch + ns - 1; ++li) {
      const int64_t cd = li - (ns - 1);  // the chunk whose last section runs in this launch
      if (li < nch) launch_fx_transpose_in(chunk_args(li), chunk_args(li).xT, s);
      // inT / coT of slot cd % kFxSlots: chunk cd - kFxSlots's allpasses are done
      if (verb && cd >= kFxSlots) AD_HIP(hipStreamWaitEvent(s, h->ev[EA][cd % kFxSlots], 0));
      FxStageArgs e = chunk_args(std::min(li, nch - 1));
      e.nparts = 0;
      for (int k = 0; k < ns; ++k) {
        const int64_t c = li - k;
        if (c < 0 || c >= nch) continue;
        const FxStageArgs ac = chunk_args(c);
        const double* in = k == 0 ? ac.xT : h->secT[k - 1][c & 1].p;
        double* out = k == ns - 1 ? (verb ? ac.inT : ac.vT) : h->secT[k][c & 1].p;
        e.part[e.nparts++] = FxEqPart{k, 1, 0, ac.len, in, out, nullptr};
      }
      launch_fx_eq_sec(e, s);
      if (cd < 0) continue;
      const FxStageArgs b = chunk_args(cd);
      if (!verb) {
        launch_fx_transpose_out(b, b.vT, s);
        continue;
      }
      kl = (int)(cd % kFxSlots);
      AD_HIP(hipEventRecord(h->ev[EE][kl], s));
      AD_HIP(hipStreamWaitEvent(sc, h->ev[EE][kl], 0));
      launch_fx_comb(b, sc);
      AD_HIP(hipEventRecord(h->ev[EC][kl], sc));
      AD_HIP(hipStreamWaitEvent(sa, h->ev[EC][kl], 0));
      launch_fx_allpass(b, sa);
      AD_HIP(hipEventRecord(h->ev[EA][kl], sa));
    }
    AD_HIP(hipGetLastError());
    if (verb) AD_HIP(hipStreamWaitEvent(s, h->ev[EA][kl], 0));
    return;
  }
  if (s1) {
    // Split K_eq: launch i runs part A (sections 0 .. s1-1) of chunk i and
    // part B (sections s1 .. ns-1 + detector) of chunk i - 1, which read A's
    // rows of chunk i - 1 from midT; chunk i - 1's later stages follow.  A
    // slot is rewritten (transpose / part A of chunk i) only after chunk
    // i - kFxSlots's allpasses, enqueued kFxSlots - 1 iterations earlier.
    const int64_t nch = (n + T - 1) / T;
    int kl = 0;
    for (int64_t ci = 0; ci <= nch; ++ci) {
      FxStageArgs e{};
      if (ci < nch) {
        const int ks = (int)(ci % kFxSlots);
        FxStageArgs a = chunk_args(ci);
        if (verb && ci >= kFxSlots) AD_HIP(hipStreamWaitEvent(s, h->ev[EA][ks], 0));
        launch_fx_transpose_in(a, a.xT, s);
        e = a;
        e.part[e.nparts++] = FxEqPart{0, s1, 0, a.len, a.xT, h->midT[ks].p, nullptr};
      }
      if (ci > 0) {
        const FxStageArgs b = chunk_args(ci - 1);
        if (ci == nch) e = b;
        e.part[e.nparts++] = FxEqPart{s1, h->nsec - s1, 1, b.len, h->midT[(ci - 1) % kFxSlots].p, b.vT, b.envT};
        if (ci == 1) e.prof = fx_prof_begin(h, kFxProfWords, s);
        launch_fx_eq_parts(e, s);
        launch_fx_gain(b, !verb, s);
        if (verb) {
          kl = (int)((ci - 1) % kFxSlots);
          AD_HIP(hipEventRecord(h->ev[EE][kl], s));
          AD_HIP(hipStreamWaitEvent(sc, h->ev[EE][kl], 0));
          launch_fx_comb(b, sc);
          AD_HIP(hipEventRecord(h->ev[EC][kl], sc));
          AD_HIP(hipStreamWaitEvent(sa, h->ev[EC][kl], 0));
          launch_fx_allpass(b, sa);
          AD_HIP(hipEventRecord(h->ev[EA][kl], sa));
        }
      } else {
        launch_fx_eq_parts(e, s);
      }
    }
    AD_HIP(hipGetLastError());
    if (verb) AD_HIP(hipStreamWaitEvent(s, h->ev[EA][kl], 0));
    return;
  }
  int64_t i = 0;
  int k = 0;
  for (int64_t t0 = 0; t0 < n; t0 += T, ++i) {
    k = (int)(i % kFxSlots);
    const bool reuse = i >= kFxSlots;  // slot k was used by chunk i - kFxSlots
    FxStageArgs a{};
    a.channels = h->channels;
    a.cpad = h->cpad;
    a.len = std::min(T, n - t0);
    a.buf = d_buf + t0;
    a.stride = stride;
    a.xT = h->xT[k].p;
    a.vT = h->vT[k].p;
    a.envT = h->envT[k].p;
    a.inT = h->inT[k].p;
    a.coT = h->coT[k].p;
    a.tmax = h->tmax;
    a.eq.nsec = h->nsec;
    a.eq.sec = h->sec_dev.p;
    a.eq.sec_ch_stride = h->eq_uniform ? 0 : (int64_t)h->nsec * kSecStride;
    a.eq.state = h->eq_state.p;
    a.cp = h->cp;
    a.cs = h->cs.p;
    a.rms_ring = h->ring.p;
    a.vp = h->vp;
    a.vs = h->vs.p;
    a.vbuf = h->vbuf.p;
    if (i == 0) a.prof = fx_prof_begin(h, kFxProfWords, s);
    if (verb && reuse) AD_HIP(hipStreamWaitEvent(s, h->ev[EA][k], 0));  // inT / coT of that chunk consumed
    if (eq || comp) {
      launch_fx_transpose_in(a, a.xT, s);
      launch_fx_eq(a, comp, (verb && !comp) ? kFxOutInT : kFxOutVT, s);
      if (comp) launch_fx_gain(a, !verb, s);
      if (!comp && !verb) launch_fx_transpose_out(a, a.vT, s);
    } else {
      launch_fx_transpose_in(a, a.inT, s);
    }
    if (verb) {
      AD_HIP(hipEventRecord(h->ev[EE][k], s));
      AD_HIP(hipStreamWaitEvent(sc, h->ev[EE][k], 0));
      launch_fx_comb(a, sc);
      AD_HIP(hipEventRecord(h->ev[EC][k], sc));
      AD_HIP(hipStreamWaitEvent(sa, h->ev[EC][k], 0));
      launch_fx_allpass(a, sa);
      AD_HIP(hipEventRecord(h->ev[EA][k], sa));
    }
  }
  AD_HIP(hipGetLastError());
  if (verb) AD_HIP(hipStreamWaitEvent(s, h->ev[EA][k], 0));  // the last chunk's allpasses follow all work
}

// The EQ's round-off noise relative to its signal, as the time-parallel
// engine's distance from the serial recurrence: eps sqrt(sum_k NG_k) over the
// sections of the worst coefficient set, NG = (1 + a2) / ((1 - a2)((1 + a2)^2 -
// a1^2)) the noise gain of a section's all-pole part (infinite for poles on or
// outside the unit circle).  Both the serial recurrence and the chained
// segment starts carry that noise, so the two differ by about this much:
// tools/tp_cond.py simulates the engine's arithmetic against the oracle, e.g.
// a 40 Hz highpass at 48 kHz (config 5) 3.5e-13 estimated vs 3.5e-13
// simulated, 40 Hz at 96 kHz 9.9e-13 vs 1.4e-12, 10 Hz at 192 kHz 2.2e-11 vs
// 3.7e-11 (the simulated distance runs up to 1.7x the estimate).  Past
// kFxTpNoiseMax the chain keeps the bit-exact staged engine.
constexpr double kFxTpNoiseMax = 4.5e-13;
double fx_eq_noise(const std::vector<double>& tab, int sets, int nsec) {
  typedef long double ld;
  double worst = 0.0;
  for (int c = 0; c < sets; ++c) {
    ld sum = 0;
    for (int k = 0; k < nsec; ++k) {
      const double* g = tab.data() + ((size_t)c * nsec + k) * kSecStride;
      const ld a1 = g[4], a2 = g[5];
      // the stability triangle |a2| < 1, |a1| < 1 + a2 (d alone is
      // also positive for a2 > 1, |a1| > 1 + a2, e.g. a pole at -3.41)
      if (!(std::fabs(a2) < 1) || !(std::fabs(a1) < 1 + a2)) return INFINITY;  // not stable: no estimate
      const ld d = (1 - a2) * ((1 + a2) * (1 + a2) - a1 * a1);
      if (!(d > 0) || !std::isfinite((double)d)) return INFINITY;
      sum += (1 + a2) / d;
    }
    worst = std::max(worst, (double)(std::sqrt(sum) * std::ldexp(1.0L, -52)));
  }
  return worst;
}

// The time-parallel engine (fx_tp.hip): per chunk of T samples, the caller's
// stream runs the input transpose and the three EQ launches (K_eqz, K_carry,
// K_eqx); st[0] the detector (serial per channel) and the gain of that chunk;
// st[1] the reverb.  So chunk i's EQ overlaps chunk i-1's detector and chunk
// i-2's reverb.  A slot is reused only after st[1] is done with it (the
// detector and the gain precede st[1]'s work on every chunk).
#ifndef AD_FX_TP_CHUNK  // tools/ A/B builds only
#define AD_FX_TP_CHUNK 49152  // config 5 (tools/fx_chunk_sweep.py, round 5 schedule + 64-row detector batches): 24576 11.7, 32768 12.3-12.4, 49152 12.5-12.6, 65536 12.4-12.5 Gsamples/s
#endif
constexpr int64_t kFxTpChunk = AD_FX_TP_CHUNK;
#ifndef AD_FX_TP_SERIAL_TAIL  // tools/ A/B builds
#define AD_FX_TP_SERIAL_TAIL 0
#endif
constexpr bool kFxTpSerialTail = AD_FX_TP_SERIAL_TAIL;  // gain + Freeverb on the caller's stream (fx_run_tp)
#ifndef AD_FX_TP_GAIN_ON_S  // tools/ A/B builds
#define AD_FX_TP_GAIN_ON_S 1
#endif
// chunk i - 1's gain on the caller's stream behind chunk i's EQ, its Freeverb on
// st[1] after it: the detector's stream runs detectors back to back (fx_run_tp)
constexpr bool kFxTpGainOnS = AD_FX_TP_GAIN_ON_S;
constexpr int kFxTpSeg = 64;     // K_eq segment (samples), at least
constexpr size_t kFxTpMatsCached = 8;  // segment lengths whose maps stay cached

// K_carry's maps for a chunk cut into nseg segments of seg samples, per
// coefficient set (layout: fx_tp_mat_stride in dsp_kernels.hpp): the cascade's
// zero-input step A (2 nsec x 2 nsec, block lower triangular: section k's
// input is section k-1's output), its segment map B = A^seg as 2 x 2 blocks,
// and per section the scan maps B(k,k)^(2^i).  Computed in
// 64-bit-mantissa long double and stored as double-double pairs.  Built once
// per segment length and coefficient table (the maps do not depend on the
// segment count).
const double* fx_tp_mats(ad_fx_chain* h, int seg, hipStream_t s) {
  {
    auto it = h->tp_mats.find(seg);
    if (it != h->tp_mats.end()) return it->second->p;
  }
  if (h->tp_mats.size() >= kFxTpMatsCached) {  // a caller cycling through chunk lengths: drop the cache
    for (hipStream_t x : h->st) AD_HIP(hipStreamSynchronize(x));
    AD_HIP(hipStreamSynchronize(s));
    h->tp_mats.clear();
  }
  auto& slot = h->tp_mats[seg];
  const int sets = h->eq_uniform ? 1 : h->channels, nsec = h->nsec, D = 2 * nsec;
  typedef long double ld;
  typedef std::vector<ld> mat;  // D x D row-major
  auto mul = [D](const mat& x, const mat& y) {
    mat r((size_t)D * D, 0);
    for (int i = 0; i < D; ++i)
      for (int k = 0; k < D; ++k) {
        const ld v = x[(size_t)i * D + k];
        if (v != 0)
          for (int j = 0; j < D; ++j) r[(size_t)i * D + j] += v * y[(size_t)k * D + j];
      }
    return r;
  };
  auto pw = [&](mat b, int e) {
    mat m((size_t)D * D, 0);
    for (int i = 0; i < D; ++i) m[(size_t)i * D + i] = 1;
    for (; e > 0; e >>= 1) {
      if (e & 1) m = mul(m, b);
      b = mul(b, b);
    }
    return m;
  };
  auto m2 = [](const ld* x, const ld* y, ld* r) {
    const ld u[4] = {x[0] * y[0] + x[1] * y[2], x[0] * y[1] + x[1] * y[3], x[2] * y[0] + x[3] * y[2],
                     x[2] * y[1] + x[3] * y[3]};
    for (int i = 0; i < 4; ++i) r[i] = u[i];
  };
  auto put = [](double* o, ld v) {
    o[0] = (double)v;
    o[1] = (double)(v - (ld)o[0]);
  };
  const int stride = fx_tp_mat_stride(nsec);
  std::vector<double> t((size_t)sets * stride, 0.0);
  for (int c = 0; c < sets; ++c) {
    const double* q = h->sec_host.data() + (size_t)c * nsec * kSecStride;
    // A's column i: one zero-input step of the cascade (section.go:47-53)
    // from the unit state e_i; state order (d0, d1) per section
    mat A((size_t)D * D, 0);
    for (int i = 0; i < D; ++i) {
      std::vector<ld> st(D, 0);
      st[i] = 1;
      ld x = 0;
      for (int k = 0; k < nsec; ++k) {
        const double* g = q + k * kSecStride;
        const ld v = x * g[0];
        const ld y = g[1] * v + st[2 * k];
        A[(size_t)(2 * k) * D + i] = g[2] * v - g[4] * y + st[2 * k + 1];
        A[(size_t)(2 * k + 1) * D + i] = g[3] * v - g[5] * y;
        x = y;
      }
    }
    const mat B = pw(A, seg);
    double* o = t.data() + (size_t)c * stride;
    for (int k = 0; k < nsec; ++k)
      for (int j = 0; j <= k; ++j)
        for (int e = 0; e < 4; ++e)
          put(o + ((size_t)k * nsec + j) * 8 + 2 * e, B[(size_t)(2 * k + e / 2) * D + 2 * j + e % 2]);
    for (int k = 0; k < nsec; ++k) {  // B(k,k) and its repeated squares
      ld P[4];
      for (int e = 0; e < 4; ++e) P[e] = B[(size_t)(2 * k + e / 2) * D + 2 * k + e % 2];
      for (int i = 0; i < kFxTpScan; ++i) {
        for (int e = 0; e < 4; ++e) put(o + ((size_t)nsec * nsec + k * kFxTpScan + i) * 8 + 2 * e, P[e]);
        m2(P, P, P);
      }
    }
  }
  slot.reset(new DevBuf<double>());
  slot->alloc(t.size());
  AD_HIP(hipMemcpy(slot->p, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
  return slot->p;
}

// K_comb warm-up: samples after which the damping filter's start value is
// below 2^-60 of the run (da^wu < 2^-60); 0 without damping; a filter that
// forgets too slowly runs each window as one segment.
int fx_comb_warmup(const VerbParams& vp) {
  const double da = std::fabs(vp.damp_a);
  if (da == 0.0) return 0;
  if (da >= 0.97) return 1 << 20;
  return (int)std::ceil(-60.0 * std::log(2.0) / std::log(da));
}

void fx_run_tp(ad_fx_chain* h, double* d_buf, int64_t stride, int64_t n, hipStream_t s) {
  const bool eq = h->nsec > 0, comp = h->comp_on, verb = h->verb_on;
  const int64_t T = std::min(h->chunk > 0 ? h->chunk : kFxTpChunk, n);
  if (!h->st[0]) {
    for (auto& x : h->st) AD_HIP(lib_stream_create(&x));
    for (auto& e2 : h->ev)
      for (auto& e : e2) AD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    AD_HIP(hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming));
  }
  {
    // each buffer's own capacity against cpad * tmax (tmax is shared with the
    // staged engine, which may have raised it; see fx_run_staged)
    const size_t r = (size_t)h->cpad * std::max(T, h->tmax);
    auto shortb = [](const DevBuf<double>& b, size_t want) { return !b.p || b.n < want; };
    bool grow = (verb && shortb(h->coC, (size_t)h->channels * 2 * kVerbCombs * kFxVerbSB)) ||
                (eq && shortb(h->tp_zs, (size_t)kFxTpMaxSeg * h->nsec * h->cpad * 2));
    for (int k = 0; k < kFxSlots; ++k)
      grow = grow || shortb(h->xT[k], r) || (eq && shortb(h->vT[k], r)) || (comp && shortb(h->envT[k], r)) ||
             (comp && verb && shortb(h->inC[k], r));
    if (grow || T > h->tmax) {  // (re)size once no stage is running
      for (hipStream_t x : h->st) AD_HIP(hipStreamSynchronize(x));
      AD_HIP(hipStreamSynchronize(s));
      fx_grow_tmax(h, std::max(T, h->tmax));
      for (int k = 0; k < kFxSlots; ++k) {
        h->xT[k].reserve(r);
        if (eq) h->vT[k].reserve(r);
        if (comp) h->envT[k].reserve(r);
        if (comp && verb) h->inC[k].reserve(r);
      }
      if (verb) h->coC.reserve((size_t)h->channels * 2 * kVerbCombs * kFxVerbSB);  // two halves (k_fxtp_verb_pipe)
      if (eq) {
        h->tp_zs.reserve((size_t)kFxTpMaxSeg * h->nsec * h->cpad * 2);
        h->tp_carry.reserve((size_t)kFxTpMaxSeg * h->nsec * h->cpad * 4);
      }
    }
  }
#ifdef AD_FX_TP_SERIAL  // tools/ builds only: every stage on the caller's stream (isolated kernel times)
  hipStream_t sd = s, sv = s;
#else
  hipStream_t sd = h->st[0], sv = h->st[1];
#endif
  enum { EE = 0, ED = 1, EA = 2 };
  if (verb && !h->verb_cm) {  // the delay lines into K_verb's channel-major layout
    h->vbufC.reserve((size_t)kVerbLen * h->channels);
    launch_vbuf_layout(h->vbuf.p, h->vbufC.p, h->cpad, h->channels, true, s);
    h->verb_cm = true;
  }
  AD_HIP(hipEventRecord(h->ev_in, s));
  AD_HIP(hipStreamWaitEvent(sd, h->ev_in, 0));
  AD_HIP(hipStreamWaitEvent(sv, h->ev_in, 0));
  const int wu = verb ? fx_comb_warmup(h->vp) : 0;
  // kFxTpSerialTail: the gain + Freeverb of a chunk on the caller's stream
  // (see the loop); slot reuse then follows from that stream's order: chunk i's
  // transpose and EQ come after chunk i - 1's (and so i - kFxSlots's) tail,
  // whose wait on the detector orders every reader of the slot before them
  FxStageArgs prev{};
  auto tail = [&](const FxStageArgs& p, int kp) {
    AD_HIP(hipStreamWaitEvent(s, h->ev[ED][kp], 0));
    FxStageArgs b = p;
    b.buf = h->inC[kp].p;
    b.stride = h->tmax;
    launch_fx_gain(b, true, s);
    launch_fxtp_verb(p, h->inC[kp].p, h->tmax, h->vbufC.p, h->coC.p, wu, s);
  };
  // kFxTpGainOnS: chunk i - 1's gain on s (it waits there for its detector,
  // by then chunk i's EQ is queued ahead of it) and its Freeverb on sv behind
  // the gain; EE[kp] is re-recorded after the gain (the detector's wait on the
  // EQ's record was already enqueued)
  // (inC[kp]'s previous reader, chunk i - 1 - kFxSlots's Freeverb, is ordered
  // before the gain by s's own wait on that slot at the top of the loop; on
  // CU-masked streams of their own, the detector and the gain measured 2x slower)
  auto gain_verb = [&](const FxStageArgs& p, int kp) {
    AD_HIP(hipStreamWaitEvent(s, h->ev[ED][kp], 0));
    FxStageArgs b = p;
    b.buf = h->inC[kp].p;
    b.stride = h->tmax;
    launch_fx_gain(b, true, s);
    AD_HIP(hipEventRecord(h->ev[EE][kp], s));
    AD_HIP(hipStreamWaitEvent(sv, h->ev[EE][kp], 0));
    launch_fxtp_verb(p, h->inC[kp].p, h->tmax, h->vbufC.p, h->coC.p, wu, sv, true);
    AD_HIP(hipEventRecord(h->ev[EA][kp], sv));
  };
  const bool gain_on_s = kFxTpGainOnS && !kFxTpSerialTail && comp && verb;
  int64_t i = 0;
  int k = 0;
  for (int64_t t0 = 0; t0 < n; t0 += T, ++i) {
    k = (int)(i % kFxSlots);
    FxStageArgs a{};
    a.channels = h->channels;
    a.cpad = h->cpad;
    a.len = std::min(T, n - t0);
    a.buf = d_buf + t0;
    a.stride = stride;
    a.xT = h->xT[k].p;
    a.vT = eq ? h->vT[k].p : h->xT[k].p;  // the EQ output (or the input)
    a.envT = h->envT[k].p;
    a.inT = nullptr;
    a.tmax = h->tmax;
    a.eq.nsec = h->nsec;
    a.eq.sec = h->sec_dev.p;
    a.eq.sec_ch_stride = h->eq_uniform ? 0 : (int64_t)h->nsec * kSecStride;
    a.eq.state = h->eq_state.p;
    a.cp = h->cp;
    a.cs = h->cs.p;
    a.rms_ring = h->ring.p;
    a.vp = h->vp;
    a.vs = h->vs.p;
    a.vbuf = h->vbuf.p;
    if (i >= kFxSlots && !(kFxTpSerialTail && comp && verb))
      AD_HIP(hipStreamWaitEvent(s, h->ev[EA][k], 0));  // slot k consumed
    if (eq || comp) launch_fx_transpose_in(a, a.xT, s);  // the rows the EQ / the detector read
    if (eq) {
      FxTpEqArgs e{};
      e.channels = h->channels;
      e.cpad = h->cpad;
      e.len = a.len;
      e.seg = (int)std::max<int64_t>(kFxTpSeg, ((a.len + kFxTpMaxSeg - 1) / kFxTpMaxSeg + 15) / 16 * 16);
      e.nseg = (int)((a.len + e.seg - 1) / e.seg);
      e.xT = a.xT;
      e.vT = a.vT;
      e.eq = a.eq;
      e.zs = h->tp_zs.p;
      e.sdd = h->tp_carry.p;
      e.mats = fx_tp_mats(h, e.seg, s);
      e.mat_sets = h->eq_uniform ? 1 : h->channels;
      launch_fxtp_eq(e, false, s);
      launch_fxtp_carry(e, s);
      launch_fxtp_eq(e, true, s);
    }
    AD_HIP(hipEventRecord(h->ev[EE][k], s));
    if (kFxTpSerialTail && comp && verb) {
      // chunk i's detector on sd; chunk i - 1's gain and Freeverb on the
      // caller's stream behind chunk i's EQ, so the chip-wide kernels never
      // share CUs with K_verb (only the 32 detector CUs run beside both)
      AD_HIP(hipStreamWaitEvent(sd, h->ev[EE][k], 0));
      launch_fxtp_det(a, sd);
      AD_HIP(hipEventRecord(h->ev[ED][k], sd));
      if (i > 0) tail(prev, (int)((i - 1) % kFxSlots));
      prev = a;
      continue;
    }
    if (gain_on_s) {
      AD_HIP(hipStreamWaitEvent(sd, h->ev[EE][k], 0));
      launch_fxtp_det(a, sd);
      AD_HIP(hipEventRecord(h->ev[ED][k], sd));
      if (i > 0) gain_verb(prev, (int)((i - 1) % kFxSlots));
      prev = a;
      continue;
    }
    if (comp) {
      AD_HIP(hipStreamWaitEvent(sd, h->ev[EE][k], 0));
      launch_fxtp_det(a, sd);
      if (verb) {
        // the compressor output channel-major into inC on the detector's
        // stream (the reverb's stream is the longer one), then Freeverb into
        // the user buffer; inC[k] is free once chunk i - kFxSlots's reverb ran
        if (i >= kFxSlots) AD_HIP(hipStreamWaitEvent(sd, h->ev[EA][k], 0));
        FxStageArgs b = a;
        b.buf = h->inC[k].p;
        b.stride = h->tmax;
        launch_fx_gain(b, true, sd);
      }
      AD_HIP(hipEventRecord(h->ev[ED][k], sd));
      AD_HIP(hipStreamWaitEvent(sv, h->ev[ED][k], 0));
      if (verb)
        launch_fxtp_verb(a, h->inC[k].p, h->tmax, h->vbufC.p, h->coC.p, wu, sv);
      else
        launch_fx_gain(a, true, sv);
    } else {  // no compressor (AD_FX_ENGINE_TIME_PARALLEL): the EQ output back, then Freeverb in place
      AD_HIP(hipStreamWaitEvent(sv, h->ev[EE][k], 0));
      if (eq) launch_fx_transpose_out(a, a.vT, sv);
      if (verb) launch_fxtp_verb(a, a.buf, a.stride, h->vbufC.p, h->coC.p, wu, sv);
    }
    AD_HIP(hipEventRecord(h->ev[EA][k], sv));
  }
  if (kFxTpSerialTail && comp && verb) {
    tail(prev, k);  // the last chunk's gain and Freeverb, on s after its detector
    AD_HIP(hipGetLastError());
    return;
  }
  if (gain_on_s) gain_verb(prev, k);  // the last chunk's
  AD_HIP(hipGetLastError());
  AD_HIP(hipStreamWaitEvent(s, h->ev[EA][k], 0));  // the last chunk's reverb / output follows all work
}

void fx_run(ad_fx_chain* h, double* d_buf, int64_t stride, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  if (!h->ev_last) AD_HIP(hipEventCreateWithFlags(&h->ev_last, hipEventDisableTiming));
  // time-parallel: by default where the chain is already a tolerance (the
  // compressor's log2 / exp2); on request for any other chain.
  // Never for an EQ whose round-off noise gain would put its distance from
  // the serial recurrence past the chain's bar (fx_eq_noise): such chains run
  // on the staged engine, which is bit-exact.
  const bool tp_ok = fx_staged_ok(h) && (h->comp_on || h->nsec > 0 || h->verb_on) && h->tp_cond_ok;
  const bool tp = tp_ok && ((h->engine == AD_FX_ENGINE_AUTO && h->comp_on) || h->engine == AD_FX_ENGINE_TIME_PARALLEL);
  if (h->verb_on && h->verb_cm && !tp) {  // the delay lines back into vbuf's layout
    launch_vbuf_layout(h->vbuf.p, h->vbufC.p, h->cpad, h->channels, false, s);
    h->verb_cm = false;
  }
  if (fx_staged_ok(h)) {
    // an EQ-only chain keeps the staged engine (bit-exact) unless asked
    if (tp) {
      fx_run_tp(h, d_buf, stride, n, s);
      h->last_engine = AD_FX_ENGINE_TIME_PARALLEL;
    } else {
      fx_run_staged(h, d_buf, stride, n, s);
      h->last_engine =
          (fx_eq_lanes(h) || fx_eq_split(h) || fx_eq_per_section(h)) ? AD_FX_ENGINE_STAGED : AD_FX_ENGINE_STAGED_NOSPLIT;
    }
    AD_HIP(hipEventRecord(h->ev_last, s));
    return;
  }
  ChainArgs a{};
  a.buf = d_buf;
  a.stride = stride;
  a.n = n;
  a.channels = h->channels;
  a.cp = h->cp;
  a.cs = h->cs.p;
  a.rms_ring = h->ring.p;
  a.vp = h->vp;
  a.vs = h->vs.p;
  a.vbuf = h->vbuf.p;
  a.prof = fx_prof_begin(h, std::max<size_t>(kFxProfWords, (size_t)((h->channels + 63) / 64) * 16), s);
  const int post = (h->comp_on ? 2 : 0) | (h->verb_on ? 4 : 0);
  // EQ sections in passes of <= kMaxSecPerPass; the last pass fuses the
  // compressor and Freeverb stages (per-sample fusion is exact, see kernels)
  int s0 = 0;
  do {
    const int ns = std::min(kMaxSecPerPass, h->nsec - s0);
    a.eq.nsec = ns;
    a.eq.sec = h->sec_dev.p ? h->sec_dev.p + (int64_t)s0 * kSecStride : nullptr;
    a.eq.sec_ch_stride = h->eq_uniform ? 0 : (int64_t)h->nsec * kSecStride;
    // state rows of this pass: the kernel indexes [c][ns][2]; keep one
    // contiguous [C][nsec][2] array by giving each pass its own slab
    a.eq.state = h->eq_state.p + (int64_t)h->channels * s0 * 2;
    const bool last = s0 + ns >= h->nsec;
    const int stages = (ns > 0 ? 1 : 0) | (last ? post : 0);
    if (stages) launch_chain(stages, a, s);
    s0 += ns;
  } while (s0 < h->nsec);
  AD_HIP(hipGetLastError());
  AD_HIP(hipEventRecord(h->ev_last, s));
  h->last_engine = AD_FX_ENGINE_FUSED;
}

}  // namespace

namespace adsp {
// Internal (not in the C ABI): an effect-chain graph whose branches run on
// several streams keeps each chain on its caller's stream, since the staged
// engine's two extra streams per chain would outnumber the hardware queues.
void fx_chain_allow_staged(ad_fx_chain* h, bool on) {
  if (h) h->staged_ok = on;
}
}  // namespace adsp

namespace {

template <class Fn>
int fx_guard(ad_fx_chain* h, Fn&& fn) {
  return guard([&] {
    if (!h) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null effect-chain handle");
    DeviceScope ds(h->device);
    fn();
  });
}

}  // namespace

extern "C" {

void ad_compressor_default_config(ad_compressor_config* c, double sample_rate) {
  // NewCompressor defaults (compressor.go:6-13, 83-98)
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->sample_rate = sample_rate;
  c->threshold_db = -20.0;
  c->ratio = 4.0;
  c->knee_db = 6.0;
  c->attack_ms = 10.0;
  c->release_ms = 100.0;
  c->rms_window_ms = 30.0;
  c->makeup_db = 0.0;
  c->auto_makeup = 1;
  c->feedback_ratio_scale = 1;
}

int ad_compressor_validate(const ad_compressor_config* cfg) {
  return guard([&] {
    if (!cfg) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil compressor config");
    check_comp_config(*cfg);
  });
}

int ad_fx_chain_create(int channels, int device, ad_fx_chain** out) {
  if (out) *out = nullptr;
  ad_fx_chain* raw = nullptr;
  const int rc = guard([&] {
    if (channels <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "channels must be positive");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_fx_chain> h(new ad_fx_chain());
    h->device = dev;
    h->channels = channels;
    h->cpad = (channels + 63) / 64 * 64;
    AD_HIP(lib_stream_create(&h->stream));
    raw = h.release();
  });
  if (rc == AD_OK && out) *out = raw;
  return rc;
}

int ad_fx_eq_noise(const double* sections, int nsec, int sets, double* noise) {
  return guard([&] {
    if (nsec < 0 || sets < 1 || (nsec > 0 && !sections) || !noise) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad EQ section table");
    const std::vector<double> tab(sections, sections + (size_t)sets * nsec * kSecStride);
    *noise = nsec > 0 ? fx_eq_noise(tab, sets, nsec) : 0.0;
  });
}

int ad_fx_chain_set_eq(ad_fx_chain* h, const double* sections, int nsec, int per_channel) {
  return fx_guard(h, [&] {
    if (nsec < 0 || (nsec > 0 && !sections)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad EQ section table");
    fx_quiesce(h);
    const bool keep_state = nsec == h->nsec;
    h->nsec = nsec;
    h->eq_uniform = !per_channel;
    h->sec_dev.alloc((size_t)(per_channel ? h->channels : 1) * nsec * kSecStride);
    if (nsec > 0) AD_HIP(hipMemcpy(h->sec_dev.p, sections, h->sec_dev.n * sizeof(double), hipMemcpyHostToDevice));
    h->sec_host.assign(sections, sections + h->sec_dev.n);
    h->tp_mats.clear();
    h->eq_noise = nsec > 0 ? fx_eq_noise(h->sec_host, per_channel ? h->channels : 1, nsec) : 0.0;
    h->tp_cond_ok = h->eq_noise <= kFxTpNoiseMax;
    // Section state survives a coefficient update with the same section
    // count, like filterRuntime.Configure (runtime_filter_pitch_reverb.go:150-165).
    if (!keep_state || !h->eq_state.p) {
      h->eq_state.alloc((size_t)std::max(1, h->channels * nsec * 2));
      AD_HIP(hipMemset(h->eq_state.p, 0, h->eq_state.n * sizeof(double)));
    }
  });
}

int ad_fx_chain_set_compressor(ad_fx_chain* h, const ad_compressor_config* cfg) {
  return fx_guard(h, [&] {
    fx_quiesce(h);
    if (!cfg) {
      h->comp_on = false;
      return;
    }
    check_comp_config(*cfg);
    const CompParams p = comp_params(*cfg);
    const bool fresh = !h->comp_on || p.rms_n != h->cp.rms_n;
    h->cp = p;
    h->comp_on = true;
    if (fresh) {
      h->cs.alloc((size_t)h->channels);
      h->ring.alloc((size_t)h->channels * p.rms_n);
      fx_reset_comp(h);
      fx_quiesce(h);
    }
  });
}

int ad_fx_chain_set_expander(ad_fx_chain* h, const ad_compressor_config* cfg, int gate, double range_db,
                             double hold_ms) {
  // NewExpander / NewGate (expander.go:70-108, gate.go:82-126) and their setters' ranges
  return fx_guard(h, [&] {
    fx_quiesce(h);
    if (!cfg) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "nil expander config");
    ad_compressor_config g = *cfg;
    check_comp_config(g);
    if (!(g.ratio >= 1.0 && g.ratio <= 100.0)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: ratio must be in [1, 100]");
    if (!(g.knee_db >= 0.0 && g.knee_db <= 24.0)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: knee must be in [0, 24] dB");
    if (!(g.attack_ms >= 0.1 && g.attack_ms <= 1000.0))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: attack must be in [0.1, 1000] ms");
    if (!(g.release_ms >= 1.0 && g.release_ms <= 5000.0))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: release must be in [1, 5000] ms");
    if (!(range_db >= -120.0 && range_db <= 0.0)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: range must be in [-120, 0] dB");
    if (gate && !(hold_ms >= 0.0 && hold_ms <= 5000.0))
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "dynamics: hold must be in [0, 5000] ms");
    // the expander/gate core: no makeup, feedback time constants not ratio-scaled
    g.auto_makeup = 0;
    g.makeup_db = 0.0;
    g.feedback_ratio_scale = 0;
    CompParams p = comp_params(g);
    p.mode = gate ? 2 : 1;
    p.ratio_m1 = g.ratio - 1.0;
    p.range_lin = std::pow(10.0, range_db / 20.0);
    p.hold_n = gate ? (int)(hold_ms * 0.001 * g.sample_rate) : 0;
    const bool fresh = !h->comp_on || p.rms_n != h->cp.rms_n;
    h->cp = p;
    h->comp_on = true;
    if (fresh) {
      h->cs.alloc((size_t)h->channels);
      h->ring.alloc((size_t)h->channels * p.rms_n);
      fx_reset_comp(h);
      fx_quiesce(h);
    }
  });
}

int ad_fx_chain_set_freeverb(ad_fx_chain* h, double wet, double dry, double room_size, double damp, double gain) {
  return fx_guard(h, [&] {
    fx_quiesce(h);
    // SetWet/SetDry/SetRoomSize/SetDamp/SetGain (reverb.go:192-220)
    h->vp.wet = wet;
    h->vp.dry = dry;
    h->vp.feedback = room_size;
    h->vp.damp_a = damp;
    h->vp.damp_b = 1.0 - damp;
    h->vp.gain = gain;
    h->vp.ap_feedback = 0.5;
    if (!h->verb_on) {
      h->verb_on = true;
      h->vs.alloc((size_t)h->channels);
      h->vbuf.alloc((size_t)kVerbLen * h->cpad);
      fx_reset_verb(h);
      fx_quiesce(h);
    }
  });
}

int ad_fx_chain_disable_freeverb(ad_fx_chain* h) {
  return fx_guard(h, [&] { h->verb_on = false; });
}

int ad_fx_chain_reset(ad_fx_chain* h) {
  return fx_guard(h, [&] {
    if (h->eq_state.p) AD_HIP(hipMemsetAsync(h->eq_state.p, 0, h->eq_state.n * sizeof(double), h->stream));
    fx_reset_comp(h);
    fx_reset_verb(h);
    fx_quiesce(h);
  });
}

int ad_fx_chain_process(ad_fx_chain* h, double* buf, int64_t n) {
  return fx_guard(h, [&] {
    if (n < 0 || (n > 0 && !buf)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad buffer");
    if (n == 0) return;
    const size_t bytes = (size_t)h->channels * n * sizeof(double);
    h->work.reserve((size_t)h->channels * n);
    AD_HIP(hipMemcpyAsync(h->work.p, buf, bytes, hipMemcpyHostToDevice, h->stream));
    fx_run(h, h->work.p, n, n, h->stream);
    AD_HIP(hipMemcpyAsync(buf, h->work.p, bytes, hipMemcpyDeviceToHost, h->stream));
    fx_quiesce(h);
  });
}

int ad_fx_chain_process_device(ad_fx_chain* h, double* d_buf, int64_t stride, int64_t n, void* stream) {
  return fx_guard(h, [&] {
    if (n < 0 || stride < n) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad buffer geometry");
    fx_run(h, d_buf, stride, n, reinterpret_cast<hipStream_t>(stream));
  });
}

int ad_fx_chain_compressor_metrics(ad_fx_chain* h, int channel, double* input_peak, double* output_peak,
                                   double* gain_reduction) {
  return fx_guard(h, [&] {
    if (!h->comp_on) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "compressor stage not configured");
    if (channel < 0 || channel >= h->channels) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "channel out of range");
    fx_quiesce(h);
    CompChState s{};
    AD_HIP(hipMemcpy(&s, h->cs.p + channel, sizeof(s), hipMemcpyDeviceToHost));
    if (input_peak) *input_peak = s.in_peak;
    if (output_peak) *output_peak = s.out_peak;
    if (gain_reduction) *gain_reduction = s.gr;
  });
}

int ad_fx_chain_eq_state(ad_fx_chain* h, double* state, int64_t cap) {
  return fx_guard(h, [&] {
    const int64_t need = (int64_t)h->channels * h->nsec * 2;
    if (cap < need) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "state buffer too small");
    if (need > 0 && !state) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null state buffer");
    fx_quiesce(h);
    std::vector<double> raw((size_t)need);
    if (need) AD_HIP(hipMemcpy(raw.data(), h->eq_state.p, need * sizeof(double), hipMemcpyDeviceToHost));
    eq_state_from_slabs(raw.data(), h->channels, h->nsec, state);
  });
}

int ad_fx_chain_set_eq_state(ad_fx_chain* h, const double* state, int64_t n) {
  // Chain.SetState (chain.go:130-138) / Section.SetState (section.go:152-155)
  // of every channel: state [channels][nsec][2] {d0, d1}, applied between
  // calls (after the previous call's work, before the next).
  return fx_guard(h, [&] {
    const int64_t need = (int64_t)h->channels * h->nsec * 2;
    if (n < need) AD_FAIL(AD_ERR_LENGTH_MISMATCH, "state buffer too small: need channels*sections*2 values");
    if (need > 0 && !state) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null state buffer");
    fx_quiesce(h);
    if (need == 0) return;
    std::vector<double> raw((size_t)need);
    eq_state_to_slabs(state, h->channels, h->nsec, raw.data());
    AD_HIP(hipMemcpy(h->eq_state.p, raw.data(), raw.size() * sizeof(double), hipMemcpyHostToDevice));
  });
}

int ad_fx_chain_set_engine(ad_fx_chain* h, int engine, int64_t chunk) {
  return fx_guard(h, [&] {
    if (engine < AD_FX_ENGINE_AUTO || engine > AD_FX_ENGINE_TIME_PARALLEL)
      AD_FAIL(AD_ERR_INVALID_ARGUMENT, "unknown effect-chain engine");
    if (chunk != 0 && chunk < 256) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "staged chunk must be 0 (default) or >= 256");
    fx_quiesce(h);
    h->engine = engine;
    h->chunk = chunk;
  });
}

int ad_fx_chain_last_engine(ad_fx_chain* h, int* engine, double* eq_noise) {
  return fx_guard(h, [&] {
    if (engine) *engine = h->last_engine;
    if (eq_noise) *eq_noise = h->eq_noise;
  });
}

int ad_fx_chain_set_profiling(ad_fx_chain* h, int enable) {
  return fx_guard(h, [&] {
    fx_quiesce(h);
    h->prof_on = enable != 0;
  });
}

int ad_fx_chain_read_profile(ad_fx_chain* h, unsigned long long* counters, int cap, int* count) {
  return fx_guard(h, [&] {
    fx_quiesce(h);
    const int n = h->prof.p ? (int)std::min<size_t>(h->prof.n, (size_t)std::max(cap, 0)) : 0;
    if (n > 0 && !counters) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null counter buffer");
    if (n > 0) AD_HIP(hipMemcpy(counters, h->prof.p, (size_t)n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    if (count) *count = n;
  });
}

void ad_fx_chain_destroy(ad_fx_chain* h) {
  if (!h) return;
  (void)guard([&] {
    DeviceScope ds(h->device);
    delete h;
  });
}

// biquad.Chain.ProcessBlock over `channels` independent chains that share one
// coefficient set (chain.go:59-70); state [channels][sections][2] in/out.
int ad_biquad_chain_process(const double* coeffs, double* state, double gain, double* buf, int channels,
                            int sections, int64_t n, int device) {
  ad_fx_chain* h = nullptr;
  int rc = ad_fx_chain_create(channels, device, &h);
  if (rc != AD_OK) return rc;
  rc = guard([&] {
    if (sections < 0 || (sections > 0 && (!coeffs || !state))) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad sections");
    std::vector<double> tab((size_t)sections * kSecStride);
    for (int s = 0; s < sections; ++s) {
      tab[(size_t)s * kSecStride] = s == 0 ? gain : 1.0;
      for (int k = 0; k < 5; ++k) tab[(size_t)s * kSecStride + 1 + k] = coeffs[s * 5 + k];
    }
    int r = ad_fx_chain_set_eq(h, tab.data(), sections, 0);
    if (r != AD_OK) throw Status{r, ad_last_error()};
    r = ad_fx_chain_set_eq_state(h, state, (int64_t)channels * sections * 2);
    if (r != AD_OK) throw Status{r, ad_last_error()};
    r = ad_fx_chain_process(h, buf, n);
    if (r != AD_OK) throw Status{r, ad_last_error()};
    r = ad_fx_chain_eq_state(h, state, (int64_t)channels * sections * 2);
    if (r != AD_OK) throw Status{r, ad_last_error()};
  });
  ad_fx_chain_destroy(h);
  return rc;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// FIR
// ---------------------------------------------------------------------------
struct ad_fir {
  int device = 0, channels = 0;
  int64_t N = 0;
  hipStream_t stream = nullptr;       // host-buffer calls
  hipStream_t last = nullptr;         // stream of the last call (valid when has_last)
  bool has_last = false;              // a call has been enqueued (last may be the NULL stream)
  hipEvent_t done = nullptr;          // recorded on `last` after each call's last operation
  DevBuf<double> h;                   // [N]
  DevBuf<double> hist[2];             // [C][N-1] delay line, ping-pong (cur = hist[cur])
  int cur = 0;
  DevBuf<double> stage;               // [C][n]: in-place calls read a copy of the input
  DevBuf<double> io_in, io_out;       // host-buffer calls
  ~ad_fir() {
    if (done) {
      (void)hipEventSynchronize(done);
      (void)hipEventDestroy(done);
    }
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)lib_stream_destroy(stream);
    }
  }
};

namespace {

// y = FIR(x) for n new samples per channel, device in/out; updates history.
// The kernel reads the old delay line and the input directly; the next
// delay line (last N-1 samples of [hist | src]) is built in the other
// history buffer first, so nothing the kernel reads is written meanwhile.
// An in-place call (dst overlaps src) reads a staged copy of src.
void fir_run(ad_fir* f, const double* d_src, int64_t src_stride, double* d_dst, int64_t dst_stride, int64_t n,
             hipStream_t s) {
  // The delay line, the staging copy and the ping-pong index are shared by
  // every stream a caller uses: a call on a new stream first waits for the
  // previous call's last operation.
  if (f->has_last && f->last != s) AD_HIP(hipStreamWaitEvent(s, f->done, 0));
  const int64_t hn = f->N - 1;
  const size_t C = (size_t)f->channels;
  const char* s0 = reinterpret_cast<const char*>(d_src);
  const char* s1 = reinterpret_cast<const char*>(d_src + (C - 1) * src_stride + n);
  const char* d0 = reinterpret_cast<const char*>(d_dst);
  const char* d1 = reinterpret_cast<const char*>(d_dst + (C - 1) * dst_stride + n);
  if (s0 < d1 && d0 < s1) {
    f->stage.reserve(C * n);
    AD_HIP(hipMemcpy2DAsync(f->stage.p, n * sizeof(double), d_src, src_stride * sizeof(double), n * sizeof(double),
                            C, hipMemcpyDeviceToDevice, s));
    d_src = f->stage.p;
    src_stride = n;
  }
  const double* hold = f->hist[f->cur].p;
  if (hn > 0) {
    double* hnew = f->hist[f->cur ^ 1].p;
    if (n >= hn) {
      AD_HIP(hipMemcpy2DAsync(hnew, hn * sizeof(double), d_src + (n - hn), src_stride * sizeof(double),
                              hn * sizeof(double), C, hipMemcpyDeviceToDevice, s));
    } else {
      AD_HIP(hipMemcpy2DAsync(hnew, hn * sizeof(double), hold + n, hn * sizeof(double), (hn - n) * sizeof(double),
                              C, hipMemcpyDeviceToDevice, s));
      AD_HIP(hipMemcpy2DAsync(hnew + (hn - n), hn * sizeof(double), d_src, src_stride * sizeof(double),
                              n * sizeof(double), C, hipMemcpyDeviceToDevice, s));
    }
  }
  FirArgs a{};
  a.h = f->h.p;
  a.N = f->N;
  a.hist = hold;
  a.src = d_src;
  a.sstride = src_stride;
  a.y = d_dst;
  a.ystride = dst_stride;
  a.n = n;
  a.channels = f->channels;
  a.reversed = f->N >= 32;
  launch_fir(a, s);
  AD_HIP(hipGetLastError());
  if (hn > 0) f->cur ^= 1;
  AD_HIP(hipEventRecord(f->done, s));
  f->last = s;
  f->has_last = true;
}

}  // namespace

extern "C" {

int ad_fir_create(const double* coeffs, int64_t n_taps, int channels, int device, ad_fir** out) {
  if (out) *out = nullptr;
  ad_fir* raw = nullptr;
  const int rc = guard([&] {
    if (n_taps < 0 || (n_taps > 0 && !coeffs)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad coefficients");
    if (channels <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "channels must be positive");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    std::unique_ptr<ad_fir> f(new ad_fir());
    f->device = dev;
    f->channels = channels;
    f->N = n_taps;
    AD_HIP(lib_stream_create(&f->stream));
    AD_HIP(hipEventCreateWithFlags(&f->done, hipEventDisableTiming));
    if (n_taps > 0) {
      f->h.alloc((size_t)n_taps);
      AD_HIP(hipMemcpy(f->h.p, coeffs, n_taps * sizeof(double), hipMemcpyHostToDevice));
    }
    if (n_taps > 1) {
      for (auto& hb : f->hist) {
        hb.alloc((size_t)channels * (n_taps - 1));
        AD_HIP(hipMemset(hb.p, 0, hb.n * sizeof(double)));
      }
    }
    raw = f.release();
  });
  if (rc == AD_OK && out) *out = raw;
  return rc;
}

int ad_fir_process_block_to(ad_fir* f, double* dst, const double* src, int64_t n) {
  return guard([&] {
    if (!f) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null FIR handle");
    if (n <= 0) return;
    if (f->N == 0) {  // filter.go:75-77 / 120-122: no taps -> output untouched
      return;
    }
    DeviceScope ds(f->device);
    const size_t cnt = (size_t)f->channels * n;
    f->io_in.reserve(cnt);
    f->io_out.reserve(cnt);
    AD_HIP(hipMemcpyAsync(f->io_in.p, src, cnt * sizeof(double), hipMemcpyHostToDevice, f->stream));
    fir_run(f, f->io_in.p, n, f->io_out.p, n, n, f->stream);
    AD_HIP(hipMemcpyAsync(dst, f->io_out.p, cnt * sizeof(double), hipMemcpyDeviceToHost, f->stream));
    AD_HIP(hipStreamSynchronize(f->stream));
  });
}

int ad_fir_process_block(ad_fir* f, double* buf, int64_t n) { return ad_fir_process_block_to(f, buf, buf, n); }

int ad_fir_process_device(ad_fir* f, const double* d_src, int64_t src_stride, double* d_dst, int64_t dst_stride,
                          int64_t n, void* stream) {
  return guard([&] {
    if (!f) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null FIR handle");
    if (n <= 0 || f->N == 0) return;
    if (src_stride < n || dst_stride < n) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad strides");
    DeviceScope ds(f->device);
    fir_run(f, d_src, src_stride, d_dst, dst_stride, n, reinterpret_cast<hipStream_t>(stream));
  });
}

int ad_fir_reset(ad_fir* f) {
  // filter.go:162-172; ordered after the last call, on the stream it used
  return guard([&] {
    if (!f) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null FIR handle");
    DeviceScope ds(f->device);
    // after the last call, whatever stream (NULL included) it was enqueued on
    if (f->has_last) AD_HIP(hipStreamWaitEvent(f->stream, f->done, 0));
    for (auto& hb : f->hist)
      if (hb.p) AD_HIP(hipMemsetAsync(hb.p, 0, hb.n * sizeof(double), f->stream));
    AD_HIP(hipEventRecord(f->done, f->stream));
    f->last = f->stream;
    f->has_last = true;
    AD_HIP(hipStreamSynchronize(f->stream));
  });
}

void ad_fir_destroy(ad_fir* f) {
  if (!f) return;
  (void)guard([&] {
    DeviceScope ds(f->device);
    delete f;
  });
}

}  // extern "C"

// ---------------------------------------------------------------------------
// IRLB f16 decode
// ---------------------------------------------------------------------------
extern "C" {

int ad_decode_f16_device(const uint16_t* d_in, int64_t frames, int channels, double* d_out, void* stream) {
  return guard([&] {
    if (frames < 0 || channels <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad f16 geometry");
    launch_decode_f16(d_in, frames, channels, d_out, reinterpret_cast<hipStream_t>(stream));
    AD_HIP(hipGetLastError());
  });
}

int ad_decode_f16(const uint16_t* in, int64_t frames, int channels, double* out, int device) {
  return guard([&] {
    if (frames < 0 || channels <= 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "bad f16 geometry");
    if (frames == 0) return;
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    const int64_t n = frames * channels;
    DevBuf<uint16_t> din;
    DevBuf<double> dout;
    din.alloc((size_t)n);
    dout.alloc((size_t)n);
    AD_HIP(hipMemcpy(din.p, in, n * sizeof(uint16_t), hipMemcpyHostToDevice));
    launch_decode_f16(din.p, frames, channels, dout.p, nullptr);
    AD_HIP(hipGetLastError());
    AD_HIP(hipMemcpy(out, dout.p, n * sizeof(double), hipMemcpyDeviceToHost));
  });
}

}  // extern "C"
