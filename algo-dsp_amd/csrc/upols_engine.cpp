// Host runtime of the UPOLS convolution engine.  See upols_engine.hpp and the
// data-flow comment at the top of conv_kernels.hip.
#include "upols_engine.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "conv_kernels.hpp"

namespace adsp {

namespace {

// K2 lane layout: one lane keeps PC partitions of a chunk in VGPRs, PC = the
// smallest power of two >= P, capped at 16 (larger P: one launch per chunk of
// 16 partitions, the later ones read-modify-writing Z).
int pick_pc(int P) {
  int pc = 1;
  while (pc < P && pc < 16) pc *= 2;
  return pc;
}

}  // namespace

Upols::Upols(int device, const double* kernels, int n_ir, int64_t K, int L, int C, const int32_t* ir_map, int jc_max,
             hipStream_t stream)
    : K_(K), L_(L), C_(C), n_ir_(n_ir), jc_max_(jc_max), stream_(stream) {
  if (L < 64 || L > 8192 || !is_pow2(L)) AD_FAIL(AD_ERR_INTERNAL, "UPOLS hop must be a power of two in [64, 8192]");
  if (n_ir < 1 || C < 1 || K < 1 || jc_max < 1) AD_FAIL(AD_ERR_INTERNAL, "UPOLS: bad geometry");
  M_ = L;
  MS_ = M_ + 8;
  P_ = (int)((K + L - 1) / L);
  NH_ = 1;
  PC_ = pick_pc(P_);
  Q_ = jc_max_ + P_ + 2 * PC_ + 1;
  R_ = 0;  // the launcher sizes runs to one resident round of waves

  // Twiddle tables, computed in long double on the host.
  std::vector<double2> tw(2 * (size_t)M_);
  const long double two_pi = 6.283185307179586476925286766559005768L;
  for (int e = 0; e < M_; ++e) {
    const long double a = -two_pi * (long double)e / (long double)M_;
    tw[e] = make_double2((double)cosl(a), (double)sinl(a));
    const long double b = -two_pi * (long double)e / (long double)(2 * M_);
    tw[M_ + e] = make_double2((double)cosl(b), (double)sinl(b));
  }
  tw_.alloc(tw.size());
  AD_HIP(hipMemcpyAsync(tw_.p, tw.data(), tw.size() * sizeof(double2), hipMemcpyHostToDevice, stream_));

  // IR partitions [n_ir*P][L], zero padded, then their spectra via K1.
  const int64_t nparts = (int64_t)n_ir_ * P_;
  std::vector<double> parts((size_t)(nparts * L_), 0.0);
  for (int r = 0; r < n_ir_; ++r)
    for (int p = 0; p < P_; ++p) {
      const int64_t start = (int64_t)p * L_;
      const int64_t cnt = std::min<int64_t>(L_, K_ - start);
      std::memcpy(&parts[(size_t)(((int64_t)r * P_ + p) * L_)], kernels + (int64_t)r * K_ + start,
                  (size_t)cnt * sizeof(double));
    }
  DevBuf<double> dparts;
  dparts.alloc(parts.size());
  AD_HIP(hipMemcpyAsync(dparts.p, parts.data(), parts.size() * sizeof(double), hipMemcpyHostToDevice, stream_));
  H_.alloc((size_t)nparts * MS_);
  AD_HIP(hipMemsetAsync(H_.p, 0, H_.n * sizeof(double2), stream_));
  RfftArgs a{};
  a.x = dparts.p;
  a.x_stride = L_;
  a.n = L_;
  a.s0 = 0;
  a.jc = 1;
  a.channels = (int)nparts;
  a.aligned = 1;
  a.X = H_.p;
  a.x_ch_stride = MS_;
  a.Q = 1;
  a.slot0 = 0;
  a.MS = MS_;
  a.twM = tw_.p;
  a.twN = tw_.p + M_;
  if (!launch_window_rfft(M_, a, stream_)) AD_FAIL(AD_ERR_INTERNAL, "unsupported FFT size");
  AD_HIP(hipGetLastError());

  X_.alloc((size_t)C_ * (Q_ + 1) * MS_);  // Q ring rows + one zero row per channel
  // Z rows: jc_max outputs + 16 rows of run overshoot (k_fdl_mac)
  Y_.alloc((size_t)C_ * (jc_max_ + 16) * MS_);
  std::vector<int> irm(C_);
  for (int c = 0; c < C_; ++c) irm[c] = ir_map ? ir_map[c] : (c % n_ir_);
  for (int c = 0; c < C_; ++c)
    if (irm[c] < 0 || irm[c] >= n_ir_) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "ir_index out of range");
  irmap_.alloc(C_);
  AD_HIP(hipMemcpyAsync(irmap_.p, irm.data(), C_ * sizeof(int), hipMemcpyHostToDevice, stream_));
  reset_stream(stream_);
  // dparts must outlive the K1 launch that reads it
  AD_HIP(hipStreamSynchronize(stream_));
}

Upols::~Upols() {
  for (auto st : ps_)
    if (st) {
      (void)hipStreamSynchronize(st);
      (void)lib_stream_destroy(st);
    }
  for (auto& row : pev_)
    for (auto e : row)
      if (e) (void)hipEventDestroy(e);
  for (auto& r : prof_recs_) {
    (void)hipEventDestroy(r.start);
    (void)hipEventDestroy(r.stop);
  }
  for (auto e : event_pool_) (void)hipEventDestroy(e);
}

hipEvent_t Upols::take_event() {
  if (!event_pool_.empty()) {
    hipEvent_t e = event_pool_.back();
    event_pool_.pop_back();
    return e;
  }
  hipEvent_t e;
  AD_HIP(hipEventCreate(&e));
  return e;
}

// The events ride in the kernel's dispatch packet (timed_launch), so the
// interval is the launch's own execution: no marker packets sit between the
// kernels of a call (those cost ~5 us per kernel and a cold start).
void Upols::prof_begin(hipStream_t, hipEvent_t* e, int kernel) {
  *e = nullptr;
  if (!prof_ || !((prof_mask_ >> kernel) & 1)) return;
  *e = take_event();
  LaunchTiming& t = launch_timing();
  t.start = *e;
  t.stop = take_event();
}

void Upols::prof_end(hipStream_t, hipEvent_t e0, int kernel, double bytes) {
  if (!e0) return;
  LaunchTiming& t = launch_timing();
  if (t.start) {  // nothing was launched
    event_pool_.push_back(e0);
    event_pool_.push_back(t.stop);
  } else {
    prof_recs_.push_back({e0, t.stop, kernel, bytes});
  }
  t.start = t.stop = nullptr;
}

void Upols::set_profiling(bool on) {
  prof_ = on;
  // pre-create events so recording inside a timed region never pays hipEventCreate
  while (on && event_pool_.size() < 512) {
    hipEvent_t e;
    AD_HIP(hipEventCreate(&e));
    event_pool_.push_back(e);
  }
}

void Upols::read_profile(double* ms, int64_t* launches, double* alg_bytes) {
  for (auto& r : prof_recs_) {
    AD_HIP(hipEventSynchronize(r.stop));
    float t = 0.f;
    AD_HIP(hipEventElapsedTime(&t, r.start, r.stop));
    acc_ms_[r.kernel] += t;
    acc_n_[r.kernel] += 1;
    acc_bytes_[r.kernel] += r.bytes;
    event_pool_.push_back(r.start);
    event_pool_.push_back(r.stop);
  }
  prof_recs_.clear();
  for (int k = 0; k < kKernels; ++k) {
    if (ms) ms[k] = acc_ms_[k];
    if (launches) launches[k] = acc_n_[k];
    if (alg_bytes) alg_bytes[k] = acc_bytes_[k];
    acc_ms_[k] = 0;
    acc_n_[k] = 0;
    acc_bytes_[k] = 0;
  }
}

void Upols::reset_stream(hipStream_t s) {
  AD_HIP(hipMemsetAsync(X_.p, 0, X_.n * sizeof(double2), s));
  g_next_ = 0;
}

void Upols::begin_offline(hipStream_t) {
  // Spectra with logical index < 0 read as zeros inside k_fdl_mac, so a new
  // signal only restarts the logical block counter (no memset).
  g_next_ = 0;
  // the schedule is fixed per signal: a request made between two segments of
  // one signal waits for the next signal, so the rings never change size
  // under a signal in flight
  sched_mode_ = req_mode_;
  pipe_jc_ = req_jc_;
  pipe_run_ = req_run_;
  sig_pipe_ = sched_mode_ != kSchedSerial && M_ >= 2048;
  if (sig_pipe_) ensure_pipe();
}

void Upols::set_schedule(int mode, int chunk, int run) {
  if (mode != kSchedSerial && mode != kSchedPipelined && mode != kSchedChunked) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "unknown schedule");
  if (chunk < 0 || run < 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "schedule: negative chunk or run length");
  req_mode_ = mode;
  // auto chunk: 128 blocks per channel of two channels keep the live rings
  // (two chunks of block spectra + two of Z rows, ~64 MiB each at hop 8192)
  // inside the 256 MiB Infinity Cache
  req_jc_ = chunk > 0 ? chunk : (int)std::max<int64_t>(32, std::min<int64_t>(jc_max_, 256 / std::max(1, C_)));
  req_jc_ = std::min(req_jc_, jc_max_);
  req_run_ = run;
}

void Upols::ensure_pipe() {
  const int Qp = 2 * pipe_jc_ + P_ + 2 * PC_ + 1;
  const int zr = pipe_jc_ + 16;
  if (Qp != Qp_ || !Xp_.p) {
    // a resized ring: no kernel of an earlier call may still read the old one
    for (auto st : ps_)
      if (st) AD_HIP(hipStreamSynchronize(st));
    Xp_.alloc((size_t)C_ * (Qp + 1) * MS_);
    // the zero rows (row Qp of each channel) must read as zeros; every other
    // row is written by K1 before any kernel reads it
    AD_HIP(hipMemsetAsync(Xp_.p, 0, Xp_.n * sizeof(double2), stream_));
    AD_HIP(hipStreamSynchronize(stream_));  // the memset precedes any call stream's use
    Qp_ = Qp;
  }
  if (zr != zrows_p_ || !Zp_.p) {
    for (auto st : ps_)
      if (st) AD_HIP(hipStreamSynchronize(st));
    Zp_.alloc((size_t)2 * C_ * zr * MS_);
    zrows_p_ = zr;
  }
  for (auto& st : ps_)
    if (!st) AD_HIP(lib_stream_create(&st));
  for (auto& row : pev_)
    for (auto& e : row)
      if (!e) AD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

void Upols::k1(const Chunk& ck, const Rings& rg, const Io& io, const StreamGate& sg, bool ordered, int runR,
               int runNy, hipStream_t s) {
  RfftArgs a{};
  a.x = io.in;
  a.x_stride = io.in_stride;
  a.n = io.n;
  a.s0 = ck.cs * L_;
  a.jc = ck.jin;
  a.channels = C_;
  a.aligned = io.in_aligned;
  a.X = rg.X;
  a.x_ch_stride = (int64_t)(rg.Q + 1) * MS_;
  a.Q = rg.Q;
  a.slot0 = (int)(ck.g0 % rg.Q);
  a.MS = MS_;
  a.twM = tw_.p;
  a.twN = tw_.p + M_;
  if (ordered) {
    a.ord_R = runR;
    a.ord_ny = runNy;
    a.ord_pc = PC_;
  }
  a.sg = sg;
  hipEvent_t e0;
  prof_begin(s, &e0, 0);
  launch_window_rfft(M_, a, s);
  // algorithmic bytes per launch: unique input samples in, M+1
  // complex128 bins out, per (channel, block)
  prof_end(s, e0, 0, (double)C_ * ck.jin * ((double)L_ * 8 + (double)M_ * 16));
}

void Upols::k2(const Chunk& ck, const Rings& rg, const StreamGate& sg, int runR, hipStream_t s) {
  MacArgs m{};
  m.X = rg.X;
  m.x_ch_stride = (int64_t)(rg.Q + 1) * MS_;
  m.Q = rg.Q;
  m.g0 = ck.g0;
  m.gend = ck.gend;
  m.MS = MS_;
  m.H = H_.p;
  m.h_ir_stride = (int64_t)P_ * MS_;
  m.ir_index = irmap_.p;
  m.n_ir = n_ir_;
  m.Y = rg.Z;
  m.y_ch_stride = (int64_t)rg.zrows * MS_;
  m.jc = ck.jc;
  m.R = runR;
  m.P = P_;
  m.M = M_;
  m.twN = tw_.p + M_;
  // Z[M/2] from K3 (split sizes, few partitions): K2 then runs pair waves only
  m.mid_in_k3 = (M_ >= 2048 && P_ <= 256) ? 1 : 0;
  m.sg = sg;
  hipEvent_t e0;
  prof_begin(s, &e0, 1);
  launch_fdl_mac(PC_, NH_, m, C_, s);
  prof_end(s, e0, 1, (double)C_ * ck.jc * (double)(M_ + 1) * 32 + (double)n_ir_ * P_ * (M_ + 1) * 16);
}

void Upols::k3(const Chunk& ck, const Rings& rg, const Io& io, const StreamGate& sg, bool ordered, int runR,
               int runNy, hipStream_t s) {
  IrfftArgs b{};
  b.Y = rg.Z;
  b.y_ch_stride = (int64_t)rg.zrows * MS_;
  b.MS = MS_;
  b.out = io.mix ? io.mix->p : io.out;
  b.out_stride = io.mix ? io.mix->stride : io.out_stride;
  b.out_len = io.out_len;
  b.o0 = ck.cs * L_;
  b.jc = ck.jc;
  b.channels = C_;
  b.aligned = io.out_aligned;
  b.accumulate = io.accumulate ? 1 : 0;
  b.twM = tw_.p;
  b.twN = tw_.p + M_;
  if (ordered) {
    b.ord_R = runR;
    b.ord_ny = runNy;
  }
  if (M_ >= 2048 && P_ <= 256) {
    b.mid.on = 1;
    b.mid.X = rg.X;
    b.mid.x_ch_stride = (int64_t)(rg.Q + 1) * MS_;
    b.mid.Q = rg.Q;
    b.mid.g0 = ck.g0;
    b.mid.gend = ck.gend;
    b.mid.H = H_.p;
    b.mid.h_ir_stride = (int64_t)P_ * MS_;
    b.mid.ir_index = irmap_.p;
    b.mid.n_ir = n_ir_;
    b.mid.P = P_;
  }
  b.sg = sg;
  const double blocks = (double)C_ * ck.jc;
  hipEvent_t e0;
  prof_begin(s, &e0, 2);
  if (io.mix) {  // every channel's Z rows in, the two mix rows out
    b.mix_parity = io.mix->first_parity & 1;
    launch_irfft_mix(M_, b, s);
    prof_end(s, e0, 2, blocks * (double)(M_ + 1) * 16 + 2.0 * ck.jc * L_ * 8);
  } else {
    launch_irfft_store(M_, b, s);
    prof_end(s, e0, 2, blocks * ((double)(M_ + 1) * 16 + (double)L_ * 8));
  }
}

void Upols::run(const double* d_in, int64_t in_stride, int64_t n, double* d_out, int64_t out_stride, int64_t out_len,
                bool use_hist, hipStream_t s, int64_t jb, int64_t je, bool accumulate, const MixOut* mix) {
  if (out_len <= 0) return;
  if (mix && (!can_mix() || accumulate || gate_on_)) AD_FAIL(AD_ERR_INTERNAL, "UPOLS: fused mixdown needs hop >= 2048");
  if (je < 0) je = (out_len + L_ - 1) / L_;
  const int64_t J = je - jb;
  if (J <= 0) return;
  Io io{};
  io.in = d_in;
  io.in_stride = in_stride;
  io.n = n;
  io.in_aligned = ((reinterpret_cast<uintptr_t>(d_in) & 15) == 0) && (in_stride % 2 == 0);
  io.out = d_out;
  io.out_stride = out_stride;
  io.out_len = out_len;
  io.accumulate = accumulate;
  io.mix = mix;
  const double* op = mix ? mix->p : d_out;
  const int64_t ostr = mix ? mix->stride : out_stride;
  io.out_aligned = ((reinterpret_cast<uintptr_t>(op) & 15) == 0) && (ostr % 2 == 0);
  // call blocks holding input samples: [0, nb_in); K1 transforms only those,
  // K2 reads every later block as zeros
  const int64_t nb_in = (std::max<int64_t>(n, 0) + L_ - 1) / L_;
  if (sig_pipe_ && pipe_call_ && !use_hist && !accumulate && !gate_on_) {
    run_pipelined(io, s, jb, J, nb_in);
    return;
  }
  StreamGate sg{};
  if (gate_on_) {
    if (J != 1 || C_ != 1 || M_ < 2048) AD_FAIL(AD_ERR_INTERNAL, "gated run: one block of one channel, hop >= 2048");
    sg = gate_;
    gate_on_ = false;
  }
  const Rings rg{X_.p, Q_, Y_.p, jc_max_ + 16};
  // balanced chunks of at most jc_max blocks (no tiny tail launch)
  const int64_t nchunks = (J + jc_max_ - 1) / jc_max_;
  const int64_t jc_even = (J + nchunks - 1) / nchunks;
  for (int64_t cr = 0; cr < J; cr += jc_even) {
    Chunk ck{};
    ck.jc = (int)std::min<int64_t>(jc_even, J - cr);
    ck.cs = jb + cr;
    ck.jin = (int)std::clamp<int64_t>(nb_in - ck.cs, 0, ck.jc);
    ck.g0 = g_next_;
    ck.gend = g_next_ - ck.cs + nb_in - 1;
    // K2's run geometry, decided here so K1 and K3 can order their items by it
    // (newest rows first for the kernel that reads them next; see RfftArgs)
    int runR = R_, runNy = 0;
    mac_run_geometry(PC_, NH_, M_, M_ >= 2048 && P_ <= 256 ? 1 : 0, C_, ck.jc, R_, &runR, &runNy);
    // worth it when the Infinity Cache (256 MiB) holds the rows of a good
    // part of a run: stereo at hop 8192 ~81 of R = 176 steps (step 0.5751 ->
    // 0.5686 ms); the 8-channel shard ~81 of R = 688 (no gain, +0.7 %)
    const int64_t rows_per_step = (int64_t)C_ * runNy;
    const int64_t steps_cached = (int64_t(256) << 20) / ((int64_t)MS_ * 16 * std::max<int64_t>(1, rows_per_step));
    const bool ordered = M_ >= 2048 && !(NH_ == 1 && ck.jc <= 2) && runNy > 1 && steps_cached * 4 >= runR && !mix;
    k1(ck, rg, io, sg, ordered, runR, runNy, s);
    k2(ck, rg, sg, runR, s);
    k3(ck, rg, io, sg, ordered, runR, runNy, s);
    AD_HIP(hipGetLastError());
    g_next_ += ck.jc;
  }
}

// The pipelined offline schedule (set_schedule): chunk k's K1 on the caller's
// stream s, its K2 on ps_[0], its K3 on ps_[1].  Ring reuse:
//   - K1(k) overwrites block-spectrum rows that K2 and K3's middle bin of
//     chunk k-2 read: s waits for K3(k-2) (which follows K2(k-2)); the rows
//     chunk k-1's kernels read (its blocks and the P + PC rows before them)
//     are disjoint from chunk k's in a ring of Qp >= 2 chunk + P + 2 PC + 1;
//   - K2(k) writes Z half k mod 2, which K3(k-2) read: ps_[0] waits for it;
//   - K2(k) waits for K1(k), K3(k) for K2(k);
//   - the caller's stream waits for the last K3, so the call's outputs are
//     complete when s passes it, as in the serial schedule, and the next
//     call's K1 (on s) follows every kernel of this one.
void Upols::run_pipelined(const Io& io, hipStream_t s, int64_t jb, int64_t J, int64_t nb_in) {
  const int jp = pipe_jc_;
  // the rings were sized for this signal's schedule at begin_offline
  if (jp < 1 || jp + 16 > zrows_p_ || 2 * jp + P_ + 2 * PC_ + 1 > Qp_)
    AD_FAIL(AD_ERR_INTERNAL, "pipelined schedule: rings smaller than the chunk");
  const int64_t nchunks = (J + jp - 1) / jp;
  const int64_t jc_even = (J + nchunks - 1) / nchunks;
  int64_t k = 0;
  for (int64_t cr = 0; cr < J; cr += jc_even, ++k) {
    Chunk ck{};
    ck.jc = (int)std::min<int64_t>(jc_even, J - cr);
    ck.cs = jb + cr;
    ck.jin = (int)std::clamp<int64_t>(nb_in - ck.cs, 0, ck.jc);
    ck.g0 = g_next_;
    ck.gend = g_next_ - ck.cs + nb_in - 1;
    const Rings rg{Xp_.p, Qp_, Zp_.p + (size_t)(k & 1) * C_ * zrows_p_ * MS_, zrows_p_};
    hipEvent_t* e1 = &pev_[0][k & 3];
    hipEvent_t* e2 = &pev_[1][k & 3];
    hipEvent_t* e3 = &pev_[2][k & 3];
    const hipEvent_t e3_prev2 = k >= 2 ? pev_[2][(k - 2) & 3] : nullptr;
    int runR = pipe_run_, runNy = 0;
    mac_run_geometry(PC_, NH_, M_, M_ >= 2048 && P_ <= 256 ? 1 : 0, C_, ck.jc, pipe_run_, &runR, &runNy);
    if (sched_mode_ == kSchedChunked) {
      k1(ck, rg, io, StreamGate{}, false, runR, runNy, s);
      k2(ck, rg, StreamGate{}, runR, s);
      k3(ck, rg, io, StreamGate{}, false, runR, runNy, s);
      AD_HIP(hipGetLastError());
      g_next_ += ck.jc;
      continue;
    }
    if (e3_prev2) AD_HIP(hipStreamWaitEvent(s, e3_prev2, 0));
    k1(ck, rg, io, StreamGate{}, false, runR, runNy, s);
    AD_HIP(hipEventRecord(*e1, s));
    AD_HIP(hipStreamWaitEvent(ps_[0], *e1, 0));
    if (e3_prev2) AD_HIP(hipStreamWaitEvent(ps_[0], e3_prev2, 0));
    k2(ck, rg, StreamGate{}, runR, ps_[0]);
    AD_HIP(hipEventRecord(*e2, ps_[0]));
    AD_HIP(hipStreamWaitEvent(ps_[1], *e2, 0));
    k3(ck, rg, io, StreamGate{}, false, runR, runNy, ps_[1]);
    AD_HIP(hipEventRecord(*e3, ps_[1]));
    AD_HIP(hipGetLastError());
    g_next_ += ck.jc;
  }
  if (sched_mode_ != kSchedChunked) AD_HIP(hipStreamWaitEvent(s, pev_[2][(k - 1) & 3], 0));
}

void Upols::save_history(const double*, int64_t, int64_t n, hipStream_t) {
  if (n < L_) AD_FAIL(AD_ERR_INTERNAL, "streaming call shorter than the hop");
}

}  // namespace adsp
