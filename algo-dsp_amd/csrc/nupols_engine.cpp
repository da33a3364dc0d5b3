// Host runtime of the non-uniformly partitioned engine (see nupols_engine.hpp).
#include "nupols_engine.hpp"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "conv_kernels.hpp"

namespace adsp {

namespace {
int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// In-place forward DFT of a power-of-two length in long double (radix-2,
// bit-reversed input reordering): the fused stages' partition spectra.
void host_fft_ld(std::vector<long double>& re, std::vector<long double>& im) {
  const size_t n = re.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) {
      std::swap(re[i], re[j]);
      std::swap(im[i], im[j]);
    }
  }
  for (size_t len = 2; len <= n; len <<= 1) {
    const long double a = -6.283185307179586476925286766559005768L / (long double)len;
    for (size_t i = 0; i < n; i += len)
      for (size_t k = 0; k < len / 2; ++k) {
        const long double wr = cosl(a * k), wi = sinl(a * k);
        const long double xr = re[i + k + len / 2] * wr - im[i + k + len / 2] * wi;
        const long double xi = re[i + k + len / 2] * wi + im[i + k + len / 2] * wr;
        re[i + k + len / 2] = re[i + k] - xr;
        im[i + k + len / 2] = im[i + k] - xi;
        re[i + k] += xr;
        im[i + k] += xi;
      }
  }
}
}  // namespace

NupolsDev::NupolsDev(int device, const double* h, int64_t K, int64_t lambda, int64_t p_max, int channels,
                     hipStream_t s)
    : C_(channels), lambda_(lambda) {
  if (lambda < 64 || !is_pow2(lambda) || p_max < lambda || !is_pow2(p_max) || p_max > 8192 || channels < 1)
    AD_FAIL(AD_ERR_INTERNAL, "NupolsDev: bad geometry");
  // stage layout: two partitions per size while the size doubles, the rest at
  // p_max; T_{s+1} = T_s + n_s p_s >= p_{s+1} - lambda holds by construction
  int64_t T = 0, p = lambda;
  while (T < K) {
    int64_t nparts = 2;
    if (p >= p_max) nparts = (K - T + p - 1) / p;
    Stage st;
    st.p = p;
    st.T = T;
    st.taps = std::min<int64_t>(nparts * p, K - T);
    st_.push_back(std::move(st));
    T += nparts * p;
    if (p < p_max) p *= 2;
  }
  std::vector<double2> tw(2048);
  for (int m = 0; m < 2048; ++m) {
    const long double a = -6.283185307179586476925286766559005768L * m / 2048.0L;
    tw[m] = make_double2((double)cosl(a), (double)sinl(a));
  }
  tw2048_.alloc(2048);
  AD_HIP(hipMemcpyAsync(tw2048_.p, tw.data(), 2048 * sizeof(double2), hipMemcpyHostToDevice, s));
  for (auto& st : st_) {
    st.fused = st.p <= 1024 && st.taps <= 2 * st.p;
    if (st.fused) {
      const int N = (int)(2 * st.p);
      std::vector<double2> hs(2 * (size_t)N);
      for (int part = 0; part < 2; ++part) {
        std::vector<long double> re(N, 0.0L), im(N, 0.0L);
        for (int64_t k = 0; k < st.p; ++k) {
          const int64_t tap = st.T + part * st.p + k;
          if (tap < st.T + st.taps) re[k] = h[tap];
        }
        host_fft_ld(re, im);
        for (int k = 0; k < N; ++k) hs[(size_t)part * N + k] = make_double2((double)re[k], (double)im[k]);
      }
      st.H.reset(new DevBuf<double2>());
      st.H->alloc(hs.size());
      AD_HIP(hipMemcpyAsync(st.H->p, hs.data(), hs.size() * sizeof(double2), hipMemcpyHostToDevice, s));
      AD_HIP(hipStreamSynchronize(s));  // hs must outlive the copy
    } else {
      // up to 64 blocks (and >= 8192 samples) per launch chunk: long calls batch
      const int jc = (int)std::max<int64_t>(64, 8192 / st.p);
      st.eng.reset(new Upols(device, h + st.T, 1, st.taps, (int)st.p, channels, nullptr, jc, s));
    }
  }
  AD_HIP(hipStreamSynchronize(s));
  reset(s);
}

void NupolsDev::reset(hipStream_t s) {
  gate_cancel(s);
  for (auto& st : st_) {
    if (st.eng) st.eng->reset_stream(s);
    st.done = 0;
  }
  received_ = emitted_ = 0;
  xin_base_ = acc_base_ = 0;
  acc_hi_ = 0;
  if (acc_[acur_].p) AD_HIP(hipMemsetAsync(acc_[acur_].p, 0, acc_[acur_].n * sizeof(double), s));
}

void NupolsDev::ensure_xin(int64_t need_hi, hipStream_t s) {
  if (need_hi - xin_base_ <= xcap_) return;
  int64_t min_done = received_;  // fused stages re-read two windows (2p) before their next block
  for (auto& st : st_) min_done = std::min(min_done, st.fused ? st.done - 2 * st.p : st.done);
  const int64_t nb = std::max<int64_t>(0, min_done) / 64 * 64;  // 16-byte alignment of every block start
  const int64_t keep = received_ - nb;
  const int64_t cap = std::max<int64_t>(round_up(2 * (need_hi - nb), 8192), xcap_);
  DevBuf<double>& dst = xin_[xcur_ ^ 1];
  dst.alloc((size_t)C_ * cap);
  if (keep > 0 && xin_[xcur_].p)
    launch_shift_cols(xin_[xcur_].p + (nb - xin_base_), xcap_, dst.p, cap, C_, keep, keep, s);
  if (cap != xcap_) xin_[xcur_].release();  // same size: kept for the next compaction
  xcur_ ^= 1;
  xcap_ = cap;
  xin_base_ = nb;
}

void NupolsDev::ensure_acc(int64_t lo_keep, int64_t need_hi, hipStream_t s) {
  if (need_hi - acc_base_ <= acap_ && acc_[acur_].p) return;
  const int64_t nb = std::max<int64_t>(acc_base_, lo_keep / 64 * 64);
  const int64_t keep = std::max<int64_t>(0, acc_hi_ - nb);
  const int64_t cap = std::max<int64_t>(round_up(2 * (need_hi - nb), 8192), acap_);
  DevBuf<double>& dst = acc_[acur_ ^ 1];
  dst.alloc((size_t)C_ * cap);
  if (acc_[acur_].p)
    launch_shift_cols(acc_[acur_].p + (nb - acc_base_), acap_, dst.p, cap, C_, keep, cap, s);
  else
    AD_HIP(hipMemsetAsync(dst.p, 0, dst.n * sizeof(double), s));
  if (cap != acap_) acc_[acur_].release();
  acur_ ^= 1;
  acap_ = cap;
  acc_base_ = nb;
}

int64_t NupolsDev::complete_upto() const {
  int64_t c = INT64_MAX;
  for (auto& st : st_) c = std::min(c, st.done + st.T);
  return c;
}

void NupolsDev::append(const double* d_in, int64_t in_stride, int64_t n, bool mapped_src, hipStream_t s) {
  ensure_xin(received_ + n, s);
  double* dst = xin_[xcur_].p + (received_ - xin_base_);
  if (mapped_src && C_ == 1) {
    launch_copy_f64(d_in, dst, n, s);  // a copy kernel reads mapped host memory fastest
  } else {
    AD_HIP(hipMemcpy2DAsync(dst, (size_t)xcap_ * sizeof(double), d_in, (size_t)in_stride * sizeof(double),
                            (size_t)n * sizeof(double), (size_t)C_, hipMemcpyDeviceToDevice, s));
  }
  received_ += n;
}

void NupolsDev::run_stages(int64_t emit_hi, hipStream_t s) {
  int64_t hi = acc_hi_;
  for (auto& st : st_) {
    const int64_t nb = (received_ - st.done) / st.p;
    if (nb > 0) hi = std::max(hi, st.done + nb * st.p + st.T);
  }
  ensure_acc(emitted_ - lambda_, std::max(hi, emit_hi), s);
  // Fused stages whose accumulator ranges are pairwise disjoint (every
  // lambda-aligned call: the stages firing together tile the time axis) go
  // in one launch; otherwise one launch each, in stage order.
  {
    PcSmallMulti m{};
    std::vector<std::pair<int64_t, int64_t>> ranges;
    bool disjoint = true;
    for (auto& st : st_) {
      const int64_t nb = (received_ - st.done) / st.p;
      if (!st.fused || nb == 0) continue;
      const int64_t lo = st.done + st.T, hi2 = lo + nb * st.p;
      for (auto& r : ranges)
        if (lo < r.second && r.first < hi2) disjoint = false;
      ranges.push_back({lo, hi2});
      if (m.nst == kPcMaxFused || (int64_t)m.first[m.nst] + nb > (1 << 30)) disjoint = false;
      if (!disjoint) break;
      PcSmallArgs& a = m.st[m.nst];
      a.xin = xin_[xcur_].p;
      a.xstride = xcap_;
      a.xbase = xin_base_;
      a.d0 = st.done;
      a.nb = (int)nb;
      a.H = st.H->p;
      a.acc = acc_[acur_].p;
      a.acc_stride = acap_;
      a.acc_off = st.done + st.T - acc_base_;
      a.tw = tw2048_.p;
      m.N[m.nst] = (int)(2 * st.p);
      m.first[m.nst + 1] = m.first[m.nst] + (int)nb;
      ++m.nst;
    }
    if (disjoint && m.nst > 1) {
      launch_pc_small_multi(m, C_, s);
      for (auto& st : st_)
        if (st.fused) st.done += (received_ - st.done) / st.p * st.p;
    }
  }
  for (auto& st : st_) {
    const int64_t nb = (received_ - st.done) / st.p;
    if (nb == 0) continue;
    const int64_t len = nb * st.p;
    if (st.fused) {
      PcSmallArgs a{};
      a.xin = xin_[xcur_].p;
      a.xstride = xcap_;
      a.xbase = xin_base_;
      a.d0 = st.done;
      a.nb = (int)nb;
      a.H = st.H->p;
      a.acc = acc_[acur_].p;
      a.acc_stride = acap_;
      a.acc_off = st.done + st.T - acc_base_;
      a.tw = tw2048_.p;
      if (!launch_pc_small((int)(2 * st.p), a, C_, s)) AD_FAIL(AD_ERR_INTERNAL, "fused stage size");
    } else {
      st.eng->run(xin_[xcur_].p + (st.done - xin_base_), xcap_, len, acc_[acur_].p + (st.done + st.T - acc_base_),
                  acap_, len, /*use_hist=*/true, s, 0, -1, /*accumulate=*/true);
    }
    st.done += len;
  }
  acc_hi_ = hi;
}

void NupolsDev::emit(const double* d_in, int64_t in_stride, double* d_out, int64_t out_stride, int64_t n, bool mix,
                     double wet, double dry, hipStream_t s) {
  const int64_t first = std::max<int64_t>(0, std::min<int64_t>(n, lambda_ - emitted_));
  launch_pc_emit(d_in, in_stride, d_out, out_stride, acc_[acur_].p, acap_, emitted_ - lambda_ - acc_base_, first, n,
                 C_, mix ? 1 : 0, wet, dry, s, nullptr, 0, true, 0);
  AD_HIP(hipGetLastError());
  emitted_ += n;
}

void NupolsDev::process(const double* d_in, int64_t in_stride, double* d_out, int64_t out_stride, int64_t n,
                        bool mix, double wet, double dry, hipStream_t s) {
  if (n <= 0) return;
  gate_preempt(this);  // another handle's armed emit must not hold up this call either
  gate_cancel(s);
  append(d_in, in_stride, n, false, s);           // 1. the block joins the input FIFO
  run_stages(emitted_ + n, s);                    // 2. every complete block of every stage (K3 adds at +T)
  emit(d_in, in_stride, d_out, out_stride, n, mix, wet, dry, s);  // 3. y[t - lambda]
}

void NupolsDev::ensure_mapped(int64_t n) {
  if (n <= map_cap_) return;
  if (map_cap_) AD_HIP(hipDeviceSynchronize());
  for (int i = 0; i < 2; ++i) {
    if (in_h_[i]) AD_HIP(hipHostFree(in_h_[i]));
    in_h_[i] = nullptr;
  }
  if (out_h_) AD_HIP(hipHostFree(out_h_));
  out_h_ = nullptr;
  map_cap_ = 0;
  const size_t bytes = (size_t)n * C_ * sizeof(double);
  for (int i = 0; i < 2; ++i) {
    AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&in_h_[i]), bytes, hipHostMallocMapped));
    AD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&in_d_[i]), in_h_[i], 0));
  }
  AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&out_h_), bytes, hipHostMallocMapped));
  AD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&out_d_), out_h_, 0));
  map_cap_ = n;
}

namespace {
uint64_t ctl_load(const uint64_t* w) { return __atomic_load_n(w, __ATOMIC_ACQUIRE); }
// Spins until pred() holds; after 2 s the stream is synchronised so that a
// device fault surfaces, then it gives up.
template <class Pred>
void ctl_spin(hipStream_t s, Pred&& pred) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 0;; ++i) {
    if (pred()) return;
    if ((i & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      AD_HIP(hipStreamSynchronize(s));
      if (pred()) return;
      AD_FAIL(AD_ERR_INTERNAL, "low-latency call: the pre-enqueued emit never reported");
    }
    __builtin_ia32_pause();
  }
}
}  // namespace

// Pre-enqueues the next host call's emit (k_pc_emit_gated), assuming it
// brings n samples again with the same mix: its slot, FIFO position and
// accumulator offset are fixed now and the bookkeeping advances as if it had
// run; gate_cancel undoes that when the next call differs.  Only when the
// accumulator is already complete for that call's range (the emit-first
// condition), for one channel, n <= 256, and while calls come back to back
// (interval EMA under 5 ms, fewer than 3 timed-out emits in a row): a paced
// caller gets ordinary launches, not a workgroup polling through its period.
void NupolsDev::gate_arm(int64_t n, bool mix, double wet, double dry, hipStream_t s) {
  // one measured call interval first (gap_ms_ > 0), and back-to-back calls only
  if (C_ != 1 || n > 256 || gp_.on || gmiss_ >= 3 || gap_ms_ <= 0 || gap_ms_ >= 5.0) return;
  if (emitted_ + n - lambda_ > complete_upto()) return;
  // the process-wide slot (ad_common.hpp): no other handle's launch waiting,
  // and no more library streams than hardware queues to spare
  if (!gctl_) {
    AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&gctl_), sizeof(GateCtl), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(gctl_, 0, sizeof(GateCtl));
    AD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&gctl_dev_), gctl_, 0));
    int dev = 0, khz = 0;
    AD_HIP(hipGetDevice(&dev));
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    gkhz_ = (uint64_t)khz;
  }
  if (!gate_acquire(this, &gctl_->go, s)) return;
  // the emit gives up after 4 call intervals (1 .. 20 ms): work that shares
  // its hardware queue waits behind it at most that long
  gtimeout_ = (uint64_t)(std::clamp(4.0 * gap_ms_, 1.0, 20.0) * (double)gkhz_);
  const int slot = in_slot_;
  in_slot_ ^= 1;
  if (in_used_[slot]) AD_HIP(hipEventSynchronize(ev_in_[slot]));
  ensure_xin(received_ + n, s);
  const int64_t first = std::max<int64_t>(0, std::min<int64_t>(n, lambda_ - emitted_));
  StreamGate g{};
  g.go = &gctl_dev_->go;
  g.k1_state = &gctl_dev_->state;
  g.done = &gctl_dev_->done;
  g.seq = ++gseq_;
  g.timeout = gtimeout_;
  launch_pc_emit_gated(in_d_[slot], out_d_, acc_[acur_].p, emitted_ - lambda_ - acc_base_, first, n, mix ? 1 : 0, wet,
                       dry, xin_[xcur_].p + (received_ - xin_base_), g, s);
  AD_HIP(hipGetLastError());
  AD_HIP(hipEventRecord(ev_in_[slot], s));
  in_used_[slot] = true;
  emitted_ += n;
  received_ += n;
  gp_.on = true;
  gp_.seq = g.seq;
  gp_.n = n;
  gp_.slot = slot;
  gp_.mix = mix;
  gp_.wet = wet;
  gp_.dry = dry;
}

// Drops a pre-enqueued emit (its workgroup exits at once) and rolls the
// bookkeeping back; the stream is idle afterwards.
void NupolsDev::gate_cancel(hipStream_t s) {
  if (!gp_.on) return;
  __atomic_store_n(&gctl_->go, kGateAbort, __ATOMIC_RELEASE);
  ctl_spin(s, [&] {
    const uint64_t v = ctl_load(&gctl_->state);
    return v == (gp_.seq | kGateSkipped) || v == gp_.seq;
  });
  AD_HIP(hipStreamSynchronize(s));
  if (ctl_load(&gctl_->state) != gp_.seq) {  // skipped: it neither emitted nor appended
    emitted_ -= gp_.n;
    received_ -= gp_.n;
  }
  gate_release(this);  // before clearing go: no stale gate_preempt abort after the clear
  __atomic_store_n(&gctl_->go, 0, __ATOMIC_RELEASE);
  gp_.on = false;
}

void NupolsDev::process_host(const double* in, double* out, int64_t n, bool mix, double wet, double dry,
                             hipStream_t s) {
  if (n <= 0) return;
  gate_preempt(this);  // another handle's armed emit must not hold up this call
  if (!ev_emit_) {
    AD_HIP(hipEventCreateWithFlags(&ev_emit_, hipEventDisableTiming));
    for (auto& e : ev_in_) AD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  {
    const auto now = std::chrono::steady_clock::now();
    if (glast_.time_since_epoch().count() != 0) {
      const double gap = std::chrono::duration<double, std::milli>(now - glast_).count();
      gap_ms_ = gap_ms_ == 0 ? gap : 0.75 * gap_ms_ + 0.25 * gap;
    }
    glast_ = now;
  }
  if (gp_.on && gp_.n == n && gp_.mix == mix && gp_.wet == wet && gp_.dry == dry) {
    // the pre-enqueued emit takes this block: publish it, then enqueue this
    // call's stage work and the next call's emit while the GPU emits
    std::memcpy(in_h_[gp_.slot], in, (size_t)n * sizeof(double));
    const uint64_t sq = gp_.seq;
    __atomic_store_n(&gctl_->go, sq, __ATOMIC_RELEASE);
    ctl_spin(s, [&] {
      const uint64_t v = ctl_load(&gctl_->state);
      return v == sq || v == (sq | kGateSkipped);
    });
    gp_.on = false;
    gate_release(this);
    if (ctl_load(&gctl_->state) == sq) {
      gmiss_ = 0;
      ++ghits_;
      run_stages(emitted_, s);
      gate_arm(n, mix, wet, dry, s);
      ctl_spin(s, [&] { return ctl_load(&gctl_->done) == sq; });
      std::memcpy(out, out_h_, (size_t)n * sizeof(double));
      return;
    }
    ++gmiss_;  // it gave up before this call came: roll back and run the ordinary path
    ++gtimeouts_;
    AD_HIP(hipStreamSynchronize(s));
    emitted_ -= n;
    received_ -= n;
    __atomic_store_n(&gctl_->go, 0, __ATOMIC_RELEASE);
  }
  gate_cancel(s);
  ensure_mapped(n);
  const int slot = in_slot_;
  in_slot_ ^= 1;
  if (in_used_[slot]) AD_HIP(hipEventSynchronize(ev_in_[slot]));  // the append that read this buffer is done
  std::memcpy(in_h_[slot], in, (size_t)n * C_ * sizeof(double));
  // The emit needs the accumulator only below emitted + n - lambda.  When the
  // previous calls' stage work already covers that (every lambda-aligned call
  // of at most lambda samples), the output goes out first and this call's
  // stage work runs behind it: the caller gets its block back while the GPU
  // convolves, and the next call finds that work done.
  const bool emit_first = emitted_ + n - lambda_ <= complete_upto();
  if (emit_first) {
    // one launch: emit from the accumulator + append the block to the FIFO
    ensure_xin(received_ + n, s);
    const int64_t first = std::max<int64_t>(0, std::min<int64_t>(n, lambda_ - emitted_));
    launch_pc_emit(in_d_[slot], n, out_d_, n, acc_[acur_].p, acap_, emitted_ - lambda_ - acc_base_, first, n, C_,
                   mix ? 1 : 0, wet, dry, s, xin_[xcur_].p + (received_ - xin_base_), xcap_, true, 0);
    AD_HIP(hipGetLastError());
    emitted_ += n;
    received_ += n;
    AD_HIP(hipEventRecord(ev_emit_, s));
    AD_HIP(hipEventRecord(ev_in_[slot], s));
    run_stages(emitted_, s);
  } else {
    append(in_d_[slot], n, n, true, s);
    AD_HIP(hipEventRecord(ev_in_[slot], s));
    run_stages(emitted_ + n, s);
    emit(in_d_[slot], n, out_d_, n, n, mix, wet, dry, s);
    AD_HIP(hipEventRecord(ev_emit_, s));
  }
  in_used_[slot] = true;
  if (gmiss_ >= 3 && gap_ms_ > 0 && gap_ms_ < 1.0) gmiss_ = 0;  // back to back again: retry (as gate_block)
  gate_arm(n, mix, wet, dry, s);
  AD_HIP(hipEventSynchronize(ev_emit_));
  std::memcpy(out, out_h_, (size_t)n * C_ * sizeof(double));
}

NupolsDev::~NupolsDev() {
  if (gp_.on && gctl_) __atomic_store_n(&gctl_->go, kGateAbort, __ATOMIC_RELEASE);  // release the waiting emit
  gate_release(this);
  if (gctl_) {
    (void)hipDeviceSynchronize();
    (void)hipHostFree(gctl_);
  }
  if (ev_emit_) {
    (void)hipDeviceSynchronize();
    (void)hipEventDestroy(ev_emit_);
    for (auto& e : ev_in_) (void)hipEventDestroy(e);
  }
  for (auto& p : in_h_)
    if (p) (void)hipHostFree(p);
  if (out_h_) (void)hipHostFree(out_h_);
}

}  // namespace adsp
