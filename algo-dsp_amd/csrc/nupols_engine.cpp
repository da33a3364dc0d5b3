// Host runtime of the non-uniformly partitioned engine (see nupols_engine.hpp).
#include "nupols_engine.hpp"

#include <algorithm>
#include <cstring>

#include "conv_kernels.hpp"

namespace adsp {

Nupols::Nupols(int device, const double* h, int64_t K, int64_t lambda, int64_t p_max)
    : device_(device), lambda_(lambda) {
  if (lambda < 64 || !is_pow2(lambda) || p_max < lambda || !is_pow2(p_max) || p_max > 8192)
    AD_FAIL(AD_ERR_INTERNAL, "Nupols: bad partition sizes");
  // Stage layout: two partitions per size while the size doubles, the rest
  // at p_max.  T_{s+1} = T_s + n_s p_s >= p_{s+1} - lambda holds by construction.
  int64_t T = 0, p = lambda;
  while (T < K) {
    int64_t n = 2;
    if (p >= p_max) n = (K - T + p - 1) / p;
    Stage s;
    s.p = p;
    s.T = T;
    s.taps = std::min<int64_t>(n * p, K - T);
    st_.push_back(std::move(s));
    T += n * p;
    if (p < p_max) p *= 2;
  }
  for (auto& s : st_) {
    AD_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    s.cap = std::max<int64_t>(1, kBatchSamples / s.p);
    s.eng.reset(new Upols(device, h + s.T, 1, s.taps, (int)s.p, 1, nullptr, (int)s.cap, s.stream));
    const size_t bytes = (size_t)(s.cap * s.p) * sizeof(double);
    AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.in_h), bytes, hipHostMallocMapped));
    AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.out_h), bytes, hipHostMallocMapped));
    AD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.in_d), s.in_h, 0));
    AD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&s.out_d), s.out_h, 0));
  }
  reset();
}

Nupols::~Nupols() {
  for (auto& s : st_) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    s.eng.reset();
    if (s.in_h) (void)hipHostFree(s.in_h);
    if (s.out_h) (void)hipHostFree(s.out_h);
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
}

void Nupols::reset() {
  for (auto& s : st_) {
    s.eng->reset_stream(s.stream);
    s.done = 0;
    s.pending = false;
  }
  for (auto& s : st_) AD_HIP(hipStreamSynchronize(s.stream));
  xin_.clear();
  xin_base_ = 0;
  received_ = 0;
  acc_.clear();
  acc_base_ = 0;
  emitted_ = 0;
}

void Nupols::process(const double* in, int64_t n, double* out) {
  xin_.insert(xin_.end(), in, in + n);
  received_ += n;
  // A stage run's block [d, d + p) first contributes to output time d + T_s,
  // and T_s + lambda >= p_s, so a run launched for a block that completes in
  // this call is never needed before the next call (the call emits up to
  // time received - 1 - lambda).  Runs are therefore left in flight across
  // calls: the device works while the caller produces the next block, and a
  // run is synchronised only when its buffers are reused, or when a call
  // emits an output it contributes to (calls longer than a stage's block).
  auto finish = [&](Stage& s) {
    AD_HIP(hipStreamSynchronize(s.stream));
    const int64_t t0 = s.pend_d + s.T;  // absolute output time of the block's first sample
    const int64_t need = t0 + s.pend_n - acc_base_;
    if ((int64_t)acc_.size() < need) acc_.resize((size_t)need, 0.0);
    double* a = acc_.data() + (t0 - acc_base_);
    for (int64_t k = 0; k < s.pend_n; ++k) a[k] += s.out_h[k];
    s.pending = false;
  };
  for (bool launched = true; launched;) {
    launched = false;
    for (auto& s : st_) {
      // every complete block of this stage (up to cap) in one launch
      const int64_t nb = std::min((received_ - s.done) / s.p, s.cap);
      if (nb == 0) continue;
      if (s.pending) finish(s);  // in_h / out_h are reused
      const int64_t len = nb * s.p, off = s.done - xin_base_;
      std::memcpy(s.in_h, xin_.data() + off, (size_t)len * sizeof(double));
      s.eng->run(s.in_d, len, len, s.out_d, len, len, /*use_hist=*/true, s.stream);
      s.pending = true;
      s.pend_d = s.done;
      s.pend_n = len;
      s.done += len;
      launched = true;
    }
  }
  const int64_t last_u = emitted_ + n - 1 - lambda_;  // latest output time this call emits
  for (auto& s : st_)
    if (s.pending && s.pend_d + s.T <= last_u) finish(s);
  // Emit: y[o] = linear conv at o - lambda (complete by the T_s + lambda >= p_s rule).
  for (int64_t i = 0; i < n; ++i) {
    const int64_t u = emitted_ + i - lambda_;
    if (u < 0) {
      out[i] = 0.0;
      continue;
    }
    const int64_t idx = u - acc_base_;
    out[i] = idx < (int64_t)acc_.size() ? acc_[(size_t)idx] : 0.0;
  }
  emitted_ += n;
  // Drop what no later output or stage needs.
  const int64_t keep_out = emitted_ - lambda_;
  const int64_t drop_acc = std::min<int64_t>(std::max<int64_t>(keep_out - acc_base_, 0), (int64_t)acc_.size());
  acc_.erase(acc_.begin(), acc_.begin() + drop_acc);
  acc_base_ += drop_acc;
  int64_t min_done = received_;
  for (auto& s : st_) min_done = std::min(min_done, s.done);
  const int64_t drop_in = std::min<int64_t>(std::max<int64_t>(min_done - xin_base_, 0), (int64_t)xin_.size());
  xin_.erase(xin_.begin(), xin_.begin() + drop_in);
  xin_base_ += drop_in;
}

// ---------------------------------------------------------------------------
// NupolsDev
// ---------------------------------------------------------------------------
namespace {
int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
}  // namespace

NupolsDev::NupolsDev(int device, const double* h, int64_t K, int64_t lambda, int64_t p_max, int channels,
                     hipStream_t s)
    : C_(channels), lambda_(lambda) {
  if (lambda < 64 || !is_pow2(lambda) || p_max < lambda || !is_pow2(p_max) || p_max > 8192 || channels < 1)
    AD_FAIL(AD_ERR_INTERNAL, "NupolsDev: bad geometry");
  // same stage layout as Nupols (two partitions per size, the rest at p_max)
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
  for (auto& st : st_) {
    // up to 64 blocks (and >= 8192 samples) per launch chunk: long calls batch
    const int jc = (int)std::max<int64_t>(64, 8192 / st.p);
    st.eng.reset(new Upols(device, h + st.T, 1, st.taps, (int)st.p, channels, nullptr, jc, s));
  }
  reset(s);
}

void NupolsDev::reset(hipStream_t s) {
  for (auto& st : st_) {
    st.eng->reset_stream(s);
    st.done = 0;
  }
  received_ = emitted_ = 0;
  xin_base_ = acc_base_ = 0;
  acc_hi_ = 0;
  if (acc_[acur_].p) AD_HIP(hipMemsetAsync(acc_[acur_].p, 0, acc_[acur_].n * sizeof(double), s));
}

void NupolsDev::ensure_xin(int64_t need_hi, hipStream_t s) {
  if (need_hi - xin_base_ <= xcap_) return;
  int64_t min_done = received_;
  for (auto& st : st_) min_done = std::min(min_done, st.done);
  const int64_t nb = min_done / 64 * 64;  // keep 16-byte alignment of every stage's block start
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

void NupolsDev::process(const double* d_in, int64_t in_stride, double* d_out, int64_t out_stride, int64_t n,
                        bool mix, double wet, double dry, hipStream_t s) {
  if (n <= 0) return;
  // 1. append the block to the input FIFO
  ensure_xin(received_ + n, s);
  AD_HIP(hipMemcpy2DAsync(xin_[xcur_].p + (received_ - xin_base_), (size_t)xcap_ * sizeof(double), d_in,
                          (size_t)in_stride * sizeof(double), (size_t)n * sizeof(double), (size_t)C_,
                          hipMemcpyDeviceToDevice, s));
  received_ += n;
  // 2. every complete block of every stage; K3 adds into the accumulator at +T
  int64_t hi = acc_hi_;
  for (auto& st : st_) {
    const int64_t nb = (received_ - st.done) / st.p;
    if (nb > 0) hi = std::max(hi, st.done + nb * st.p + st.T);
  }
  ensure_acc(emitted_ - lambda_, std::max(hi, emitted_ + n), s);
  for (auto& st : st_) {
    const int64_t nb = (received_ - st.done) / st.p;
    if (nb == 0) continue;
    const int64_t len = nb * st.p;
    st.eng->run(xin_[xcur_].p + (st.done - xin_base_), xcap_, len, acc_[acur_].p + (st.done + st.T - acc_base_),
                acap_, len, /*use_hist=*/true, s, 0, -1, /*accumulate=*/true);
    st.done += len;
  }
  acc_hi_ = hi;
  // 3. emit y[t - lambda] for t in [emitted, emitted + n)
  const int64_t first = std::max<int64_t>(0, std::min<int64_t>(n, lambda_ - emitted_));
  launch_pc_emit(d_in, in_stride, d_out, out_stride, acc_[acur_].p, acap_, emitted_ - lambda_ - acc_base_, first, n,
                 C_, mix ? 1 : 0, wet, dry, s);
  AD_HIP(hipGetLastError());
  emitted_ += n;
}

}  // namespace adsp
