// Host runtime of the non-uniformly partitioned engine (see nupols_engine.hpp).
#include "nupols_engine.hpp"

#include <algorithm>
#include <cstring>

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

}  // namespace adsp
