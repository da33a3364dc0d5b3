// Chunked, overlapped host-buffer path of the offline convolution (see
// host_pipeline.hpp).  Reference entry points served: OverlapSave.Process /
// ProcessTo (dsp/conv/overlap_save.go:126-272), OverlapAdd.Process / ProcessTo
// (overlap_add.go:108-182), and the many-channel form of the same.
#include "host_pipeline.hpp"

#include <chrono>
#include <exception>

#include <algorithm>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>

namespace adsp {

namespace {

// A fixed pool of worker threads for host memcpy (created on first use).
class Pool {
 public:
  static Pool& get() {
    static Pool p;
    return p;
  }
  void run(int64_t n, const std::function<void(int64_t)>& fn, int workers) {
    if (n <= 0) return;
    const int w = (int)std::min<int64_t>(std::min<int64_t>(workers, (int64_t)threads_.size()), n - 1);
    if (w <= 0) {
      for (int64_t i = 0; i < n; ++i) fn(i);
      return;
    }
    std::mutex m;
    std::condition_variable cv;
    int64_t next = 0;
    int active = w;
    auto body = [&] {
      for (;;) {
        int64_t i;
        {
          std::lock_guard<std::mutex> g(m);
          if (next >= n) break;
          i = next++;
        }
        fn(i);
      }
    };
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int k = 0; k < w; ++k)
        tasks_.push_back([&] {
          body();
          std::lock_guard<std::mutex> g2(m);
          if (--active == 0) cv.notify_all();
        });
    }
    cv_.notify_all();
    body();
    std::unique_lock<std::mutex> lk(m);
    cv.wait(lk, [&] { return active == 0; });
  }

 private:
  Pool() {
    const unsigned hw = std::max(2u, std::thread::hardware_concurrency());
    const int n = (int)std::min(7u, hw - 1);
    for (int i = 0; i < n; ++i) threads_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  void loop() {
    for (;;) {
      std::function<void()> t;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !tasks_.empty(); });
        if (stop_ && tasks_.empty()) return;
        t = std::move(tasks_.front());
        tasks_.pop_front();
      }
      t();
    }
  }
  std::vector<std::thread> threads_;
  std::deque<std::function<void()>> tasks_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

// Copies a [C][len] column range between the caller's per-channel buffers and
// a packed [C][len] pinned buffer, split into ~1 MiB pieces over the pool.
void copy_in(double* pin, const double* const* in, int C, int64_t col0, int64_t len, int workers) {
  const int64_t piece = std::max<int64_t>(1, (int64_t(1) << 17));  // doubles (1 MiB)
  const int64_t per = (len + piece - 1) / piece;
  parallel_for((int64_t)C * per, [&](int64_t k) {
    const int c = (int)(k / per);
    const int64_t a = (k % per) * piece, b = std::min(len, a + piece);
    std::memcpy(pin + (int64_t)c * len + a, in[c] + col0 + a, (size_t)(b - a) * sizeof(double));
  }, workers);
}
void copy_out(double* const* out, const double* pin, int C, int64_t col0, int64_t len, int workers) {
  const int64_t piece = int64_t(1) << 17;
  const int64_t per = (len + piece - 1) / piece;
  parallel_for((int64_t)C * per, [&](int64_t k) {
    const int c = (int)(k / per);
    const int64_t a = (k % per) * piece, b = std::min(len, a + piece);
    std::memcpy(out[c] + col0 + a, pin + (int64_t)c * len + a, (size_t)(b - a) * sizeof(double));
  }, workers);
}

}  // namespace

void parallel_for(int64_t n, const std::function<void(int64_t)>& fn, int workers) {
  Pool::get().run(n, fn, workers);
}

namespace {
// Process-wide registry of the caller ranges page-locked by calls in flight.
// hipHostRegister is process-wide, so two threads that pass the same (or an
// overlapping) array must not register it twice or unregister it under each
// other's copies: a range is registered once, every call holding it takes a
// reference, and it is unregistered when the last reference goes.  A call
// whose range only partly overlaps a registered one does not register its own
// (its copies stay pageable) but still holds the overlapping entries, so their
// pages stay locked while its copies run.
struct PinEntry {
  uintptr_t lo, hi;
  int refs;
};
std::mutex g_pin_mu;
std::vector<PinEntry> g_pins;

bool pin_acquire(const void* ptr, size_t bytes, std::vector<uintptr_t>& held) {
  const uintptr_t lo = (uintptr_t)ptr, hi = lo + bytes;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  bool covered = false, overlap = false;
  for (PinEntry& e : g_pins)
    if (e.lo < hi && lo < e.hi) {
      overlap = true;
      covered = covered || (e.lo <= lo && hi <= e.hi);
      ++e.refs;
      held.push_back(e.lo);
    }
  if (overlap) return covered;
  if (hipHostRegister(const_cast<void*>(ptr), bytes, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  g_pins.push_back(PinEntry{lo, hi, 1});
  held.push_back(lo);
  return true;
}

void pin_release(std::vector<uintptr_t>& held) {
  std::lock_guard<std::mutex> lk(g_pin_mu);
  for (uintptr_t k : held)
    for (size_t i = 0; i < g_pins.size(); ++i)
      if (g_pins[i].lo == k) {
        if (--g_pins[i].refs == 0) {
          (void)hipHostUnregister((void*)k);
          g_pins.erase(g_pins.begin() + (ptrdiff_t)i);
        }
        break;
      }
  held.clear();
}
}  // namespace

HostPin::HostPin(const void* ptr, size_t bytes, size_t min_bytes) {
#ifdef AD_HOSTPIN_OFF  // tools/ A/B builds only
  return;
#endif
  if (!ptr || bytes < min_bytes) return;
  ok = pin_acquire(ptr, bytes, held);
}
HostPin::~HostPin() {
  if (held.empty()) return;
  // unwinding from an error: copies into or out of these pages may still be
  // queued, and the caller may free them as soon as the error returns
  if (std::uncaught_exceptions() > 0) (void)hipDeviceSynchronize();
  pin_release(held);
}

HostPipeline::HostPipeline(int) {
  AD_HIP(lib_stream_create(&s_in_));
  AD_HIP(lib_stream_create(&s_out_));
  for (int i = 0; i < 2; ++i) {
    AD_HIP(hipEventCreateWithFlags(&ev_in_[i], hipEventDisableTiming));
    AD_HIP(hipEventCreateWithFlags(&ev_out_[i], hipEventDisableTiming));
  }
  AD_HIP(hipEventCreateWithFlags(&ev_comp_, hipEventDisableTiming));
}

HostPipeline::~HostPipeline() {
  if (s_in_) (void)hipStreamSynchronize(s_in_);
  if (s_out_) (void)hipStreamSynchronize(s_out_);
  for (int i = 0; i < 2; ++i) {
    if (pin_in_[i]) (void)hipHostFree(pin_in_[i]);
    if (pin_out_[i]) (void)hipHostFree(pin_out_[i]);
    if (ev_in_[i]) (void)hipEventDestroy(ev_in_[i]);
    if (ev_out_[i]) (void)hipEventDestroy(ev_out_[i]);
  }
  if (ev_comp_) (void)hipEventDestroy(ev_comp_);
  if (s_in_) (void)lib_stream_destroy(s_in_);
  if (s_out_) (void)lib_stream_destroy(s_out_);
}

void HostPipeline::ensure_pinned(int64_t doubles) {
  if (doubles <= pin_cap_) return;
  for (int i = 0; i < 2; ++i) {
    if (pin_in_[i]) AD_HIP(hipHostFree(pin_in_[i]));
    if (pin_out_[i]) AD_HIP(hipHostFree(pin_out_[i]));
    pin_in_[i] = pin_out_[i] = nullptr;
  }
  pin_cap_ = 0;
  for (int i = 0; i < 2; ++i) {
    AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&pin_in_[i]), (size_t)doubles * sizeof(double), hipHostMallocDefault));
    AD_HIP(hipHostMalloc(reinterpret_cast<void**>(&pin_out_[i]), (size_t)doubles * sizeof(double), hipHostMallocDefault));
  }
  pin_cap_ = doubles;
}

namespace {
// Page-locks [p, p + bytes) for the scope of one call (hipHostRegister);
// `ok` is false when the runtime refuses, and the caller then stages.
// Shares the process-wide registry with HostPin (another thread may hold
// the same arrays).
struct Registration {
  std::vector<uintptr_t> held;
  bool ok = true;
  void add(const void* p, size_t bytes) {
    if (!ok) return;
    ok = pin_acquire(p, bytes, held);
  }
  void release() { pin_release(held); }
  ~Registration() { release(); }
};

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}
}  // namespace

void HostPipeline::offline(Upols& eng, const double* const* in, int C, int64_t n, double* const* out,
                           int64_t out_len, hipStream_t s) {
  const int64_t L = eng.hop();
  if (C != eng.channels()) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "channel count differs from the engine's");
  const int mode = mode_;
  const int64_t bytes = (int64_t)C * (n + out_len) * 8;
  last_reg_ms_ = last_xfer_ms_ = last_unreg_ms_ = 0;
  if (mode == kRegister || (mode == kAuto && bytes >= (int64_t(64) << 20))) {
    auto t0 = std::chrono::steady_clock::now();
    Registration reg;
    for (int c = 0; c < C && reg.ok; ++c) {
      reg.add(in[c], (size_t)n * sizeof(double));
      if (static_cast<const void*>(out[c]) != static_cast<const void*>(in[c]))
        reg.add(out[c], (size_t)out_len * sizeof(double));
    }
    last_reg_ms_ = ms_since(t0);
    if (reg.ok) {
      t0 = std::chrono::steady_clock::now();
      try {
        offline_direct(eng, in, C, n, out, out_len, s);
      } catch (...) {
        // DMAs into / out of the caller's pages may still be queued: drain
        // every stream of the call before ~Registration unlocks those pages
        // (the caller may free them as soon as the error returns)
        (void)hipStreamSynchronize(s_in_);
        (void)hipStreamSynchronize(s_out_);
        (void)hipStreamSynchronize(s);
        throw;
      }
      last_xfer_ms_ = ms_since(t0);
      t0 = std::chrono::steady_clock::now();
      reg.release();
      last_unreg_ms_ = ms_since(t0);
      return;
    }
  }
  const auto t_stage = std::chrono::steady_clock::now();
  struct StageTime {
    double* dst;
    std::chrono::steady_clock::time_point t;
    ~StageTime() { *dst = ms_since(t); }
  } stage_time{&last_xfer_ms_, t_stage};
  // chunk: S input samples per channel (a multiple of L), C*S doubles <= kChunkBytes
  int64_t S = std::max<int64_t>(L, (kChunkBytes / 8 / C) / L * L);
  // at least ~4 chunks when the signal allows (transfers overlap the compute
  // only across chunks); small calls: small pinned buffers
  S = std::min(S, std::max<int64_t>(L, ((n + 3) / 4 + L - 1) / L * L));
  const int64_t nblocks = (out_len + L - 1) / L;
  ensure_pinned((int64_t)C * S);
  din_.reserve((size_t)C * n);
  dout_.reserve((size_t)C * out_len);
  eng.begin_offline(s);

  // Output pieces of <= S samples, each waiting for the compute event of the
  // segment that produced it.  Piece k goes through pin_out_[k % 2].
  struct Piece {
    int64_t o0, len;
  };
  std::vector<Piece> pending;  // enqueued on s_out_, not yet copied to the caller
  int64_t out_issued = 0;      // output samples enqueued for D2H
  int64_t nout = 0;            // pieces enqueued so far
  auto drain_one = [&] {       // completes the oldest pending piece
    const Piece p = pending.front();
    const int slot = (int)((nout - (int64_t)pending.size()) % 2);
    AD_HIP(hipEventSynchronize(ev_out_[slot]));
    copy_out(out, pin_out_[slot], C, p.o0, p.len, workers_);
    pending.erase(pending.begin());
  };
  auto issue_output = [&](int64_t upto) {  // D2H of output [out_issued, upto), after ev_comp_
    AD_HIP(hipStreamWaitEvent(s_out_, ev_comp_, 0));
    while (out_issued < upto) {
      if (pending.size() == 2) drain_one();  // pin_out slot reuse
      const int slot = (int)(nout % 2);
      const int64_t len = std::min(S, upto - out_issued);
      AD_HIP(hipMemcpy2DAsync(pin_out_[slot], (size_t)len * sizeof(double), dout_.p + out_issued,
                              (size_t)out_len * sizeof(double), (size_t)len * sizeof(double), (size_t)C,
                              hipMemcpyDeviceToHost, s_out_));
      AD_HIP(hipEventRecord(ev_out_[slot], s_out_));
      pending.push_back({out_issued, len});
      out_issued += len;
      ++nout;
    }
  };

  const int64_t nin = (n + S - 1) / S;
  int64_t jdone = 0;
  for (int64_t i = 0; i < nin; ++i) {
    const int slot = (int)(i % 2);
    const int64_t c0 = i * S, len = std::min(S, n - c0);
    if (i >= 2) AD_HIP(hipEventSynchronize(ev_in_[slot]));  // pin_in slot free again
    copy_in(pin_in_[slot], in, C, c0, len, workers_);
    AD_HIP(hipMemcpy2DAsync(din_.p + c0, (size_t)n * sizeof(double), pin_in_[slot], (size_t)len * sizeof(double),
                            (size_t)len * sizeof(double), (size_t)C, hipMemcpyHostToDevice, s_in_));
    AD_HIP(hipEventRecord(ev_in_[slot], s_in_));
    // blocks whose windows end inside the data on the device: j + 1 <= (c0 + len) / L
    const int64_t je = (i == nin - 1) ? nblocks : std::min(nblocks, (c0 + len) / L);
    if (je > jdone) {
      AD_HIP(hipStreamWaitEvent(s, ev_in_[slot], 0));
      eng.run(din_.p, n, n, dout_.p, out_len, out_len, /*use_hist=*/false, s, jdone, je);
      AD_HIP(hipEventRecord(ev_comp_, s));
      jdone = je;
      issue_output(std::min(out_len, je * L));
    }
    // keep the host busy with the previous output while the device works
    while (pending.size() > 1) drain_one();
  }
  if (jdone < nblocks) {  // (only when n == 0, which the callers reject)
    eng.run(din_.p, n, n, dout_.p, out_len, out_len, false, s, jdone, nblocks);
    AD_HIP(hipEventRecord(ev_comp_, s));
    issue_output(out_len);
  }
  while (!pending.empty()) drain_one();
  // nothing of this call may still read din_/dout_ when the next call starts
  AD_HIP(hipStreamSynchronize(s_in_));
}

// Registered form: the caller's pages are locked for this call, so the chunks
// go straight between them and the device (no host memcpy).  Same chunking
// and stream overlap as the staged form.
void HostPipeline::offline_direct(Upols& eng, const double* const* in, int C, int64_t n, double* const* out,
                                  int64_t out_len, hipStream_t s) {
  const int64_t L = eng.hop();
  int64_t S = std::max<int64_t>(L, (kChunkBytes / 8 / C) / L * L);
  S = std::min(S, std::max<int64_t>(L, ((n + 3) / 4 + L - 1) / L * L));
  const int64_t nblocks = (out_len + L - 1) / L;
  din_.reserve((size_t)C * n);
  dout_.reserve((size_t)C * out_len);
  eng.begin_offline(s);
  const int64_t nin = (n + S - 1) / S;
  int64_t jdone = 0, out_issued = 0;
  for (int64_t i = 0; i < nin; ++i) {
    const int64_t c0 = i * S, len = std::min(S, n - c0);
    for (int c = 0; c < C; ++c)
      AD_HIP(hipMemcpyAsync(din_.p + (int64_t)c * n + c0, in[c] + c0, (size_t)len * sizeof(double),
                            hipMemcpyHostToDevice, s_in_));
    AD_HIP(hipEventRecord(ev_in_[0], s_in_));
    const int64_t je = (i == nin - 1) ? nblocks : std::min(nblocks, (c0 + len) / L);
    if (je > jdone) {
      AD_HIP(hipStreamWaitEvent(s, ev_in_[0], 0));
      eng.run(din_.p, n, n, dout_.p, out_len, out_len, /*use_hist=*/false, s, jdone, je);
      AD_HIP(hipEventRecord(ev_comp_, s));
      jdone = je;
      const int64_t upto = std::min(out_len, je * L);
      AD_HIP(hipStreamWaitEvent(s_out_, ev_comp_, 0));
      for (int c = 0; c < C; ++c)
        AD_HIP(hipMemcpyAsync(out[c] + out_issued, dout_.p + (int64_t)c * out_len + out_issued,
                              (size_t)(upto - out_issued) * sizeof(double), hipMemcpyDeviceToHost, s_out_));
      out_issued = upto;
    }
  }
  AD_HIP(hipStreamSynchronize(s_out_));
  AD_HIP(hipStreamSynchronize(s_in_));
}

}  // namespace adsp
