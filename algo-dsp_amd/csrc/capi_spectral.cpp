// C ABI of the spectral-division / correlation row:
// CorrelateFFT (dsp/conv/correlate.go:111-172), Deconvolve with its naive,
// regularised and Wiener methods (deconvolve.go:72-323) and InverseFilter
// (deconvolve.go:354-394), on the device FFT of bigfft.hip.  Each call copies
// its host inputs in, runs forward FFTs of the zero-padded real inputs (two
// transforms in one batched launch per pass), one pointwise kernel, one
// inverse FFT whose last pass writes the scaled real part, and copies out.
#pragma clang fp contract(off)  // host-side variance/NSR arithmetic as Go computes it

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <exception>
#include <mutex>
#include <string>

#include "ad_common.hpp"
#include "bigfft.hpp"
#include "host_pipeline.hpp"

using namespace adsp;

namespace {

// deconvolve.go:326-349 variance (two passes, sequential sums)
double go_variance(const double* x, int64_t n) {
  if (n == 0) return 0;
  double mean = 0;
  for (int64_t i = 0; i < n; ++i) mean += x[i];
  mean /= (double)n;
  double sum = 0;
  for (int64_t i = 0; i < n; ++i) {
    const double d = x[i] - mean;
    sum += d * d;
  }
  return sum / (double)n;
}

// Per-device cache of FFT plans (twiddle tables) and grow-only work buffers,
// so repeated calls of one size allocate nothing.  One lock per call: the
// reference's functions are stateless, the cache is an implementation detail.
struct DeviceCache {
  std::mutex mu;
  std::map<int64_t, std::unique_ptr<BigFft>> plans;
  DevBuf<double2> spec, scratch;
  DevBuf<double> xr, res;
  DevBuf<unsigned long long> bad, amax;
  // The work buffers (and the first pass's max-abs counter, which the kernel
  // resets itself) are shared by every call on the device, whatever its
  // stream: a call waits for the previous call's last launch when that was
  // enqueued on another stream (two CorrelateFFT calls on two
  // streams interleaved the counter's increments).
  hipEvent_t last = nullptr;
  hipStream_t last_stream = nullptr;
  bool pending = false;  // `last` covers a device call that may still run
};

// Orders a call on stream s after the previous call on the device; on
// destruction records the call's end (device calls) or, for host calls that
// synchronised s, clears it.
struct CallOrder {
  DeviceCache& dc;
  hipStream_t s;
  bool async;
  CallOrder(DeviceCache& c, hipStream_t st, bool device_call) : dc(c), s(st), async(device_call) {
    if (dc.pending && dc.last_stream != s) AD_HIP(hipStreamWaitEvent(s, dc.last, 0));
  }
  ~CallOrder() {
    if (!async) {
      if (std::uncaught_exceptions() == 0) dc.pending = false;
      return;
    }
    if (!dc.last && hipEventCreateWithFlags(&dc.last, hipEventDisableTiming) != hipSuccess) return;
    if (hipEventRecord(dc.last, s) == hipSuccess) {
      dc.last_stream = s;
      dc.pending = true;
    }
  }
};
DeviceCache& cache(int dev) {
  static std::mutex m;
  static std::map<int, std::unique_ptr<DeviceCache>> all;
  std::lock_guard<std::mutex> g(m);
  auto& c = all[dev];
  if (!c) c.reset(new DeviceCache);
  return *c;
}

// Forward FFTs of `batch` zero-padded real arrays in xr ([batch][N]); inverse
// of spec[0..N) into res (real part, 1/N as algo-fft's Inverse).
struct SpectralRun {
  int64_t N;
  DeviceCache& dc;
  BigFft* fft;
  SpectralRun(DeviceCache& c, int64_t n) : N(n), dc(c) {
    auto& p = dc.plans[n];
    if (!p) p.reset(new BigFft(n));
    fft = p.get();
  }
  void forward(const double* xr_dev, int batch, hipStream_t s) {
    dc.spec.reserve((size_t)(N * batch));
    dc.scratch.reserve((size_t)(2 * N * batch));
    fft->run(true, nullptr, xr_dev, N, N, dc.spec.p, nullptr, N, 1.0, batch, dc.scratch.p, s);
  }
  void inverse(hipStream_t s) {
    dc.res.reserve((size_t)N);
    fft->run(false, dc.spec.p, nullptr, 0, N, nullptr, dc.res.p, N, 1.0 / (double)N, 1, dc.scratch.p, s);
  }
  // CorrelateFFT with fused edges: one forward transform of a + i b, the
  // inverse of the Hermitian product at half length (N >= 32: both plans
  // have passes)
  bool fused() const { return N >= 32; }
  void correlate(const double* a, int64_t n, const double* b, int64_t m, double* out, hipStream_t s) {
    auto& h = dc.plans[N / 2];
    if (!h) h.reset(new BigFft(N / 2));
    dc.spec.reserve((size_t)N);
    dc.scratch.reserve((size_t)(2 * N));
    if (dc.amax.n < (size_t)kAbsmaxWords) {  // zeroed once: the kernel resets its counter itself
      dc.amax.reserve(kAbsmaxWords);
      AD_HIP(hipMemsetAsync(dc.amax.p, 0, dc.amax.n * sizeof(unsigned long long), s));
    }
    fft->correlate_half(*h, a, n, b, m, dc.spec.p, out, dc.scratch.p, dc.amax.p, s);
  }
  // Deconvolve / InverseFilter through the same structure (x: n, h: m real
  // samples, h may be null): the first n_front real outputs to out.
  void spectral(int op, double eps, unsigned long long* bad, const double* x, int64_t n, const double* h, int64_t m,
                int64_t n_front, double* out, hipStream_t s) {
    auto& hp = dc.plans[N / 2];
    if (!hp) hp.reset(new BigFft(N / 2));
    const bool two = h != nullptr;  // Deconvolve: separate transforms of x and h
    dc.spec.reserve((size_t)(two ? 2 * N : N));
    dc.scratch.reserve((size_t)(two ? 4 * N : 2 * N));
    fft->spectral_half(*hp, op, eps, bad, !two, x, n, h, h ? m : 0, n_front, 0, N, dc.spec.p, out, dc.scratch.p, s);
  }
  double2* spec() const { return dc.spec.p; }
  double* res() const { return dc.res.p; }
};

// Stages host arrays into one zero-padded [count][N] device buffer.
void stage_real(DevBuf<double>& buf, int64_t N, const double* const* src, const int64_t* len, int count,
                hipStream_t s) {
  buf.reserve((size_t)(N * count));
  AD_HIP(hipMemsetAsync(buf.p, 0, (size_t)(N * count) * sizeof(double), s));
  for (int i = 0; i < count; ++i)
    if (len[i] > 0)
      AD_HIP(hipMemcpyAsync(buf.p + (int64_t)i * N, src[i], (size_t)len[i] * sizeof(double), hipMemcpyHostToDevice,
                            s));
}

}  // namespace

extern "C" {

ad_deconv_options ad_deconv_default_options(void) {
  // deconvolve.go:57-63 DefaultDeconvOptions
  ad_deconv_options o;
  o.method = AD_DECONV_REGULARIZED;
  o.epsilon = 1e-6;
  o.noise_variance = 0;
  o.signal_variance = 0;
  return o;
}

int ad_correlate_fft(const double* a, int64_t n, const double* b, int64_t m, double* out, int device) {
  return guard([&] {
    if (n <= 0 || m <= 0 || !a || !b) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (!out) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null output");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    DeviceCache& dc = cache(dev);
    std::lock_guard<std::mutex> g(dc.mu);
    hipStream_t s = nullptr;
    CallOrder order(dc, s, /*device_call=*/false);
    const int64_t N = next_pow2(n + m - 1);  // correlate.go:119
    SpectralRun run(dc, N);
    // the caller's arrays page-locked for the call: DMA, not pageable staging
    // (a fresh output array otherwise faults its pages in during the copy)
    const HostPin pa(a, (size_t)n * 8), pb(b, (size_t)m * 8), po(out, (size_t)(n + m - 1) * 8);
    if (run.fused()) {
      // a and b to the device unpadded, the fused transforms (see the device
      // form below), the n + m - 1 lags back in one copy
      dc.xr.reserve((size_t)(n + m));
      dc.res.reserve((size_t)(n + m - 1));
      AD_HIP(hipMemcpyAsync(dc.xr.p, a, (size_t)n * sizeof(double), hipMemcpyHostToDevice, s));
      AD_HIP(hipMemcpyAsync(dc.xr.p + n, b, (size_t)m * sizeof(double), hipMemcpyHostToDevice, s));
      run.correlate(dc.xr.p, n, dc.xr.p + n, m, dc.res.p, s);
      AD_HIP(hipMemcpyAsync(out, dc.res.p, (size_t)(n + m - 1) * sizeof(double), hipMemcpyDeviceToHost, s));
      AD_HIP(hipStreamSynchronize(s));
      return;
    }
    const double* src[2] = {a, b};
    const int64_t len[2] = {n, m};
    stage_real(dc.xr, N, src, len, 2, s);
    run.forward(dc.xr.p, 2, s);
    launch_spec_op(kSpecCorr, run.spec(), run.spec() + N, N, 0.0, nullptr, s);
    run.inverse(s);
    // correlate.go:165-171: lags 0..n-1 from the front, -(m-1)..-1 from the back
    AD_HIP(hipMemcpyAsync(out + (m - 1), run.res(), (size_t)n * sizeof(double), hipMemcpyDeviceToHost, s));
    if (m > 1)
      AD_HIP(hipMemcpyAsync(out, run.res() + (N - m + 1), (size_t)(m - 1) * sizeof(double), hipMemcpyDeviceToHost,
                            s));
    AD_HIP(hipStreamSynchronize(s));
  });
}

int ad_correlate_fft_device(const double* a, int64_t n, const double* b, int64_t m, double* out, int device,
                            void* stream) {
  return guard([&] {
    if (n <= 0 || m <= 0 || !a || !b) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (!out) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null output");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    DeviceCache& dc = cache(dev);
    std::lock_guard<std::mutex> g(dc.mu);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    CallOrder order(dc, s, /*device_call=*/true);
    const int64_t N = next_pow2(n + m - 1);
    SpectralRun run(dc, N);
    if (run.fused()) {
      // one forward transform of a + i b straight from the caller's arrays, the
      // inverse of A conj(B) at half length, its outputs written in lag order
      run.correlate(a, n, b, m, out, s);
      return;
    }
    dc.xr.reserve((size_t)(2 * N));
    AD_HIP(hipMemsetAsync(dc.xr.p, 0, (size_t)(2 * N) * sizeof(double), s));
    AD_HIP(hipMemcpyAsync(dc.xr.p, a, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, s));
    AD_HIP(hipMemcpyAsync(dc.xr.p + N, b, (size_t)m * sizeof(double), hipMemcpyDeviceToDevice, s));
    run.forward(dc.xr.p, 2, s);
    launch_spec_op(kSpecCorr, run.spec(), run.spec() + N, N, 0.0, nullptr, s);
    run.inverse(s);
    AD_HIP(hipMemcpyAsync(out + (m - 1), run.res(), (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, s));
    if (m > 1)
      AD_HIP(hipMemcpyAsync(out, run.res() + (N - m + 1), (size_t)(m - 1) * sizeof(double), hipMemcpyDeviceToDevice,
                            s));
    // asynchronous on the caller's stream: the cached work buffers are reused
    // only by later calls, which the lock and CallOrder serialise
  });
}

int ad_deconvolve(const double* signal, int64_t n, const double* kernel, int64_t m, const ad_deconv_options* opts,
                  double* out, int64_t out_cap, int64_t* out_len, int device) {
  return guard([&] {
    // deconvolve.go:72-101
    if (n <= 0 || !signal) AD_FAIL(AD_ERR_EMPTY_INPUT, "conv: empty input");
    if (m <= 0 || !kernel) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    ad_deconv_options o = opts ? *opts : ad_deconv_default_options();
    int op = kSpecReg;
    double eps = o.epsilon;
    switch (o.method) {
      case AD_DECONV_NAIVE:
        op = kSpecNaive;
        break;
      case AD_DECONV_REGULARIZED:
        if (eps <= 0) eps = 1e-6;
        break;
      case AD_DECONV_WIENER: {  // deconvolve.go:235-262
        double noise = o.noise_variance, sig = o.signal_variance;
        if (sig <= 0) sig = go_variance(signal, n);
        if (noise <= 0) noise = sig * 0.01;
        double nsr = noise / sig;
        if (nsr <= 0) nsr = 1e-6;
        eps = nsr;
        break;
      }
      default:
        eps = 1e-6;
        break;
    }
    const int64_t N = next_pow2(n);  // deconvolve.go:114,180,264: the SIGNAL length
    if (m > N) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "conv: kernel longer than the transform (reference indexes out of range)");
    int64_t olen = n - m + 1;
    if (olen <= 0) olen = n;
    if (out_len) *out_len = olen;
    if (!out || out_cap < olen) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "output capacity too small");
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    DeviceCache& dc = cache(dev);
    std::lock_guard<std::mutex> g(dc.mu);
    hipStream_t s = nullptr;
    CallOrder order(dc, s, /*device_call=*/false);
    SpectralRun run(dc, N);
    const HostPin ps(signal, (size_t)n * 8), pk(kernel, (size_t)m * 8), po(out, (size_t)olen * 8);
    if (run.fused()) {
      // one forward transform of signal + i kernel, the division fused into
      // the inverse's first pass, the inverse at half length, olen outputs
      dc.xr.reserve((size_t)(n + m));
      dc.res.reserve((size_t)olen);
      AD_HIP(hipMemcpyAsync(dc.xr.p, signal, (size_t)n * sizeof(double), hipMemcpyHostToDevice, s));
      AD_HIP(hipMemcpyAsync(dc.xr.p + n, kernel, (size_t)m * sizeof(double), hipMemcpyHostToDevice, s));
      if (op == kSpecNaive) {
        dc.bad.reserve(1);
        AD_HIP(hipMemsetAsync(dc.bad.p, 0xff, sizeof(unsigned long long), s));
      }
      run.spectral(op, eps, op == kSpecNaive ? dc.bad.p : nullptr, dc.xr.p, n, dc.xr.p + n, m, olen, dc.res.p, s);
      if (op == kSpecNaive) {
        unsigned long long first = 0;
        AD_HIP(hipMemcpyAsync(&first, dc.bad.p, sizeof(first), hipMemcpyDeviceToHost, s));
        AD_HIP(hipStreamSynchronize(s));
        if (first != ~0ull)
          AD_FAIL(AD_ERR_DIVISION_BY_ZERO,
                  "conv: division by zero in deconvolution: at frequency bin " + std::to_string(first));
      }
      AD_HIP(hipMemcpyAsync(out, dc.res.p, (size_t)olen * sizeof(double), hipMemcpyDeviceToHost, s));
      AD_HIP(hipStreamSynchronize(s));
      return;
    }
    const double* src[2] = {signal, kernel};
    const int64_t len[2] = {n, m};
    stage_real(dc.xr, N, src, len, 2, s);
    run.forward(dc.xr.p, 2, s);
    if (op == kSpecNaive) {
      dc.bad.reserve(1);
      AD_HIP(hipMemsetAsync(dc.bad.p, 0xff, sizeof(unsigned long long), s));
    }
    launch_spec_op(op, run.spec(), run.spec() + N, N, eps, op == kSpecNaive ? dc.bad.p : nullptr, s);
    if (op == kSpecNaive) {
      unsigned long long first = 0;
      AD_HIP(hipMemcpyAsync(&first, dc.bad.p, sizeof(first), hipMemcpyDeviceToHost, s));
      AD_HIP(hipStreamSynchronize(s));
      if (first != ~0ull)
        AD_FAIL(AD_ERR_DIVISION_BY_ZERO,
                "conv: division by zero in deconvolution: at frequency bin " + std::to_string(first));
    }
    run.inverse(s);
    AD_HIP(hipMemcpyAsync(out, run.res(), (size_t)olen * sizeof(double), hipMemcpyDeviceToHost, s));
    AD_HIP(hipStreamSynchronize(s));
  });
}

int ad_inverse_filter(const double* kernel, int64_t m, int64_t length, double epsilon, double* out, int device) {
  return guard([&] {
    // deconvolve.go:354-394
    if (m <= 0 || !kernel) AD_FAIL(AD_ERR_EMPTY_KERNEL, "conv: empty kernel");
    if (length < 0) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "negative inverse-filter length");
    if (epsilon <= 0) epsilon = 1e-6;
    if (length == 0) return;
    if (!out) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "null output");
    const int64_t N = next_pow2(length);
    const int dev = pick_device(device);
    DeviceScope ds(dev);
    DeviceCache& dc = cache(dev);
    std::lock_guard<std::mutex> g(dc.mu);
    hipStream_t s = nullptr;
    CallOrder order(dc, s, /*device_call=*/false);
    SpectralRun run(dc, N);
    const int64_t mk = m < N ? m : N;  // kernel truncated to the transform (:367)
    const HostPin pk(kernel, (size_t)mk * 8), po(out, (size_t)length * 8);
    if (run.fused()) {
      dc.xr.reserve((size_t)mk);
      dc.res.reserve((size_t)length);
      AD_HIP(hipMemcpyAsync(dc.xr.p, kernel, (size_t)mk * sizeof(double), hipMemcpyHostToDevice, s));
      run.spectral(kSpecInvFilt, epsilon, nullptr, dc.xr.p, mk, nullptr, 0, length, dc.res.p, s);
      AD_HIP(hipMemcpyAsync(out, dc.res.p, (size_t)length * sizeof(double), hipMemcpyDeviceToHost, s));
      AD_HIP(hipStreamSynchronize(s));
      return;
    }
    const double* src[1] = {kernel};
    const int64_t len[1] = {mk};
    stage_real(dc.xr, N, src, len, 1, s);
    run.forward(dc.xr.p, 1, s);
    launch_spec_op(kSpecInvFilt, run.spec(), nullptr, N, epsilon, nullptr, s);
    run.inverse(s);
    AD_HIP(hipMemcpyAsync(out, run.res(), (size_t)length * sizeof(double), hipMemcpyDeviceToHost, s));
    AD_HIP(hipStreamSynchronize(s));
  });
}

}  // extern "C"
