/*
 * or_spectral.c — CPU restatement of dsp/conv/correlate.go and
 * dsp/conv/deconvolve.go (TEST INFRASTRUCTURE ONLY; see oracle.h).
 * Complex arithmetic follows Go's complex128 semantics: products as
 * (ac - bd, ad + bc); quotients by the Go runtime's complex128div (Smith's
 * algorithm, runtime/complex.go); cmplx.Abs = math.Hypot (scaled form).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int64_t sp_next_pow2(int64_t n) { /* conv.go:250-261 */
  if (n <= 1) return 1;
  int64_t p = 1;
  while (p < n) p *= 2;
  return p;
}
static or_c128 go_mul(or_c128 a, or_c128 b) {
  or_c128 r = {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
  return r;
}
static or_c128 go_div(or_c128 n, or_c128 m) { /* runtime complex128div, finite operands */
  double e, f;
  if (fabs(m.re) >= fabs(m.im)) {
    const double ratio = m.im / m.re;
    const double denom = m.re + ratio * m.im;
    e = (n.re + n.im * ratio) / denom;
    f = (n.im - n.re * ratio) / denom;
  } else {
    const double ratio = m.re / m.im;
    const double denom = m.im + ratio * m.re;
    e = (n.re * ratio + n.im) / denom;
    f = (n.im * ratio - n.re) / denom;
  }
  or_c128 r = {e, f};
  return r;
}
static double go_hypot(double p, double q) { /* math.hypot (pure Go form) */
  p = fabs(p);
  q = fabs(q);
  if (isinf(p) || isinf(q)) return INFINITY;
  if (isnan(p) || isnan(q)) return NAN;
  if (p < q) {
    const double t = p;
    p = q;
    q = t;
  }
  if (p == 0) return 0;
  q = q / p;
  return p * sqrt(1 + q * q);
}

/* zero-padded complex copy of a real array */
static or_c128* pad_complex(const double* x, int64_t n, int64_t size) {
  or_c128* z = (or_c128*)calloc((size_t)size, sizeof(or_c128));
  for (int64_t i = 0; i < n && i < size; ++i) z[i].re = x[i];
  return z;
}

/* CorrelateFFT correlate.go:111-172 */
int or_correlate_fft(const double* a, int64_t n, const double* b, int64_t m, double* out) {
  if (n == 0 || m == 0) return OR_ERR_EMPTY_INPUT;
  const int64_t N = sp_next_pow2(n + m - 1);
  or_c128* ap = pad_complex(a, n, N);
  or_c128* bp = pad_complex(b, m, N);
  or_c128* af = (or_c128*)malloc((size_t)N * sizeof(or_c128));
  or_c128* bf = (or_c128*)malloc((size_t)N * sizeof(or_c128));
  or_fft(ap, af, N, 0);
  or_fft(bp, bf, N, 0);
  for (int64_t i = 0; i < N; ++i) { /* :150-156 */
    const or_c128 bc = {bf[i].re, -bf[i].im};
    af[i] = go_mul(af[i], bc);
  }
  or_fft(af, ap, N, 1);
  for (int64_t i = 0; i < n; ++i) out[m - 1 + i] = ap[i].re; /* :165-171 */
  for (int64_t i = 0; i < m - 1; ++i) out[i] = ap[N - m + 1 + i].re;
  free(ap);
  free(bp);
  free(af);
  free(bf);
  return OR_OK;
}

/* variance deconvolve.go:326-349 */
static double go_variance(const double* x, int64_t n) {
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

/* Deconvolve deconvolve.go:72-101 with deconvolveNaive :104-166,
 * deconvolveRegularized :170-230 and deconvolveWiener :235-323.
 * method: 0 naive, 1 regularized, 2 wiener, other -> regularized(1e-6).
 * bad_bin (nullable) receives the first naive bin with |H| < 1e-15. */
int or_deconvolve(const double* signal, int64_t n, const double* kernel, int64_t m, int method, double epsilon,
                  double noise_var, double signal_var, double* out, int64_t out_cap, int64_t* out_len,
                  int64_t* bad_bin) {
  if (n == 0) return OR_ERR_EMPTY_INPUT;
  if (m == 0) return OR_ERR_EMPTY_KERNEL;
  double eps = epsilon;
  int naive = 0;
  if (method == 0) {
    naive = 1;
  } else if (method == 1) {
    if (eps <= 0) eps = 1e-6;
  } else if (method == 2) {
    double sv = signal_var, nv = noise_var;
    if (sv <= 0) sv = go_variance(signal, n);
    if (nv <= 0) nv = sv * 0.01;
    double nsr = nv / sv;
    if (nsr <= 0) nsr = 1e-6;
    eps = nsr;
  } else {
    eps = 1e-6;
  }
  const int64_t N = sp_next_pow2(n);
  if (m > N) return OR_ERR_INVALID_ARGUMENT; /* the reference indexes out of range */
  int64_t olen = n - m + 1;
  if (olen <= 0) olen = n;
  if (out_len) *out_len = olen;
  if (out_cap < olen) return OR_ERR_LENGTH_MISMATCH;
  or_c128* sp = pad_complex(signal, n, N);
  or_c128* kp = pad_complex(kernel, m, N);
  or_c128* sf = (or_c128*)malloc((size_t)N * sizeof(or_c128));
  or_c128* kf = (or_c128*)malloc((size_t)N * sizeof(or_c128));
  or_fft(sp, sf, N, 0);
  or_fft(kp, kf, N, 0);
  int rc = OR_OK;
  for (int64_t i = 0; i < N; ++i) {
    if (naive) { /* :146-154 */
      if (go_hypot(kf[i].re, kf[i].im) < 1e-15) {
        if (bad_bin) *bad_bin = i;
        rc = OR_ERR_DIVISION_BY_ZERO;
        break;
      }
      sf[i] = go_div(sf[i], kf[i]);
    } else { /* :208-213, :298-303 */
      const or_c128 hc = {kf[i].re, -kf[i].im};
      const double mag2 = kf[i].re * kf[i].re + kf[i].im * kf[i].im;
      const or_c128 d = {mag2 + eps, 0.0};
      sf[i] = go_div(go_mul(sf[i], hc), d);
    }
  }
  if (rc == OR_OK) {
    or_fft(sf, sp, N, 1);
    for (int64_t i = 0; i < olen; ++i) out[i] = sp[i].re;
  }
  free(sp);
  free(kp);
  free(sf);
  free(kf);
  return rc;
}

/* InverseFilter deconvolve.go:354-394 */
int or_inverse_filter(const double* kernel, int64_t m, int64_t length, double epsilon, double* out) {
  if (m == 0) return OR_ERR_EMPTY_KERNEL;
  if (length < 0) return OR_ERR_INVALID_ARGUMENT;
  if (epsilon <= 0) epsilon = 1e-6;
  const int64_t N = sp_next_pow2(length);
  or_c128* kp = pad_complex(kernel, m, N);
  or_c128* kf = (or_c128*)malloc((size_t)N * sizeof(or_c128));
  or_fft(kp, kf, N, 0);
  for (int64_t i = 0; i < N; ++i) {
    const or_c128 hc = {kf[i].re, -kf[i].im};
    const double mag2 = kf[i].re * kf[i].re + kf[i].im * kf[i].im;
    const or_c128 d = {mag2 + epsilon, 0.0};
    kf[i] = go_div(hc, d);
  }
  or_fft(kf, kp, N, 1);
  for (int64_t i = 0; i < length; ++i) out[i] = kp[i].re;
  free(kp);
  free(kf);
  return OR_OK;
}
