/*
 * or_conv.c — CPU restatement of dsp/conv (TEST INFRASTRUCTURE ONLY; see oracle.h).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int64_t next_pow2(int64_t n) { /* conv.go:250-261 */
  if (n <= 1) return 1;
  int64_t p = 1;
  while (p < n) p *= 2;
  return p;
}
static int is_pow2(int64_t n) { return n > 0 && (n & (n - 1)) == 0; } /* conv.go:264-266 */
static int64_t imax(int64_t a, int64_t b) { return a > b ? a : b; }
static int64_t imin(int64_t a, int64_t b) { return a < b ? a : b; }

static or_c128 cmul(or_c128 a, or_c128 b) { /* Go complex128 '*' (no FMA on amd64) */
  or_c128 r;
  r.re = a.re * b.re - a.im * b.im;
  r.im = a.re * b.im + a.im * b.re;
  return r;
}

/* ------------------------------------------------------------------------- */
/* algo-fft restatement: iterative radix-2 decimation-in-time complex FFT.    */
/* Forward: X[k] = sum x[n] exp(-2 pi i k n / N); inverse: conj twiddles, 1/N. */
/* ------------------------------------------------------------------------- */
int or_fft(const or_c128* src, or_c128* dst, int64_t n, int inverse) {
  if (!is_pow2(n)) return OR_ERR_INVALID_BLOCK_SIZE;
  or_c128* tmp = (or_c128*)malloc((size_t)n * sizeof(or_c128));
  int lg = 0;
  while (((int64_t)1 << lg) < n) ++lg;
  for (int64_t i = 0; i < n; ++i) {
    int64_t r = 0, v = i;
    for (int b = 0; b < lg; ++b) {
      r = (r << 1) | (v & 1);
      v >>= 1;
    }
    tmp[r] = src[i];
  }
  const double sign = inverse ? 1.0 : -1.0;
  for (int64_t len = 2; len <= n; len <<= 1) {
    const int64_t half = len >> 1;
    for (int64_t k = 0; k < half; ++k) {
      const double ang = sign * 2.0 * M_PI * (double)k / (double)len;
      or_c128 w = {cos(ang), sin(ang)};
      for (int64_t s = 0; s < n; s += len) {
        or_c128 u = tmp[s + k];
        or_c128 t = cmul(w, tmp[s + k + half]);
        tmp[s + k].re = u.re + t.re;
        tmp[s + k].im = u.im + t.im;
        tmp[s + k + half].re = u.re - t.re;
        tmp[s + k + half].im = u.im - t.im;
      }
    }
  }
  if (inverse) {
    const double sc = 1.0 / (double)n;
    for (int64_t i = 0; i < n; ++i) {
      tmp[i].re *= sc;
      tmp[i].im *= sc;
    }
  }
  memcpy(dst, tmp, (size_t)n * sizeof(or_c128));
  free(tmp);
  return OR_OK;
}

/* ------------------------------------------------------------------------- */
/* conv.go                                                                   */
/* ------------------------------------------------------------------------- */

/* DirectTo conv.go:97-154: dst cleared, then for each a[i] (increasing i)
 * temp = b*a[i] (ScaleBlock), dst[i:i+m] += temp (AddBlockInPlace).  The
 * scalar path (m < 16, :117-123) accumulates in the same order. */
static void direct_to(double* dst, const double* a, int64_t n, const double* b, int64_t m) {
  for (int64_t i = 0; i < n + m - 1; ++i) dst[i] = 0;
  if (m >= 16) {
    double* temp = (double*)malloc((size_t)m * sizeof(double));
    for (int64_t i = 0; i < n; ++i) {
      for (int64_t j = 0; j < m; ++j) temp[j] = b[j] * a[i];
      for (int64_t j = 0; j < m; ++j) dst[i + j] += temp[j];
    }
    free(temp);
  } else {
    for (int64_t i = 0; i < n; ++i)
      for (int64_t j = 0; j < m; ++j) dst[i + j] += a[i] * b[j];
  }
}

int or_direct(const double* a, int64_t n, const double* b, int64_t m, double* dst) { /* conv.go:76-93 */
  if (n == 0) return OR_ERR_EMPTY_INPUT;
  if (m == 0) return OR_ERR_EMPTY_KERNEL;
  direct_to(dst, a, n, b, m);
  return OR_OK;
}

int or_direct_circular(const double* a, int64_t n, const double* b, int64_t m, double* dst) { /* conv.go:158-189 */
  if (n == 0 || m == 0) return OR_ERR_EMPTY_INPUT;
  if (n != m) return OR_ERR_LENGTH_MISMATCH;
  for (int64_t i = 0; i < n; ++i) dst[i] = 0;
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < n; ++j) dst[(i + j) % n] += a[i] * b[j];
  return OR_OK;
}

void or_direct_ld(const double* a, int64_t n, const double* b, int64_t m, double* dst) {
  /* golden reference: long double with Kahan compensation */
  for (int64_t k = 0; k < n + m - 1; ++k) {
    long double s = 0.0L, c = 0.0L;
    const int64_t lo = imax(0, k - m + 1), hi = imin(k, n - 1);
    for (int64_t i = lo; i <= hi; ++i) {
      long double y = (long double)a[i] * (long double)b[k - i] - c;
      long double t = s + y;
      c = (t - s) - y;
      s = t;
    }
    dst[k] = (double)s;
  }
}

/* ------------------------------------------------------------------------- */
/* overlap_add.go                                                            */
/* ------------------------------------------------------------------------- */
struct or_ola {
  or_c128* kernel_fft;
  int64_t kernel_len, block_size, fft_size;
  or_c128 *input_padded, *output_padded;
};

static void ola_init(or_ola* oa, const double* kernel, int64_t K, int64_t block_size, int64_t fft_size) {
  /* NewOverlapAdd overlap_add.go:44-89 / initOverlapAdd :256-294 */
  oa->kernel_len = K;
  oa->block_size = block_size;
  oa->fft_size = fft_size;
  oa->kernel_fft = (or_c128*)calloc((size_t)fft_size, sizeof(or_c128));
  oa->input_padded = (or_c128*)calloc((size_t)fft_size, sizeof(or_c128));
  oa->output_padded = (or_c128*)calloc((size_t)fft_size, sizeof(or_c128));
  or_c128* kp = (or_c128*)calloc((size_t)fft_size, sizeof(or_c128));
  for (int64_t i = 0; i < K; ++i) kp[i].re = kernel[i];
  or_fft(kp, oa->kernel_fft, fft_size, 0);
  free(kp);
}

int or_ola_new(const double* kernel, int64_t K, int64_t block_size, or_ola** out) {
  *out = NULL;
  if (K == 0) return OR_ERR_EMPTY_KERNEL;
  if (block_size <= 0) block_size = imax(next_pow2(K), 256);
  const int64_t fft_size = next_pow2(block_size + K - 1);
  or_ola* oa = (or_ola*)calloc(1, sizeof(or_ola));
  ola_init(oa, kernel, K, block_size, fft_size);
  *out = oa;
  return OR_OK;
}

int or_ola_process(or_ola* oa, const double* input, int64_t n, double* output) { /* overlap_add.go:108-164 */
  if (n == 0) return OR_ERR_EMPTY_INPUT;
  const int64_t output_len = n + oa->kernel_len - 1;
  for (int64_t i = 0; i < output_len; ++i) output[i] = 0;
  const int64_t num_blocks = (n + oa->block_size - 1) / oa->block_size;
  for (int64_t bi = 0; bi < num_blocks; ++bi) {
    const int64_t start = bi * oa->block_size;
    const int64_t end = imin(start + oa->block_size, n);
    const int64_t block_len = end - start;
    memset(oa->input_padded, 0, (size_t)oa->fft_size * sizeof(or_c128));
    for (int64_t i = 0; i < block_len; ++i) oa->input_padded[i].re = input[start + i];
    or_fft(oa->input_padded, oa->input_padded, oa->fft_size, 0);
    for (int64_t i = 0; i < oa->fft_size; ++i) oa->output_padded[i] = cmul(oa->input_padded[i], oa->kernel_fft[i]);
    or_fft(oa->output_padded, oa->output_padded, oa->fft_size, 1);
    const int64_t result_len = block_len + oa->kernel_len - 1;
    for (int64_t i = 0; i < result_len && start + i < output_len; ++i) output[start + i] += oa->output_padded[i].re;
  }
  return OR_OK;
}

int64_t or_ola_block_size(const or_ola* h) { return h->block_size; }
int64_t or_ola_fft_size(const or_ola* h) { return h->fft_size; }

void or_ola_free(or_ola* h) {
  if (!h) return;
  free(h->kernel_fft);
  free(h->input_padded);
  free(h->output_padded);
  free(h);
}

int or_ola_convolve(const double* signal, int64_t n, const double* kernel, int64_t K, double* out) {
  /* OverlapAddConvolve overlap_add.go:221-253 */
  if (K == 0) return OR_ERR_EMPTY_KERNEL;
  const int64_t block_size = imax(next_pow2(K), 256);
  const int64_t fft_size = next_pow2(block_size + K - 1);
  or_ola oa;
  ola_init(&oa, kernel, K, block_size, fft_size);
  const int rc = or_ola_process(&oa, signal, n, out);
  free(oa.kernel_fft);
  free(oa.input_padded);
  free(oa.output_padded);
  return rc;
}

/* Convolve conv.go:194-216 + ConvolveMode/trimToMode :219-247 */
int or_convolve(const double* a, int64_t n, const double* b, int64_t m, int mode, double* dst, int64_t dst_cap,
                int64_t* dst_len) {
  if (n == 0) return OR_ERR_EMPTY_INPUT;
  if (m == 0) return OR_ERR_EMPTY_KERNEL;
  const double *la = a, *lb = b;
  int64_t ln = n, lm = m;
  if (lm > ln) {
    la = b;
    lb = a;
    ln = m;
    lm = n;
  }
  const int64_t full_len = ln + lm - 1;
  double* full = (double*)malloc((size_t)full_len * sizeof(double));
  int rc = (lm <= 64) ? or_direct(la, ln, lb, lm, full) : or_ola_convolve(la, ln, lb, lm, full);
  if (rc != OR_OK) {
    free(full);
    return rc;
  }
  int64_t start = 0, len = full_len;
  if (mode == 1) { /* ModeSame */
    start = (m - 1) / 2;
    len = n;
  } else if (mode == 2) { /* ModeValid */
    if (n >= m) {
      start = m - 1;
      len = n - (m - 1);
    } else {
      start = n - 1;
      len = m - (n - 1);
    }
  }
  if (dst_len) *dst_len = len;
  if (dst_cap < len) {
    free(full);
    return OR_ERR_LENGTH_MISMATCH;
  }
  memcpy(dst, full + start, (size_t)len * sizeof(double));
  free(full);
  return OR_OK;
}

/* ------------------------------------------------------------------------- */
/* overlap_save.go                                                           */
/* ------------------------------------------------------------------------- */
struct or_ols {
  or_c128* kernel_fft;
  int64_t kernel_len, fft_size, step_size;
  or_c128 *input_buffer, *output_buffer;
  double* history;
};

int or_ols_new(const double* kernel, int64_t K, int64_t fft_size, or_ols** out) { /* overlap_save.go:53-107 */
  *out = NULL;
  if (K == 0) return OR_ERR_EMPTY_KERNEL;
  if (fft_size <= 0) fft_size = imax(next_pow2(2 * K), 256);
  if (!is_pow2(fft_size)) return OR_ERR_INVALID_BLOCK_SIZE;
  if (fft_size < 2 * K) fft_size = next_pow2(2 * K);
  or_ols* os = (or_ols*)calloc(1, sizeof(or_ols));
  os->kernel_len = K;
  os->fft_size = fft_size;
  os->step_size = fft_size - K + 1;
  os->kernel_fft = (or_c128*)calloc((size_t)fft_size, sizeof(or_c128));
  os->input_buffer = (or_c128*)calloc((size_t)fft_size, sizeof(or_c128));
  os->output_buffer = (or_c128*)calloc((size_t)fft_size, sizeof(or_c128));
  os->history = (double*)calloc((size_t)(K > 1 ? K - 1 : 1), sizeof(double));
  or_c128* kp = (or_c128*)calloc((size_t)fft_size, sizeof(or_c128));
  for (int64_t i = 0; i < K; ++i) kp[i].re = kernel[i];
  or_fft(kp, os->kernel_fft, fft_size, 0);
  free(kp);
  *out = os;
  return OR_OK;
}

int or_ols_process(or_ols* os, const double* input, int64_t n, double* output) { /* overlap_save.go:126-254 */
  if (n == 0) return OR_ERR_EMPTY_INPUT;
  const int64_t K = os->kernel_len, N = os->fft_size, step = os->step_size;
  const int64_t output_len = n + K - 1;
  for (int64_t i = 0; i < output_len; ++i) output[i] = 0;
  for (int64_t i = 0; i < K - 1; ++i) os->history[i] = 0;
  int64_t input_pos = 0, output_pos = 0;
  while (input_pos < n) {
    memset(os->input_buffer, 0, (size_t)N * sizeof(or_c128));
    for (int64_t i = 0; i < K - 1; ++i) os->input_buffer[i].re = os->history[i];
    int64_t new_samples = step;
    if (input_pos + new_samples > n) new_samples = n - input_pos;
    for (int64_t i = 0; i < new_samples; ++i) os->input_buffer[K - 1 + i].re = input[input_pos + i];
    or_fft(os->input_buffer, os->input_buffer, N, 0);
    for (int64_t i = 0; i < N; ++i) os->output_buffer[i] = cmul(os->input_buffer[i], os->kernel_fft[i]);
    or_fft(os->output_buffer, os->output_buffer, N, 1);
    const int64_t valid_start = K - 1;
    for (int64_t i = 0; i < new_samples && output_pos + i < output_len; ++i)
      output[output_pos + i] = os->output_buffer[valid_start + i].re;
    /* history update, first form (:190-201) */
    const int64_t history_start = imax(new_samples, 0);
    for (int64_t i = 0; i < K - 1; ++i) {
      const int64_t idx = history_start + i;
      if (idx < step && input_pos + idx < n) {
        os->history[i] = input[input_pos + idx];
      } else if (input_pos + new_samples + i - step >= 0 && input_pos + new_samples + i - step < n) {
        os->history[i] = input[input_pos + new_samples + i - step];
      } else {
        os->history[i] = 0;
      }
    }
    /* second form overrides it (:205-215) */
    const int64_t actual = input_pos + new_samples - (K - 1);
    for (int64_t i = 0; i < K - 1; ++i) {
      const int64_t idx = actual + i;
      if (idx >= 0 && idx < n)
        os->history[i] = input[idx];
      else
        os->history[i] = 0;
    }
    input_pos += new_samples;
    output_pos += new_samples;
  }
  if (output_pos < output_len) { /* tail (:224-251) */
    memset(os->input_buffer, 0, (size_t)N * sizeof(or_c128));
    for (int64_t i = 0; i < K - 1; ++i) os->input_buffer[i].re = os->history[i];
    or_fft(os->input_buffer, os->input_buffer, N, 0);
    for (int64_t i = 0; i < N; ++i) os->output_buffer[i] = cmul(os->input_buffer[i], os->kernel_fft[i]);
    or_fft(os->output_buffer, os->output_buffer, N, 1);
    const int64_t valid_start = K - 1;
    for (int64_t i = 0; output_pos + i < output_len && valid_start + i < N; ++i)
      output[output_pos + i] = os->output_buffer[valid_start + i].re;
  }
  return OR_OK;
}

int64_t or_ols_fft_size(const or_ols* h) { return h->fft_size; }
int64_t or_ols_step_size(const or_ols* h) { return h->step_size; }

void or_ols_free(or_ols* h) {
  if (!h) return;
  free(h->kernel_fft);
  free(h->input_buffer);
  free(h->output_buffer);
  free(h->history);
  free(h);
}

/* ------------------------------------------------------------------------- */
/* streaming_overlap_save.go / streaming_overlap_add.go                      */
/* ------------------------------------------------------------------------- */
struct or_stream {
  int is_ola;
  or_c128* kernel_fft;
  int64_t kernel_len, block_size, fft_size;
  or_c128 *in_buf, *out_buf;
  double* history;     /* OLS: last K-1 inputs */
  double* tail;        /* OLA: K-1 tail */
  double* conv_result; /* OLA: B+K-1 */
};

static int stream_new(int is_ola, const double* kernel, int64_t K, int64_t B, or_stream** out) {
  /* NewStreamingOverlapSaveT streaming_overlap_save.go:45-84,
   * NewStreamingOverlapAddT streaming_overlap_add.go:43-83 */
  *out = NULL;
  if (K == 0) return OR_ERR_EMPTY_KERNEL;
  if (B <= 0) return OR_ERR_INVALID_ARGUMENT;
  or_stream* s = (or_stream*)calloc(1, sizeof(or_stream));
  s->is_ola = is_ola;
  s->kernel_len = K;
  s->block_size = B;
  s->fft_size = next_pow2(B + K - 1);
  const int64_t N = s->fft_size;
  s->kernel_fft = (or_c128*)calloc((size_t)N, sizeof(or_c128));
  s->in_buf = (or_c128*)calloc((size_t)N, sizeof(or_c128));
  s->out_buf = (or_c128*)calloc((size_t)N, sizeof(or_c128));
  s->history = (double*)calloc((size_t)(K > 1 ? K - 1 : 1), sizeof(double));
  s->tail = (double*)calloc((size_t)(K > 1 ? K - 1 : 1), sizeof(double));
  s->conv_result = (double*)calloc((size_t)(B + K - 1), sizeof(double));
  or_c128* kp = (or_c128*)calloc((size_t)N, sizeof(or_c128));
  for (int64_t i = 0; i < K; ++i) kp[i].re = kernel[i];
  or_fft(kp, s->kernel_fft, N, 0);
  free(kp);
  *out = s;
  return OR_OK;
}

int or_sols_new(const double* kernel, int64_t K, int64_t B, or_stream** out) { return stream_new(0, kernel, K, B, out); }
int or_sola_new(const double* kernel, int64_t K, int64_t B, or_stream** out) { return stream_new(1, kernel, K, B, out); }

static void sols_core(or_stream* s, double* dst, const double* input) { /* streaming_overlap_save.go:100-133 */
  const int64_t K = s->kernel_len, B = s->block_size, N = s->fft_size;
  memset(s->in_buf, 0, (size_t)N * sizeof(or_c128));
  for (int64_t i = 0; i < K - 1; ++i) s->in_buf[i].re = s->history[i];
  for (int64_t i = 0; i < B; ++i) s->in_buf[K - 1 + i].re = input[i];
  or_fft(s->in_buf, s->in_buf, N, 0);
  for (int64_t i = 0; i < N; ++i) s->out_buf[i] = cmul(s->in_buf[i], s->kernel_fft[i]);
  or_fft(s->out_buf, s->out_buf, N, 1);
  const int64_t vs = K - 1;
  for (int64_t i = 0; i < B; ++i) dst[i] = s->out_buf[vs + i].re;
  if (B >= K - 1) {
    for (int64_t i = 0; i < K - 1; ++i) s->history[i] = input[B - K + 1 + i];
  } else {
    memmove(s->history, s->history + B, (size_t)(K - 1 - B) * sizeof(double));
    for (int64_t i = 0; i < B; ++i) s->history[K - 1 - B + i] = input[i];
  }
}

static void sola_core(or_stream* s, const double* input) { /* streaming_overlap_add.go:98-133 */
  const int64_t K = s->kernel_len, B = s->block_size, N = s->fft_size;
  memset(s->in_buf, 0, (size_t)N * sizeof(or_c128));
  for (int64_t i = 0; i < B; ++i) s->in_buf[i].re = input[i];
  or_fft(s->in_buf, s->in_buf, N, 0);
  for (int64_t i = 0; i < N; ++i) s->out_buf[i] = cmul(s->in_buf[i], s->kernel_fft[i]);
  or_fft(s->out_buf, s->out_buf, N, 1);
  const int64_t result_len = B + K - 1;
  for (int64_t i = 0; i < result_len; ++i) s->conv_result[i] = s->out_buf[i].re;
  const int64_t tail_len = K - 1;
  for (int64_t i = 0; i < tail_len && i < result_len; ++i) s->conv_result[i] += s->tail[i];
  const int64_t new_tail = result_len - B;
  for (int64_t i = 0; i < new_tail; ++i) s->tail[i] = s->conv_result[B + i];
  for (int64_t i = new_tail; i < tail_len; ++i) s->tail[i] = 0;
}

int or_stream_process_block(or_stream* s, const double* in, int64_t in_len, double* out, int64_t out_len) {
  if (in_len != s->block_size) return OR_ERR_LENGTH_MISMATCH;
  if (out_len != s->block_size) return OR_ERR_LENGTH_MISMATCH;
  if (s->is_ola) {
    sola_core(s, in);
    memcpy(out, s->conv_result, (size_t)s->block_size * sizeof(double));
  } else {
    double* tmp = (double*)malloc((size_t)s->block_size * sizeof(double));
    sols_core(s, tmp, in);
    memcpy(out, tmp, (size_t)s->block_size * sizeof(double));
    free(tmp);
  }
  return OR_OK;
}

void or_stream_reset(or_stream* s) {
  const int64_t K = s->kernel_len;
  if (K > 1) {
    memset(s->history, 0, (size_t)(K - 1) * sizeof(double));
    memset(s->tail, 0, (size_t)(K - 1) * sizeof(double));
  }
}

int64_t or_stream_fft_size(const or_stream* s) { return s->fft_size; }

void or_stream_free(or_stream* s) {
  if (!s) return;
  free(s->kernel_fft);
  free(s->in_buf);
  free(s->out_buf);
  free(s->history);
  free(s->tail);
  free(s->conv_result);
  free(s);
}

/* ------------------------------------------------------------------------- */
/* partitioned.go                                                            */
/* ------------------------------------------------------------------------- */
typedef struct {
  int fft_order;
  int64_t fft_size, part_size, output_pos, latency;
  int64_t mod, mod_and;
  int64_t count;
  or_c128** ir_spectra;
  or_c128 *signal_buf, *signal_freq;
  double* conv_time;
} or_stage;

struct or_pc {
  int64_t kernel_len, kernel_len_padded, latency;
  int min_order, max_order;
  double *input_buffer, *output_buffer;
  int64_t input_len, output_len;
  int64_t block_pos;
  int nstages;
  or_stage* stages;
};

static int trunc_log2(int64_t n) { /* partitioned.go:186-199 */
  if (n <= 0) return 0;
  int r = 0;
  while (n > 1) {
    n >>= 1;
    ++r;
  }
  return r;
}
static int64_t bit_count_to_bits(int n) { return ((int64_t)2 << n) - 1; } /* partitioned.go:202-204 */

static void stage_init(or_stage* s, int order, int64_t start_pos, int64_t latency, int64_t count, const double* kernel,
                       int64_t K) {
  /* newPartStage :77-108 + calculateIRSpectra :113-130 */
  s->fft_order = order;
  s->part_size = (int64_t)1 << order;
  s->fft_size = (int64_t)1 << (order + 1);
  s->output_pos = start_pos;
  s->latency = latency;
  s->mod = 0;
  s->mod_and = s->part_size / latency - 1;
  s->count = count;
  s->ir_spectra = (or_c128**)calloc((size_t)count, sizeof(or_c128*));
  s->signal_buf = (or_c128*)calloc((size_t)s->fft_size, sizeof(or_c128));
  s->signal_freq = (or_c128*)calloc((size_t)s->fft_size, sizeof(or_c128));
  s->conv_time = (double*)calloc((size_t)s->fft_size, sizeof(double));
  for (int64_t b = 0; b < count; ++b) {
    s->ir_spectra[b] = (or_c128*)calloc((size_t)s->fft_size, sizeof(or_c128));
    memset(s->signal_buf, 0, (size_t)s->fft_size * sizeof(or_c128));
    const int64_t ks = s->output_pos + b * s->part_size;
    const int64_t ke = imin(ks + s->part_size, K);
    if (ks < K) {
      for (int64_t i = 0; i < ke - ks; ++i) s->signal_buf[s->part_size + i].re = kernel[ks + i];
    }
    or_fft(s->signal_buf, s->ir_spectra[b], s->fft_size, 0);
  }
}

static void stage_process(or_stage* s, const double* input_buf, int64_t in_len, double* output_buf, int64_t out_len) {
  /* partStageT.process :134-183 */
  if (s->mod != 0) {
    s->mod = (s->mod + 1) & s->mod_and;
    return;
  }
  const int64_t N = s->fft_size, p = s->part_size;
  const int64_t input_start = in_len - N;
  memset(s->signal_buf, 0, (size_t)N * sizeof(or_c128));
  for (int64_t i = 0; i < N; ++i) s->signal_buf[i].re = input_buf[input_start + i];
  or_fft(s->signal_buf, s->signal_freq, N, 0);
  for (int64_t b = 0; b < s->count; ++b) {
    for (int64_t i = 0; i < N; ++i) s->signal_buf[i] = cmul(s->signal_freq[i], s->ir_spectra[b][i]);
    or_fft(s->signal_buf, s->signal_buf, N, 1);
    for (int64_t i = 0; i < N; ++i) s->conv_time[i] = s->signal_buf[i].re;
    const int64_t out_pos = s->output_pos + s->latency - p + b * p;
    if (out_pos >= 0 && out_pos + p <= out_len) {
      for (int64_t i = 0; i < p; ++i) output_buf[out_pos + i] += s->conv_time[i];
    }
  }
  s->mod = (s->mod + 1) & s->mod_and;
}

int or_pc_new(const double* kernel, int64_t K, int min_order, int max_order, or_pc** out) {
  /* NewPartitionedConvolutionT :212-266, partitionIR :269-332 */
  *out = NULL;
  if (K == 0) return OR_ERR_EMPTY_IMPULSE_RESPONSE;
  if (min_order < 1) return OR_ERR_INVALID_BLOCK_ORDER;
  if (max_order < min_order) return OR_ERR_INVALID_BLOCK_ORDER;
  const int64_t latency = (int64_t)1 << min_order;
  const int64_t min_block = latency;
  const int64_t padded = ((K + min_block - 1) / min_block) * min_block;

  int max_ir = trunc_log2(padded + min_block) - 1;
  int64_t res = padded - (bit_count_to_bits(max_ir) - bit_count_to_bits(min_order - 1));
  if (res > 0 && ((res >> max_ir) & 1) == 0 && max_ir > min_order) --max_ir;
  if (max_ir > max_order) max_ir = max_order;
  res = padded - (bit_count_to_bits(max_ir) - bit_count_to_bits(min_order - 1));

  or_pc* pc = (or_pc*)calloc(1, sizeof(or_pc));
  pc->stages = (or_stage*)calloc((size_t)(max_ir - min_order + 2), sizeof(or_stage));
  int ns = 0;
  int64_t start = 0;
  for (int order = min_order; order < max_ir; ++order) {
    const int64_t count = 1 + ((res >> order) & 1);
    stage_init(&pc->stages[ns++], order, start, latency, count, kernel, K);
    start += count * ((int64_t)1 << order);
    res -= (count - 1) * ((int64_t)1 << order);
  }
  int64_t count = 1;
  if (max_ir > 0) {
    count = 1 + res / ((int64_t)1 << max_ir);
    if (count < 1) count = 1;
  }
  stage_init(&pc->stages[ns++], max_ir, start, latency, count, kernel, K);
  pc->nstages = ns;

  int max_ord_used = pc->stages[ns - 1].fft_order;
  pc->kernel_len = K;
  pc->kernel_len_padded = padded;
  pc->latency = latency;
  pc->min_order = min_order;
  pc->max_order = max_order;
  pc->input_len = (int64_t)2 << max_ord_used;
  const int64_t out_hist = imax(0, padded - latency);
  pc->output_len = out_hist + latency;
  pc->input_buffer = (double*)calloc((size_t)pc->input_len, sizeof(double));
  pc->output_buffer = (double*)calloc((size_t)pc->output_len, sizeof(double));
  pc->block_pos = 0;
  *out = pc;
  return OR_OK;
}

int or_pc_process_block(or_pc* p, const double* input, double* output, int64_t n) { /* :348-396 */
  int64_t in_pos = 0, remaining = n;
  const int64_t latency = p->latency;
  while (remaining > 0) {
    const int64_t chunk = imin(latency - p->block_pos, remaining);
    const int64_t ib_end = p->input_len;
    memcpy(p->input_buffer + (ib_end - latency + p->block_pos), input + in_pos, (size_t)chunk * sizeof(double));
    memcpy(output + in_pos, p->output_buffer + p->block_pos, (size_t)chunk * sizeof(double));
    p->block_pos += chunk;
    in_pos += chunk;
    remaining -= chunk;
    if (p->block_pos == latency) {
      const int64_t out_len = p->output_len;
      memmove(p->output_buffer, p->output_buffer + latency, (size_t)(out_len - latency) * sizeof(double));
      memset(p->output_buffer + out_len - latency, 0, (size_t)latency * sizeof(double));
      for (int s = 0; s < p->nstages; ++s)
        stage_process(&p->stages[s], p->input_buffer, p->input_len, p->output_buffer, p->output_len);
      memmove(p->input_buffer, p->input_buffer + latency, (size_t)(p->input_len - latency) * sizeof(double));
      memset(p->input_buffer + p->input_len - latency, 0, (size_t)latency * sizeof(double));
      p->block_pos = 0;
    }
  }
  return OR_OK;
}

void or_pc_reset(or_pc* p) { /* :399-407 */
  memset(p->input_buffer, 0, (size_t)p->input_len * sizeof(double));
  memset(p->output_buffer, 0, (size_t)p->output_len * sizeof(double));
  p->block_pos = 0;
  for (int s = 0; s < p->nstages; ++s) p->stages[s].mod = 0;
}

int64_t or_pc_latency(const or_pc* p) { return p->latency; }
int or_pc_stage_count(const or_pc* p) { return p->nstages; }
int or_pc_stage_info(const or_pc* p, int index, int64_t* part_size, int64_t* block_count) {
  if (index < 0 || index >= p->nstages) return OR_ERR_STAGE_INDEX_OUT_OF_RANGE;
  *part_size = p->stages[index].part_size;
  *block_count = p->stages[index].count;
  return OR_OK;
}

void or_pc_free(or_pc* p) {
  if (!p) return;
  for (int s = 0; s < p->nstages; ++s) {
    or_stage* st = &p->stages[s];
    for (int64_t b = 0; b < st->count; ++b) free(st->ir_spectra[b]);
    free(st->ir_spectra);
    free(st->signal_buf);
    free(st->signal_freq);
    free(st->conv_time);
  }
  free(p->stages);
  free(p->input_buffer);
  free(p->output_buffer);
  free(p);
}
