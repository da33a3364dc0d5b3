/*
 * or_filters.c — CPU restatement of dsp/filter/fir and dsp/filter/biquad
 * (TEST INFRASTRUCTURE ONLY; see oracle.h).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ---- dsp/filter/fir/filter.go ---- */
struct or_fir {
  double* coeffs;
  double* delay;
  double* linear;
  int64_t n, pos;
};

or_fir* or_fir_new(const double* coeffs, int64_t n) { /* filter.go:20-30 */
  or_fir* f = (or_fir*)calloc(1, sizeof(or_fir));
  f->n = n;
  f->coeffs = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  if (n > 0) memcpy(f->coeffs, coeffs, (size_t)n * sizeof(double));
  f->delay = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  f->linear = (double*)calloc((size_t)(n > 0 ? 2 * n : 1), sizeof(double));
  return f;
}

double or_fir_process_sample(or_fir* f, double x) { /* filter.go:36-59 */
  f->delay[f->pos] = x;
  double y = 0;
  const int64_t n = f->n;
  int64_t p = f->pos;
  for (int64_t k = 0; k < n; ++k) {
    y += f->coeffs[k] * f->delay[p];
    --p;
    if (p < 0) p = n - 1;
  }
  ++f->pos;
  if (f->pos >= n) f->pos = 0;
  return y;
}

/* vecmath.DotProduct restated as a sequential sum (algo-vecmath v0.1.0 is not
 * vendored; its SIMD summation order is unknown -> tolerance parity). */
static double dot(const double* a, const double* b, int64_t n) {
  double s = 0;
  for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

static void fir_block(or_fir* f, double* dst, const double* src, int64_t len) { /* filter.go:64-104, 109-149 */
  const int64_t n = f->n;
  if (n == 0) return;
  if (n < 32) {
    for (int64_t i = 0; i < len; ++i) dst[i] = or_fir_process_sample(f, src[i]);
    return;
  }
  for (int64_t i = 0; i < len; ++i) {
    const double x = src[i];
    f->linear[f->pos] = x;
    f->linear[f->pos + n] = x;
    f->delay[f->pos] = x;
    const int64_t start = f->pos + 1;
    dst[i] = dot(f->coeffs, f->linear + start, n);
    ++f->pos;
    if (f->pos >= n) f->pos = 0;
  }
}

void or_fir_process_block(or_fir* f, double* buf, int64_t n) { fir_block(f, buf, buf, n); }
void or_fir_process_block_to(or_fir* f, double* dst, const double* src, int64_t n) { fir_block(f, dst, src, n); }

void or_fir_reset(or_fir* f) { /* filter.go:152-162 */
  memset(f->delay, 0, (size_t)(f->n > 0 ? f->n : 1) * sizeof(double));
  memset(f->linear, 0, (size_t)(f->n > 0 ? 2 * f->n : 1) * sizeof(double));
  f->pos = 0;
}

void or_fir_free(or_fir* f) {
  if (!f) return;
  free(f->coeffs);
  free(f->delay);
  free(f->linear);
  free(f);
}

/* ---- dsp/filter/biquad ---- */
double or_biquad_process_sample(const double* c, double* st, double x) { /* section.go:47-53 */
  const double y = c[0] * x + st[0];
  st[0] = c[1] * x - c[3] * y + st[1];
  st[1] = c[2] * x - c[4] * y;
  return y;
}

/* amd64 "avx2" registry kernel: 4x-unrolled scalar DF-II-T
 * (internal/arch/amd64/avx2/register.go:23-66) */
void or_biquad_process_block(const double* c, double* st, double* buf, int64_t n) {
  const double b0 = c[0], b1 = c[1], b2 = c[2], a1 = c[3], a2 = c[4];
  double d0 = st[0], d1 = st[1];
  int64_t i = 0;
  for (; i + 3 < n; i += 4) {
    const double x0 = buf[i];
    const double y0 = b0 * x0 + d0;
    const double d0n0 = b1 * x0 - a1 * y0 + d1;
    const double d1n0 = b2 * x0 - a2 * y0;
    const double x1 = buf[i + 1];
    const double y1 = b0 * x1 + d0n0;
    const double d0n1 = b1 * x1 - a1 * y1 + d1n0;
    const double d1n1 = b2 * x1 - a2 * y1;
    const double x2 = buf[i + 2];
    const double y2 = b0 * x2 + d0n1;
    const double d0n2 = b1 * x2 - a1 * y2 + d1n1;
    const double d1n2 = b2 * x2 - a2 * y2;
    const double x3 = buf[i + 3];
    const double y3 = b0 * x3 + d0n2;
    d0 = b1 * x3 - a1 * y3 + d1n2;
    d1 = b2 * x3 - a2 * y3;
    buf[i] = y0;
    buf[i + 1] = y1;
    buf[i + 2] = y2;
    buf[i + 3] = y3;
  }
  for (; i < n; ++i) {
    const double x = buf[i];
    const double y = b0 * x + d0;
    d0 = b1 * x - a1 * y + d1;
    d1 = b2 * x - a2 * y;
    buf[i] = y;
  }
  st[0] = d0;
  st[1] = d1;
}

/* generic registry kernel (internal/arch/generic/register.go:18-49), 2x unroll */
void or_biquad_process_block_generic(const double* c, double* st, double* buf, int64_t n) {
  const double b0 = c[0], b1 = c[1], b2 = c[2], a1 = c[3], a2 = c[4];
  double d0 = st[0], d1 = st[1];
  int64_t i = 0;
  for (; i + 1 < n; i += 2) {
    const double x0 = buf[i];
    const double y0 = b0 * x0 + d0;
    const double d0n = b1 * x0 - a1 * y0 + d1;
    const double d1n = b2 * x0 - a2 * y0;
    const double x1 = buf[i + 1];
    const double y1 = b0 * x1 + d0n;
    d0 = b1 * x1 - a1 * y1 + d1n;
    d1 = b2 * x1 - a2 * y1;
    buf[i] = y0;
    buf[i + 1] = y1;
  }
  if (i < n) {
    const double x = buf[i];
    const double y = b0 * x + d0;
    d0 = b1 * x - a1 * y + d1;
    d1 = b2 * x - a2 * y;
    buf[i] = y;
  }
  st[0] = d0;
  st[1] = d1;
}

void or_biquad_process_block_to(const double* c, double* st, double* dst, const double* src, int64_t n) {
  /* section.go:130-138 */
  for (int64_t i = 0; i < n; ++i) {
    const double x = src[i];
    const double y = c[0] * x + st[0];
    st[0] = c[1] * x - c[3] * y + st[1];
    st[1] = c[2] * x - c[4] * y;
    dst[i] = y;
  }
}

void or_biquad_chain_process_block(const double* coeffs, double* state, int sections, double gain, double* buf,
                                   int64_t n) { /* chain.go:59-70 */
  if (gain != 1) {
    for (int64_t i = 0; i < n; ++i) buf[i] = buf[i] * gain;
  }
  for (int s = 0; s < sections; ++s) or_biquad_process_block(coeffs + 5 * s, state + 2 * s, buf, n);
}

double or_biquad_chain_process_sample(const double* coeffs, double* state, int sections, double gain, double x) {
  /* chain.go:49-56 */
  x *= gain;
  for (int s = 0; s < sections; ++s) x = or_biquad_process_sample(coeffs + 5 * s, state + 2 * s, x);
  return x;
}
