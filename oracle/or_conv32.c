/*
 * or_conv32.c — float32 / complex64 restatement of the streaming and
 * partitioned convolvers (TEST INFRASTRUCTURE ONLY; see oracle.h).
 *
 * The reference instantiates the same generic code with F = float32 and
 * C = complex64:
 *   NewStreamingOverlapSave32  dsp/conv/streaming_overlap_save.go:94 (core :100-133)
 *   NewStreamingOverlapAdd32   dsp/conv/streaming_overlap_add.go:93 (core :98-133)
 *   NewPartitionedConvolution32 dsp/conv/partitioned.go:340 (stages :77-183, ProcessBlock :348-396)
 * so every buffer is float32 / complex64 and every arithmetic operation rounds
 * to float32 (Go evaluates complex64 products in float32; no FMA on amd64).
 * The complex64 FFT is algo-fft's (absent here): restated as the same radix-2
 * transform as or_fft with float32 butterflies and twiddles rounded from
 * float64 -- bit-level parity with algo-fft is unpinned, as for float64; the
 * reference's own float32 tests bound the error at 1e-4 (streaming_test.go:175-265).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  float re, im;
} c64;

static int64_t nextp2(int64_t n) {
  int64_t p = 1;
  while (p < n) p *= 2;
  return p;
}
static int64_t mn(int64_t a, int64_t b) { return a < b ? a : b; }
static int64_t mx(int64_t a, int64_t b) { return a > b ? a : b; }

static c64 cmul32(c64 a, c64 b) {
  c64 r;
  r.re = a.re * b.re - a.im * b.im;
  r.im = a.re * b.im + a.im * b.re;
  return r;
}

static void fft32(c64* x, int64_t n, int inverse) {
  int lg = 0;
  while (((int64_t)1 << lg) < n) ++lg;
  c64* t = (c64*)malloc((size_t)n * sizeof(c64));
  for (int64_t i = 0; i < n; ++i) {
    int64_t r = 0, v = i;
    for (int b = 0; b < lg; ++b) {
      r = (r << 1) | (v & 1);
      v >>= 1;
    }
    t[r] = x[i];
  }
  const double sign = inverse ? 1.0 : -1.0;
  for (int64_t len = 2; len <= n; len <<= 1) {
    const int64_t half = len >> 1;
    for (int64_t k = 0; k < half; ++k) {
      const double ang = sign * 2.0 * M_PI * (double)k / (double)len;
      const c64 w = {(float)cos(ang), (float)sin(ang)};
      for (int64_t s = 0; s < n; s += len) {
        const c64 u = t[s + k];
        const c64 v = cmul32(w, t[s + k + half]);
        t[s + k].re = u.re + v.re;
        t[s + k].im = u.im + v.im;
        t[s + k + half].re = u.re - v.re;
        t[s + k + half].im = u.im - v.im;
      }
    }
  }
  if (inverse) {
    const float sc = 1.0f / (float)n;
    for (int64_t i = 0; i < n; ++i) {
      t[i].re *= sc;
      t[i].im *= sc;
    }
  }
  memcpy(x, t, (size_t)n * sizeof(c64));
  free(t);
}

/* ---- streaming OLS / OLA -------------------------------------------------- */
struct or_stream32 {
  int is_ola;
  int64_t K, B, N;
  c64 *kfft, *in, *out;
  float *hist, *tail, *conv;
};

int or_stream32_new(int is_ola, const float* kernel, int64_t K, int64_t B, or_stream32** out) {
  *out = NULL;
  if (K == 0) return OR_ERR_EMPTY_KERNEL;
  if (B <= 0) return OR_ERR_INVALID_ARGUMENT;
  or_stream32* s = (or_stream32*)calloc(1, sizeof(*s));
  s->is_ola = is_ola;
  s->K = K;
  s->B = B;
  s->N = nextp2(B + K - 1);
  s->kfft = (c64*)calloc((size_t)s->N, sizeof(c64));
  s->in = (c64*)calloc((size_t)s->N, sizeof(c64));
  s->out = (c64*)calloc((size_t)s->N, sizeof(c64));
  s->hist = (float*)calloc((size_t)mx(K - 1, 1), sizeof(float));
  s->tail = (float*)calloc((size_t)mx(K - 1, 1), sizeof(float));
  s->conv = (float*)calloc((size_t)(B + K - 1), sizeof(float));
  for (int64_t i = 0; i < K; ++i) s->kfft[i].re = kernel[i];
  fft32(s->kfft, s->N, 0);
  *out = s;
  return OR_OK;
}

int or_stream32_process_block(or_stream32* s, const float* in, float* out, int64_t n) {
  if (n != s->B) return OR_ERR_LENGTH_MISMATCH;
  const int64_t K = s->K, B = s->B, N = s->N;
  memset(s->in, 0, (size_t)N * sizeof(c64));
  if (!s->is_ola) { /* streaming_overlap_save.go:100-133 */
    for (int64_t i = 0; i < K - 1; ++i) s->in[i].re = s->hist[i];
    for (int64_t i = 0; i < B; ++i) s->in[K - 1 + i].re = in[i];
  } else { /* streaming_overlap_add.go:98-133 */
    for (int64_t i = 0; i < B; ++i) s->in[i].re = in[i];
  }
  fft32(s->in, N, 0);
  for (int64_t i = 0; i < N; ++i) s->out[i] = cmul32(s->in[i], s->kfft[i]);
  fft32(s->out, N, 1);
  if (!s->is_ola) {
    float* tmp = (float*)malloc((size_t)B * sizeof(float));
    for (int64_t i = 0; i < B; ++i) tmp[i] = s->out[K - 1 + i].re;
    if (B >= K - 1) {
      for (int64_t i = 0; i < K - 1; ++i) s->hist[i] = in[B - K + 1 + i];
    } else {
      memmove(s->hist, s->hist + B, (size_t)(K - 1 - B) * sizeof(float));
      for (int64_t i = 0; i < B; ++i) s->hist[K - 1 - B + i] = in[i];
    }
    memcpy(out, tmp, (size_t)B * sizeof(float));
    free(tmp);
  } else {
    const int64_t rl = B + K - 1;
    for (int64_t i = 0; i < rl; ++i) s->conv[i] = s->out[i].re;
    for (int64_t i = 0; i < K - 1 && i < rl; ++i) s->conv[i] += s->tail[i];
    for (int64_t i = 0; i < K - 1; ++i) s->tail[i] = s->conv[B + i];
    memcpy(out, s->conv, (size_t)B * sizeof(float));
  }
  return OR_OK;
}

int64_t or_stream32_fft_size(const or_stream32* s) { return s->N; }

void or_stream32_free(or_stream32* s) {
  if (!s) return;
  free(s->kfft);
  free(s->in);
  free(s->out);
  free(s->hist);
  free(s->tail);
  free(s->conv);
  free(s);
}

/* ---- partitioned (partitioned.go:77-396, float32) -------------------------- */
typedef struct {
  int64_t fft_size, part_size, output_pos, latency, mod, mod_and, count;
  c64 **irs, *sig, *freq;
} st32;

struct or_pc32 {
  int64_t latency, input_len, output_len, block_pos;
  float *inbuf, *outbuf;
  int nst;
  st32* st;
};

static int tlog2(int64_t n) {
  int r = 0;
  while (n > 1) {
    n >>= 1;
    ++r;
  }
  return r;
}
static int64_t bits(int n) { return ((int64_t)2 << n) - 1; }

static void st32_init(st32* s, int order, int64_t start, int64_t lat, int64_t count, const float* k, int64_t K) {
  s->part_size = (int64_t)1 << order;
  s->fft_size = (int64_t)1 << (order + 1);
  s->output_pos = start;
  s->latency = lat;
  s->mod = 0;
  s->mod_and = s->part_size / lat - 1;
  s->count = count;
  s->irs = (c64**)calloc((size_t)count, sizeof(c64*));
  s->sig = (c64*)calloc((size_t)s->fft_size, sizeof(c64));
  s->freq = (c64*)calloc((size_t)s->fft_size, sizeof(c64));
  for (int64_t b = 0; b < count; ++b) {
    s->irs[b] = (c64*)calloc((size_t)s->fft_size, sizeof(c64));
    const int64_t ks = start + b * s->part_size, ke = mn(ks + s->part_size, K);
    for (int64_t i = 0; ks < K && i < ke - ks; ++i) s->irs[b][s->part_size + i].re = k[ks + i];
    fft32(s->irs[b], s->fft_size, 0);
  }
}

static void st32_process(st32* s, const float* ib, int64_t in_len, float* ob, int64_t out_len) {
  if (s->mod != 0) {
    s->mod = (s->mod + 1) & s->mod_and;
    return;
  }
  const int64_t N = s->fft_size, p = s->part_size;
  for (int64_t i = 0; i < N; ++i) {
    s->freq[i].re = ib[in_len - N + i];
    s->freq[i].im = 0;
  }
  fft32(s->freq, N, 0);
  for (int64_t b = 0; b < s->count; ++b) {
    for (int64_t i = 0; i < N; ++i) s->sig[i] = cmul32(s->freq[i], s->irs[b][i]);
    fft32(s->sig, N, 1);
    const int64_t op = s->output_pos + s->latency - p + b * p;
    if (op >= 0 && op + p <= out_len)
      for (int64_t i = 0; i < p; ++i) ob[op + i] += s->sig[i].re;
  }
  s->mod = (s->mod + 1) & s->mod_and;
}

int or_pc32_new(const float* kernel, int64_t K, int min_order, int max_order, or_pc32** out) {
  *out = NULL;
  if (K == 0) return OR_ERR_EMPTY_IMPULSE_RESPONSE;
  if (min_order < 1 || max_order < min_order) return OR_ERR_INVALID_BLOCK_ORDER;
  const int64_t lat = (int64_t)1 << min_order;
  const int64_t padded = ((K + lat - 1) / lat) * lat;
  int max_ir = tlog2(padded + lat) - 1;
  int64_t res = padded - (bits(max_ir) - bits(min_order - 1));
  if (res > 0 && ((res >> max_ir) & 1) == 0 && max_ir > min_order) --max_ir;
  if (max_ir > max_order) max_ir = max_order;
  res = padded - (bits(max_ir) - bits(min_order - 1));
  or_pc32* pc = (or_pc32*)calloc(1, sizeof(*pc));
  pc->st = (st32*)calloc((size_t)mx(max_ir - min_order + 2, 1), sizeof(st32));
  int64_t start = 0;
  for (int order = min_order; order < max_ir; ++order) {
    const int64_t count = 1 + ((res >> order) & 1);
    st32_init(&pc->st[pc->nst++], order, start, lat, count, kernel, K);
    start += count * ((int64_t)1 << order);
    res -= (count - 1) * ((int64_t)1 << order);
  }
  int64_t count = 1;
  if (max_ir > 0) count = mx(1, 1 + res / ((int64_t)1 << max_ir));
  st32_init(&pc->st[pc->nst++], max_ir, start, lat, count, kernel, K);
  pc->latency = lat;
  pc->input_len = (int64_t)2 << tlog2(pc->st[pc->nst - 1].part_size);
  pc->output_len = mx(0, padded - lat) + lat;
  pc->inbuf = (float*)calloc((size_t)pc->input_len, sizeof(float));
  pc->outbuf = (float*)calloc((size_t)pc->output_len, sizeof(float));
  *out = pc;
  return OR_OK;
}

int or_pc32_process_block(or_pc32* p, const float* input, float* output, int64_t n) {
  int64_t pos = 0, rem = n;
  const int64_t lat = p->latency;
  while (rem > 0) {
    const int64_t chunk = mn(lat - p->block_pos, rem);
    memcpy(p->inbuf + (p->input_len - lat + p->block_pos), input + pos, (size_t)chunk * sizeof(float));
    memcpy(output + pos, p->outbuf + p->block_pos, (size_t)chunk * sizeof(float));
    p->block_pos += chunk;
    pos += chunk;
    rem -= chunk;
    if (p->block_pos == lat) {
      memmove(p->outbuf, p->outbuf + lat, (size_t)(p->output_len - lat) * sizeof(float));
      memset(p->outbuf + p->output_len - lat, 0, (size_t)lat * sizeof(float));
      for (int s = 0; s < p->nst; ++s) st32_process(&p->st[s], p->inbuf, p->input_len, p->outbuf, p->output_len);
      memmove(p->inbuf, p->inbuf + lat, (size_t)(p->input_len - lat) * sizeof(float));
      memset(p->inbuf + p->input_len - lat, 0, (size_t)lat * sizeof(float));
      p->block_pos = 0;
    }
  }
  return OR_OK;
}

void or_pc32_free(or_pc32* p) {
  if (!p) return;
  for (int s = 0; s < p->nst; ++s) {
    for (int64_t b = 0; b < p->st[s].count; ++b) free(p->st[s].irs[b]);
    free(p->st[s].irs);
    free(p->st[s].sig);
    free(p->st[s].freq);
  }
  free(p->st);
  free(p->inbuf);
  free(p->outbuf);
  free(p);
}
