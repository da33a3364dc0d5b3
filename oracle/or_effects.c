/*
 * or_effects.c — CPU restatement of dsp/effects/dynamics (Compressor +
 * dynamicsCore), dsp/effects/reverb (Freeverb) and the IRLB reader of
 * internal/webdemo (TEST INFRASTRUCTURE ONLY; see oracle.h).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ------------------------------------------------------------------------- */
/* dynamics                                                                  */
/* ------------------------------------------------------------------------- */
#define LOG2_OF_10_DIV_20 0.166096404744 /* compressor.go:27 (truncated literal) */
#define MIN_FEEDBACK_GAIN_MEMORY 1e-9     /* core.go:13 */

/* Go math.Log2 structure (frexp split, then Log(frac)/Ln2 + exp). */
static double go_log2(double x) {
  int e;
  const double frac = frexp(x, &e);
  if (frac == 0.5) return (double)(e - 1);
  return log(frac) * (1.0 / M_LN2) + (double)e;
}

typedef struct {
  int enabled;
  double alpha, state;
} onepole;

static void lp_configure(onepole* f, double cutoff, double fs) { /* core.go:606-617 */
  if (cutoff <= 0) {
    f->enabled = 0;
    f->alpha = 0;
    f->state = 0;
    return;
  }
  f->enabled = 1;
  f->alpha = 1.0 - exp(-2.0 * M_PI * cutoff / fs);
}
static double lp_process(onepole* f, double x) { /* core.go:619-627 */
  if (!f->enabled) return x;
  f->state += f->alpha * (x - f->state);
  return f->state;
}

struct or_comp {
  or_comp_cfg cfg;
  double envelope, attack, release, fb_attack, fb_release;
  int64_t rms_n, rms_index, rms_filled;
  double* rms_sq;
  double rms_sum;
  double threshold_log2, knee_width_log2, inv_knee_width_log2, makeup_db, makeup_lin;
  double previous_gain, previous_abs;
  onepole lp;        /* sidechain high-cut */
  int hp_enabled;    /* sidechain low-cut = x - lp(x) */
  onepole hp_lp;
  double m_in_peak, m_out_peak, m_gr;
  int mode;              /* 0 compressor, 1 expander, 2 gate */
  double range_lin;      /* expander/gate floor (mathPower10(rangeDB/20)) */
  int64_t hold_samples;  /* gate: int(holdMs * 0.001 * fs) */
  int64_t hold_counter;
};

void or_comp_default_cfg(or_comp_cfg* c, double fs) { /* NewCompressor compressor.go:77-127 */
  memset(c, 0, sizeof(*c));
  c->sample_rate = fs;
  c->threshold_db = -20.0;
  c->ratio = 4.0;
  c->knee_db = 6.0;
  c->attack_ms = 10.0;
  c->release_ms = 100.0;
  c->makeup_db = 0.0;
  c->rms_window_ms = 30.0;
  c->auto_makeup = 1;
  c->topology = 0;
  c->detector_mode = 0;
  c->feedback_ratio_scale = 1;
}

static void comp_recalc(or_comp* c) { /* core.go:404-540 */
  const or_comp_cfg* g = &c->cfg;
  const double fs = g->sample_rate;
  c->attack = 1.0 - exp(-M_LN2 / (g->attack_ms * 0.001 * fs));
  c->release = exp(-M_LN2 / (g->release_ms * 0.001 * fs));
  if (g->feedback_ratio_scale) {
    c->fb_attack = 1.0 - exp(-M_LN2 / (g->attack_ms * 0.001 * fs * g->ratio));
    c->fb_release = exp(-M_LN2 / (g->release_ms * 0.001 * fs * g->ratio));
  } else {
    c->fb_attack = c->attack;
    c->fb_release = c->release;
  }
  int64_t n = (int64_t)round(g->rms_window_ms * 0.001 * fs);
  if (n < 1) n = 1;
  if (n != c->rms_n) {
    free(c->rms_sq);
    c->rms_sq = (double*)calloc((size_t)n, sizeof(double));
    c->rms_n = n;
    c->rms_index = 0;
    c->rms_filled = 0;
    c->rms_sum = 0;
  }
  c->threshold_log2 = g->threshold_db * LOG2_OF_10_DIV_20;
  c->knee_width_log2 = g->knee_db * LOG2_OF_10_DIV_20;
  c->inv_knee_width_log2 = g->knee_db > 0 ? 1.0 / c->knee_width_log2 : 0;
  if (g->auto_makeup) {
    const double reduction = g->threshold_db * (1.0 - 1.0 / g->ratio);
    c->makeup_db = -reduction;
  } else {
    c->makeup_db = g->makeup_db;
  }
  c->makeup_lin = pow(10.0, c->makeup_db / 20.0);
  lp_configure(&c->hp_lp, g->sidechain_low_cut_hz, fs);
  c->hp_enabled = g->sidechain_low_cut_hz > 0;
  lp_configure(&c->lp, g->sidechain_high_cut_hz, fs);
}

void or_comp_reset(or_comp* c) { /* core.go:572-586 + Compressor.Reset */
  c->envelope = 0;
  c->previous_gain = 1.0;
  c->previous_abs = 0;
  c->rms_index = 0;
  c->rms_filled = 0;
  c->rms_sum = 0;
  if (c->rms_sq) memset(c->rms_sq, 0, (size_t)c->rms_n * sizeof(double));
  c->hp_lp.state = 0;
  c->lp.state = 0;
  c->m_in_peak = 0;
  c->m_out_peak = 0;
  c->m_gr = 1.0;
  c->hold_counter = 0;
}

or_comp* or_comp_new(const or_comp_cfg* cfg) {
  or_comp* c = (or_comp*)calloc(1, sizeof(or_comp));
  c->cfg = *cfg;
  comp_recalc(c);
  or_comp_reset(c);
  return c;
}

static double gain_for_level(const or_comp* c, double level) { /* core.go:288-329 */
  if (level <= 0) return 1.0;
  const double level_log2 = go_log2(level);
  const double overshoot = level_log2 - c->threshold_log2;
  double cf = 1.0 - 1.0 / c->cfg.ratio;
  if (c->cfg.topology == 1 && c->cfg.feedback_ratio_scale) cf = c->cfg.ratio - 1.0;
  if (c->cfg.knee_db <= 0) {
    if (overshoot <= 0) return 1.0;
    return pow(2.0, -overshoot * cf);
  }
  const double half = c->knee_width_log2 * 0.5;
  double eff;
  if (overshoot < -half) return 1.0;
  if (overshoot > half) {
    eff = overshoot;
  } else {
    const double s = overshoot + half;
    eff = s * s * 0.5 * c->inv_knee_width_log2;
  }
  return pow(2.0, -eff * cf);
}

/* calculateDownwardExpansionGain expander.go:358-411 */
static double expansion_gain(const or_comp* c, double level) {
  if (level <= 0) return c->range_lin;
  const double undershoot = c->threshold_log2 - go_log2(level);
  const double rf = c->cfg.ratio - 1.0;
  if (c->cfg.knee_db <= 0) {
    if (undershoot <= 0) return 1.0;
    const double g = pow(2.0, -undershoot * rf);
    return g < c->range_lin ? c->range_lin : g;
  }
  const double half = c->knee_width_log2 * 0.5;
  double eff;
  if (undershoot < -half) return 1.0;
  if (undershoot > half) {
    eff = undershoot;
  } else {
    const double s = undershoot + half;
    eff = s * s * 0.5 * c->inv_knee_width_log2;
  }
  const double g = pow(2.0, -eff * rf);
  return g < c->range_lin ? c->range_lin : g;
}

double or_comp_gain_for_level(const or_comp* c, double level) {
  return c->mode ? expansion_gain(c, level) : gain_for_level(c, level);
}

void or_comp_set_expander(or_comp* c, int mode, double range_db, double hold_ms) {
  /* NewExpander / NewGate: core with autoMakeup off, makeup 0 dB
   * (expander.go:88-104, gate.go:106-122); the feedback-scaled time
   * constants are not enabled by these constructors */
  c->mode = mode;
  c->cfg.auto_makeup = 0;
  c->cfg.makeup_db = 0.0;
  c->cfg.feedback_ratio_scale = 0;
  comp_recalc(c);
  c->range_lin = pow(10.0, range_db / 20.0);
  c->hold_samples = mode == 2 ? (int64_t)(hold_ms * 0.001 * c->cfg.sample_rate) : 0;
  c->hold_counter = 0;
}

int or_comp_hold_counter(const or_comp* c) { return (int)c->hold_counter; }

static double update_rms(or_comp* c, double source) { /* core.go:361-388 */
  if (c->rms_n == 0) return source;
  const double sq = source * source;
  if (c->rms_filled == c->rms_n)
    c->rms_sum -= c->rms_sq[c->rms_index];
  else
    c->rms_filled++;
  c->rms_sq[c->rms_index] = sq;
  c->rms_sum += sq;
  c->rms_index++;
  if (c->rms_index >= c->rms_n) c->rms_index = 0;
  const double mean = c->rms_sum / (double)c->rms_n;
  if (mean <= 0) return 0;
  return sqrt(mean);
}

double or_comp_process_sample(or_comp* c, double x) {
  /* Compressor.ProcessSample -> ProcessSampleSidechain compressor.go:348-359,
   * dynamicsCore.ProcessSample core.go:274-286 */
  double src;
  if (c->cfg.topology == 1) {
    src = c->previous_abs;
  } else {
    double s = x; /* applyPrefilter core.go:390-400: lp then hp */
    s = lp_process(&c->lp, s);
    if (c->hp_enabled) s = s - lp_process(&c->hp_lp, s);
    src = fabs(s);
  }
  if (c->cfg.detector_mode == 1) src = update_rms(c, src);
  double a = c->attack, r = c->release;
  if (c->cfg.topology == 1 && c->cfg.feedback_ratio_scale) {
    a = c->fb_attack;
    r = c->fb_release;
  }
  if (src > c->envelope)
    c->envelope += (src - c->envelope) * a;
  else
    c->envelope = src + (c->envelope - src) * r;
  double gain, out;
  if (c->mode == 0) {
    gain = gain_for_level(c, c->envelope);
    out = x * gain * c->makeup_lin;
    if (c->cfg.topology == 1) {
      c->previous_gain = gain > MIN_FEEDBACK_GAIN_MEMORY ? gain : MIN_FEEDBACK_GAIN_MEMORY;
      c->previous_abs = fabs(out);
    }
  } else {
    /* Expander/Gate.ProcessSampleSidechain (expander.go, gate.go:354-375):
     * only previousGain is kept for the feedback topology */
    gain = expansion_gain(c, c->envelope);
    if (c->mode == 2) {
      if (gain >= 1.0) {
        c->hold_counter = c->hold_samples;
      } else if (c->hold_counter > 0) {
        c->hold_counter--;
        gain = 1.0;
      }
    }
    if (c->cfg.topology == 1) c->previous_gain = gain > MIN_FEEDBACK_GAIN_MEMORY ? gain : MIN_FEEDBACK_GAIN_MEMORY;
    out = x * gain;
  }
  /* updateMetrics compressor.go:411-423 */
  const double il = fabs(x), ol = fabs(out);
  if (il > c->m_in_peak) c->m_in_peak = il;
  if (ol > c->m_out_peak) c->m_out_peak = ol;
  if (c->m_gr == 1.0 || gain < c->m_gr) c->m_gr = gain;
  return out;
}

void or_comp_process_in_place(or_comp* c, double* buf, int64_t n) { /* compressor.go:362-366 */
  for (int64_t i = 0; i < n; ++i) buf[i] = or_comp_process_sample(c, buf[i]);
}

void or_comp_metrics(const or_comp* c, double* ip, double* op, double* gr) {
  if (ip) *ip = c->m_in_peak;
  if (op) *op = c->m_out_peak;
  if (gr) *gr = c->m_gr;
}

void or_comp_params(const or_comp* c, double* thr, double* knee, double* att, double* rel, double* mk) {
  if (thr) *thr = c->threshold_log2;
  if (knee) *knee = c->knee_width_log2;
  if (att) *att = c->attack;
  if (rel) *rel = c->release;
  if (mk) *mk = c->makeup_lin;
}

void or_comp_free(or_comp* c) {
  if (!c) return;
  free(c->rms_sq);
  free(c);
}

/* ------------------------------------------------------------------------- */
/* reverb.go (Freeverb)                                                      */
/* ------------------------------------------------------------------------- */
static const int kCombTuning[8] = {1116, 1188, 1277, 1356, 1422, 1491, 1557, 1617}; /* reverb.go:12-19 */
static const int kAllpassTuning[4] = {556, 441, 341, 225};                           /* reverb.go:21-24 */

typedef struct {
  double feedback, filter_store, damp_a, damp_b;
  double* buf;
  int size, index;
} comb_t;
typedef struct {
  double feedback;
  double* buf;
  int size, index;
} allpass_t;

struct or_verb {
  double wet, dry, room, damp, gain;
  comb_t combs[8];
  allpass_t ap[4];
};

or_verb* or_verb_new(void) { /* NewReverb reverb.go:129-155 */
  or_verb* r = (or_verb*)calloc(1, sizeof(or_verb));
  r->gain = 0.015;
  for (int i = 0; i < 8; ++i) {
    r->combs[i].size = kCombTuning[i];
    r->combs[i].buf = (double*)calloc((size_t)kCombTuning[i], sizeof(double));
  }
  for (int i = 0; i < 4; ++i) {
    r->ap[i].size = kAllpassTuning[i];
    r->ap[i].buf = (double*)calloc((size_t)kAllpassTuning[i], sizeof(double));
    r->ap[i].feedback = 0.5;
  }
  or_verb_set(r, 0.22, 1.0, 0.72, 0.45, 0.015);
  return r;
}

void or_verb_set(or_verb* r, double wet, double dry, double room, double damp, double gain) {
  /* SetWet/SetDry/SetRoomSize/SetDamp/SetGain reverb.go:192-220 */
  r->wet = wet;
  r->dry = dry;
  r->room = room;
  r->damp = damp;
  r->gain = gain;
  for (int i = 0; i < 8; ++i) {
    r->combs[i].feedback = room;
    r->combs[i].damp_a = damp;
    r->combs[i].damp_b = 1 - damp;
  }
}

static double comb_process(comb_t* c, double input) { /* reverb.go:101-117 */
  const double output = c->buf[c->index];
  c->filter_store = output * c->damp_b + c->filter_store * c->damp_a;
  if (fabs(c->filter_store) < 1e-23) c->filter_store = 0;
  c->buf[c->index] = input + c->filter_store * c->feedback;
  if (++c->index >= c->size) c->index = 0;
  return output;
}

static double allpass_process(allpass_t* a, double input) { /* reverb.go:57-68 */
  const double buf_out = a->buf[a->index];
  const double output = buf_out - input;
  a->buf[a->index] = input + buf_out * a->feedback;
  if (++a->index >= a->size) a->index = 0;
  return output;
}

double or_verb_process_sample(or_verb* r, double input) { /* reverb.go:169-182 */
  const double x = r->gain * input;
  double acc = 0;
  for (int i = 0; i < 8; ++i) acc += comb_process(&r->combs[i], x);
  for (int i = 0; i < 4; ++i) acc = allpass_process(&r->ap[i], acc);
  return acc * r->wet + input * r->dry;
}

void or_verb_process_in_place(or_verb* r, double* buf, int64_t n) { /* reverb.go:185-189 */
  for (int64_t i = 0; i < n; ++i) buf[i] = or_verb_process_sample(r, buf[i]);
}

void or_verb_reset(or_verb* r) { /* reverb.go:158-166 */
  for (int i = 0; i < 8; ++i) {
    memset(r->combs[i].buf, 0, (size_t)r->combs[i].size * sizeof(double));
    r->combs[i].index = 0;
    r->combs[i].filter_store = 0;
  }
  for (int i = 0; i < 4; ++i) {
    memset(r->ap[i].buf, 0, (size_t)r->ap[i].size * sizeof(double));
    r->ap[i].index = 0;
  }
}

void or_verb_free(or_verb* r) {
  if (!r) return;
  for (int i = 0; i < 8; ++i) free(r->combs[i].buf);
  for (int i = 0; i < 4; ++i) free(r->ap[i].buf);
  free(r);
}

/* ------------------------------------------------------------------------- */
/* internal/webdemo/irlib.go                                                 */
/* ------------------------------------------------------------------------- */
float or_decode_f16(uint16_t h) { /* irlib.go:68-97, subnormal exponent kept as written (:87) */
  const uint32_t sign = (uint32_t)(h >> 15) << 31;
  const int e16 = (h >> 10) & 0x1F;
  const uint32_t frac = h & 0x3FF;
  uint32_t bits;
  if (e16 == 0) {
    if (frac == 0) {
      bits = sign;
    } else {
      int e = 0;
      uint32_t m = frac;
      while ((m & 0x400) == 0) {
        m <<= 1;
        ++e;
      }
      bits = sign | ((uint32_t)(127 - 14 - e + 1) << 23) | ((m & 0x3FF) << 13);
    }
  } else if (e16 == 31) {
    bits = sign | 0x7F800000u | (frac << 13);
  } else {
    bits = sign | ((uint32_t)(e16 + 112) << 23) | (frac << 13);
  }
  float f;
  memcpy(&f, &bits, 4);
  return f;
}

typedef struct {
  const uint8_t* p;
  int64_t size, pos;
  int err;
} rd_t;
static void rd_bytes(rd_t* r, void* dst, int64_t n) {
  if (r->pos + n > r->size || r->pos < 0) {
    r->err = 1;
    memset(dst, 0, (size_t)n);
    return;
  }
  memcpy(dst, r->p + r->pos, (size_t)n);
  r->pos += n;
}
static uint16_t rd_u16(rd_t* r) { uint16_t v; rd_bytes(r, &v, 2); return v; }
static uint32_t rd_u32(rd_t* r) { uint32_t v; rd_bytes(r, &v, 4); return v; }
static uint64_t rd_u64(rd_t* r) { uint64_t v; rd_bytes(r, &v, 8); return v; }
static double rd_f64(rd_t* r) { double v; rd_bytes(r, &v, 8); return v; }
static void rd_string(rd_t* r, char* dst, int cap) { /* readString irlib.go:100-120 */
  const uint16_t len = rd_u16(r);
  if (r->pos + len > r->size) {
    r->err = 1;
    return;
  }
  if (dst && cap > 0) {
    const int n = len < cap - 1 ? len : cap - 1;
    memcpy(dst, r->p + r->pos, (size_t)n);
    dst[n] = 0;
  }
  r->pos += len;
}

typedef struct {
  uint64_t offset;
  double sample_rate;
  uint32_t channels, length;
} idx_t;

static int read_index(const uint8_t* data, int64_t size, idx_t* out, int cap) { /* readIRLib irlib.go:136-250 */
  rd_t r = {data, size, 0, 0};
  char magic[4];
  rd_bytes(&r, magic, 4);
  if (r.err || memcmp(magic, "IRLB", 4) != 0) return -1;
  if (rd_u16(&r) != 1) return -1;
  (void)rd_u32(&r); /* ir_count */
  const uint64_t index_offset = rd_u64(&r);
  if (r.err) return -1;
  r.pos = (int64_t)index_offset;
  rd_bytes(&r, magic, 4);
  if (r.err || memcmp(magic, "INDX", 4) != 0) return -1;
  const uint64_t indx_size = rd_u64(&r);
  uint64_t read = 0;
  int n = 0;
  while (read < indx_size && !r.err) {
    idx_t e;
    e.offset = rd_u64(&r);
    e.sample_rate = rd_f64(&r);
    e.channels = rd_u32(&r);
    e.length = rd_u32(&r);
    read += 24;
    const int64_t p0 = r.pos;
    rd_string(&r, NULL, 0);
    read += (uint64_t)(r.pos - p0);
    const int64_t p1 = r.pos;
    rd_string(&r, NULL, 0);
    read += (uint64_t)(r.pos - p1);
    if (r.err) return -1;
    if (out && n < cap) out[n] = e;
    ++n;
  }
  return n;
}

/* readIRChunk irlib.go:269-451.  Returns 0 on success. */
static int read_chunk(const uint8_t* data, int64_t size, const idx_t* e, char* name, int name_cap, double* fs,
                      int* channels, int64_t* length, double* dst) {
  rd_t r = {data, size, (int64_t)e->offset, 0};
  char magic[4];
  rd_bytes(&r, magic, 4);
  if (r.err || memcmp(magic, "IR--", 4) != 0) return -1;
  const uint64_t chunk_size = rd_u64(&r);
  uint64_t chunk_read = 0;
  int has_meta = 0, has_audio = 0;
  int meta_ch = 0;
  while (chunk_read < chunk_size) {
    rd_bytes(&r, magic, 4);
    if (r.err) break;
    chunk_read += 4;
    const uint32_t sub = rd_u32(&r);
    if (r.err) break;
    chunk_read += 4;
    if (memcmp(magic, "META", 4) == 0) {
      const double sr = rd_f64(&r);
      const uint32_t ch = rd_u32(&r);
      const uint32_t len = rd_u32(&r);
      rd_string(&r, name, name_cap);
      rd_string(&r, NULL, 0); /* description */
      rd_string(&r, NULL, 0); /* category */
      const uint16_t tags = rd_u16(&r);
      for (int i = 0; i < tags; ++i) rd_string(&r, NULL, 0);
      if (r.err) return -1;
      if (fs) *fs = sr;
      meta_ch = (int)ch;
      (void)len;
      has_meta = 1;
    } else if (memcmp(magic, "AUDI", 4) == 0) {
      if (r.pos + sub > r.size) return -1;
      const uint8_t* raw = r.p + r.pos;
      const int ch = has_meta ? meta_ch : (int)e->channels;
      const int64_t total = sub / 2;
      const int64_t frames = ch > 0 ? total / ch : 0;
      r.pos += sub;
      if (frames == 0) {
        chunk_read += sub;
        continue;
      }
      if (channels) *channels = ch;
      if (length) *length = frames;
      if (dst) {
        for (int64_t i = 0; i < total; ++i) {
          const uint16_t h = (uint16_t)(raw[2 * i] | (raw[2 * i + 1] << 8));
          const double v = (double)or_decode_f16(h);
          const int64_t c = i % ch, f = i / ch;
          if (f < frames) dst[c * frames + f] = v;
        }
      }
      has_audio = 1;
    } else {
      r.pos += sub;
    }
    chunk_read += sub;
  }
  return (has_meta && has_audio) ? 0 : -1;
}

int or_irlib_count(const uint8_t* data, int64_t size) {
  const int n = read_index(data, size, NULL, 0);
  if (n < 0) return -1;
  idx_t* e = (idx_t*)calloc((size_t)(n > 0 ? n : 1), sizeof(idx_t));
  read_index(data, size, e, n);
  int ok = 0;
  for (int i = 0; i < n; ++i)
    if (read_chunk(data, size, &e[i], NULL, 0, NULL, NULL, NULL, NULL) == 0) ++ok;
  free(e);
  return ok;
}

int or_irlib_get(const uint8_t* data, int64_t size, int index, char* name, int name_cap, double* fs, int* channels,
                 int64_t* length, double* dst) {
  const int n = read_index(data, size, NULL, 0);
  if (n < 0) return -1;
  idx_t* e = (idx_t*)calloc((size_t)(n > 0 ? n : 1), sizeof(idx_t));
  read_index(data, size, e, n);
  int ok = -1;
  for (int i = 0; i < n; ++i) {
    /* bad chunks are skipped (irlib.go:255-263), so `index` counts good ones */
    if (read_chunk(data, size, &e[i], NULL, 0, NULL, NULL, NULL, NULL) != 0) continue;
    if (++ok == index) {
      read_chunk(data, size, &e[i], name, name_cap, fs, channels, length, dst);
      free(e);
      return 0;
    }
  }
  free(e);
  return -1;
}
