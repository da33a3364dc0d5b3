/*
 * oracle.h — CPU restatement of the algo-dsp reference algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * engine (tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg).
 * It is never linked into, loaded by, or used as a fallback for the product
 * library (algo-dsp_amd/libalgodsp_hip.so).
 *
 * Each function restates the reference Go code line by line; the file:line
 * it follows (relative to the reference repo root) is cited at its
 * definition.  Build flags: -O2 -ffp-contract=off -fno-fast-math, matching
 * the reference's amd64 GOAMD64=v1 arithmetic (no FMA fusion).
 *
 * Third-party arithmetic restated from its published algorithm:
 *   github.com/cwbudde/algo-fft v0.6.10 (go.mod:6) — complex FFT plans.  The
 *   reference relies on: forward unnormalised DFT, inverse with 1/N
 *   (dsp/conv/overlap_add.go:138-160).  Restated as an iterative radix-2 DIT
 *   FFT.  Bit-level parity with algo-fft is unpinned; the reference's own
 *   tests pin FFT paths only by tolerance (1e-7 .. 1e-10) against Direct.
 *   github.com/cwbudde/algo-vecmath v0.1.0 — ScaleBlock/AddBlockInPlace are
 *   elementwise (exactly restatable); DotProduct summation order unknown
 *   (restated as sequential sum).
 */
#ifndef ALGODSP_ORACLE_H_
#define ALGODSP_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  double re, im;
} or_c128;

/* status codes: identical to include/algodsp.h */
enum {
  OR_OK = 0,
  OR_ERR_EMPTY_INPUT = 1,
  OR_ERR_EMPTY_KERNEL = 2,
  OR_ERR_LENGTH_MISMATCH = 3,
  OR_ERR_INVALID_BLOCK_SIZE = 4,
  OR_ERR_INVALID_BLOCK_ORDER = 5,
  OR_ERR_EMPTY_IMPULSE_RESPONSE = 6,
  OR_ERR_STAGE_INDEX_OUT_OF_RANGE = 7,
  OR_ERR_INVALID_ARGUMENT = 8,
  OR_ERR_DIVISION_BY_ZERO = 9
};

/* ---- FFT (algo-fft restatement) ---- */
int or_fft(const or_c128* src, or_c128* dst, int64_t n, int inverse);

/* ---- dsp/conv/conv.go ---- */
int or_direct(const double* a, int64_t n, const double* b, int64_t m, double* dst);
int or_direct_circular(const double* a, int64_t n, const double* b, int64_t m, double* dst);
int or_convolve(const double* a, int64_t n, const double* b, int64_t m, int mode, double* dst, int64_t dst_cap,
                int64_t* dst_len);
/* ---- dsp/conv/correlate.go, deconvolve.go (or_spectral.c) ---- */
int or_correlate_fft(const double* a, int64_t n, const double* b, int64_t m, double* out);
int or_deconvolve(const double* signal, int64_t n, const double* kernel, int64_t m, int method, double epsilon,
                  double noise_var, double signal_var, double* out, int64_t out_cap, int64_t* out_len,
                  int64_t* bad_bin);
int or_inverse_filter(const double* kernel, int64_t m, int64_t length, double epsilon, double* out);
/* high-precision (long double, compensated) full linear convolution: golden reference */
void or_direct_ld(const double* a, int64_t n, const double* b, int64_t m, double* dst);

/* ---- dsp/conv/overlap_add.go ---- */
typedef struct or_ola or_ola;
int or_ola_new(const double* kernel, int64_t K, int64_t block_size, or_ola** out);
int or_ola_process(or_ola* h, const double* in, int64_t n, double* out); /* out: n+K-1 */
int64_t or_ola_block_size(const or_ola* h);
int64_t or_ola_fft_size(const or_ola* h);
void or_ola_free(or_ola* h);
int or_ola_convolve(const double* signal, int64_t n, const double* kernel, int64_t K, double* out);

/* ---- dsp/conv/overlap_save.go ---- */
typedef struct or_ols or_ols;
int or_ols_new(const double* kernel, int64_t K, int64_t fft_size, or_ols** out);
int or_ols_process(or_ols* h, const double* in, int64_t n, double* out); /* out: n+K-1 */
int64_t or_ols_fft_size(const or_ols* h);
int64_t or_ols_step_size(const or_ols* h);
void or_ols_free(or_ols* h);

/* ---- float32 / complex64 instantiations (or_conv32.c): NewStreamingOverlapSave32
 * streaming_overlap_save.go:94, NewStreamingOverlapAdd32 streaming_overlap_add.go:93,
 * NewPartitionedConvolution32 partitioned.go:340 ---- */
typedef struct or_stream32 or_stream32;
int or_stream32_new(int is_ola, const float* kernel, int64_t K, int64_t B, or_stream32** out);
int or_stream32_process_block(or_stream32* h, const float* in, float* out, int64_t n);
int64_t or_stream32_fft_size(const or_stream32* h);
void or_stream32_free(or_stream32* h);
typedef struct or_pc32 or_pc32;
int or_pc32_new(const float* kernel, int64_t K, int min_order, int max_order, or_pc32** out);
int or_pc32_process_block(or_pc32* p, const float* input, float* output, int64_t n);
void or_pc32_free(or_pc32* p);

/* ---- dsp/conv/streaming_overlap_{save,add}.go ---- */
typedef struct or_stream or_stream;
int or_sols_new(const double* kernel, int64_t K, int64_t B, or_stream** out);
int or_sola_new(const double* kernel, int64_t K, int64_t B, or_stream** out);
int or_stream_process_block(or_stream* h, const double* in, int64_t in_len, double* out, int64_t out_len);
void or_stream_reset(or_stream* h);
int64_t or_stream_fft_size(const or_stream* h);
void or_stream_free(or_stream* h);

/* ---- dsp/conv/partitioned.go ---- */
typedef struct or_pc or_pc;
int or_pc_new(const double* kernel, int64_t K, int min_order, int max_order, or_pc** out);
int or_pc_process_block(or_pc* h, const double* in, double* out, int64_t n);
void or_pc_reset(or_pc* h);
int64_t or_pc_latency(const or_pc* h);
int or_pc_stage_count(const or_pc* h);
int or_pc_stage_info(const or_pc* h, int index, int64_t* part_size, int64_t* block_count);
void or_pc_free(or_pc* h);

/* ---- dsp/filter/fir/filter.go ---- */
typedef struct or_fir or_fir;
or_fir* or_fir_new(const double* coeffs, int64_t n);
double or_fir_process_sample(or_fir* f, double x);
void or_fir_process_block(or_fir* f, double* buf, int64_t n);
void or_fir_process_block_to(or_fir* f, double* dst, const double* src, int64_t n);
void or_fir_reset(or_fir* f);
void or_fir_free(or_fir* f);

/* ---- dsp/filter/biquad ---- */
/* coeffs: [b0,b1,b2,a1,a2]; state: [d0,d1] updated in place */
double or_biquad_process_sample(const double* coeffs, double* state, double x);
void or_biquad_process_block(const double* coeffs, double* state, double* buf, int64_t n); /* avx2 4x unroll */
void or_biquad_process_block_generic(const double* coeffs, double* state, double* buf, int64_t n); /* 2x unroll */
void or_biquad_process_block_to(const double* coeffs, double* state, double* dst, const double* src, int64_t n);
/* Chain: coeffs [sec][5], state [sec][2] */
void or_biquad_chain_process_block(const double* coeffs, double* state, int sections, double gain, double* buf,
                                   int64_t n);
double or_biquad_chain_process_sample(const double* coeffs, double* state, int sections, double gain, double x);

/* ---- dsp/effects/dynamics Compressor (feed-forward defaults + full core) ---- */
typedef struct or_comp_cfg {
  double sample_rate, threshold_db, ratio, knee_db, attack_ms, release_ms, rms_window_ms, makeup_db;
  double sidechain_low_cut_hz, sidechain_high_cut_hz;
  int topology;       /* 0 feed-forward, 1 feedback */
  int detector_mode;  /* 0 peak, 1 rms */
  int feedback_ratio_scale;
  int auto_makeup;
} or_comp_cfg;
typedef struct or_comp or_comp;
void or_comp_default_cfg(or_comp_cfg* cfg, double sample_rate);
or_comp* or_comp_new(const or_comp_cfg* cfg);
double or_comp_process_sample(or_comp* c, double x);
void or_comp_process_in_place(or_comp* c, double* buf, int64_t n);
void or_comp_reset(or_comp* c);
void or_comp_metrics(const or_comp* c, double* input_peak, double* output_peak, double* gain_reduction_db);
void or_comp_params(const or_comp* c, double* threshold_log2, double* knee_width_log2, double* attack_coeff,
                    double* release_coeff, double* makeup_lin);
void or_comp_free(or_comp* c);
/* dynamics.Expander / dynamics.Gate (expander.go, gate.go): the same detector
 * core with the downward-expansion gain (expander.go:358-411), no makeup,
 * range floor; the gate adds a hold counter (gate.go:354-375).
 * mode 1 = expander, 2 = gate.  Resets the hold counter. */
void or_comp_set_expander(or_comp* c, int mode, double range_db, double hold_ms);
int or_comp_hold_counter(const or_comp* c);
double or_comp_gain_for_level(const or_comp* c, double level);

/* ---- dsp/effects/reverb Freeverb ---- */
typedef struct or_verb or_verb;
or_verb* or_verb_new(void);
void or_verb_set(or_verb* r, double wet, double dry, double room, double damp, double gain);
double or_verb_process_sample(or_verb* r, double x);
void or_verb_process_in_place(or_verb* r, double* buf, int64_t n);
void or_verb_reset(or_verb* r);
void or_verb_free(or_verb* r);

/* ---- internal/webdemo/irlib.go ---- */
float or_decode_f16(uint16_t h);
/* Parses an IRLB image; returns the number of IRs (or -1).  For IR `index`
 * fills length/channels/sample_rate and, when dst != NULL, the samples
 * [channels][length] as float64. */
int or_irlib_count(const uint8_t* data, int64_t size);
int or_irlib_get(const uint8_t* data, int64_t size, int index, char* name, int name_cap, double* sample_rate,
                 int* channels, int64_t* length, double* dst);

#ifdef __cplusplus
}
#endif

#endif
