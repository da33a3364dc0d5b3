// Device-side argument blocks of the per-sample processors (biquad chains,
// compressor, Freeverb, their fused chain) and of the FIR block filter.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace adsp {

// Biquad sections as they run per sample: x *= pre_gain; DF-II-T section.
// A biquad.Chain with gain g becomes pre_gain = g on its first section and 1
// on the others (x * 1.0 == x exactly, so the reference's `gain != 1` skip,
// chain.go:59-64, is reproduced bit for bit).
constexpr int kSecStride = 6;  // {pre_gain, b0, b1, b2, a1, a2}
constexpr int kMaxSecPerPass = 8;

struct EqArgs {
  const double* sec;      // [channels][nsec][6]; a table shared by all channels has stride 0
  int64_t sec_ch_stride;  // elements between channels' tables
  double* state;          // [channels][nsec][2]  {d0, d1}
  int nsec;               // <= kMaxSecPerPass in one launch
};

// dynamicsCore parameters, precomputed on the host exactly as
// recalculateDetectorCoefficients / recalculateGainComputer do
// (dsp/effects/dynamics/core.go:480-540).
struct CompParams {
  double threshold_log2, knee_width_log2, inv_knee_width_log2, half_knee;
  double cf;  // 1 - 1/ratio, or ratio - 1 (feedback topology with ratio scaling)
  double makeup_lin;
  double attack, release;  // already the feedback pair when that topology is scaled
  // the envelope step as env' = c2 |src - env| + (k1 env + c1 src) (env_step,
  // dsp_device.hpp): c1 = (attack + b) / 2, c2 = (attack - b) / 2, k1 = 1 - c1,
  // b = 1 - release
  double env_c1, env_c2, env_k1;
  double lp_alpha, hp_alpha;
  int knee_on, topology_fb, detector_rms, lp_on, hp_on, rms_n;
  // dynamics.Expander / dynamics.Gate (expander.go, gate.go): mode 1 / 2 use
  // the downward-expansion gain (ratio_m1 = ratio - 1, floor range_lin), no
  // makeup (makeup_lin = 1), and the gate holds the gain at 1 for hold_n
  // samples after it was last >= 1.  mode 0 is the compressor.
  int mode;
  double ratio_m1, range_lin;
  int hold_n;
};

struct CompChState {
  double env, lp, hp, rms_sum, prev_abs, prev_gain, in_peak, out_peak, gr;
  int rms_index, rms_filled;
  int hold;  // gate hold counter
};

// reverb.Reverb (Freeverb) parameters and per-channel state.
constexpr int kVerbCombs = 8, kVerbAllpass = 4;
constexpr int kVerbLen = 1116 + 1188 + 1277 + 1356 + 1422 + 1491 + 1557 + 1617 + 556 + 441 + 341 + 225;  // 12587
constexpr int kCombLen[kVerbCombs] = {1116, 1188, 1277, 1356, 1422, 1491, 1557, 1617};  // reverb.go:12-19
constexpr int kApLen[kVerbAllpass] = {556, 441, 341, 225};                             // reverb.go:21-24
// delay lines of one channel column in vbuf ([pos][cpad]): combs, then allpasses
__host__ __device__ constexpr int comb_off(int i) { return i == 0 ? 0 : comb_off(i - 1) + kCombLen[i - 1]; }
__host__ __device__ constexpr int ap_off(int i) {
  return i == 0 ? comb_off(kVerbCombs) : ap_off(i - 1) + kApLen[i - 1];
}
static_assert(ap_off(kVerbAllpass) == kVerbLen, "Freeverb delay-line layout");
struct VerbParams {
  double wet, dry, gain, feedback, damp_a, damp_b, ap_feedback;
};
struct VerbChState {
  double filter_store[kVerbCombs];
  int comb_idx[kVerbCombs];
  int ap_idx[kVerbAllpass];
};

struct ChainArgs {
  double* buf;  // [channels][stride], n samples processed in place
  int64_t stride, n;
  int channels;
  EqArgs eq;
  CompParams cp;
  CompChState* cs;  // [channels]
  double* rms_ring;  // [channels][rms_n]
  VerbParams vp;
  VerbChState* vs;  // [channels]
  double* vbuf;     // [channels][kVerbLen]
  unsigned long long* prof;  // diagnostics only (AD_FX_PROF): per wave {busy, total} clock ticks
};

// stages: bit 0 EQ, bit 1 compressor, bit 2 Freeverb
void launch_chain(int stages, const ChainArgs& a, hipStream_t s);

// Staged effect chain (fx_staged.hip): the chain split by recurrence into
// kernels that run concurrently on their own streams over time chunks, each
// stage on its own CUs.  Chunk-local buffers are time-major [t][cpad].
// One K_eq pipeline: sections [s0, s0 + ns) of the chain, then (det) the
// compressor's detector/envelope, over one chunk.  A launch runs one part per
// blockIdx.y: the whole chain, or (split, fx_run_staged) sections 0 .. s1-1
// of chunk i beside sections s1 .. ns-1 + the detector of chunk i - 1, so the
// EQ recurrences of a channel group get two CUs.
struct FxEqPart {
  int s0, ns;
  int det;
  int64_t len;       // samples of this part's chunk
  const double* in;  // input rows [len][cpad]
  double* out;       // rows of the last section's output (ns = 0: the input)
  double* env;       // envelope rows (det)
};

struct FxStageArgs {
  int channels, cpad;
  int64_t len;           // samples in this chunk
  double* buf;           // user buffer at the chunk start, [channels][stride]
  int64_t stride;
  double* xT;            // chunk input        [len][cpad] (transposed user buffer)
  double* vT;            // EQ output          [len][cpad]
  double* envT;          // envelope           [len][cpad]
  double* inT;           // reverb input       [len][cpad] (compressor output / EQ output / input)
  double* coT;           // comb outputs   [8][tmax][cpad]
  int64_t tmax;
  EqArgs eq;
  CompParams cp;
  CompChState* cs;
  double* rms_ring;
  VerbParams vp;
  VerbChState* vs;
  double* vbuf;
  unsigned long long* prof;  // diagnostics only (AD_FX_PROF): K_eq per wave {compute, barrier wait} clock ticks
  FxEqPart part[kMaxSecPerPass];  // K_eq parts (launch_fx_eq_parts)
  int nparts;
};
// stage kernels; `mode` selects where a stage writes (see fx_staged.hip)
void launch_fx_eq(const FxStageArgs& a, bool comp, int out_mode, hipStream_t s);
void launch_fx_eq_parts(const FxStageArgs& a, hipStream_t s);  // a.part[0 .. nparts)
// one section per part (part.s0, ns = 1, no detector), a workgroup each (EQ-only pipeline)
void launch_fx_eq_sec(const FxStageArgs& a, hipStream_t s);
void launch_fx_gain(const FxStageArgs& a, bool to_user, hipStream_t s);
// EQ-only chains with the cascade's sections across lanes (fx_eq_lanes.hip):
// the user buffer [channels][stride] filtered in place, state eq.state
// [channels][nsec][2]; g1: every section after the first has pre-gain 1.0
struct FxEqLaneArgs {
  double* buf;
  int64_t stride, n;
  int channels;
  EqArgs eq;
  double* dump;  // kFxEqLaneDump doubles of scratch (stores outside the signal)
};
constexpr int kFxEqLaneDump = 256;
void launch_fx_eq_lanes(const FxEqLaneArgs& a, bool g1, hipStream_t s);
void launch_fx_transpose_in(const FxStageArgs& a, double* dstT, hipStream_t s);   // user -> dstT
void launch_fx_transpose_out(const FxStageArgs& a, const double* srcT, hipStream_t s);  // srcT -> user
void launch_fx_comb(const FxStageArgs& a, hipStream_t s);
void launch_fx_allpass(const FxStageArgs& a, hipStream_t s);
constexpr int kFxOutVT = 1, kFxOutInT = 2;

// Time-parallel engine (fx_tp.hip; host: fx_run_tp).  The EQ cascade of a
// chunk cut into nseg <= 256 segments of `seg` samples runs in three launches:
// K_eqz the cascade's zero-state runs (end states to `zs`), K_carry the
// segment start states of every section (double-double, to `sdd`), K_eqx the
// exact cascade from those starts (rows to vT, chunk-end states to eq.state).
struct FxTpEqArgs {
  int channels, cpad;
  int64_t len;
  int seg, nseg;
  const double* xT;  // chunk input rows [len][cpad]
  double* vT;        // EQ output rows [len][cpad]
  EqArgs eq;
  double* zs;          // [nseg][nsec][cpad][d0, d1]
  double* sdd;         // [nseg][nsec][cpad][d0.hi, d0.lo, d1.hi, d1.lo]
  const double* mats;  // [mat_sets][fx_tp_mat_stride(nsec)] (host fx_tp_mats)
  int mat_sets;        // 1 (one coefficient table) or channels
};
constexpr int kFxTpMaxSeg = 256;  // segments per chunk, at most (K_carry: one thread each)
constexpr int kFxTpScan = 8;      // K_carry scan steps (log2 kFxTpMaxSeg)
// per coefficient set: the segment map's 2 x 2 blocks B(k, j) (section k's end
// state from section j's start, j <= k; [nsec][nsec]), then per section the
// scan maps B(k, k)^(2^i), i < kFxTpScan; every block 4
// double-double entries (row-major), i.e. 8 doubles
__host__ __device__ constexpr int fx_tp_mat_stride(int nsec) { return nsec * (nsec + kFxTpScan) * 8; }
constexpr int kFxVerbSB = 4096;     // K_verb sub-block (samples)
void launch_fxtp_eq(const FxTpEqArgs& a, bool exact, hipStream_t s);  // K_eqz (exact = false) or K_eqx
void launch_fxtp_carry(const FxTpEqArgs& a, hipStream_t s);
void launch_fxtp_det(const FxStageArgs& a, hipStream_t s);           // vT -> envT (+ detector state)
// Freeverb, one channel per workgroup: xC [channels][xstride] (channel-major
// reverb input) -> user buffer, delay lines in vbufC [channels][kVerbLen],
// comb outputs through coC [channels][8][kFxVerbSB] (scratch)
// pipe: k_fxtp_verb_pipe, the comb and allpass phases of consecutive
// sub-blocks overlapped (faster beside the config-5 pipeline's other stages:
// 12.5 -> 13.0 Gsamples/s; slower alone: Freeverb-only 22.3 -> 20.1)
void launch_fxtp_verb(const FxStageArgs& a, const double* xC, int64_t xstride, double* vbufC, double* coC, int wu,
                      hipStream_t s, bool pipe = false);
void launch_vbuf_layout(double* vbuf, double* vbufC, int cpad, int channels, bool to_cm, hipStream_t s);

// Fan-in average of an effect-chain graph node (mixParentEdgesInto,
// chain_process.go:295-318): dst = (0 + src0 + src1 + ...) * (1/nsrc).
struct FxMixArgs {
  const double* src[8];
  int64_t src_stride[8];
  int nsrc;
  double* dst;
  int64_t dst_stride, n;
  int channels;
};
void launch_fx_mix(const FxMixArgs& a, hipStream_t s);

// FIR block filter over [hist (N-1) | block (n)] per channel.
struct FirArgs {
  const double* h;     // [N]
  int64_t N;
  const double* hist;  // [channels][N-1]: the delay line before this block
  const double* src;   // [channels][sstride]: n new samples
  int64_t sstride;
  double* y;           // [channels][ystride]
  int64_t ystride, n;
  int channels;
  int reversed;  // taps >= 32: y[i] = sum_j h[j] x[i-N+1+j]; else sum_k h[k] x[i-k]
};
void launch_fir(const FirArgs& a, hipStream_t s);

// IRLB f16 decode: in [frames][channels] (interleaved) -> out [channels][frames]
void launch_decode_f16(const uint16_t* in, int64_t frames, int channels, double* out, hipStream_t s);

}  // namespace adsp
