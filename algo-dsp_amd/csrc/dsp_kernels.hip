// Per-sample processors of the algo-dsp hot path, hand-written for gfx950:
//   biquad.Chain / biquad.Section ProcessBlock   dsp/filter/biquad/chain.go:59-70, section.go:56-138
//   dynamics.Compressor ProcessInPlace            dsp/effects/dynamics/compressor.go:348-366,
//                                                  core.go:274-400
//   reverb.Reverb (Freeverb) ProcessInPlace       dsp/effects/reverb/reverb.go:57-189
//   effectchain filter -> dyn-compressor -> reverb-freeverb, fused per sample
//                                                  dsp/effectchain/chain_process.go:11-33
//   fir.Filter ProcessBlock / ProcessBlockTo      dsp/filter/fir/filter.go:46-159
//
// The recurrences are serial in time, so the parallel axis is the channel:
// one lane per channel, state and coefficients in VGPRs for the whole call.  Fusing the chain's stages per
// sample gives the same result bit for bit as the reference's stage-by-stage
// block passes (each stage is causal and only sees its predecessor's output
// of the same sample), and reads/writes each sample once instead of once per
// stage.  `#pragma clang fp contract(off)`: the reference (amd64, no FMA
// fusion) rounds every product and sum separately, and so do these kernels,
// which makes the biquad, Freeverb and FIR (taps < 32) paths bit-exact.
//
// Freeverb delay lines are stored position-major, channel-minor
// ([pos][Cpad]): all channels advance their ring indices in lockstep, so the
// 12 delay-line reads and 12 writes per sample are 512-byte coalesced wave
// accesses.  The reads of a chunk of D samples are issued together at the
// chunk start (a line is rewritten only `size` >= 225 samples after it is
// read, so a D <= 8 lookahead never reads a stale value).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "blocked_dot.hpp"
#include "dsp_device.hpp"
#include "dsp_kernels.hpp"

namespace adsp {

namespace {

constexpr int kVerbD = 2;                                                              // samples per chunk


template <bool EQ, bool COMP, bool VERB>
__global__ __launch_bounds__(64) void k_chain(ChainArgs a) {
#pragma clang fp contract(off)
  const int c = blockIdx.x * 64 + threadIdx.x;
  const bool active = c < a.channels;
  const int cc = active ? c : a.channels - 1;  // inactive lanes shadow the last channel, never store
  double* xb = a.buf + (int64_t)cc * a.stride;

  // --- EQ state / coefficients (up to kMaxSecPerPass sections per launch),
  // held in VGPRs for the whole call (a shared table has channel stride 0)
  double d0[kMaxSecPerPass], d1[kMaxSecPerPass], q[kMaxSecPerPass][kSecStride];
  if constexpr (EQ) {
    const double* sec = a.eq.sec + (int64_t)cc * a.eq.sec_ch_stride;
#pragma unroll
    for (int s = 0; s < kMaxSecPerPass; ++s) {
      d0[s] = s < a.eq.nsec ? a.eq.state[((int64_t)cc * a.eq.nsec + s) * 2] : 0.0;
      d1[s] = s < a.eq.nsec ? a.eq.state[((int64_t)cc * a.eq.nsec + s) * 2 + 1] : 0.0;
#pragma unroll
      for (int k = 0; k < kSecStride; ++k) q[s][k] = s < a.eq.nsec ? sec[s * kSecStride + k] : 0.0;
    }
  }
  // --- compressor state
  CompChState cs{};
  double* ring = nullptr;
  if constexpr (COMP) {
    cs = a.cs[cc];
    ring = a.rms_ring + (int64_t)cc * a.cp.rms_n;
  }
  // --- Freeverb state
  VerbChState vs{};
  const int cpad = (a.channels + 63) / 64 * 64;
  if constexpr (VERB) vs = a.vs[cc];

  // Chunks of kVerbD samples, double-buffered: the input samples and the
  // Freeverb delay-line values of chunk k+1 are loaded (branch-free, clamped)
  // while chunk k computes.  Fixed ping-pong buffers (A/B) instead of a
  // loop-carried copy keep the loads in flight across the chunk.
  auto load_chunk = [&](double (&x)[kVerbD], double (&dl)[kVerbCombs + kVerbAllpass][kVerbD], int64_t t0,
                        int ahead) {
#pragma unroll
    for (int d = 0; d < kVerbD; ++d) x[d] = xb[min(t0 + d, a.n - 1)];
    if constexpr (VERB) {
#pragma unroll
      for (int i = 0; i < kVerbCombs; ++i) {
        int p = vs.comb_idx[i] + ahead;
        if (p >= kCombLen[i]) p -= kCombLen[i];
#pragma unroll
        for (int d = 0; d < kVerbD; ++d) {
          dl[i][d] = a.vbuf[(int64_t)(comb_off(i) + p) * cpad + c];
          if (++p >= kCombLen[i]) p = 0;
        }
      }
#pragma unroll
      for (int i = 0; i < kVerbAllpass; ++i) {
        int p = vs.ap_idx[i] + ahead;
        if (p >= kApLen[i]) p -= kApLen[i];
#pragma unroll
        for (int d = 0; d < kVerbD; ++d) {
          dl[kVerbCombs + i][d] = a.vbuf[(int64_t)(ap_off(i) + p) * cpad + c];
          if (++p >= kApLen[i]) p = 0;
        }
      }
    }
  };
  auto compute_chunk = [&](double (&x)[kVerbD], double (&dl)[kVerbCombs + kVerbAllpass][kVerbD], int64_t t0) {
    const int nd = (int)min((int64_t)kVerbD, a.n - t0);
#pragma unroll
    for (int d = 0; d < kVerbD; ++d) {
      if (d >= nd) break;
      double v = x[d];
      if constexpr (EQ) {
#pragma unroll
        for (int s = 0; s < kMaxSecPerPass; ++s) {
          if (s >= a.eq.nsec) break;
          v = v * q[s][0];                                // chain gain (1.0 is exact)
          const double y = q[s][1] * v + d0[s];           // section.go:47-53
          d0[s] = q[s][2] * v - q[s][4] * y + d1[s];
          d1[s] = q[s][3] * v - q[s][5] * y;
          v = y;
        }
      }
      if constexpr (COMP) {  // Compressor.ProcessSample (compressor.go:348-359, core.go:274-286)
        const CompParams& p = a.cp;
        double src;
        if (p.topology_fb) {
          src = cs.prev_abs;
        } else {
          double s = v;  // applyPrefilter core.go:390-400
          if (p.lp_on) {
            cs.lp += p.lp_alpha * (s - cs.lp);
            s = cs.lp;
          }
          if (p.hp_on) {
            cs.hp += p.hp_alpha * (s - cs.hp);
            s = s - cs.hp;
          }
          src = fabs(s);
        }
        if (p.detector_rms) {  // updateRMS core.go:361-388
          const double sq = src * src;
          if (cs.rms_filled == p.rms_n)
            cs.rms_sum -= ring[cs.rms_index];
          else
            cs.rms_filled++;
          ring[cs.rms_index] = sq;
          cs.rms_sum += sq;
          if (++cs.rms_index >= p.rms_n) cs.rms_index = 0;
          const double mean = cs.rms_sum / (double)p.rms_n;
          src = mean <= 0.0 ? 0.0 : sqrt(mean);
        }
        cs.env = env_step(p, cs.env, src);
        double g = gain_for_level(p, cs.env);
        if (p.mode == 2) {  // gate hold (gate.go:361-366)
          if (g >= 1.0) {
            cs.hold = p.hold_n;
          } else if (cs.hold > 0) {
            cs.hold--;
            g = 1.0;
          }
        }
        const double out = v * g * p.makeup_lin;  // makeup_lin = 1 for the expander and gate
        if (p.topology_fb) {
          cs.prev_gain = g > 1e-9 ? g : 1e-9;
          if (!p.mode) cs.prev_abs = fabs(out);  // the expander and gate keep only previousGain
        }
        const double il = fabs(v), ol = fabs(out);  // updateMetrics compressor.go:411-423
        if (il > cs.in_peak) cs.in_peak = il;
        if (ol > cs.out_peak) cs.out_peak = ol;
        if (cs.gr == 1.0 || g < cs.gr) cs.gr = g;
        v = out;
      }
      if constexpr (VERB) {  // Reverb.ProcessSample reverb.go:169-182
        const VerbParams& p = a.vp;
        const double in = v;
        const double xg = p.gain * in;
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < kVerbCombs; ++i) {  // comb.process reverb.go:101-117
          const double output = dl[i][d];
          double fs = output * p.damp_b + vs.filter_store[i] * p.damp_a;
          if (fabs(fs) < 1e-23) fs = 0.0;
          vs.filter_store[i] = fs;
          if (active)
            a.vbuf[(int64_t)(comb_off(i) + vs.comb_idx[i]) * cpad + c] = xg + fs * p.feedback;
          if (++vs.comb_idx[i] >= kCombLen[i]) vs.comb_idx[i] = 0;
          acc += output;
        }
#pragma unroll
        for (int i = 0; i < kVerbAllpass; ++i) {  // allpass.process reverb.go:57-68
          const double bo = dl[kVerbCombs + i][d];
          const double output = bo - acc;
          if (active) a.vbuf[(int64_t)(ap_off(i) + vs.ap_idx[i]) * cpad + c] = acc + bo * p.ap_feedback;
          if (++vs.ap_idx[i] >= kApLen[i]) vs.ap_idx[i] = 0;
          acc = output;
        }
        v = acc * p.wet + in * p.dry;
      }
      x[d] = v;
    }
    if (active) {
#pragma unroll
      for (int d = 0; d < kVerbD; ++d)
        if (d < nd) xb[t0 + d] = x[d];
    }
    };
  double xa[kVerbD], xbb[kVerbD];
  double dla[kVerbCombs + kVerbAllpass][kVerbD], dlb[kVerbCombs + kVerbAllpass][kVerbD];
  load_chunk(xa, dla, 0, 0);
  for (int64_t t0 = 0; t0 < a.n; t0 += 2 * kVerbD) {
    load_chunk(xbb, dlb, t0 + kVerbD, kVerbD);
    compute_chunk(xa, dla, t0);
    if (t0 + kVerbD >= a.n) break;
    load_chunk(xa, dla, t0 + 2 * kVerbD, kVerbD);
    compute_chunk(xbb, dlb, t0 + kVerbD);
  }

  if (!active) return;
  if constexpr (EQ) {
#pragma unroll
    for (int s = 0; s < kMaxSecPerPass; ++s) {
      if (s >= a.eq.nsec) break;
      a.eq.state[((int64_t)c * a.eq.nsec + s) * 2] = d0[s];
      a.eq.state[((int64_t)c * a.eq.nsec + s) * 2 + 1] = d1[s];
    }
  }
  if constexpr (COMP) a.cs[c] = cs;
  if constexpr (VERB) a.vs[c] = vs;
}

// ---------------------------------------------------------------------------
// Wave-pipelined effect chain (EQ -> feed-forward Compressor -> Freeverb).
// One workgroup of five waves serves 64 channels; each wave runs one stage
// of every sample and the chunks of kPipeD samples flow through LDS rings:
//   wave 0  EQ sections + compressor side-chain filters, detector, envelope
//           (the serial recurrences)          -> v, env
//   wave 1  gain(env) = 2^(-cf*knee(log2 env - T)), out = v*g*makeup,
//           metrics (independent per sample given env) -> out
//   wave 2  Freeverb combs 0-3 (delay-line reads a chunk ahead) -> c0+..+c3
//   wave 3  Freeverb combs 4-7                                  -> c4..c7
//   wave 4  comb sum, allpasses, wet/dry mix, store
// At step k wave w works on chunk k - w; one barrier per step.  Every
// value is computed with the same operations in the same order as the fused
// one-wave kernel, so results are identical; the four stages just run on
// four SIMDs at once instead of one after the other.
// ---------------------------------------------------------------------------
constexpr int kPipeD = 8;
constexpr int kRing = 4;

__global__ __launch_bounds__(320) void k_chain_pipe(ChainArgs a) {
#pragma clang fp contract(off)
  __shared__ double ring_v[kRing][kPipeD][64];
  __shared__ double ring_env[kRing][kPipeD][64];
  __shared__ double ring_out[kRing][kPipeD][64];
  __shared__ double ring_acc[kRing][kPipeD][64];     // combs 0-3 partial sum
  __shared__ double ring_c47[kRing][4][kPipeD][64];  // outputs of combs 4-7
  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + l;
  const bool active = c < a.channels;
  const int cc = active ? c : a.channels - 1;
  const int cpad = (a.channels + 63) / 64 * 64;
  double* xb = a.buf + (int64_t)cc * a.stride;
  const int64_t nch = (a.n + kPipeD - 1) / kPipeD;
  const CompParams& p = a.cp;
  const VerbParams& vp = a.vp;
  unsigned long long t_busy = 0, t_mark = clock64(), t_start = t_mark;
  // step barrier; with AD_FX_PROF the wave's busy time (excluding the wait) is accumulated
#define PIPE_SYNC()                                 \
  do {                                              \
    if (a.prof) t_busy += clock64() - t_mark;       \
    __syncthreads();                                \
    if (a.prof) t_mark = clock64();                 \
  } while (0)

  if (w == 0) {
    // ---- EQ + detector
    double d0[kMaxSecPerPass], d1[kMaxSecPerPass], q[kMaxSecPerPass][kSecStride];
    const double* sec = a.eq.sec + (int64_t)cc * a.eq.sec_ch_stride;
#pragma unroll
    for (int s = 0; s < kMaxSecPerPass; ++s) {
      d0[s] = s < a.eq.nsec ? a.eq.state[((int64_t)cc * a.eq.nsec + s) * 2] : 0.0;
      d1[s] = s < a.eq.nsec ? a.eq.state[((int64_t)cc * a.eq.nsec + s) * 2 + 1] : 0.0;
#pragma unroll
      for (int k = 0; k < kSecStride; ++k) q[s][k] = s < a.eq.nsec ? sec[s * kSecStride + k] : 0.0;
    }
    CompChState cs = a.cs[cc];
    double* rring = a.rms_ring + (int64_t)cc * p.rms_n;
    double xn[kPipeD], xn2[kPipeD];  // the next two chunks of input
#pragma unroll
    for (int d = 0; d < kPipeD; ++d) {
      xn[d] = xb[min((int64_t)d, a.n - 1)];
      xn2[d] = xb[min((int64_t)(kPipeD + d), a.n - 1)];
    }
    for (int64_t k = 0; k < nch + 3; ++k) {
      if (k < nch) {
        const int r = (int)(k % kRing);
        const int64_t t0 = k * kPipeD;
        double x[kPipeD];
#pragma unroll
        for (int d = 0; d < kPipeD; ++d) {
          x[d] = xn[d];
          xn[d] = xn2[d];
        }
#pragma unroll
        for (int d = 0; d < kPipeD; ++d) xn2[d] = xb[min(t0 + 2 * kPipeD + d, a.n - 1)];
#pragma unroll
        for (int d = 0; d < kPipeD; ++d) {
          const bool real = t0 + d < a.n;  // padding of the last chunk leaves every state untouched
          double v = x[d];
#pragma unroll
          for (int s = 0; s < kMaxSecPerPass; ++s) {
            if (s >= a.eq.nsec) break;
            v = v * q[s][0];
            const double y = q[s][1] * v + d0[s];
            const double n0 = q[s][2] * v - q[s][4] * y + d1[s];
            const double n1 = q[s][3] * v - q[s][5] * y;
            d0[s] = real ? n0 : d0[s];
            d1[s] = real ? n1 : d1[s];
            v = y;
          }
          double sc = v;  // applyPrefilter core.go:390-400
          if (p.lp_on) {
            const double nl = cs.lp + p.lp_alpha * (sc - cs.lp);
            sc = nl;
            if (real) cs.lp = nl;
          }
          if (p.hp_on) {
            const double nh = cs.hp + p.hp_alpha * (sc - cs.hp);
            sc = sc - nh;
            if (real) cs.hp = nh;
          }
          double src = fabs(sc);
          if (p.detector_rms) {  // updateRMS core.go:361-388
            if (real) {
              const double sq = src * src;
              if (cs.rms_filled == p.rms_n)
                cs.rms_sum -= rring[cs.rms_index];
              else
                cs.rms_filled++;
              rring[cs.rms_index] = sq;
              cs.rms_sum += sq;
              if (++cs.rms_index >= p.rms_n) cs.rms_index = 0;
              const double mean = cs.rms_sum / (double)p.rms_n;
              src = mean <= 0.0 ? 0.0 : sqrt(mean);
            }
          }
          if (real) cs.env = env_step(p, cs.env, src);
          ring_v[r][d][l] = v;
          ring_env[r][d][l] = cs.env;
        }
      }
      PIPE_SYNC();
    }
    if (active) {  // each wave stores only the state fields it owns
#pragma unroll
      for (int s = 0; s < kMaxSecPerPass; ++s) {
        if (s >= a.eq.nsec) break;
        a.eq.state[((int64_t)c * a.eq.nsec + s) * 2] = d0[s];
        a.eq.state[((int64_t)c * a.eq.nsec + s) * 2 + 1] = d1[s];
      }
      CompChState* o = a.cs + c;
      o->env = cs.env;
      o->lp = cs.lp;
      o->hp = cs.hp;
      o->rms_sum = cs.rms_sum;
      o->rms_index = cs.rms_index;
      o->rms_filled = cs.rms_filled;
    }
  } else if (w == 1) {
    // ---- gain + metrics
    CompChState cs = a.cs[cc];
    for (int64_t k = 0; k < nch + 3; ++k) {
      const int64_t my = k - 1;
      if (my >= 0 && my < nch) {
        const int r = (int)(my % kRing);
        const int64_t t0 = my * kPipeD;
#pragma unroll 4
        for (int d = 0; d < kPipeD; ++d) {
          const double v = ring_v[r][d][l];
          double g = gain_for_level(p, ring_env[r][d][l]);
          if (p.mode == 2 && t0 + d < a.n) {  // gate hold (gate.go:361-366)
            if (g >= 1.0) {
              cs.hold = p.hold_n;
            } else if (cs.hold > 0) {
              cs.hold--;
              g = 1.0;
            }
          }
          const double out = v * g * p.makeup_lin;
          if (t0 + d < a.n) {
            const double il = fabs(v), ol = fabs(out);
            if (il > cs.in_peak) cs.in_peak = il;
            if (ol > cs.out_peak) cs.out_peak = ol;
            if (cs.gr == 1.0 || g < cs.gr) cs.gr = g;
          }
          ring_out[r][d][l] = out;
        }
      }
      PIPE_SYNC();
    }
    if (active) {
      a.cs[c].hold = cs.hold;
      a.cs[c].in_peak = cs.in_peak;
      a.cs[c].out_peak = cs.out_peak;
      a.cs[c].gr = cs.gr;
    }
  } else if (w == 2 || w == 3) {
    // ---- combs: wave 2 runs combs 0-3 and passes their running sum, wave 3
    // runs combs 4-7 and passes each output; the allpass wave finishes the
    // reference's sequential sum acc = (((c0+c1)+c2)+...)+c7 in order.
    // Branch-free vmem: lanes past the channel count shadow the last channel
    // (same state, same input, so identical values to identical addresses),
    // and padding samples of the last chunk write back the value they read
    // (a no-op), so every chunk issues the same loads and stores and the
    // prefetch wait never drains the previous chunk's stores.
    const int i0 = w == 2 ? 0 : 4;
    const int col = cc;
    VerbChState vs = a.vs[cc];
    int cidx[4];  // write positions (advance on padding too)
    double fst[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      cidx[i] = vs.comb_idx[i0 + i];
      fst[i] = vs.filter_store[i0 + i];
    }
    auto comb_len = [&](int i) { return w == 2 ? kCombLen[i] : kCombLen[4 + i]; };
    auto comb_base = [&](int i) { return w == 2 ? comb_off(i) : comb_off(4 + i); };
    auto prefetch = [&](double (&dl)[4][kPipeD], int ahead) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int len = comb_len(i);
        int pp = cidx[i] + ahead;
        if (pp >= len) pp -= len;
#pragma unroll
        for (int d = 0; d < kPipeD; ++d) {
          dl[i][d] = a.vbuf[(int64_t)(comb_base(i) + pp) * cpad + col];
          if (++pp >= len) pp = 0;
        }
      }
    };
    // Three delay-line buffers in rotation, chunk m in b[m % 3]: the loads
    // of chunk m+2 are issued while chunk m computes and are first waited on
    // two steps later.  The step loop is unrolled by three so the rotation is
    // a compile-time renaming (a runtime copy would wait on them at once).
    auto step = [&](int64_t my, double (&cur)[4][kPipeD], double (&pre)[4][kPipeD]) {
      if (my < 0 || my >= nch) return;
      const int r = (int)(my % kRing);
      const int64_t t0 = my * kPipeD;
      prefetch(pre, 2 * kPipeD);  // lines are rewritten only >= 225 samples after they are read
#pragma unroll
      for (int d = 0; d < kPipeD; ++d) {
        const double xg = vp.gain * ring_out[r][d][l];
        const bool real = t0 + d < a.n;
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double output = cur[i][d];
          double fs = output * vp.damp_b + fst[i] * vp.damp_a;
          if (fabs(fs) < 1e-23) fs = 0.0;
          fst[i] = real ? fs : fst[i];
          const double wv = xg + fs * vp.feedback;
          a.vbuf[(int64_t)(comb_base(i) + cidx[i]) * cpad + col] = real ? wv : output;
          if (++cidx[i] >= comb_len(i)) cidx[i] = 0;
          if (w == 2)
            acc += output;
          else
            ring_c47[r][i][d][l] = output;
        }
        if (w == 2) ring_acc[r][d][l] = acc;
      }
    };
    double b0[4][kPipeD], b1[4][kPipeD], b2[4][kPipeD];
    prefetch(b0, 0);
    prefetch(b1, kPipeD);
    for (int64_t k = 0; k < nch + 3; k += 3) {  // chunk my = k - 2 + j, my % 3 = (1 + j) % 3
      step(k - 2, b1, b0);
      PIPE_SYNC();
      if (k + 1 < nch + 3) {
        step(k - 1, b2, b1);
        PIPE_SYNC();
      }
      if (k + 2 < nch + 3) {
        step(k, b0, b2);
        PIPE_SYNC();
      }
    }
    if (active) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a.vs[c].filter_store[i0 + i] = fst[i];
        a.vs[c].comb_idx[i0 + i] = (int)((vs.comb_idx[i0 + i] + a.n) % comb_len(i));
      }
    }
  } else {
    // ---- allpasses + mix + store (branch-free vmem, as the combs wave)
    const int col = cc;
    int ap_idx[kVerbAllpass];
#pragma unroll
    for (int i = 0; i < kVerbAllpass; ++i) ap_idx[i] = a.vs[cc].ap_idx[i];
    const int ap0[kVerbAllpass] = {ap_idx[0], ap_idx[1], ap_idx[2], ap_idx[3]};
    auto prefetch = [&](double (&dl)[kVerbAllpass][kPipeD], int ahead) {
#pragma unroll
      for (int i = 0; i < kVerbAllpass; ++i) {
        int pp = ap_idx[i] + ahead;
        if (pp >= kApLen[i]) pp -= kApLen[i];
#pragma unroll
        for (int d = 0; d < kPipeD; ++d) {
          dl[i][d] = a.vbuf[(int64_t)(ap_off(i) + pp) * cpad + col];
          if (++pp >= kApLen[i]) pp = 0;
        }
      }
    };
    auto step = [&](int64_t my, double (&cur)[kVerbAllpass][kPipeD], double (&pre)[kVerbAllpass][kPipeD]) {
      if (my < 0 || my >= nch) return;
      const int r = (int)(my % kRing);
      const int64_t t0 = my * kPipeD;
      prefetch(pre, 2 * kPipeD);
        double last = 0.0;
#pragma unroll
        for (int d = 0; d < kPipeD; ++d) {
          double acc = ring_acc[r][d][l];
#pragma unroll
          for (int i = 0; i < 4; ++i) acc += ring_c47[r][i][d][l];
          const double in = ring_out[r][d][l];
          const bool real = t0 + d < a.n;
#pragma unroll
          for (int i = 0; i < kVerbAllpass; ++i) {
            const double bo = cur[i][d];
            const double output = bo - acc;
            a.vbuf[(int64_t)(ap_off(i) + ap_idx[i]) * cpad + col] = real ? acc + bo * vp.ap_feedback : bo;
            if (++ap_idx[i] >= kApLen[i]) ap_idx[i] = 0;
            acc = output;
          }
          const double y = acc * vp.wet + in * vp.dry;
          last = real ? y : last;  // padding rewrites the last real sample with its own value
          xb[min(t0 + d, a.n - 1)] = last;
        }
    };
    double b0[kVerbAllpass][kPipeD], b1[kVerbAllpass][kPipeD], b2[kVerbAllpass][kPipeD];
    prefetch(b0, 0);
    prefetch(b1, kPipeD);
    for (int64_t k = 0; k < nch + 3; k += 3) {  // chunk my = k - 3 + j, my % 3 = j
      step(k - 3, b0, b2);
      PIPE_SYNC();
      if (k + 1 < nch + 3) {
        step(k - 2, b1, b0);
        PIPE_SYNC();
      }
      if (k + 2 < nch + 3) {
        step(k - 1, b2, b1);
        PIPE_SYNC();
      }
    }
    if (active) {
#pragma unroll
      for (int i = 0; i < kVerbAllpass; ++i) a.vs[c].ap_idx[i] = (int)((ap0[i] + a.n) % kApLen[i]);
    }
  }
  if (a.prof && l == 0) {
    a.prof[(blockIdx.x * 8 + w) * 2] = t_busy;
    a.prof[(blockIdx.x * 8 + w) * 2 + 1] = clock64() - t_start;
  }
#undef PIPE_SYNC
}
// fir.Filter block paths (filter.go:64-104 / 109-149).  Output-parallel: a
// workgroup owns 256 consecutive outputs of one channel, one lane per output
// sample, summing in the reference's term order q = 0, 1, ... with a rounded
// product and a rounded add:
//   reversed (taps >= 32, the block path's dot): term q = h[q] * x[i-(N-1)+q]
//   ring     (taps <  32, ProcessSample's loop): term q = h[q] * x[i-q]
// where x[< 0] is the delay line.  Taps are walked in chunks of FQ; the input
// window a chunk meets (256 + FQ - 1 samples, from the delay line and the new
// block) is staged in LDS, and h[q] is wave-uniform (scalar loads).
//
// A lane owns R consecutive outputs (blocked_dot.hpp): the window slides by
// one sample per term, so one R-wide LDS read feeds R*R products and the
// reversed path is bound by the FP64 VALU rather than LDS bandwidth.
constexpr int FQ = 1024;
template <int R>
__global__ __launch_bounds__(256) void k_fir(FirArgs a) {
#pragma clang fp contract(off)
  constexpr int DT = 256 * R;
  __shared__ __attribute__((aligned(32))) double w[DT + FQ + 8];
  const int t = threadIdx.x;
  const int c = blockIdx.y;
  const int64_t i0 = (int64_t)blockIdx.x * DT;
  const int64_t hn = a.N - 1;
  const double* hc = a.hist + (int64_t)c * hn;
  const double* xc = a.src + (int64_t)c * a.sstride;
  double acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0;
  for (int64_t q0 = 0; q0 < a.N; q0 += FQ) {
    const int cq = (int)(a.N - q0 < FQ ? a.N - q0 : FQ);
    // window start: reversed w[1 + v] = x[i0 - hn + q0 + v]; ring w[1 + v] = x[i0 - q0 - cq + 1 + v]
    const int64_t g0 = a.reversed ? i0 - hn + q0 : i0 - q0 - cq + 1;
    __syncthreads();
    for (int v = t; v < DT + cq - 1; v += 256) {
      const int64_t g = g0 + v;
      w[1 + v] = g < 0 ? hc[hn + g] : (g < a.n ? xc[g] : 0.0);
    }
    __syncthreads();
    const double* hq = a.h + q0;
    const double* wt = w + 1 + t * R;
    if (a.reversed) {
      blocked_dot<R, 1>(hq, wt, cq, acc);  // term q0 + u of output r: wt[u + r]
    } else {
      for (int u = 0; u < cq; ++u) {  // term q0 + u of output r: wt[r + cq - 1 - u]
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const double p = hq[u] * wt[r + cq - 1 - u];
          acc[r] = acc[r] + p;
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = i0 + t * R + r;
    if (i < a.n) a.y[(int64_t)c * a.ystride + i] = acc[r];
  }
}

// decodeF16 (internal/webdemo/irlib.go:68-97), reference quirk kept: a
// subnormal is normalised with exponent 127-14-e+1 (one more than IEEE).
__device__ __forceinline__ float decode_f16(uint32_t h) {
  const uint32_t sign = (h >> 15) << 31;
  const uint32_t ex = (h >> 10) & 0x1F;
  const uint32_t frac = h & 0x3FF;
  uint32_t bits;
  if (ex == 0) {
    if (frac == 0) {
      bits = sign;
    } else {
      const int e = __clz(frac) - 21;  // shifts until bit 10 is set
      bits = sign | ((uint32_t)(127 - 14 - e + 1) << 23) | (((frac << e) & 0x3FF) << 13);
    }
  } else if (ex == 31) {
    bits = sign | 0x7F800000u | (frac << 13);
  } else {
    bits = sign | ((ex + 112) << 23) | (frac << 13);
  }
  return __uint_as_float(bits);
}

// readIRChunk's AUDI loop (irlib.go:414-451): sample i belongs to channel
// i % ch, frame i / ch; output is channel-major float64.
__global__ __launch_bounds__(256) void k_decode_f16(const uint16_t* __restrict__ in, int64_t frames, int channels,
                                                    double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= frames * channels) return;
  const int64_t f = i / channels;
  const int c = (int)(i - f * channels);
  out[(int64_t)c * frames + f] = (double)decode_f16(in[i]);
}

// Mono / stereo form: a lane decodes 4 whole frames (one 8- or 16-byte load
// of the interleaved codes) and stores 4 consecutive doubles per channel.
template <int CH>
__global__ __launch_bounds__(256) void k_decode_f16_v(const uint16_t* __restrict__ in, int64_t frames,
                                                      double* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;  // frames 4g .. 4g+3
  const int64_t f0 = 4 * g;
  if (f0 >= frames) return;
  if (f0 + 4 <= frames) {
    uint32_t w[2 * CH];
    if constexpr (CH == 1) {
      const uint2 v = *reinterpret_cast<const uint2*>(in + f0);
      w[0] = v.x;
      w[1] = v.y;
    } else {
      const uint4 v = *reinterpret_cast<const uint4*>(in + 2 * f0);
      w[0] = v.x;
      w[1] = v.y;
      w[2] = v.z;
      w[3] = v.w;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      double d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = j * CH + c;  // code index within the 4 frames
        d[j] = (double)decode_f16((w[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
      }
      double2* o = reinterpret_cast<double2*>(out + (int64_t)c * frames + f0);
      o[0] = make_double2(d[0], d[1]);
      o[1] = make_double2(d[2], d[3]);
    }
  } else {
    for (int64_t f = f0; f < frames; ++f)
      for (int c = 0; c < CH; ++c) out[(int64_t)c * frames + f] = (double)decode_f16(in[f * CH + c]);
  }
}

}  // namespace

// Fan-in average (mixParentEdgesInto, chain_process.go:295-318): the Go code
// zeroes mixBuf, adds each parent's block in edge order, then scales by
// 1/len(parents); the same rounded adds and one rounded multiply here.
__global__ __launch_bounds__(256) void k_fx_mix(FxMixArgs a) {
#pragma clang fp contract(off)
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  if (t >= a.n) return;
  double acc = 0.0;
  for (int k = 0; k < a.nsrc; ++k) acc += a.src[k][(int64_t)c * a.src_stride[k] + t];
  a.dst[(int64_t)c * a.dst_stride + t] = acc * (1.0 / (double)a.nsrc);
}

void launch_fx_mix(const FxMixArgs& a, hipStream_t s) {
  if (a.n <= 0 || a.channels <= 0) return;
  hipLaunchKernelGGL(k_fx_mix, dim3((unsigned)((a.n + 255) / 256), (unsigned)a.channels), dim3(256), 0, s, a);
}

void launch_decode_f16(const uint16_t* in, int64_t frames, int channels, double* out, hipStream_t s) {
  const int64_t n = frames * channels;
  if (n <= 0) return;
  // vector form when every row and the input are 16-byte aligned
  const bool al = ((uintptr_t)in % 16 == 0) && ((uintptr_t)out % 16 == 0) && frames % 2 == 0;
  const unsigned g4 = (unsigned)((frames + 1023) / 1024);
  if (al && channels == 1) {
    hipLaunchKernelGGL(k_decode_f16_v<1>, dim3(g4), dim3(256), 0, s, in, frames, out);
  } else if (al && channels == 2) {
    hipLaunchKernelGGL(k_decode_f16_v<2>, dim3(g4), dim3(256), 0, s, in, frames, out);
  } else {
    hipLaunchKernelGGL(k_decode_f16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, frames, channels, out);
  }
}

template <bool EQ, bool COMP, bool VERB>
static void chain_go(const ChainArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((k_chain<EQ, COMP, VERB>), dim3((unsigned)((a.channels + 63) / 64)), dim3(64), 0, s, a);
}

bool chain_pipe_ok(int stages, const ChainArgs& a) {
  return stages == 7 && !a.cp.topology_fb && a.eq.nsec <= kMaxSecPerPass;
}

void launch_chain(int stages, const ChainArgs& a, hipStream_t s) {
  if (a.channels <= 0 || a.n <= 0) return;
  if (chain_pipe_ok(stages, a)) {
    hipLaunchKernelGGL(k_chain_pipe, dim3((unsigned)((a.channels + 63) / 64)), dim3(320), 0, s, a);
    return;
  }
  switch (stages) {
    case 1: chain_go<true, false, false>(a, s); break;
    case 2: chain_go<false, true, false>(a, s); break;
    case 3: chain_go<true, true, false>(a, s); break;
    case 4: chain_go<false, false, true>(a, s); break;
    case 5: chain_go<true, false, true>(a, s); break;
    case 6: chain_go<false, true, true>(a, s); break;
    case 7: chain_go<true, true, true>(a, s); break;
    default: break;
  }
}

void launch_fir(const FirArgs& a, hipStream_t s) {
  if (a.channels <= 0 || a.n <= 0) return;
  // R = 4 outputs per lane once that still gives >= 2 workgroups per CU
  const int64_t work = a.n * a.channels;
  if (work >= 512 * 1024)
    hipLaunchKernelGGL(k_fir<4>, dim3((unsigned)((a.n + 1023) / 1024), (unsigned)a.channels), dim3(256), 0, s, a);
  else if (work >= 512 * 512)
    hipLaunchKernelGGL(k_fir<2>, dim3((unsigned)((a.n + 511) / 512), (unsigned)a.channels), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_fir<1>, dim3((unsigned)((a.n + 255) / 256), (unsigned)a.channels), dim3(256), 0, s, a);
}

}  // namespace adsp
