// Time-parallel effect chain: biquad EQ -> feed-forward Compressor ->
// Freeverb over time chunks, with the serial recurrences broken up in time
// where their algebra allows it (host side: fx_run_tp in capi_dsp.cpp).
//
// Reference behaviour:
//   biquad.Chain.ProcessBlock        dsp/filter/biquad/chain.go:59-70, section.go:47-53
//   Compressor.ProcessSample         dsp/effects/dynamics/compressor.go:348-359, core.go:274-400
//   Reverb.ProcessSample (Freeverb)  dsp/effects/reverb/reverb.go:57-117, 169-182
//
// At config 5 (256 channels) one lane per channel gives four 64-channel
// waves: a one-lane-per-channel engine is bound by its recurrences' issue
// and latency on a handful of CUs.  Here time is a parallel axis too:
//
//   K_eq   a DF-II-T section is linear in its state s = (d0, d1): over a
//          segment of L samples, s_end = A^L s_start + s_zs, where s_zs is
//          the zero-state run of the segment and A = [[-a1, 1], [-a2, 0]].
//          Launch k runs, for every (segment, channel), the exact section k-1
//          from its true start state (the reference operations, so only the
//          start state carries rounding) fused with the zero-state run of
//          section k; the last workgroup to finish then chains the segment
//          start states of section k (S steps of a 2 x 2 map per channel).
//          nsec + 1 launches over the whole chip per chunk.
//   K_det  the envelope follower is not linear (attack or release by the
//          sign of src - env): one wave per 64 channels, serial.
//   K_verb a comb reads its line D >= 1116 samples back, so between two
//          wraps of its ring index every line value read is known before
//          the first sample; only the one-pole damping filter
//          fs = out*db + fs*da chains samples, and it forgets its start value
//          geometrically (da = damp < 1).  Such a piece is cut into up to 16
//          lane segments; segment w > 0 starts its filter `wu` samples early
//          from zero (da^wu < 2^-60: by its first output the run has met the
//          serial value, to the last bit in every case tested), segment 0
//          continues the exact carried value.  Every allpass delay is >= 225
//          samples, so the 225 samples of a window are independent.  One
//          channel per workgroup with all its delay lines in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dsp_device.hpp"
#include "dsp_kernels.hpp"
#include "fft_device.hpp"

namespace adsp {

namespace {

#define AD_TPG __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ AD_TPG T* gptr(T* p) {
  return (AD_TPG T*)p;
}
__device__ __forceinline__ int wave_of_thread() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// One DF-II-T step with the reference operations (section.go:47-53; the
// chain gain as pre-gain, kSecStride layout).
__device__ __forceinline__ double sec_step(const double (&q)[kSecStride], double& d0, double& d1, double x) {
#pragma clang fp contract(off)
  const double v = x * q[0];
  const double y = q[1] * v + d0;
  d0 = q[2] * v - q[4] * y + d1;
  d1 = q[3] * v - q[5] * y;
  return y;
}

constexpr int kTpSegB = 16;  // K_eq: rows per load batch

__global__ __launch_bounds__(256) void k_fxtp_eq(FxTpEqArgs a) {
#pragma clang fp contract(off)
  const int w = wave_of_thread();
  const int l = threadIdx.x & 63;
  const int g = blockIdx.y;
  const int c = g * 64 + l;
  const bool active = c < a.channels;
  const int cc = active ? c : a.channels - 1;
  const unsigned uc = (unsigned)c;
  const int cp = a.cpad;
  const int sg = blockIdx.x * 4 + w;  // segment
  const int k = a.k, nsec = a.eq.nsec;
  const bool p3 = k >= 1, p1 = k < nsec;
  if (sg < a.nseg) {
    const int64_t n0 = (int64_t)sg * a.seg, n1 = min(a.len, n0 + a.seg);
    const double* secs = a.eq.sec + (int64_t)cc * a.eq.sec_ch_stride;
    double q3[kSecStride], q1[kSecStride];
#pragma unroll
    for (int j = 0; j < kSecStride; ++j) {
      q3[j] = p3 ? secs[(k - 1) * kSecStride + j] : 0.0;
      q1[j] = p1 ? secs[k * kSecStride + j] : 0.0;
    }
    double d0 = 0.0, d1 = 0.0, z0 = 0.0, z1 = 0.0;
    if (p3) {
      const double2 s = reinterpret_cast<const double2*>(a.carry)[(int64_t)sg * cp + c];
      d0 = s.x;
      d1 = s.y;
    }
    // section k-1's input: the chunk input for section 0, else the rows the
    // previous launch wrote (in place: a lane rewrites only rows it has read)
    const AD_TPG double* src = gptr(k >= 2 ? (const double*)a.vT : a.xT);
    AD_TPG double* dst = gptr(a.vT);
    double xb[2][kTpSegB];
    auto load = [&](double (&b)[kTpSegB], int64_t r0) {
#pragma unroll
      for (int j = 0; j < kTpSegB; ++j) b[j] = src[min(r0 + j, a.len - 1) * cp + uc];
    };
    auto run = [&](double (&b)[kTpSegB], int64_t r0) {
      const int nb = (int)min((int64_t)kTpSegB, n1 - r0);
#pragma unroll
      for (int j = 0; j < kTpSegB; ++j) {
        if (j < nb) {
          double x = b[j];
          if (p3) {
            x = sec_step(q3, d0, d1, x);
            dst[(r0 + j) * cp + uc] = x;
          }
          if (p1) (void)sec_step(q1, z0, z1, x);
        }
      }
    };
    if (n0 < n1) load(xb[0], n0);
    for (int64_t r = n0; r < n1; r += 2 * kTpSegB) {
      if (r + kTpSegB < n1) load(xb[1], r + kTpSegB);
      run(xb[0], r);
      if (r + kTpSegB >= n1) break;
      if (r + 2 * kTpSegB < n1) load(xb[0], r + 2 * kTpSegB);
      run(xb[1], r + kTpSegB);
    }
    if (p3 && sg == a.nseg - 1 && active) {  // the chunk-end state of section k-1
      double* st = a.eq.state + ((int64_t)c * nsec + (k - 1)) * 2;
      st[0] = d0;
      st[1] = d1;
    }
    if (p1) reinterpret_cast<double2*>(a.zs)[(int64_t)sg * cp + c] = make_double2(z0, z1);
  }
}

// Double-double arithmetic (Dekker / Knuth error-free transforms with FMA)
// for K_carry.  A low-frequency section is far from normal: its poles sit
// near z = 1, 2 r sin(theta) apart, so A^n grows to ~1/(2 sin theta) (about
// 100 for the 40 Hz highpass at 48 kHz) before it decays, and M = A^seg has
// entries of ~50.  Chained in double, each step M s + z would add ~50 eps |s|
// to the start states and the rerun would amplify that by the same growth:
// measured 5e-12 relative on the EQ output.  Chained in double-double the
// start states carry one rounding (eps |s|), as the serial recurrence's do.
struct dd {
  double hi, lo;
};
__device__ __forceinline__ dd dd_two_sum(double a, double b) {
#pragma clang fp contract(off)
  const double s = a + b, bb = s - a;
  return dd{s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ dd dd_norm(double hi, double lo) {
#pragma clang fp contract(off)
  const double s = hi + lo;
  return dd{s, lo - (s - hi)};
}
__device__ __forceinline__ dd dd_add(dd x, dd y) {
#pragma clang fp contract(off)
  const dd s = dd_two_sum(x.hi, y.hi);
  return dd_norm(s.hi, s.lo + (x.lo + y.lo));
}
__device__ __forceinline__ dd dd_mul(dd x, dd y) {
#pragma clang fp contract(off)
  const double p = x.hi * y.hi;
  const double e = __builtin_fma(x.hi, y.hi, -p);
  return dd_norm(p, e + (x.hi * y.lo + x.lo * y.hi));
}
struct dd2x2 {
  dd m[4];
};
// s' = M s + z
__device__ __forceinline__ void dd_step(const dd2x2& M, dd& s0, dd& s1, dd z0, dd z1) {
  const dd t0 = dd_add(dd_add(dd_mul(M.m[0], s0), dd_mul(M.m[1], s1)), z0);
  const dd t1 = dd_add(dd_add(dd_mul(M.m[2], s0), dd_mul(M.m[3], s1)), z1);
  s0 = t0;
  s1 = t1;
}

// K_carry (after the launch that ran section k's zero-state segments): one
// workgroup of kCyW waves per 64 channels chains section k's segment start
// states in double-double, carry[0] = the chunk-start state,
// carry[v + 1] = M carry[v] + zs[v], M = A^seg.  Wave u takes Q = nseg/kCyW
// consecutive segments: it chains its zs from zero (e_u), the start of its
// range is M^Q-chained over e_0 .. e_{u-1} (LDS), then it walks its range
// again writing the starts rounded to double.
constexpr int kCyW = kFxTpCarryWaves;  // 16 KiB of LDS, so it fits beside a K_verb workgroup
__global__ __launch_bounds__(64 * kCyW) void k_fxtp_carry(FxTpEqArgs a) {
  const int w = wave_of_thread();
  const int l = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + l;
  const int cc = c < a.channels ? c : a.channels - 1;
  const int cp = a.cpad;
  const int k = a.k, nsec = a.eq.nsec;
  __shared__ dd agg[kCyW][2][64];
  // M = A^seg and M^Q, A the zero-input step [[-a1, 1], [-a2, 0]] (host, fx_tp_mats)
  const double* mt = a.mats + ((int64_t)k * a.mat_sets + (a.mat_sets > 1 ? cc : 0)) * 16;
  dd2x2 M, MQ;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    M.m[i] = dd{mt[2 * i], mt[2 * i + 1]};
    MQ.m[i] = dd{mt[8 + 2 * i], mt[8 + 2 * i + 1]};
  }
  const int Q = (a.nseg + kCyW - 1) / kCyW;
  const int v0 = w * Q, nv = max(0, min(a.nseg - v0, Q));
  const double2* zs = reinterpret_cast<const double2*>(a.zs) + (int64_t)v0 * cp + c;
  // zs streamed twice (8 loads ahead): chain from zero, then walk from the true start
  auto walk = [&](dd& s0, dd& s1, bool store) {
    double2* cy = reinterpret_cast<double2*>(a.carry) + (int64_t)v0 * cp + c;
    for (int j0 = 0; j0 < nv; j0 += 8) {
      double2 zr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) zr[j] = zs[(int64_t)min(j0 + j, nv - 1) * cp];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j0 + j < nv) {
          if (store) cy[(int64_t)(j0 + j) * cp] = make_double2(s0.hi + s0.lo, s1.hi + s1.lo);
          dd_step(M, s0, s1, dd{zr[j].x, 0}, dd{zr[j].y, 0});
        }
      }
    }
  };
  dd e0{0, 0}, e1{0, 0};
  walk(e0, e1, false);
  agg[w][0][l] = e0;
  agg[w][1][l] = e1;
  __syncthreads();
  const double* st = a.eq.state + ((int64_t)cc * nsec + k) * 2;
  dd s0{st[0], 0}, s1{st[1], 0};
  for (int u = 0; u < w; ++u) dd_step(MQ, s0, s1, agg[u][0][l], agg[u][1][l]);
  walk(s0, s1, true);
}

// ---------------------------------------------------------------------------
// K_det: side-chain prefilters, detector and envelope (core.go:274-286,
// 331-400), serial over the chunk, kDetCh channels per workgroup (lanes of
// wave 0; the other lanes repeat them): a 64-channel group would need
// ~40 GB/s of row traffic into one CU at the detector's pace.  Wave 1 keeps
// kDetNB batches of row loads in flight in registers (every load covers
// 64 / kDetCh rows of kDetCh channels; <= 63 outstanding) and puts each
// batch into a small LDS ring one step before the detector reads it; one
// barrier per batch.  The lookahead (kDetNB batches) is what hides the
// memory latency: 10 batches of 16 measured 481 us per chunk, 14 370 us.
// ---------------------------------------------------------------------------
constexpr int kDetCh = 8;      // channels per workgroup
constexpr int kDetB = 16;      // rows per batch
constexpr int kDetLd = kDetB * kDetCh / 64;  // loads per batch (2)
constexpr int kDetNB = 28;     // batches in flight in the loader (56 loads outstanding)
constexpr int kDetSlots = 4;   // LDS ring slots (a batch lives there for one step)
__device__ __forceinline__ void lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ __launch_bounds__(128) void k_fxtp_det(FxStageArgs a) {
#pragma clang fp contract(off)
  __shared__ double ring[kDetSlots][kDetB][kDetCh];
  const int w = wave_of_thread();
  const int l = threadIdx.x & 63;
  const int c0 = blockIdx.x * kDetCh;
  const int cp = a.cpad;
  const int64_t len = a.len;
  const int64_t nb = (len + kDetB - 1) / kDetB;
  const int64_t nbp = (nb + kDetNB - 1) / kDetNB * kDetNB;
  if (w == 0) {
    // lanes >= kDetCh repeat lanes 0..kDetCh-1 (same channel, same values,
    // same stores): no branch around the stores, so the ring reads of a
    // batch are issued together ahead of the envelope chain
    const int c = c0 + (l & (kDetCh - 1));
    const bool active = l < kDetCh && c < a.channels;
    const int cc = c < a.channels ? c : a.channels - 1;
    const unsigned uc = (unsigned)c;
    const int li = l & (kDetCh - 1);
    const CompParams& p = a.cp;
    CompChState cs = a.cs[cc];
    AD_TPG double* rring = gptr(a.rms_ring) + (int64_t)cc * p.rms_n;
    AD_TPG double* eo = gptr(a.envT);
    const bool bare = !p.lp_on && !p.hp_on && !p.detector_rms;
    __builtin_amdgcn_s_waitcnt(0);  // the state loads land before the step loop
    lds_bar();                      // the loader's prologue
    // nbp steps (nb rounded up to the loader's unroll): the barrier counts match
    for (int64_t k = 0; k < nbp; ++k) {
      const int slot = (int)(k % kDetSlots);
      const int64_t r0 = k * kDetB;
      const int n = (int)max((int64_t)0, min((int64_t)kDetB, len - r0));
      if (bare && n == kDetB) {
        double xv[kDetB], ev[kDetB];
#pragma unroll
        for (int d = 0; d < kDetB; ++d) xv[d] = ring[slot][d][li];
#pragma unroll
        for (int d = 0; d < kDetB; ++d) {
          cs.env = env_step(p, cs.env, fabs(xv[d]));
          ev[d] = cs.env;
        }
        // kDetLd stores per batch, not kDetB: lane l stores row
        // l / kDetCh + RS i of its channel (every lane holds its channel's
        // whole batch), picked out of ev[] by selects
        constexpr int RS = 64 / kDetCh;
        const int rq = l / kDetCh;
#pragma unroll
        for (int i = 0; i < kDetLd; ++i) {
          double v = ev[RS * i];
#pragma unroll
          for (int q = 1; q < RS; ++q) v = rq == q ? ev[RS * i + q] : v;
          eo[(r0 + rq + RS * i) * cp + uc] = v;
        }
      } else {
        for (int d = 0; d < n; ++d) {
          double sc = ring[slot][d][li];  // applyPrefilter core.go:390-400
          if (p.lp_on) {
            cs.lp = cs.lp + p.lp_alpha * (sc - cs.lp);
            sc = cs.lp;
          }
          if (p.hp_on) {
            cs.hp = cs.hp + p.hp_alpha * (sc - cs.hp);
            sc = sc - cs.hp;
          }
          double src = fabs(sc);
          if (p.detector_rms) {  // updateRMS core.go:361-388
            const double sq = src * src;
            if (cs.rms_filled == p.rms_n)
              cs.rms_sum -= rring[cs.rms_index];
            else
              cs.rms_filled++;
            if (active) rring[cs.rms_index] = sq;
            cs.rms_sum += sq;
            if (++cs.rms_index >= p.rms_n) cs.rms_index = 0;
            const double mean = cs.rms_sum / (double)p.rms_n;
            src = mean <= 0.0 ? 0.0 : sqrt(mean);
          }
          cs.env = env_step(p, cs.env, src);
          if (l < kDetCh) eo[(r0 + d) * cp + uc] = cs.env;
        }
      }
      lds_bar();
    }
    if (active) {  // only the fields this stage owns
      AD_TPG CompChState* o = gptr(a.cs) + c;
      o->env = cs.env;
      o->lp = cs.lp;
      o->hp = cs.hp;
      o->rms_sum = cs.rms_sum;
      o->rms_index = cs.rms_index;
      o->rms_filled = cs.rms_filled;
    }
  } else {
    // loader: lane l covers row (l / kDetCh) + (64 / kDetCh) i of a batch,
    // channel l % kDetCh; its register ring holds kDetNB batches, entry =
    // batch mod kDetNB
    const AD_TPG double* vin = gptr((const double*)a.vT);
    const unsigned col = (unsigned)(c0 + (l & (kDetCh - 1)));
    const int rl = l / kDetCh;
    constexpr int RS = 64 / kDetCh;  // rows per load
    double buf[kDetNB][kDetLd];
    auto load = [&](double (&r)[kDetLd], int64_t b) {
#pragma unroll
      for (int i = 0; i < kDetLd; ++i) r[i] = vin[min(b * kDetB + rl + RS * i, len - 1) * cp + col];
    };
    // branch-free: every step loads (rows past the chunk re-read its last
    // row) and stores one batch, so the compiler's vmcnt waits stay counted
    // (a conditional put or load made it drain every load at every step);
    // a batch past the last lands in a slot whose batch was already consumed
    auto put = [&](const double (&r)[kDetLd], int64_t b) {
      const int slot = (int)(b % kDetSlots);
#pragma unroll
      for (int i = 0; i < kDetLd; ++i) ring[slot][rl + RS * i][l & (kDetCh - 1)] = r[i];
    };
#pragma unroll
    for (int e = 0; e < kDetNB; ++e) load(buf[e], e);
    put(buf[0], 0);
    load(buf[0], kDetNB);
    lds_bar();
    // step k (det consumes batch k): batch k + 1 goes into its slot, batch
    // k + 1 + kDetNB is requested into the freed entry
    for (int64_t k = 0; k < nbp; k += kDetNB) {
#pragma unroll
      for (int u = 0; u < kDetNB; ++u) {
        put(buf[(u + 1) % kDetNB], k + u + 1);
        load(buf[(u + 1) % kDetNB], k + u + 1 + kDetNB);
        lds_bar();
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K_verb: Freeverb for one channel per workgroup (reverb.go:57-189), every
// delay line of the channel in LDS for the whole chunk (12587 positions,
// 98 KiB): no delay-line traffic to memory inside the chunk, and the comb
// and allpass recurrences wait on LDS, not HBM.  Input and output are
// channel-major (the gain stage writes the compressor output that way).
// Sub-blocks of kVbSB samples (the input staged in LDS):
//   waves 0..7  comb i (comb.process reverb.go:101-117): each piece of the
//               sub-block between two wraps of the ring index (a whole
//               window but at the sub-block's ends) runs as up to 32 lane
//               segments of >= wu samples (lane 0 continues the exact carried
//               filter value, lane w > 0 warms up `wu` samples from zero; see
//               the file comment); outputs to coC (global, channel-major),
//               8 consecutive samples per lane store
//   waves 8..11 after a full barrier: the ordered comb sum
//               (((0 + c0) + c1) + ... + c7), the four allpasses in series
//               (allpass.process reverb.go:57-68) and the wet/dry mix, in
//               windows of 225 samples (the shortest allpass delay: a
//               window's samples are independent), one lane each, the next
//               window's comb outputs loaded during the current one
// ---------------------------------------------------------------------------
constexpr int kVbSB = kFxVerbSB;
constexpr int kVbSeg = 32;  // comb segments per piece, at most
constexpr int kVbThreads = 64 * (kVerbCombs + 4);
constexpr int kVbXr = (kVbSB + kVbThreads - 1) / kVbThreads;  // input values per thread per sub-block
__device__ __forceinline__ double comb_fs(const VerbParams& p, double out, double fs) {
#pragma clang fp contract(off)
  double f = out * p.damp_b + fs * p.damp_a;
  if (fabs(f) < 1e-23) f = 0.0;
  return f;
}

__global__ __launch_bounds__(kVbThreads) void k_fxtp_verb(FxStageArgs a, const double* __restrict__ xC, int64_t xstride,
                                                          double* __restrict__ vbufC, double* __restrict__ coC,
                                                          int wu) {
#pragma clang fp contract(off)
  __shared__ double lines[kVerbLen];
  __shared__ double xs[kVbSB];
  const int w = wave_of_thread();
  const int l = threadIdx.x & 63;
  const int tid = threadIdx.x;
  const int c = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const VerbParams& p = a.vp;
  const int64_t len = a.len;
  double* vl = vbufC + (int64_t)c * kVerbLen;
  for (int e = tid; e < kVerbLen; e += kVbThreads) lines[e] = vl[e];
  const double* xc = xC + (int64_t)c * xstride;
  // [comb][kVbSB] of this channel, reused by every sub-block: 67 MB at 256
  // channels, rewritten while still in the Infinity Cache (a chunk-long
  // buffer left ~1 GB of dirty lines per 64K-sample chunk to reach HBM)
  double* coc = coC + (int64_t)c * kVerbCombs * kVbSB;
  double xr[kVbXr];
#pragma unroll
  for (int q = 0; q < kVbXr; ++q) {
    const int e = q * kVbThreads + tid;
    xr[q] = e < kVbSB && e < len ? xc[e] : 0.0;
  }
  // comb wave i: ring index (uniform) and the exact filter value carried
  // between pieces; allpass waves: their four ring indices
  const int ci = w < kVerbCombs ? w : 0;
  int idx = a.vs[c].comb_idx[ci];
  double carry = a.vs[c].filter_store[ci];
  int apx[kVerbAllpass];
#pragma unroll
  for (int i = 0; i < kVerbAllpass; ++i) apx[i] = a.vs[c].ap_idx[i];
  for (int64_t t0 = 0; t0 < len; t0 += kVbSB) {
    const int sb = (int)min((int64_t)kVbSB, len - t0);
#pragma unroll
    for (int q = 0; q < kVbXr; ++q) {
      const int e = q * kVbThreads + tid;
      if (e < sb) xs[e] = xr[q];
    }
#pragma unroll
    for (int q = 0; q < kVbXr; ++q) {  // the next sub-block's input, in flight during this one
      const int e = q * kVbThreads + tid;
      if (e < kVbSB && t0 + kVbSB + e < len) xr[q] = xc[t0 + kVbSB + e];
    }
    __syncthreads();  // (the first time also the lines)
#ifndef AD_VB_NOCOMB  // tools/ A/B builds only
    if (w < kVerbCombs) {
#else
    if (w < 0) {
#endif
      const int D = kCombLen[w];
      double* L = lines + comb_off(w);
      double* cw = coc + (int64_t)w * kVbSB;
      for (int r = 0; r < sb;) {
        const int pos0 = idx;
        const int m = min(sb - r, D - pos0);
        const int nw = wu > 0 ? max(1, min(kVbSeg, m / wu)) : min(kVbSeg, m);
        // odd segment length: the lanes' LDS addresses (stride Lw doubles) fall in distinct banks
        const int Lw = ((m + nw - 1) / nw) | 1;
        const int s0 = l * Lw, s1 = min(m, s0 + Lw);
        const bool mine = l < nw && s0 < s1;
        double fs = l == 0 ? carry : 0.0;
        // batches of 8: the line values are read before the filter chain
        // needs them (LDS latency off the chain)
        if (mine && l > 0) {  // warm-up: the wu samples before the segment (inside the piece: Lw >= wu)
          int j = s0 - wu;
          for (; j + 8 <= s0; j += 8) {
            double ov[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) ov[t] = L[pos0 + j + t];
#pragma unroll
            for (int t = 0; t < 8; ++t) fs = comb_fs(p, ov[t], fs);
          }
          for (; j < s0; ++j) fs = comb_fs(p, L[pos0 + j], fs);
        }
        if (mine) {
          int j = s0;
          for (; j + 8 <= s1; j += 8) {
            double ov[8], xv[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              ov[t] = L[pos0 + j + t];
              xv[t] = xs[r + j + t];
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) {
              fs = comb_fs(p, ov[t], fs);
              L[pos0 + j + t] = p.gain * xv[t] + fs * p.feedback;
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) cw[r + j + t] = ov[t];
          }
          for (; j < s1; ++j) {
            const double out = L[pos0 + j];
            fs = comb_fs(p, out, fs);
            L[pos0 + j] = p.gain * xs[r + j] + fs * p.feedback;
            cw[r + j] = out;
          }
        }
        const int lastl = (m - 1) / Lw;
        carry = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(fs), lastl),
                                 __builtin_amdgcn_readlane(__double2loint(fs), lastl));
        idx = pos0 + m == D ? 0 : pos0 + m;
        r += m;
      }
    }
    __syncthreads();  // the comb outputs (global, this workgroup's) are complete
    const int j = (w - kVerbCombs) * 64 + l;
    const bool apw = w >= kVerbCombs && j < 225;
    double cv[kVerbCombs];
    auto loadc = [&](int r) {
#pragma unroll
      for (int i = 0; i < kVerbCombs; ++i) cv[i] = coc[(int64_t)i * kVbSB + min(r + j, sb - 1)];
    };
    if (apw) loadc(0);
    for (int r = 0; r < sb; r += 225) {
      const int m = min(225, sb - r);
#ifndef AD_VB_NOAP  // tools/ A/B builds only
      if (apw && j < m) {
#else
      if (w < 0) {
#endif
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < kVerbCombs; ++i) acc += cv[i];
        int off = comb_off(kVerbCombs);
#pragma unroll
        for (int i = 0; i < kVerbAllpass; ++i) {
          int q = apx[i] + j;
          if (q >= kApLen[i]) q -= kApLen[i];
          const double bo = lines[off + q];
          const double output = bo - acc;
          lines[off + q] = acc + bo * p.ap_feedback;
          acc = output;
          off += kApLen[i];
        }
        a.buf[(int64_t)c * a.stride + t0 + r + j] = acc * p.wet + xs[r + j] * p.dry;
      }
      if (apw && r + 225 < sb) loadc(r + 225);
#pragma unroll
      for (int i = 0; i < kVerbAllpass; ++i) {
        apx[i] += m;
        if (apx[i] >= kApLen[i]) apx[i] -= kApLen[i];
      }
      lds_bar();  // allpass lines of this window before the next (LDS only: no drain of the loads in flight)
    }
  }
  for (int e = tid; e < kVerbLen; e += kVbThreads) vl[e] = lines[e];
  if (w < kVerbCombs && l == 0) {
    a.vs[c].comb_idx[w] = idx;
    a.vs[c].filter_store[w] = carry;
  }
  if (w == kVerbCombs && l == 0) {
#pragma unroll
    for (int i = 0; i < kVerbAllpass; ++i) a.vs[c].ap_idx[i] = apx[i];
  }
}

// Freeverb delay lines between the engines' layouts: position-major
// vbuf [pos][cpad] (fused and staged kernels) <-> channel-major vbufC
// [channels][kVerbLen] (K_verb).
__global__ __launch_bounds__(256) void k_vbuf_layout(double* vbuf, double* vbufC, int cpad, int channels, int to_cm) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)kVerbLen * channels) return;
  const int pos = (int)(e % kVerbLen), c = (int)(e / kVerbLen);
  if (to_cm)
    vbufC[e] = vbuf[(int64_t)pos * cpad + c];
  else
    vbuf[(int64_t)pos * cpad + c] = vbufC[e];
}

}  // namespace

void launch_fxtp_eq(const FxTpEqArgs& a, hipStream_t s) {
  if (a.len <= 0) return;
  const dim3 grid((unsigned)((a.nseg + 3) / 4), (unsigned)((a.channels + 63) / 64));
  hipLaunchKernelGGL(k_fxtp_eq, grid, dim3(256), 0, s, a);
}

void launch_fxtp_carry(const FxTpEqArgs& a, hipStream_t s) {
  if (a.len <= 0) return;
  hipLaunchKernelGGL(k_fxtp_carry, dim3((unsigned)((a.channels + 63) / 64)), dim3(64 * kCyW), 0, s, a);
}

void launch_fxtp_det(const FxStageArgs& a, hipStream_t s) {
  if (a.len <= 0) return;
  hipLaunchKernelGGL(k_fxtp_det, dim3((unsigned)((a.channels + kDetCh - 1) / kDetCh)), dim3(128), 0, s, a);
}

void launch_fxtp_verb(const FxStageArgs& a, const double* xC, int64_t xstride, double* vbufC, double* coC, int wu,
                      hipStream_t s) {
  if (a.len <= 0) return;
  hipLaunchKernelGGL(k_fxtp_verb, dim3((unsigned)a.channels), dim3(kVbThreads), 0, s, a, xC, xstride, vbufC, coC, wu);
}

void launch_vbuf_layout(double* vbuf, double* vbufC, int cpad, int channels, bool to_cm, hipStream_t s) {
  const int64_t n = (int64_t)kVerbLen * channels;
  hipLaunchKernelGGL(k_vbuf_layout, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, vbuf, vbufC, cpad, channels,
                     to_cm ? 1 : 0);
}

}  // namespace adsp
