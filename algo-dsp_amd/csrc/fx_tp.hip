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
//   K_eq   the biquad cascade is linear in its state S (2 values per
//          section): over a segment of L samples S_end = B S_start + Z, with
//          Z the cascade's zero-state run of the segment and B = A^L (A the
//          cascade's zero-input step, block lower triangular).  K_eqz runs
//          every (segment, channel) from zero (Z); K_carry chains the segment
//          start states in double-double (an LDS scan over the segments per
//          section, the earlier sections' starts folded in through B's
//          off-diagonal blocks); K_eqx reruns the cascade from those starts
//          with the reference operations (only the start states carry
//          rounding).  Three launches and two passes over the chunk.
//   K_det  the envelope follower is not linear (attack or release by the
//          sign of src - env): serial per channel, 8 channels per workgroup.
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

constexpr int kTpSegB = 16;  // K_eqz / K_eqx: rows per load batch

// K_eqz (EXACT = false): the whole cascade from zero states over each
// (segment, channel), end states of every section to zs.  K_eqx (EXACT):
// the cascade from the segment start states K_carry chained (rounded from
// double-double), the reference operations per sample, rows to vT; the last
// segment leaves the chunk-end states in eq.state.  One wave per segment,
// one lane per channel.
template <bool EXACT>
__global__ __launch_bounds__(256) void k_fxtp_eq(FxTpEqArgs a) {
#pragma clang fp contract(off)
  const int w = wave_of_thread();
  const int l = threadIdx.x & 63;
  const int c = blockIdx.y * 64 + l;
  const bool active = c < a.channels;
  const int cc = active ? c : a.channels - 1;
  const unsigned uc = (unsigned)c;
  const int cp = a.cpad;
  const int sg = blockIdx.x * 4 + w;  // segment
  const int nsec = a.eq.nsec;
  if (sg >= a.nseg) return;
  const int64_t n0 = (int64_t)sg * a.seg, n1 = min(a.len, n0 + a.seg);
  const double* secs = a.eq.sec + (int64_t)cc * a.eq.sec_ch_stride;
  double q[kMaxSecPerPass][kSecStride], d0[kMaxSecPerPass], d1[kMaxSecPerPass];
#pragma unroll
  for (int k = 0; k < kMaxSecPerPass; ++k) {
#pragma unroll
    for (int j = 0; j < kSecStride; ++j) q[k][j] = k < nsec ? secs[k * kSecStride + j] : 0.0;
    d0[k] = d1[k] = 0.0;
    if (EXACT && k < nsec) {
      const double4 s = reinterpret_cast<const double4*>(a.sdd)[((int64_t)sg * nsec + k) * cp + c];
      d0[k] = s.x + s.y;
      d1[k] = s.z + s.w;
    }
  }
  const AD_TPG double* src = gptr(a.xT);
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
#pragma unroll
        for (int k = 0; k < kMaxSecPerPass; ++k)
          if (k < nsec) x = sec_step(q[k], d0[k], d1[k], x);
        if (EXACT) dst[(r0 + j) * cp + uc] = x;
      }
    }
  };
  load(xb[0], n0);
  for (int64_t r = n0; r < n1; r += 2 * kTpSegB) {
    if (r + kTpSegB < n1) load(xb[1], r + kTpSegB);
    run(xb[0], r);
    if (r + kTpSegB >= n1) break;
    if (r + 2 * kTpSegB < n1) load(xb[0], r + 2 * kTpSegB);
    run(xb[1], r + kTpSegB);
  }
#pragma unroll
  for (int k = 0; k < kMaxSecPerPass; ++k) {
    if (k >= nsec) break;
    if (EXACT) {
      if (sg == a.nseg - 1 && active) {  // the chunk-end state of section k
        double* st = a.eq.state + ((int64_t)c * nsec + k) * 2;
        st[0] = d0[k];
        st[1] = d1[k];
      }
    } else {
      reinterpret_cast<double2*>(a.zs)[((int64_t)sg * nsec + k) * cp + c] = make_double2(d0[k], d1[k]);
    }
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
__device__ __forceinline__ dd2x2 dd_block(const double* p) {
  dd2x2 b;
#pragma unroll
  for (int i = 0; i < 4; ++i) b.m[i] = dd{p[2 * i], p[2 * i + 1]};
  return b;
}
// (t0, t1) += B (s0, s1)
__device__ __forceinline__ void dd_madd(const dd2x2& B, dd s0, dd s1, dd& t0, dd& t1) {
  t0 = dd_add(t0, dd_add(dd_mul(B.m[0], s0), dd_mul(B.m[1], s1)));
  t1 = dd_add(t1, dd_add(dd_mul(B.m[2], s0), dd_mul(B.m[3], s1)));
}
struct dd2v {
  dd a, b;
};

// K_carry: one workgroup per channel, one thread per segment v, the
// sections in turn.  Over a segment the cascade state S = (s_0 .. s_{nsec-1})
// maps as S' = B S + Z (B block lower triangular, Z the zero-state end states
// from K_eqz), so section k's start states obey
//   s_k(v+1) = B(k,k) s_k(v) + u_k(v),  u_k(v) = Z_k(v) + sum_{j<k} B(k,j) s_j(v).
// Thread v keeps the cross terms of the later sections in registers (acc[k]),
// adding B(k,j) s_j(v) as soon as s_j(v) is known.  The chain itself is an
// inclusive scan over the segments in LDS (Hillis-Steele, maps B(k,k)^(2^i)),
// with the chunk-start state folded into segment 0.
__global__ __launch_bounds__(kFxTpMaxSeg) void k_fxtp_carry(FxTpEqArgs a) {
  const int v = threadIdx.x;  // segment
  const int c = blockIdx.x;   // channel
  const int cp = a.cpad, nsec = a.eq.nsec;
  const bool live = v < a.nseg;
  __shared__ dd2v scan[2][kFxTpMaxSeg];
  const double* ms = a.mats + (int64_t)(a.mat_sets > 1 ? c : 0) * fx_tp_mat_stride(nsec);
  const double2* zs = reinterpret_cast<const double2*>(a.zs);
  double4* sdd = reinterpret_cast<double4*>(a.sdd);
  dd acc0[kMaxSecPerPass], acc1[kMaxSecPerPass];
#pragma unroll
  for (int k = 0; k < kMaxSecPerPass; ++k) {
    acc0[k] = acc1[k] = dd{0, 0};
    if (k < nsec && live) {
      const double2 z = zs[((int64_t)v * nsec + k) * cp + c];
      acc0[k] = dd{z.x, 0};
      acc1[k] = dd{z.y, 0};
    }
  }
#pragma unroll
  for (int k = 0; k < kMaxSecPerPass; ++k) {
    if (k >= nsec) break;
    const double* st = a.eq.state + ((int64_t)c * nsec + k) * 2;
    const dd S0{st[0], 0}, S1{st[1], 0};
    dd e0 = acc0[k], e1 = acc1[k];
    if (v == 0) dd_madd(dd_block(ms + ((int64_t)k * nsec + k) * 8), S0, S1, e0, e1);
    // inclusive scan: E_v = sum_{v' <= v} B(k,k)^(v - v') e_v'  (segment v's end state)
    int cur = 0;
    scan[cur][v] = dd2v{e0, e1};
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kFxTpScan; ++i) {
      const int d = 1 << i;
      if (v >= d) {
        const dd2v p = scan[cur][v - d];
        dd_madd(dd_block(ms + ((int64_t)nsec * nsec + k * kFxTpScan + i) * 8), p.a, p.b, e0, e1);
      }
      scan[cur ^ 1][v] = dd2v{e0, e1};
      cur ^= 1;
      __syncthreads();
    }
    // segment v's start: segment v - 1's end, the chunk-start state for v = 0
    dd s0 = S0, s1 = S1;
    if (v > 0) {
      const dd2v p = scan[cur][v - 1];
      s0 = p.a;
      s1 = p.b;
    }
    if (live) sdd[((int64_t)v * nsec + k) * cp + c] = make_double4(s0.hi, s0.lo, s1.hi, s1.lo);
    // the later sections' cross terms
#pragma unroll
    for (int k2 = k + 1; k2 < kMaxSecPerPass; ++k2)
      if (k2 < nsec) dd_madd(dd_block(ms + ((int64_t)k2 * nsec + k) * 8), s0, s1, acc0[k2], acc1[k2]);
    __syncthreads();  // scan[] is rewritten by the next section
  }
}

// ---------------------------------------------------------------------------
// K_det: side-chain prefilters, detector and envelope (core.go:274-286,
// 331-400), serial over the chunk, kDetCh channels per workgroup (lanes of
// wave 0; the other lanes repeat them): a 64-channel group would need
// ~40 GB/s of row traffic into one CU at the detector's pace.  Three waves:
//   wave 1 (loader) keeps kDetNB batches of row loads in flight in registers
//          (every load covers 64 / kDetCh rows of kDetCh channels; 64
//          outstanding at 8 batches of 64 rows: the 64th issue waits for the
//          6-bit vmcnt) and puts each batch into a small LDS ring two steps
//          before the detector consumes it (kDetNB even: the steps run in pairs);
//   wave 0 (detector) reads batch k + 1 out of the ring before it runs the
//          envelope chain over batch k (the LDS latency hides under the
//          chain) and puts the batch's envelopes into a second ring;
//   wave 2 (storer) writes the envelopes of batch k - 1 to memory with two
//          full-width stores (no selects or address arithmetic on the
//          detector's issue slots, and no stores in the loader's vmcnt).
// One barrier per batch.  The lookahead (kDetNB batches) is what hides the
// memory latency: 10 batches of 16 measured 481 us per chunk, 14 370 us.
// ---------------------------------------------------------------------------
constexpr int kDetCh = 8;      // channels per workgroup
#ifndef AD_DET_B  // tools/ A/B builds may override (the one-wave form's batch; the three-wave
                  // kernel below is instantiated at 64 and 32 rows, launch_fxtp_det picks)
#define AD_DET_B 32
#endif
constexpr int kDetB = AD_DET_B;  // rows per batch of the one-wave form (k_fxtp_det1)
constexpr int kDetSlots = 4;   // input ring slots (put two steps ahead, read one step ahead)
__device__ __forceinline__ void lds_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// DB rows per batch, DNB batches in flight (DNB even: the steps run in pairs).
// Round 5, with the detector's stream running detectors only (config 5, same
// box, profiles/r05_fx_det_batch_ab.txt): 16 rows 11.39, 32 rows 12.16, 64
// rows 12.29-12.31 Gsamples/s; but 64-row batches take 256 VGPRs, and where
// the channel groups outnumber the CUs occupancy wins (16384 channels:
// 63.2 -> 56.4 Gsamples/s on the compressor-only chain), so launch_fxtp_det
// takes 64 rows for up to 256 groups and 32 above.
template <int DB, int DNB>
__global__ __launch_bounds__(192) void k_fxtp_det(FxStageArgs a) {
#pragma clang fp contract(off)
  constexpr int kDetB = DB, kDetNB = DNB;
  constexpr int kDetLd = kDetB * kDetCh / 64;  // loads per batch
  static_assert(kDetNB % 2 == 0 && kDetLd * kDetNB <= 64, "detector batches: an even count, <= 64 loads in flight");
  __shared__ double ring[kDetSlots][kDetB][kDetCh];
  __shared__ double evr[2][kDetB][kDetCh];  // envelopes of a bare full batch, for the storer
  const int w = wave_of_thread();
  const int l = threadIdx.x & 63;
  const int c0 = blockIdx.x * kDetCh;
  const int cp = a.cpad;
  const int64_t len = a.len;
  const int64_t nb = (len + kDetB - 1) / kDetB;
  const int64_t nbp = (nb + kDetNB - 1) / kDetNB * kDetNB;
  const CompParams& p = a.cp;
  const bool bare = !p.lp_on && !p.hp_on && !p.detector_rms;
  constexpr int RS = 64 / kDetCh;  // rows per load / store
  if (w == 0) {
    // lanes >= kDetCh repeat lanes 0..kDetCh-1 (same channel, same values)
    const int c = c0 + (l & (kDetCh - 1));
    const bool active = l < kDetCh && c < a.channels;
    const int cc = c < a.channels ? c : a.channels - 1;
    const unsigned uc = (unsigned)c;
    const int li = l & (kDetCh - 1);
    CompChState cs = a.cs[cc];
    AD_TPG double* rring = gptr(a.rms_ring) + (int64_t)cc * p.rms_n;
    AD_TPG double* eo = gptr(a.envT);
#ifdef AD_DET_PRIO  // tools/ A/B builds only
    __builtin_amdgcn_s_setprio(AD_DET_PRIO);
#endif
    __builtin_amdgcn_s_waitcnt(0);  // the state loads land before the step loop
    lds_bar();                      // the loader's prologue (batches 0 and 1)
    // one step: batch k from cur (read one step earlier), batch k + 1 into nxt
    auto step = [&](int64_t k, double (&cur)[kDetB], double (&nxt)[kDetB]) {
      const int slot = (int)(k % kDetSlots), sn = (int)((k + 1) % kDetSlots);
      const int64_t r0 = k * kDetB;
      const int n = (int)max((int64_t)0, min((int64_t)kDetB, len - r0));
      if (bare && n == kDetB) {
#pragma unroll
        for (int d = 0; d < kDetB; ++d) nxt[d] = ring[sn][d][li];
        double ev[kDetB];
#pragma unroll
        for (int d = 0; d < kDetB; ++d) {
          cs.env = env_step(p, cs.env, fabs(cur[d]));
          ev[d] = cs.env;
        }
        // one masked region per batch: lanes >= kDetCh would write the same
        // addresses again (8-way conflicts on every write)
        if (l < kDetCh) {
          double(*e)[kDetCh] = evr[k & 1];
#pragma unroll
          for (int d = 0; d < kDetB; ++d) e[d][li] = ev[d];
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
#pragma unroll
        for (int d = 0; d < kDetB; ++d) nxt[d] = ring[sn][d][li];
      }
      lds_bar();
    };
    double xa[kDetB], xb[kDetB];
#pragma unroll
    for (int d = 0; d < kDetB; ++d) xa[d] = ring[0][d][li];
    // nbp steps (nb rounded up to the loader's unroll, an even count): the
    // barrier counts match
    for (int64_t k = 0; k < nbp; k += 2) {
      step(k, xa, xb);
      step(k + 1, xb, xa);
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
  } else if (w == 1) {
    // loader: lane l covers row (l / kDetCh) + RS i of a batch, channel
    // l % kDetCh; its register ring holds kDetNB batches, entry = batch mod kDetNB
    const AD_TPG double* vin = gptr((const double*)a.vT);
    const unsigned col = (unsigned)(c0 + (l & (kDetCh - 1)));
    const int rl = l / kDetCh;
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
    put(buf[1], 1);
    load(buf[1], kDetNB + 1);
    lds_bar();
    // step k (the detector consumes batch k and reads k + 1): batch k + 2
    // goes into its slot, batch k + 2 + kDetNB is requested into the freed entry
    for (int64_t k = 0; k < nbp; k += kDetNB) {
#pragma unroll
      for (int u = 0; u < kDetNB; ++u) {
        put(buf[(u + 2) % kDetNB], k + u + 2);
        load(buf[(u + 2) % kDetNB], k + u + 2 + kDetNB);
        lds_bar();
      }
    }
  } else {
    // storer: after step k's barrier, the envelopes of batch k (a bare full
    // batch) go out, lane l rows (l / kDetCh) + RS i of channel l % kDetCh
    AD_TPG double* eo = gptr(a.envT);
    const unsigned col = (unsigned)(c0 + (l & (kDetCh - 1)));
    const int rl = l / kDetCh;
    auto flush = [&](int64_t k) {
      const int64_t r0 = k * kDetB;
      if (!bare || r0 + kDetB > len) return;
      double v[kDetLd];
#pragma unroll
      for (int i = 0; i < kDetLd; ++i) v[i] = evr[k & 1][rl + RS * i][l & (kDetCh - 1)];
#pragma unroll
      for (int i = 0; i < kDetLd; ++i) eo[(r0 + rl + RS * i) * cp + col] = v[i];
    };
    lds_bar();
    for (int64_t k = 0; k < nbp; ++k) {
      if (k > 0) flush(k - 1);
      lds_bar();
    }
    flush(nbp - 1);
  }
}

// ---------------------------------------------------------------------------
// K_det, one wave (the bare detector: peak level, no side-chain filters, the
// config-5 compressor).  The three-wave form above spends
// 43 clocks per sample against the envelope chain's 24.5: one barrier per
// batch and the LDS hand-offs between its waves.  Here one wave does it all
// for kDetCh channels, with no barrier:
//   - batch k's rows (32 rows x 8 channels, 2 KiB) arrive in an LDS ring by
//     LDS-DMA (global_load_lds_dwordx4: lane l fetches 16 B of row l / 4, so
//     two instructions fill a batch), issued kDet1D batches ahead;
//   - the wave reads batch k + 1 out of the ring (lane = channel) before it
//     runs the chain over batch k, puts batch k's envelopes into a small LDS
//     staging area and stores batch k - 1's from there as four full-width
//     stores (lane l: row l / 8 + 8 i, channel l % 8);
//   - the vector-memory counter retires in issue order and the wave issues 4
//     stores then 2 DMAs per step (4 dummy DMAs into a scratch line stand in
//     for the stores before the first step), so "batch k + 1 has landed" is
//     the constant wait vmcnt(6 (kDet1D - 1)) at every step (the DMAs are inline asm,
//     as K2's X ring: hipcc would drain them with vmcnt(0) before the first LDS
//     read).  A slot is refilled kDet1D + 1 steps after it was read.
// Same operations per sample as the three-wave kernel (env_step), so the same
// bits.  Full batches only; a chunk's last partial batch runs lane-serially
// after a vmcnt(0).
// ---------------------------------------------------------------------------
// Measured (round 5, one box, tools/fx_iso_prof.sh on AD_FX_TP_SERIAL builds,
// profiles/r05_det_onewave.txt): 1646 us per 64K-sample chunk at 256 channels
// against 1144 us for the three-wave kernel (60 against 42 clocks per
// sample), config 5 8.1 against 10.9 Gsamples/s: the chain wave also issuing
// the ring DMAs, their address arithmetic, the masked envelope writes and the
// stores costs more than the barrier it saves.  Kept for A/B builds only.
#ifndef AD_DET_ONEWAVE  // tools/ A/B builds: 1 = this kernel for the bare detector
#define AD_DET_ONEWAVE 0
#endif
#if AD_DET_B == 32  // the one-wave form needs 32-row batches of 8 channels (two 1-KiB DMAs)
typedef __attribute__((address_space(3))) void lds_void_t;
constexpr int kDet1D = 8;                 // batches in flight (DMA issued this many batches ahead)
constexpr int kDet1Slots = kDet1D + 2;    // ring slots
constexpr int kDet1Wait = 6 * (kDet1D - 1);  // ops issued after batch k + 1's DMAs, at step k
static_assert(kDetB == 32 && kDetCh == 8, "one-wave detector: 32-row batches of 8 channels (two 1-KiB DMAs)");
static_assert(kDet1Wait <= 63, "vmcnt holds 6 bits");

__device__ __forceinline__ void det1_dma(const double* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds)
               : "memory");
}

__global__ __launch_bounds__(64) void k_fxtp_det1(FxStageArgs a) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) double ring[kDet1Slots][kDetB][kDetCh];
  __shared__ __attribute__((aligned(16))) double evr[2][kDetB][kDetCh];
  __shared__ __attribute__((aligned(16))) double scratch[128];  // the dummy DMAs' target (1 KiB)
  const int l = threadIdx.x;
  const int li = l & (kDetCh - 1);
  const int c0 = blockIdx.x * kDetCh;
  const int cp = a.cpad;
  const int64_t len = a.len;
  const int64_t nbf = len / kDetB;  // full batches
  const CompParams& p = a.cp;
  const int c = c0 + li;
  const int cc = c < a.channels ? c : a.channels - 1;
  CompChState cs = a.cs[cc];
  const double* vin = a.vT;
  double* eo = a.envT;
  // this lane's 16 B of a DMA: row (l >> 2), channels c0 + 2 (l & 3) .. + 1
  const double* gl = vin + (int64_t)(l >> 2) * cp + c0 + 2 * (l & 3);
  auto dma = [&](int64_t b) {  // batch b into its slot (rows past the chunk re-read its last row)
    const int slot = (int)(b % kDet1Slots);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t row = min(b * kDetB + 16 * h + (l >> 2), len - 1) - (l >> 2);
      det1_dma(gl + row * cp, (unsigned)(uintptr_t)(lds_void_t*)&ring[slot][16 * h][0]);
    }
  };
  auto dummy4 = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) det1_dma(vin + c0, (unsigned)(uintptr_t)(lds_void_t*)&scratch[0]);
  };
  // envelopes of batch b from the staging area to memory (four full-width stores)
  auto flush = [&](int64_t b) {
    double v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = evr[b & 1][(l >> 3) + 8 * i][l & 7];
#pragma unroll
    for (int i = 0; i < 4; ++i) eo[(b * kDetB + (l >> 3) + 8 * i) * cp + c0 + (l & 7)] = v[i];
  };
  __builtin_amdgcn_s_waitcnt(0);  // the state load has landed: from here on only counted ops
  if (nbf > 0) {
    dma(0);
    for (int j = 1; j <= kDet1D; ++j) {
      dummy4();
      dma(j);
    }
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDet1Wait + 6) : "memory");  // batch 0
    double xa[kDetB], xb[kDetB];
#pragma unroll
    for (int d = 0; d < kDetB; ++d) xa[d] = ring[0][d][li];
    auto step = [&](int64_t k, double (&cur)[kDetB], double (&nxt)[kDetB]) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDet1Wait) : "memory");  // batch k + 1 has landed
      const int sn = (int)((k + 1) % kDet1Slots);
      double ev[kDetB];
      // the chain over batch k with batch k + 1's ring reads interleaved (they
      // issue in the chain's dependency stalls; one wave issues in order)
#pragma unroll
      for (int d = 0; d < kDetB; ++d) {
        cs.env = env_step(p, cs.env, fabs(cur[d]));
        ev[d] = cs.env;
        nxt[d] = ring[sn][d][li];
        __builtin_amdgcn_sched_barrier(0);
      }
      if (l < kDetCh) {
#pragma unroll
        for (int d = 0; d < kDetB; ++d) evr[k & 1][d][li] = ev[d];
      }
      // per step: 4 stores, then 2 DMAs (the order kDet1Wait counts)
      if (k > 0)
        flush(k - 1);
      else
        dummy4();
      dma(k + 1 + kDet1D);
    };
    int64_t k = 0;
    for (; k + 1 < nbf; k += 2) {
      step(k, xa, xb);
      step(k + 1, xb, xa);
    }
    if (k < nbf) step(k, xa, xb);
    flush(nbf - 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the chunk's last partial batch, lane-serially from memory
  for (int64_t r = nbf * kDetB; r < len; ++r) {
    const double x = vin[r * cp + cc];
    cs.env = env_step(p, cs.env, fabs(x));
    if (l < kDetCh && c < a.channels) eo[r * cp + c] = cs.env;
  }
  if (l < kDetCh && c < a.channels) {
    CompChState* o = a.cs + c;
    o->env = cs.env;
  }
}

#endif  // AD_DET_B == 32

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
#ifndef AD_VB_PIPE
#define AD_VB_PIPE 1  // k_fxtp_verb_pipe (where the caller asks): comb and allpass phases of consecutive sub-blocks overlapped
#endif
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

// K_verb with its two phases overlapped across sub-blocks (AD_VB_PIPE): in
// step b the comb waves run sub-block b while the allpass waves run sub-block
// b - 1 (the comb and allpass delay lines are separate LDS regions).  The comb
// outputs alternate between two halves of coC ([2][comb][kVbSB] per channel);
// the allpass waves read the dry input of their sub-block from the input
// buffer (each lane reads its sample before it writes the output there, so the
// in-place call stays exact), and order their 225-sample windows among
// themselves with an LDS counter instead of the workgroup barrier, which the
// comb waves only meet once per step.  Same operations per sample in the same
// order as k_fxtp_verb: the same bits.
__global__ __launch_bounds__(kVbThreads) void k_fxtp_verb_pipe(FxStageArgs a, const double* __restrict__ xC,
                                                               int64_t xstride, double* __restrict__ vbufC,
                                                               double* __restrict__ coC, int wu) {
#pragma clang fp contract(off)
  __shared__ double lines[kVerbLen];
  __shared__ double xs[kVbSB];
  __shared__ unsigned apbar;  // allpass windows done x 4 (one increment per allpass wave and window)
  const int w = wave_of_thread();
  const int l = threadIdx.x & 63;
  const int tid = threadIdx.x;
  const int c = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  const VerbParams& p = a.vp;
  const int64_t len = a.len;
  double* vl = vbufC + (int64_t)c * kVerbLen;
  for (int e = tid; e < kVerbLen; e += kVbThreads) lines[e] = vl[e];
  if (tid == 0) apbar = 0u;
  const double* xc = xC + (int64_t)c * xstride;
  double* cocb = coC + (int64_t)c * 2 * kVerbCombs * kVbSB;  // [2][comb][kVbSB]
  double xr[kVbXr];
#pragma unroll
  for (int q = 0; q < kVbXr; ++q) {
    const int e = q * kVbThreads + tid;
    xr[q] = e < kVbSB && e < len ? xc[e] : 0.0;
  }
  const int ci = w < kVerbCombs ? w : 0;
  int idx = a.vs[c].comb_idx[ci];
  double carry = a.vs[c].filter_store[ci];
  int apx[kVerbAllpass];
#pragma unroll
  for (int i = 0; i < kVerbAllpass; ++i) apx[i] = a.vs[c].ap_idx[i];
  unsigned nwin = 0;  // allpass windows this wave has finished
  // set if a window barrier's spin ever expires (cannot happen with all waves
  // resident in one workgroup): every later output of the wave is NaN, so a
  // broken barrier shows as an error instead of silently stale allpass lines
  bool spin_lost = false;
  const int64_t nsb = (len + kVbSB - 1) / kVbSB;
  for (int64_t b = 0; b <= nsb; ++b) {
    const int64_t t0 = b * kVbSB;
    const int sb = b < nsb ? (int)min((int64_t)kVbSB, len - t0) : 0;
    __syncthreads();  // step b - 1's comb reads of xs and comb outputs are done (the first time: the lines)
    if (sb > 0) {
#pragma unroll
      for (int q = 0; q < kVbXr; ++q) {
        const int e = q * kVbThreads + tid;
        if (e < sb) xs[e] = xr[q];
      }
#pragma unroll
      for (int q = 0; q < kVbXr; ++q) {  // the next sub-block's input, in flight during this step
        const int e = q * kVbThreads + tid;
        if (e < kVbSB && t0 + kVbSB + e < len) xr[q] = xc[t0 + kVbSB + e];
      }
    }
    __syncthreads();  // xs holds sub-block b
    if (w < kVerbCombs) {
      if (sb > 0) {
        const int D = kCombLen[w];
        double* L = lines + comb_off(w);
        double* cw = cocb + ((int64_t)(b & 1) * kVerbCombs + w) * kVbSB;
        for (int r = 0; r < sb;) {
          const int pos0 = idx;
          const int m = min(sb - r, D - pos0);
          const int nw = wu > 0 ? max(1, min(kVbSeg, m / wu)) : min(kVbSeg, m);
          const int Lw = ((m + nw - 1) / nw) | 1;
          const int s0 = l * Lw, s1 = min(m, s0 + Lw);
          const bool mine = l < nw && s0 < s1;
          double fs = l == 0 ? carry : 0.0;
          if (mine && l > 0) {
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
    } else if (b > 0) {  // the allpass waves: sub-block b - 1
      const int64_t tp = (b - 1) * kVbSB;
      const int sbp = (int)min((int64_t)kVbSB, len - tp);
      const double* coc = cocb + (int64_t)((b - 1) & 1) * kVerbCombs * kVbSB;
      const int j = (w - kVerbCombs) * 64 + l;
      const bool apw = j < 225;
      double cv[kVerbCombs], xd = 0.0;
      auto loadc = [&](int r) {
        const int e = min(r + j, sbp - 1);
#pragma unroll
        for (int i = 0; i < kVerbCombs; ++i) cv[i] = coc[(int64_t)i * kVbSB + e];
        xd = xc[tp + e];
      };
      if (apw) loadc(0);
      for (int r = 0; r < sbp; r += 225) {
        const int m = min(225, sbp - r);
        if (apw && j < m) {
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
          a.buf[(int64_t)c * a.stride + tp + r + j] = spin_lost ? __builtin_nan("") : acc * p.wet + xd * p.dry;
        }
        if (apw && r + 225 < sbp) loadc(r + 225);
#pragma unroll
        for (int i = 0; i < kVerbAllpass; ++i) {
          apx[i] += m;
          if (apx[i] >= kApLen[i]) apx[i] -= kApLen[i];
        }
        // the four allpass waves' window barrier (LDS counter; bounded spin,
        // an expiry poisons the wave's outputs, see spin_lost)
        ++nwin;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (l == 0) __hip_atomic_fetch_add(&apbar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        bool met = false;
        for (int it = 0; it < (1 << 22); ++it) {
          if (__hip_atomic_load(&apbar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= 4u * nwin) {
            met = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        spin_lost |= !met;
      }
    }
  }
  __syncthreads();
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

void launch_fxtp_eq(const FxTpEqArgs& a, bool exact, hipStream_t s) {
  if (a.len <= 0) return;
  const dim3 grid((unsigned)((a.nseg + 3) / 4), (unsigned)((a.channels + 63) / 64));
  if (exact)
    hipLaunchKernelGGL(k_fxtp_eq<true>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_fxtp_eq<false>, grid, dim3(256), 0, s, a);
}

void launch_fxtp_carry(const FxTpEqArgs& a, hipStream_t s) {
  if (a.len <= 0) return;
  // the host keeps nseg <= kFxTpMaxSeg (one thread per segment)
  hipLaunchKernelGGL(k_fxtp_carry, dim3((unsigned)a.channels), dim3(kFxTpMaxSeg), 0, s, a);
}

void launch_fxtp_det(const FxStageArgs& a, hipStream_t s) {
  if (a.len <= 0) return;
#if AD_DET_B == 32
  const CompParams& p = a.cp;
  const bool bare = !p.lp_on && !p.hp_on && !p.detector_rms;
  if (AD_DET_ONEWAVE && bare)
    hipLaunchKernelGGL(k_fxtp_det1, dim3((unsigned)((a.channels + kDetCh - 1) / kDetCh)), dim3(64), 0, s, a);
  else
#endif
  {
    const unsigned groups = (unsigned)((a.channels + kDetCh - 1) / kDetCh);
    if (groups <= 256)
      hipLaunchKernelGGL((k_fxtp_det<64, 8>), dim3(groups), dim3(192), 0, s, a);
    else
      hipLaunchKernelGGL((k_fxtp_det<32, 14>), dim3(groups), dim3(192), 0, s, a);
  }
}

void launch_fxtp_verb(const FxStageArgs& a, const double* xC, int64_t xstride, double* vbufC, double* coC, int wu,
                      hipStream_t s, bool pipe) {
  if (a.len <= 0) return;
  if (AD_VB_PIPE && pipe)
    hipLaunchKernelGGL(k_fxtp_verb_pipe, dim3((unsigned)a.channels), dim3(kVbThreads), 0, s, a, xC, xstride, vbufC, coC,
                       wu);
  else
    hipLaunchKernelGGL(k_fxtp_verb, dim3((unsigned)a.channels), dim3(kVbThreads), 0, s, a, xC, xstride, vbufC, coC, wu);
}

void launch_vbuf_layout(double* vbuf, double* vbufC, int cpad, int channels, bool to_cm, hipStream_t s) {
  const int64_t n = (int64_t)kVerbLen * channels;
  hipLaunchKernelGGL(k_vbuf_layout, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, vbuf, vbufC, cpad, channels,
                     to_cm ? 1 : 0);
}

}  // namespace adsp
