// Staged effect chain: biquad EQ -> feed-forward Compressor -> Freeverb,
// split by recurrence into stage kernels that run concurrently on their own
// streams over time chunks (host side: fx_run_staged in capi_dsp.cpp).
//
// Reference behaviour (all bit-for-bit the same operations as the fused
// kernels in dsp_kernels.hip, which restate these files):
//   biquad.Chain.ProcessBlock        dsp/filter/biquad/chain.go:59-70, section.go:47-53
//   Compressor.ProcessSample         dsp/effects/dynamics/compressor.go:348-359, core.go:274-400
//   updateMetrics                    compressor.go:411-423
//   Reverb.ProcessSample (Freeverb)  dsp/effects/reverb/reverb.go:57-117, 169-182
//
// Why stages: at config 5 (256 channels) one lane per channel gives four
// 64-channel waves, and the fused kernels keep one CU per 64 channels busy
// issuing ~300 dependent FP64 instructions per sample.  Only some of that is
// serial in time:
//   K_eq    EQ sections (one wave per section, LDS ring between them) and
//           the compressor detector / envelope            serial, 1 CU / 64 ch
//   K_gain  gain(env) = 2^(-cf*knee(log2 env - T)), out = v*g*makeup,
//           metrics                                       parallel over samples
//   K_comb  one wave per comb filter (8 per 64 channels)  serial, 8 CUs / 64 ch
//   K_ap    ordered comb sum, 4 allpasses, wet/dry mix    parallel within blocks
//           of 128 samples (every allpass delay is >= 225)
// so each stage gets its own CUs, and the transcendental-heavy gain stage
// runs on the whole chip.  Chunk buffers between stages are time-major
// [t][cpad] (one 512-byte row per sample per 64 channels); the user buffer
// is channel-major [c][stride].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "dsp_device.hpp"
#include "dsp_kernels.hpp"

namespace adsp {

namespace {

constexpr int kEqP = 8;    // samples per pipeline step of K_eq
constexpr int kEqPF = 4;   // K_eq input prefetch depth (steps)
constexpr int kApB = 128;  // K_ap block (<= the shortest allpass delay, 225)
constexpr int kApW = 8;    // waves of K_ap
constexpr int kCombB = 16; // K_comb samples per load/store batch

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Global-address-space view of a buffer.  Plain HIP pointers are generic:
// where the compiler cannot prove the space it emits flat loads and stores,
// which count in BOTH the vector-memory and the LDS/scalar counters, so every
// LDS wait (lgkmcnt) also waits for the flat accesses in flight, and the
// waits it inserts at merges degrade to vmcnt(0).  That drained the
// prefetched delay-line batches of K_comb and made K_eq's last section and
// detector wait each step for the previous step's row stores.  Every stage
// buffer below is accessed through these pointers (global_load / store only).
#define AD_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ AD_GLOBAL T* glob(T* p) {
  return (AD_GLOBAL T*)p;
}

// A pointer the compiler can prove wave-uniform (SGPR pair), so that p[lane]
// becomes a scalar-base + 32-bit VGPR-offset access with no 64-bit VALU add.
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a release /
// acquire fence at workgroup scope: it waits for every outstanding global
// load and store of the wave (vmcnt(0)), i.e. one HBM round trip per
// barrier, and it drains the input prefetch.  Here only the LDS writes must
// land before the other waves read them.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------------------
// K_eq: waves 0 .. ns-1 run EQ section w on step k - w (a step is kEqP
// samples); wave ns (COMP) runs the side-chain prefilter, detector and
// envelope.  Consecutive waves hand over through a two-slot LDS ring: at
// step k wave w writes slot (k - w) & 1 and wave w + 1 reads slot
// (k - w - 1) & 1, one barrier per step.  Input xT, output (the last
// section's, or the input when ns = 0) vT or inT, envelope envT: all
// time-major rows, so every access is one coalesced 512-byte row.  Full
// steps take a branch-free path; only a chunk's last step masks samples.
// ---------------------------------------------------------------------------
template <bool FULL>
__device__ __forceinline__ void eq_section_step(const double (&q)[kSecStride], double& d0, double& d1,
                                                const double (&x)[kEqP], double (&y)[kEqP], int nreal) {
#pragma clang fp contract(off)
#pragma unroll
  for (int d = 0; d < kEqP; ++d) {
    const double v = x[d] * q[0];
    const double yy = q[1] * v + d0;
    const double n0 = q[2] * v - q[4] * yy + d1;
    const double n1 = q[3] * v - q[5] * yy;
    if (FULL || d < nreal) {  // padding leaves the state untouched
      d0 = n0;
      d1 = n1;
    }
    y[d] = yy;
  }
}

template <bool COMP>
__global__ __launch_bounds__(64 * (kMaxSecPerPass + 2)) void k_fx_eq(FxStageArgs a) {
#pragma clang fp contract(off)
  __shared__ double ring[kMaxSecPerPass][2][kEqP][64];
  __shared__ double xring[2][kEqP][64];  // input rows, written by the loader wave one step ahead
  const FxEqPart& P = a.part[blockIdx.y];
  const int wid = wave_id();
  const int l = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + l;
  const bool active = c < a.channels;
  const int cc = active ? c : a.channels - 1;
  const int ns = P.ns;
  const bool det = COMP && P.det;
  const int W = ns + (det ? 1 : 0);  // compute waves; wave W is the loader
  // Pipeline role of this wave: sections 0 .. ns-1, detector ns, loader W
  // (waves past W idle through the barriers: the launch's other part is
  // wider).  Waves land on SIMD wid % 4; with three or more sections the
  // detector (the longest recurrence) takes wave 3 so that its SIMD is its own.
  const int w = (wid >= W || !det || ns < 3) ? wid : (wid == 3 ? ns : (wid < 3 ? wid : wid - 1));
  const int64_t len = P.len;
  const int64_t nst = (len + kEqP - 1) / kEqP;
  const int64_t steps = nst + W - 1;
  const int cp = a.cpad;
  const unsigned uc = (unsigned)c;
  const AD_GLOBAL double* xin = glob(P.in);  // uniform row pointers; a lane indexes [uc]
  AD_GLOBAL double* tmo = glob(P.out);

  // Wave 0's input comes from xring, filled by the loader wave (wave W):
  // it loads each step's rows kEqPF steps before it writes them to LDS, in
  // register buffers named at compile time (its loop is unrolled by kEqPF),
  // so its waits are on loads issued kEqPF steps earlier, and its own short
  // body keeps it ahead of the barrier lockstep.
  auto take_input = [&](int64_t my, double (&x)[kEqP]) {
#pragma unroll
    for (int d = 0; d < kEqP; ++d) x[d] = xring[(my & 1)][d][l];
  };
  // time-major rows of step `my`: full steps walk a uniform row pointer
  auto put_rows = [&](AD_GLOBAL double* base, int64_t my, const double (&y)[kEqP], int nreal) {
    AD_GLOBAL double* o = uniform_ptr(base + my * kEqP * cp);
    if (nreal == kEqP) {
#pragma unroll
      for (int d = 0; d < kEqP; ++d) {
        o[uc] = y[d];
        o += cp;
      }
    } else {
#pragma unroll
      for (int d = 0; d < kEqP; ++d)
        if (d < nreal) o[(int64_t)d * cp + uc] = y[d];
    }
  };
  auto emit = [&](int64_t my, const double (&y)[kEqP], int nreal) { put_rows(tmo, my, y, nreal); };

  if (w > W) {
    // ---- idle: the barrier count of the part's waves (prologue + one per step)
    for (int64_t k = 0; k <= steps; ++k) lds_barrier();
  } else if (w == W) {
    // ---- loader
    double buf[kEqPF][kEqP];
    // Branch-free: every call issues exactly kEqP loads (rows past the chunk
    // re-read its last row), so the compiler's vmcnt bookkeeping stays exact
    // across the unrolled buffers and each put waits only for its own step.
    auto fetch = [&](double (&dst)[kEqP], int64_t step) {
#pragma unroll
      for (int d = 0; d < kEqP; ++d) {
        const int64_t row = __builtin_amdgcn_readfirstlane(min(step * kEqP + d, len - 1));
        dst[d] = uniform_ptr(xin + row * cp)[uc];
      }
    };
    auto put = [&](const double (&src)[kEqP], int64_t step) {
      if (step < nst) {
#pragma unroll
        for (int d = 0; d < kEqP; ++d) xring[(step & 1)][d][l] = src[d];
      }
    };
#pragma unroll
    for (int b = 0; b < kEqPF; ++b) fetch(buf[b], b);
    put(buf[0], 0);
    fetch(buf[0], kEqPF);
    lds_barrier();
    // at step k: write step k+1 (from buf[(k+1) % PF]), then load step k+1+PF into it
    for (int64_t k = 0; k < steps; k += kEqPF) {
#pragma unroll
      for (int u = 0; u < kEqPF; ++u) {
        if (k + u < steps) {
          const int b = (u + 1) % kEqPF;
          put(buf[b], k + u + 1);
          fetch(buf[b], k + u + 1 + kEqPF);
          lds_barrier();
        }
      }
    }
  } else if (w < ns) {
    // ---- EQ section P.s0 + w (section.go:47-53 with the chain gain as pre-gain)
    const int gs = P.s0 + w;  // the section's index in the chain
    const AD_GLOBAL double* sec = glob(a.eq.sec) + (int64_t)cc * a.eq.sec_ch_stride + gs * kSecStride;
    double q[kSecStride];
#pragma unroll
    for (int k = 0; k < kSecStride; ++k) q[k] = sec[k];
    AD_GLOBAL double* st = glob(a.eq.state) + ((int64_t)cc * a.eq.nsec + gs) * 2;
    double d0 = st[0], d1 = st[1];
    // the coefficient and state loads land here, before the step loop: left
    // pending, the loop-head merge with the stores in flight made the
    // compiler wait vmcnt(0) at every step (the last section's row stores)
    __builtin_amdgcn_s_waitcnt(0);
    const bool to_ring = w < ns - 1 || det;
    const bool last = w == ns - 1;
    unsigned long long tc = 0, tb = 0;
    lds_barrier();  // the loader's prologue (step 0 in xring)
    for (int64_t k = 0; k < steps; ++k) {
      const unsigned long long t0c = a.prof ? clock64() : 0;
      const int64_t my = k - w;
      if (my >= 0 && my < nst) {
        double x[kEqP], y[kEqP];
        if (w == 0) {
          take_input(my, x);
        } else {
#pragma unroll
          for (int d = 0; d < kEqP; ++d) x[d] = ring[w - 1][(my & 1)][d][l];
        }
        const int nreal = (int)min((int64_t)kEqP, len - my * kEqP);
        if (nreal == kEqP)
          eq_section_step<true>(q, d0, d1, x, y, nreal);
        else
          eq_section_step<false>(q, d0, d1, x, y, nreal);
        if (to_ring) {
#pragma unroll
          for (int d = 0; d < kEqP; ++d) ring[w][(my & 1)][d][l] = y[d];
        }
        if (last) emit(my, y, nreal);
      }
      const unsigned long long t1c = a.prof ? clock64() : 0;
      lds_barrier();
      if (a.prof) {
        tc += t1c - t0c;
        tb += clock64() - t1c;
      }
    }
    if (a.prof && l == 0 && blockIdx.x == 0) {
      a.prof[2 * gs] = tc;
      a.prof[2 * gs + 1] = tb;
    }
    if (active) {
      st[0] = d0;
      st[1] = d1;
    }
  } else if (det) {
    // ---- detector + envelope (core.go:274-286, 331-400)
    const CompParams& p = a.cp;
    CompChState cs = a.cs[cc];  // generic load: drained by the wait below
    AD_GLOBAL double* rring = glob(a.rms_ring) + (int64_t)cc * p.rms_n;
    AD_GLOBAL double* eo = glob(P.env);
    __builtin_amdgcn_s_waitcnt(0);  // state loads land before the step loop (see the section waves)
    lds_barrier();  // the loader's prologue (step 0 in xring)
    unsigned long long tc = 0, tb = 0;
    for (int64_t k = 0; k < steps; ++k) {
      const unsigned long long t0c = a.prof ? clock64() : 0;
      const int64_t my = k - w;
      if (my >= 0 && my < nst) {
        double x[kEqP], e[kEqP];
        const int nreal = (int)min((int64_t)kEqP, len - my * kEqP);
        if (ns == 0) {
          take_input(my, x);
          emit(my, x, nreal);  // v = the input
        } else {
#pragma unroll
          for (int d = 0; d < kEqP; ++d) x[d] = ring[ns - 1][(my & 1)][d][l];
        }
        if (!p.lp_on && !p.hp_on && !p.detector_rms && nreal == kEqP) {
          // peak detector, no side-chain filters, a full step: the bare recurrence
#pragma unroll
          for (int d = 0; d < kEqP; ++d) {
            const double src = fabs(x[d]);
            const double ne = env_step(p, cs.env, src);
            cs.env = ne;
            e[d] = ne;
          }
        } else {
#pragma unroll
        for (int d = 0; d < kEqP; ++d) {
          const bool real = d < nreal;
          double sc = x[d];  // applyPrefilter core.go:390-400
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
          if (p.detector_rms && real) {  // updateRMS core.go:361-388
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
          const double ne = env_step(p, cs.env, src);
          if (real) cs.env = ne;
          e[d] = ne;
        }
        }
        put_rows(eo, my, e, nreal);
      }
      const unsigned long long t1c = a.prof ? clock64() : 0;
      lds_barrier();
      if (a.prof) {
        tc += t1c - t0c;
        tb += clock64() - t1c;
      }
    }
    if (a.prof && l == 0 && blockIdx.x == 0) {
      a.prof[2 * (P.s0 + ns)] = tc;
      a.prof[2 * (P.s0 + ns) + 1] = tb;
    }
    if (active) {  // only the fields this stage owns
      AD_GLOBAL CompChState* o = glob(a.cs) + c;
      o->env = cs.env;
      o->lp = cs.lp;
      o->hp = cs.hp;
      o->rms_sum = cs.rms_sum;
      o->rms_index = cs.rms_index;
      o->rms_filled = cs.rms_filled;
    }
  }
}

// ---------------------------------------------------------------------------
// K_sec: one EQ section of 64 channels per workgroup (the EQ-only chains'
// per-section pipeline, fx_run_staged): part blockIdx.y runs section
// part.s0 over its own chunk, so the sections of a cascade run on different
// CUs in one launch.  Two waves:
//   wave 0 (section) only reads its input rows out of an LDS ring, runs the
//          DF-II-T recurrence with the reference operations (eq_section_step)
//          and writes its outputs into a second ring; on its SIMD alone, its
//          time is the section's dependency chain;
//   wave 1 (I/O) loads input rows kSecPF steps ahead (16-B loads: lanes
//          0-31 row r, lanes 32-63 row r + 1, two channels each), puts them
//          into the ring one step ahead, and stores the section's outputs of
//          the previous step.
// One LDS-only barrier per step of kSecP samples.  Rows past the chunk are
// re-read (loads) and never stored.
// ---------------------------------------------------------------------------
#ifndef AD_SEC_P
#define AD_SEC_P 32
#endif
constexpr int kSecP = AD_SEC_P;   // samples per step
constexpr int kSecPF = 2;   // I/O wave: steps of input loads in flight
__global__ __launch_bounds__(128) void k_fx_eq_sec(FxStageArgs a) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) double xr[2][kSecP][64];
  __shared__ __attribute__((aligned(16))) double yr[2][kSecP][64];
  const FxEqPart& P = a.part[blockIdx.y];
  const int wid = wave_id();
  const int l = threadIdx.x & 63;
  const int g0 = blockIdx.x * 64;  // first channel of the group
  const int64_t len = P.len;
  const int64_t nst = (len + kSecP - 1) / kSecP;
  const int cp = a.cpad;
  if (wid == 0) {
    const int c = g0 + l;
    const int cc = c < a.channels ? c : a.channels - 1;
    const int gs = P.s0;
    const AD_GLOBAL double* sec = glob(a.eq.sec) + (int64_t)cc * a.eq.sec_ch_stride + gs * kSecStride;
    double q[kSecStride];
#pragma unroll
    for (int k = 0; k < kSecStride; ++k) q[k] = sec[k];
    AD_GLOBAL double* st = glob(a.eq.state) + ((int64_t)cc * a.eq.nsec + gs) * 2;
    double d0 = st[0], d1 = st[1];
    __builtin_amdgcn_s_waitcnt(0);
    lds_barrier();  // step 0's rows are in xr[0]
    for (int64_t k = 0; k <= nst; ++k) {
      if (k < nst) {
        const int nreal = (int)min((int64_t)kSecP, len - k * kSecP);
        double x[kSecP], y[kSecP];
#pragma unroll
        for (int d = 0; d < kSecP; ++d) x[d] = xr[k & 1][d][l];
        if (nreal == kSecP) {
#pragma unroll
          for (int h = 0; h < kSecP / kEqP; ++h)
            eq_section_step<true>(q, d0, d1, *reinterpret_cast<const double(*)[kEqP]>(x + h * kEqP),
                                  *reinterpret_cast<double(*)[kEqP]>(y + h * kEqP), kEqP);
        } else {
#pragma unroll
          for (int h = 0; h < kSecP / kEqP; ++h)
            eq_section_step<false>(q, d0, d1, *reinterpret_cast<const double(*)[kEqP]>(x + h * kEqP),
                                   *reinterpret_cast<double(*)[kEqP]>(y + h * kEqP), nreal - h * kEqP);
        }
#pragma unroll
        for (int d = 0; d < kSecP; ++d) yr[k & 1][d][l] = y[d];
      }
      lds_barrier();
    }
    if (c < a.channels) {
      st[0] = d0;
      st[1] = d1;
    }
  } else {
    // I/O wave: lane l covers channels g0 + 2 (l & 31) .. + 1 of row 2 i + (l >> 5)
    const AD_GLOBAL double* xin = glob(P.in);
    AD_GLOBAL double* yo = glob(P.out);
    const int cl = 2 * (l & 31), rh = l >> 5;
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 buf[kSecPF][kSecP / 2];
    auto fetch = [&](d2 (&dst)[kSecP / 2], int64_t step) {  // branch-free: rows past the chunk re-read its last
#pragma unroll
      for (int i = 0; i < kSecP / 2; ++i) {
        const int64_t row = min(step * kSecP + 2 * i + rh, len - 1);
        dst[i] = *reinterpret_cast<const AD_GLOBAL d2*>(xin + row * cp + g0 + cl);
      }
    };
    auto put = [&](const d2 (&src)[kSecP / 2], int64_t step) {
#pragma unroll
      for (int i = 0; i < kSecP / 2; ++i) *reinterpret_cast<d2*>(&xr[step & 1][2 * i + rh][cl]) = src[i];
    };
    auto flush = [&](int64_t step) {  // the section's outputs of `step`
      const int64_t r0 = step * kSecP;
      const int nreal = (int)min((int64_t)kSecP, len - r0);
      d2 v[kSecP / 2];
#pragma unroll
      for (int i = 0; i < kSecP / 2; ++i) v[i] = *reinterpret_cast<const d2*>(&yr[step & 1][2 * i + rh][cl]);
      if (nreal == kSecP) {
#pragma unroll
        for (int i = 0; i < kSecP / 2; ++i) *reinterpret_cast<AD_GLOBAL d2*>(yo + (r0 + 2 * i + rh) * cp + g0 + cl) = v[i];
      } else {
#pragma unroll
        for (int i = 0; i < kSecP / 2; ++i)
          if (2 * i + rh < nreal) *reinterpret_cast<AD_GLOBAL d2*>(yo + (r0 + 2 * i + rh) * cp + g0 + cl) = v[i];
      }
    };
#pragma unroll
    for (int b = 0; b < kSecPF; ++b) fetch(buf[b], b);
    put(buf[0], 0);
    fetch(buf[0], kSecPF);
    lds_barrier();
    // step k: rows of step k + 1 into xr, loads of step k + 1 + PF, outputs of step k - 1
    for (int64_t k = 0; k <= nst; k += kSecPF) {
#pragma unroll
      for (int u = 0; u < kSecPF; ++u) {
        const int64_t kk = k + u;
        if (kk <= nst) {
          const int b = (u + 1) % kSecPF;
          if (kk + 1 < nst) put(buf[b], kk + 1);
          fetch(buf[b], kk + 1 + kSecPF);
          if (kk >= 1) flush(kk - 1);
          lds_barrier();
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K_gain: out = v * g(env) * makeup per (channel, sample), parallel.  A
// workgroup takes a 64-sample x 64-channel tile (lane = channel, wave w =
// samples 16w .. 16w+15).  to_user: the tile is transposed through LDS and
// stored channel-major into the user buffer; otherwise it goes to inT.
// Metrics (updateMetrics): input/output peaks are maxima of non-negative
// values and the gain reduction is the minimum gain (every g <= 1 since the
// ratio >= 1, so `gr == 1 || g < gr` is a min from gr = 1); they combine with
// integer atomics on the IEEE bit patterns, which order like the values.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void atomic_max_pos(double* p, double v) {
  atomicMax(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v));
}
__device__ __forceinline__ void atomic_min_pos(double* p, double v) {
  atomicMin(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v));
}

template <bool TO_USER>
__global__ __launch_bounds__(256) void k_fx_gain(FxStageArgs a, int tiles_per_wg) {
#pragma clang fp contract(off)
  __shared__ double tile[64][65];
  __shared__ double red[3][4][64];
  const int w = wave_id();
  const int l = threadIdx.x & 63;
  const int c = blockIdx.y * 64 + l;
  const CompParams& p = a.cp;
  double ip = 0.0, op = 0.0, gr = 1.0;
  // tiles_per_wg consecutive 64-sample tiles: one set of metric atomics per
  // workgroup and channel for all of them (the atomics on a channel's three
  // words serialise in the L2)
  for (int q = 0; q < tiles_per_wg; ++q) {
    const int64_t t0 = ((int64_t)blockIdx.x * tiles_per_wg + q) * 64;
    if (t0 >= a.len) break;  // uniform
#pragma unroll 4
    for (int j = 0; j < 16; ++j) {
      const int tl = w * 16 + j;
      const int64_t t = t0 + tl;
      double out = 0.0;
      if (t < a.len) {
        const double v = a.vT[t * a.cpad + c];
        const double g = gain_for_level(p, a.envT[t * a.cpad + c]);
        out = v * g * p.makeup_lin;
        const double il = fabs(v), ol = fabs(out);
        if (il > ip) ip = il;
        if (ol > op) op = ol;
        if (g < gr) gr = g;
        if (!TO_USER) a.inT[t * a.cpad + c] = out;
      }
      if (TO_USER) tile[tl][l] = out;
    }
    if (TO_USER) {
      __syncthreads();
      // lane = sample, wave w = channels 16w .. 16w+15 of the tile
      const int64_t t = t0 + l;
#pragma unroll 4
      for (int j = 0; j < 16; ++j) {
        const int cl = w * 16 + j;
        const int ch = blockIdx.y * 64 + cl;
        if (ch < a.channels && t < a.len) a.buf[(int64_t)ch * a.stride + t] = tile[l][cl];
      }
      __syncthreads();  // the tile's reads before the next tile's writes
    }
  }
  red[0][w][l] = ip;
  red[1][w][l] = op;
  red[2][w][l] = gr;
  __syncthreads();
  if (w == 0 && c < a.channels) {
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      if (red[0][k][l] > ip) ip = red[0][k][l];
      if (red[1][k][l] > op) op = red[1][k][l];
      if (red[2][k][l] < gr) gr = red[2][k][l];
    }
    CompChState* cs = a.cs + c;
    if (ip > 0.0) atomic_max_pos(&cs->in_peak, ip);
    if (op > 0.0) atomic_max_pos(&cs->out_peak, op);
    if (gr < 1.0) atomic_min_pos(&cs->gr, gr);
  }
}

// user buffer [c][t] <-> time-major [t][cpad], 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void k_fx_transpose_in(FxStageArgs a, double* dstT) {
  __shared__ double tile[64][65];
  const int w = wave_id();
  const int l = threadIdx.x & 63;
  const int64_t t0 = (int64_t)blockIdx.x * 64;
  const int cb = blockIdx.y * 64;
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {  // lane = sample
    const int cl = w * 16 + j;
    const int ch = min(cb + cl, a.channels - 1);
    const int64_t t = min(t0 + l, a.len - 1);
    tile[cl][l] = a.buf[(int64_t)ch * a.stride + t];
  }
  __syncthreads();
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {  // lane = channel
    const int64_t t = t0 + w * 16 + j;
    if (t < a.len) dstT[t * a.cpad + cb + l] = tile[l][w * 16 + j];
  }
}

__global__ __launch_bounds__(256) void k_fx_transpose_out(FxStageArgs a, const double* srcT) {
  __shared__ double tile[64][65];
  const int w = wave_id();
  const int l = threadIdx.x & 63;
  const int64_t t0 = (int64_t)blockIdx.x * 64;
  const int cb = blockIdx.y * 64;
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {  // lane = channel
    const int64_t t = min(t0 + w * 16 + j, a.len - 1);
    tile[w * 16 + j][l] = srcT[t * a.cpad + cb + l];
  }
  __syncthreads();
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {  // lane = sample
    const int cl = w * 16 + j;
    const int64_t t = t0 + l;
    if (cb + cl < a.channels && t < a.len) a.buf[(int64_t)(cb + cl) * a.stride + t] = tile[l][cl];
  }
}

// ---------------------------------------------------------------------------
// K_comb: comb filter i (blockIdx.y) of 64 channels, one wave, serial in
// time (comb.process reverb.go:101-117):
//   output = line[idx]; fs = output*damp_b + fs*damp_a (flushed below 1e-23);
//   line[idx] = gain*in + fs*feedback; idx = (idx+1) mod len
// The line is read kCombB samples at a time (the values were written >= 1116
// samples earlier) two batches ahead, and written back after the batch.  Lanes
// past the channel count work on their own padding column of vbuf and
// never store state.  Output: coT[i][t][c].
// ---------------------------------------------------------------------------
template <bool FULL>
__device__ __forceinline__ void comb_batch(const VerbParams& p, double& fs, const double (&dl)[kCombB],
                                           const double (&xg)[kCombB], double (&nv)[kCombB], int nb) {
#pragma clang fp contract(off)
#pragma unroll
  for (int j = 0; j < kCombB; ++j) {
    const double output = dl[j];
    double f = output * p.damp_b + fs * p.damp_a;
    if (fabs(f) < 1e-23) f = 0.0;
    if (FULL || j < nb) fs = f;
    nv[j] = p.gain * xg[j] + fs * p.feedback;
  }
}

__global__ __launch_bounds__(64) void k_fx_comb(FxStageArgs a) {
#pragma clang fp contract(off)
  const int i = blockIdx.y;
  const int l = threadIdx.x;
  const int c = blockIdx.x * 64 + l;
  const bool active = c < a.channels;
  const int cc = active ? c : a.channels - 1;
  const int clen = kCombLen[i];
  const unsigned uc = (unsigned)c;  // zero-extended lane offset: lets loads use scalar base + 32-bit VGPR offset
  const int cp = a.cpad;
  // Row pointers are wave-uniform (scalar registers); a lane adds only its
  // channel c, so every access is a saddr + lane-offset load or store.  All
  // channels of a handle advance their delay lines together (every call
  // processes every channel over the same samples, Reset clears all), so
  // the ring index is uniform and lane 0's copy drives the addresses.
  AD_GLOBAL double* line = glob(a.vbuf) + (int64_t)comb_off(i) * cp;
  AD_GLOBAL double* co = glob(a.coT) + (int64_t)i * a.tmax * cp;
  const AD_GLOBAL double* in = glob(a.inT);
  const VerbParams& p = a.vp;
  AD_GLOBAL VerbChState* vs = glob(a.vs);
  int idx = __builtin_amdgcn_readfirstlane(vs[cc].comb_idx[i]);
  double fs = vs[cc].filter_store[i];
  const int64_t len = a.len;
  // three batches in flight: batch m sits in buffer m % 3 and is loaded two
  // batches before it runs (~100 samples of lead at ~80 cycles/sample).
  // A batch whose line positions do not wrap and whose samples are all real
  // (all but ~1.5 % at kCombB = 16, clen >= 1116) walks uniform row pointers
  // by one row per sample: no per-sample wrap test, clamp or multiply.
  double dl[3][kCombB], xg[3][kCombB];
  int lpos = idx;     // line position of the next batch to load
  int64_t lt = 0;     // its first sample
  auto load = [&](int b) {
    int pos = lpos;
    if (pos + kCombB <= clen && lt + kCombB <= len) {
      const AD_GLOBAL double* lr = uniform_ptr(line + (int64_t)pos * cp);
      const AD_GLOBAL double* ir = uniform_ptr(in + lt * cp);
#pragma unroll
      for (int j = 0; j < kCombB; ++j) {
        dl[b][j] = lr[uc];
        xg[b][j] = ir[uc];
        lr += cp;
        ir += cp;
      }
      pos += kCombB;
      if (pos >= clen) pos -= clen;
    } else {
#pragma unroll
      for (int j = 0; j < kCombB; ++j) {
        dl[b][j] = (line + (int64_t)pos * cp)[uc];
        xg[b][j] = (in + min(lt + j, len - 1) * cp)[uc];
        if (++pos >= clen) pos = 0;
      }
    }
    lpos = pos;
    lt += kCombB;
  };
  auto run = [&](int b, int64_t t0) {
    const int nb = (int)min((int64_t)kCombB, len - t0);
    double nv[kCombB];
    if (nb == kCombB && idx + kCombB <= clen) {
      comb_batch<true>(p, fs, dl[b], xg[b], nv, nb);
      AD_GLOBAL double* cr = uniform_ptr(co + t0 * cp);
      AD_GLOBAL double* lr = uniform_ptr(line + (int64_t)idx * cp);
#pragma unroll
      for (int j = 0; j < kCombB; ++j) {
        cr[uc] = dl[b][j];
        lr[uc] = nv[j];
        cr += cp;
        lr += cp;
      }
    } else {
      if (nb == kCombB)
        comb_batch<true>(p, fs, dl[b], xg[b], nv, nb);
      else
        comb_batch<false>(p, fs, dl[b], xg[b], nv, nb);
      int pos = idx;
#pragma unroll
      for (int j = 0; j < kCombB; ++j) {
        if (j < nb) {
          (co + (t0 + j) * cp)[uc] = dl[b][j];
          (line + (int64_t)pos * cp)[uc] = nv[j];
        }
        if (++pos >= clen) pos = 0;
      }
    }
    idx += nb;
    if (idx >= clen) idx -= clen;
  };
  load(0);
  load(1);
  for (int64_t t0 = 0; t0 < len; t0 += 3 * kCombB) {
    load(2);
    run(0, t0);
    if (t0 + kCombB >= len) break;
    load(0);
    run(1, t0 + kCombB);
    if (t0 + 2 * kCombB >= len) break;
    load(1);
    run(2, t0 + 2 * kCombB);
  }
  if (active) {
    vs[uc].comb_idx[i] = idx;
    vs[uc].filter_store[i] = fs;
  }
}

// ---------------------------------------------------------------------------
// K_ap: acc = (((0 + c0) + c1) + ... + c7), the four allpasses in series
// (allpass.process reverb.go:57-68: out = line[idx] - acc;
// line[idx] = acc + line[idx]*0.5), y = acc*wet + in*dry.  Within a block of
// kApB = 128 samples every (channel, sample) is independent: an allpass
// reads its line 225..556 samples back, i.e. before the block, and no two
// samples of a block touch the same line position.  So a workgroup serves
// only 16 channels (16 workgroups at 256 channels: the stage is bound by
// memory round trips, and more CUs keep more of them in flight): lane =
// channel (16) x sample phase (4); wave w, phase h takes samples
// 4w + h + 32j, j = 0..3, of a block, with all 52 loads of its four samples
// issued before the arithmetic.  y is transposed through LDS and stored
// channel-major.
// ---------------------------------------------------------------------------
constexpr int kApCh = 16;
__global__ __launch_bounds__(64 * kApW) void k_fx_allpass(FxStageArgs a) {
#pragma clang fp contract(off)
  constexpr int J = kApB / (kApW * 4);  // samples per lane per block
  __shared__ double tile[kApCh][kApB + 1];
  const int w = wave_id();
  const int l = threadIdx.x & 63;
  const int cl = l & (kApCh - 1), ph = l >> 4;
  const int c = blockIdx.x * kApCh + cl;
  const bool active = c < a.channels;
  const int cc = active ? c : a.channels - 1;
  const int cp = a.cpad;
  const VerbParams& p = a.vp;
  int base[kVerbAllpass];  // line position of the block's first sample (uniform, see K_comb)
#pragma unroll
  for (int i = 0; i < kVerbAllpass; ++i) base[i] = __builtin_amdgcn_readfirstlane(a.vs[cc].ap_idx[i]);
  const int64_t len = a.len;
  const int64_t cstride = a.tmax * cp;
  for (int64_t b0 = 0; b0 < len; b0 += kApB) {
    double cv[J][kVerbCombs], bo[J][kVerbAllpass], xin[J];
    int pos[J][kVerbAllpass];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int tl = 4 * w + ph + 32 * j;
      const int64_t t = min(b0 + tl, len - 1);  // clamped rows are never stored
      const double* cot = a.coT + t * cp + c;
#pragma unroll
      for (int i = 0; i < kVerbCombs; ++i) cv[j][i] = cot[i * cstride];
#pragma unroll
      for (int i = 0; i < kVerbAllpass; ++i) {
        int q = base[i] + tl;
        if (q >= kApLen[i]) q -= kApLen[i];
        pos[j][i] = q;
        bo[j][i] = a.vbuf[(int64_t)(ap_off(i) + q) * cp + c];
      }
      xin[j] = a.inT[t * cp + c];
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int tl = 4 * w + ph + 32 * j;
      const bool real = b0 + tl < len;
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < kVerbCombs; ++i) acc += cv[j][i];
#pragma unroll
      for (int i = 0; i < kVerbAllpass; ++i) {
        const double output = bo[j][i] - acc;
        if (real) a.vbuf[(int64_t)(ap_off(i) + pos[j][i]) * cp + c] = acc + bo[j][i] * p.ap_feedback;
        acc = output;
      }
      tile[cl][tl] = acc * p.wet + xin[j] * p.dry;
    }
    lds_barrier();  // the tile (LDS only)
    // consecutive threads = consecutive samples of one channel
#pragma unroll
    for (int r = 0; r < kApCh * kApB / (64 * kApW); ++r) {
      const int e = r * 64 * kApW + threadIdx.x;
      const int ch = e / kApB, tl = e % kApB;
      const int cg = blockIdx.x * kApCh + ch;
      if (cg < a.channels && b0 + tl < len) a.buf[(int64_t)cg * a.stride + b0 + tl] = tile[ch][tl];
    }
#pragma unroll
    for (int i = 0; i < kVerbAllpass; ++i) {
      base[i] += kApB;
      if (base[i] >= kApLen[i]) base[i] -= kApLen[i];
    }
    __syncthreads();  // line writes of this block are read by other waves 225+ samples on
  }
  if (active && w == 0 && ph == 0) {
#pragma unroll
    for (int i = 0; i < kVerbAllpass; ++i) a.vs[c].ap_idx[i] = (int)((a.vs[c].ap_idx[i] + len % kApLen[i]) % kApLen[i]);
  }
}

}  // namespace

// The serial stages (K_eq, K_comb, K_ap) are issue/latency bound per wave:
// their workgroups claim over half a CU's LDS so that no two of them share a
// CU (config 5: +1.5 %).
int fx_excl_lds(int own) { return std::max(0, 82 * 1024 - own); }

void launch_fx_eq_parts(const FxStageArgs& a, hipStream_t s) {
  int waves = 0;
  bool det = false;
  for (int i = 0; i < a.nparts; ++i) {
    waves = std::max(waves, a.part[i].ns + (a.part[i].det ? 1 : 0) + 1);  // + the loader
    det = det || a.part[i].det;
  }
  if (a.nparts <= 0 || waves <= 1) return;
  const dim3 grid((unsigned)((a.channels + 63) / 64), (unsigned)a.nparts), block((unsigned)(64 * waves));
  const int dyn = fx_excl_lds(72 * 1024);
  if (det)
    hipLaunchKernelGGL(k_fx_eq<true>, grid, block, dyn, s, a);
  else
    hipLaunchKernelGGL(k_fx_eq<false>, grid, block, dyn, s, a);
}

void launch_fx_eq_sec(const FxStageArgs& a, hipStream_t s) {
  if (a.nparts <= 0) return;
  const dim3 grid((unsigned)((a.channels + 63) / 64), (unsigned)a.nparts);
  hipLaunchKernelGGL(k_fx_eq_sec, grid, dim3(128), 0, s, a);
}

void launch_fx_eq(const FxStageArgs& a, bool comp, int out_mode, hipStream_t s) {
  if (a.len <= 0) return;
  FxStageArgs b = a;
  b.nparts = 1;
  b.part[0] = FxEqPart{0, a.eq.nsec, comp ? 1 : 0, a.len, a.xT, out_mode == kFxOutInT ? a.inT : a.vT, a.envT};
  launch_fx_eq_parts(b, s);
}

#ifndef AD_FX_GAIN_TPW
#define AD_FX_GAIN_TPW 8  // 64-sample tiles per K_gain workgroup, at most
#endif
#ifndef AD_FX_GAIN_MINWG
#define AD_FX_GAIN_MINWG 1024  // while the grid keeps at least this many workgroups
#endif
void launch_fx_gain(const FxStageArgs& a, bool to_user, hipStream_t s) {
  if (a.len <= 0) return;
  const int64_t tiles = (a.len + 63) / 64, cgroups = (a.channels + 63) / 64;
  // several tiles per workgroup while the grid keeps AD_FX_GAIN_MINWG workgroups
  int tpw = 1;
  while (tpw < AD_FX_GAIN_TPW && (tiles / (2 * tpw)) * cgroups >= AD_FX_GAIN_MINWG) tpw *= 2;
  const dim3 grid((unsigned)((tiles + tpw - 1) / tpw), (unsigned)cgroups);
  if (to_user)
    hipLaunchKernelGGL(k_fx_gain<true>, grid, dim3(256), 0, s, a, tpw);
  else
    hipLaunchKernelGGL(k_fx_gain<false>, grid, dim3(256), 0, s, a, tpw);
}

void launch_fx_transpose_in(const FxStageArgs& a, double* dstT, hipStream_t s) {
  if (a.len <= 0) return;
  const dim3 grid((unsigned)((a.len + 63) / 64), (unsigned)((a.channels + 63) / 64));
  hipLaunchKernelGGL(k_fx_transpose_in, grid, dim3(256), 0, s, a, dstT);
}

void launch_fx_transpose_out(const FxStageArgs& a, const double* srcT, hipStream_t s) {
  if (a.len <= 0) return;
  const dim3 grid((unsigned)((a.len + 63) / 64), (unsigned)((a.channels + 63) / 64));
  hipLaunchKernelGGL(k_fx_transpose_out, grid, dim3(256), 0, s, a, srcT);
}

void launch_fx_comb(const FxStageArgs& a, hipStream_t s) {
  if (a.len <= 0) return;
  hipLaunchKernelGGL(k_fx_comb, dim3((unsigned)((a.channels + 63) / 64), kVerbCombs), dim3(64), fx_excl_lds(0), s, a);
}

void launch_fx_allpass(const FxStageArgs& a, hipStream_t s) {
  if (a.len <= 0) return;
  hipLaunchKernelGGL(k_fx_allpass, dim3((unsigned)((a.channels + kApCh - 1) / kApCh)), dim3(64 * kApW),
                     fx_excl_lds(kApCh * (kApB + 1) * 8), s, a);
}

}  // namespace adsp
