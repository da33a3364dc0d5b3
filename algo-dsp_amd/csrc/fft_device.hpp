// LDS-resident FP64 Stockham FFT building blocks for gfx950 (CDNA4).
//
// Replaces the third-party `github.com/cwbudde/algo-fft v0.6.10` complex128
// plans the reference calls from dsp/conv/streaming.go:57-98 (fftEngine) and
// overlap_{add,save}.go (NewPlan64). Semantics kept: forward transform is
// unnormalised (exp(-2*pi*i*k*n/N)), the inverse carries the 1/N factor
// (overlap_add.go:138-160 uses real(IFFT(.)) as the convolution result).
//
// Design (MI355X-first, not a translation of the Go code):
//   * one M-point complex FFT is done by M/V threads, each holding V = 8 or
//     16 complex128 values in VGPRs; passes are radix-V (the first pass may
//     be radix 2/4/8), so M = 4096 at V = 16 takes three passes;
//   * the LDS image is interleaved double2 with an XOR swizzle inside each
//     aligned 16-element block (lds_slot) so every lane group of a
//     ds_read_b128 (16 lanes over 16 slots of 16 B) and of a ds_write_b128
//     (8 lanes over 8 slots) -- the consecutive accesses and the stride-NS
//     Stockham stores of every pass -- hits distinct slots (no padding);
//   * a workgroup of max(M/V, 256) threads carries max(1, 256V/M) FFTs
//     (fft_kernels.hip splits M >= 2048 into two M/2 transforms so that two
//     workgroups share a CU);
//   * butterfly twiddles come from one W_M table read once per butterfly and
//     powered by complex multiplies in registers (FP64 sincos is far too
//     expensive on the VALU).
#pragma once

#include <hip/hip_runtime.h>

namespace adsp {

struct cplx {
  double x, y;
};

// Non-temporal 16-byte load/store (streams touched once: nt keeps them from
// displacing lines another kernel is about to reuse).
typedef double d2v_t __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ double2 ld2(const double2* p) {
  if constexpr (NT) {
    const d2v_t t = __builtin_nontemporal_load(reinterpret_cast<const d2v_t*>(p));
    return make_double2(t.x, t.y);
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void st2(double2* p, double2 v) {
  if constexpr (NT)
    __builtin_nontemporal_store(d2v_t{v.x, v.y}, reinterpret_cast<d2v_t*>(p));
  else
    *p = v;
}

__device__ __forceinline__ double2 c_add(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 c_sub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 c_mul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 c_conj(double2 a) { return make_double2(a.x, -a.y); }
__device__ __forceinline__ double2 c_scale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }

// cos(2*pi*k/16), k = 0..15
__device__ constexpr double kCos16[16] = {
    1.0,
    0.92387953251128675613,
    0.70710678118654752440,
    0.38268343236508977173,
    0.0,
    -0.38268343236508977173,
    -0.70710678118654752440,
    -0.92387953251128675613,
    -1.0,
    -0.92387953251128675613,
    -0.70710678118654752440,
    -0.38268343236508977173,
    0.0,
    0.38268343236508977173,
    0.70710678118654752440,
    0.92387953251128675613,
};

// a * W16^E with W16 = exp(-2*pi*i/16) for the forward direction (conjugate
// for the inverse). Trivial rotations are special-cased so no multiply by an
// exact 0/1 is ever issued.
template <int E, bool FWD>
__device__ __forceinline__ double2 tw16(double2 a) {
  constexpr int e = E & 15;
  constexpr double R2 = 0.70710678118654752440;
  if constexpr (e == 0) {
    return a;
  } else if constexpr (e == 4) {
    return FWD ? make_double2(a.y, -a.x) : make_double2(-a.y, a.x);
  } else if constexpr (e == 8) {
    return make_double2(-a.x, -a.y);
  } else if constexpr (e == 12) {
    return FWD ? make_double2(-a.y, a.x) : make_double2(a.y, -a.x);
  } else if constexpr (e == 2) {
    return FWD ? make_double2((a.x + a.y) * R2, (a.y - a.x) * R2) : make_double2((a.x - a.y) * R2, (a.y + a.x) * R2);
  } else if constexpr (e == 6) {
    return FWD ? make_double2((a.y - a.x) * R2, -(a.x + a.y) * R2) : make_double2(-(a.x + a.y) * R2, (a.x - a.y) * R2);
  } else if constexpr (e == 10) {
    return FWD ? make_double2(-(a.x + a.y) * R2, (a.x - a.y) * R2) : make_double2((a.y - a.x) * R2, -(a.x + a.y) * R2);
  } else if constexpr (e == 14) {
    return FWD ? make_double2((a.x - a.y) * R2, (a.y + a.x) * R2) : make_double2((a.x + a.y) * R2, (a.y - a.x) * R2);
  } else {
    constexpr double c = kCos16[e];
    constexpr double s0 = kCos16[(e + 12) & 15];  // sin(2*pi*e/16)
    constexpr double s = FWD ? -s0 : s0;
    return make_double2(a.x * c - a.y * s, a.x * s + a.y * c);
  }
}

// In-register DFT of R = 1,2,4,8,16 points, natural order in and out.
// Radix-2 decimation in time, fully unrolled at compile time.
template <int R, bool FWD>
struct Dft {
  template <int I = 0>
  __device__ static __forceinline__ void combine(double2* v, const double2* e, const double2* o) {
    if constexpr (I < R / 2) {
      const double2 t = tw16<I*(16 / R), FWD>(o[I]);
      v[I] = c_add(e[I], t);
      v[I + R / 2] = c_sub(e[I], t);
      combine<I + 1>(v, e, o);
    }
  }
  __device__ static __forceinline__ void run(double2* v) {
    double2 e[R / 2], o[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      e[i] = v[2 * i];
      o[i] = v[2 * i + 1];
    }
    Dft<R / 2, FWD>::run(e);
    Dft<R / 2, FWD>::run(o);
    combine(v, e, o);
  }
};
template <bool FWD>
struct Dft<1, FWD> {
  __device__ static __forceinline__ void run(double2*) {}
};

// ---------------------------------------------------------------------------
// Mixed-radix Stockham plan for M = 2^m, 16 <= M <= 8192, V values per thread
// (V = 16: radix-16 passes; V = 8: radix-8 passes, half the VGPRs per lane and
// twice the threads).  Passes: first radix R0 = M / V^(passes-1), then radix V.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int ilog2c(int v) { return v <= 1 ? 0 : 1 + ilog2c(v >> 1); }
template <int M, int V = 16>
struct FftPlan {
  static_assert(M >= 16 && M <= 8192 && (M & (M - 1)) == 0, "FFT size must be a power of two in [16, 8192]");
  static_assert(V == 4 || V == 8 || V == 16, "4, 8 or 16 values per thread");
  static constexpr int LOGV = ilog2c(V);
  static constexpr int LOG = ilog2c(M);
  static constexpr int NPASS = (LOG + LOGV - 1) / LOGV;
  static constexpr int R0 = 1 << (LOG - LOGV * (NPASS - 1));
  static constexpr int T = M / V;                  // threads per FFT
  static constexpr int BLOCK = T > 256 ? T : 256;  // workgroup size
  static constexpr int F = BLOCK / T;              // FFTs per workgroup
  // LDS elements per FFT: several FFTs share a 16-lane group when T < 16; the
  // stride T (mod 16) puts each one on its own part of the bank row
  static constexpr int MP = M + (T < 16 ? T : 0);
  static constexpr int radix(int p) { return p == 0 ? R0 : V; }
  static constexpr int ns(int p) { return p == 0 ? 1 : R0 * (1 << (LOGV * (p - 1))); }
};

// Workgroups are dealt round-robin over the 8 XCDs (b % 8 share one L2).
// Remap the hardware index so each XCD owns a contiguous run of logical
// indices: neighbouring blocks (which share input samples / X rows) then run
// on the same XCD at about the same time.  Bijective for any grid size; a
// different placement changes speed only, never results.
__device__ __forceinline__ int xcd_remap(int b, int G) {
  const int xcd = b & 7, r = b >> 3;
  const int q = G >> 3, rem = G & 7;
  return (xcd < rem) ? xcd * (q + 1) + r : rem * (q + 1) + (xcd - rem) * q + r;
}

// Swizzled LDS index, a bijection on each aligned 16-block (tools/lds_conflicts.py
// checks the plans against the banking model).
#ifndef AD_LDS_SWZ
#define AD_LDS_SWZ 1  // 0: the round-1 swizzle g(i >> 4) (tools/ A/B builds)
#endif
__device__ __forceinline__ int lds_slot(int i) {
#if AD_LDS_SWZ
  // i ^ x(t), t = bits 3..6 of i: x's low three bits are 3 t0 ^ 5 t1 ^ 7 t2 ^ 4 t3 and
  // its bit 3 is t1 ^ t2 ^ t3 (a bijection on each aligned 16-block, since bit 3
  // flips on bits >= 4 only); the 16 values of x packed in one 64-bit constant.
  // Under the banking of MI355X_MICROARCH.md (ds_read_b128: 16-lane groups over
  // 16 slots of 16 B; ds_write_b128: 8-lane groups over 8 slots) every Stockham
  // store and load of the V = 4 and 8 plans (M = 64 ... 8192) is conflict-free
  // (tools/lds_conflicts.py).
  const int t = (i >> 3) & 15;
  return i ^ (int)((0xde0321fc12cfed30ull >> (4 * t)) & 15);
#else
  const int q = i >> 4;
  return i ^ ((q ^ ((q & 4) << 1)) & 15);
#endif
}
// lds_slot is linear over GF(2) (x(t) is an XOR of per-bit constants; checked
// for every t pair), so for a base and an offset with disjoint bits
// lds_slot(base + off) == lds_slot(base) ^ lds_slot(off).  The Stockham indices
// below are all of that form (base < the offset's lowest bit, or a multiple of
// a power of two above its highest), with the offset known at compile time:
// one swizzle per butterfly and one XOR per access instead of the shift / mask
// chain per access.
__device__ __forceinline__ int lds_slot_split(int swz_base, int off) { return swz_base ^ lds_slot(off); }
// Twiddle-table slot: stride-8 reads (the NS = 64 pass at M = 4096) and
// consecutive reads both spread over 16 slots.
__device__ __forceinline__ int tw_slot(int i) { return i ^ ((i >> 3) & 7); }

// Twiddle sources.  TwGlobal reads W_M^e from the HBM table.  TwLds reads it
// from two small LDS tables, W^e = lo[e mod 2^S] * hi[e >> S] (S = ceil(log2 M / 2),
// 2^S + M/2^S entries): no global load inside the passes, so the only vector
// memory traffic of a persistent FFT workgroup is its own prefetch and stores,
// and waiting on a twiddle never drains them (vmcnt is in-order on gfx950).
// One extra rounding vs the direct table (~1 ulp), far inside the 1e-7 gate.
struct TwGlobal {
  const double2* __restrict__ t;
  __device__ __forceinline__ double2 operator()(int e) const { return t[e]; }
};
template <int M>
struct TwSplit {
  static constexpr int S = (ilog2c(M) + 1) / 2;
  static constexpr int NLO = 1 << S;
  static constexpr int NHI = M >> S;
  static constexpr int N = NLO + NHI;  // LDS entries per table
};
template <int M>
struct TwLds {
  const double2* lo;  // LDS: W^i, i < 2^S
  const double2* hi;  // LDS: W^(i 2^S), i < M / 2^S
  __device__ __forceinline__ double2 operator()(int e) const {
    using Sp = TwSplit<M>;
    if constexpr (Sp::NHI == 1) return lo[tw_slot(e)];
    const double2 a = lo[tw_slot(e & (Sp::NLO - 1))];
    const double2 b = hi[e >> Sp::S];
    return c_mul(a, b);
  }
};
// Fills an LDS table pair from a full W_M table in HBM (all threads of the
// workgroup take part; the caller barriers before the first use).
// STRIDE > 1 reads W_M^e as g[e * STRIDE] from a finer table (W_{M*STRIDE}).
template <int M, int STRIDE = 1>
__device__ __forceinline__ TwLds<M> tw_lds_fill(double2* ltab, const double2* __restrict__ g, int tid, int nthreads) {
  using Sp = TwSplit<M>;
  for (int i = tid; i < Sp::N; i += nthreads) {
    if (i < Sp::NLO)
      ltab[tw_slot(i)] = g[i * STRIDE];
    else
      ltab[i] = g[((i - Sp::NLO) << Sp::S) * STRIDE];
  }
  return TwLds<M>{ltab, ltab + Sp::NLO};
}

// Same tables computed in the kernel (sincospi; <= 1 ulp from the rounded
// table, far inside the 1e-7 gate): no global load ahead of a workgroup's
// data loads, so its first transform waits for one memory round trip only.
template <int M>
__device__ __forceinline__ TwLds<M> tw_lds_compute(double2* ltab, int tid, int nthreads) {
  using Sp = TwSplit<M>;
  for (int i = tid; i < Sp::N; i += nthreads) {
    const int e = i < Sp::NLO ? i : ((i - Sp::NLO) << Sp::S);
    double sn, cs;
    sincospi(-2.0 * (double)e / (double)M, &sn, &cs);
    ltab[i < Sp::NLO ? tw_slot(i) : i] = make_double2(cs, sn);
  }
  return TwLds<M>{ltab, ltab + Sp::NLO};
}

// Twiddle multiply for butterfly jb of a pass with stride NS and radix R:
// v[r] *= W_{NS*R}^{(jb mod NS) * r} = W_M^{e*r}, e = (jb mod NS) * M/(NS*R).
template <int M, int R, int NS, bool FWD, class TW>
__device__ __forceinline__ void apply_twiddles(double2* v, int jb, const TW& tw) {
  if constexpr (NS > 1) {
    const int e = (jb & (NS - 1)) * (M / (NS * R));
    double2 w = tw(e);
    if (!FWD) w = c_conj(w);
    double2 wr = w;
#pragma unroll
    for (int r = 1; r < R; ++r) {
      v[r] = c_mul(v[r], wr);
      if (r + 1 < R) wr = c_mul(wr, w);
    }
  }
}

// One in-register pass on the thread's V values (V/R butterflies of radix R),
// followed by the Stockham store into the LDS image of this FFT.
template <int M, int V, int P, bool FWD, class TW>
__device__ __forceinline__ void pass_compute_store(double2* v, int tid, double2* lds, const TW& twM) {
  using Plan = FftPlan<M, V>;
  constexpr int R = Plan::radix(P);
  constexpr int NS = Plan::ns(P);
  constexpr int NB = V / R;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int jb = tid + b * Plan::T;
    apply_twiddles<M, R, NS, FWD, TW>(v + b * R, jb, twM);
    Dft<R, FWD>::run(v + b * R);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int jb = tid + b * Plan::T;
    const int base = (jb / NS) * NS * R + (jb & (NS - 1));  // bits disjoint from r * NS
    const int sb = lds_slot(base);
#pragma unroll
    for (int r = 0; r < R; ++r) lds[lds_slot_split(sb, r * NS)] = v[b * R + r];
  }
}

// Load the thread's V values of pass P from the LDS image.
template <int M, int V, int P>
__device__ __forceinline__ void pass_load(double2* v, int tid, const double2* lds) {
  using Plan = FftPlan<M, V>;
  constexpr int R = Plan::radix(P);
  constexpr int NB = V / R;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int jb = tid + b * Plan::T;  // < M / R: bits disjoint from r * (M / R)
    const int sb = lds_slot(jb);
#pragma unroll
    for (int r = 0; r < R; ++r) v[b * R + r] = lds[lds_slot_split(sb, r * (M / R))];
  }
}

// Index (in the natural-order input) of value slot s of the thread for pass 0.
template <int M, int V = 16>
__device__ __forceinline__ int pass0_index(int tid, int s) {
  using Plan = FftPlan<M, V>;
  constexpr int R = Plan::R0;
  const int b = s / R, r = s % R;
  return tid + b * Plan::T + r * (M / R);
}

// lds_slot(pass0_index(tid, s)): jb = tid + b T < M / R and r (M / R) have disjoint bits.
template <int M, int V = 16>
__device__ __forceinline__ int pass0_slot(int tid, int s) {
  using Plan = FftPlan<M, V>;
  constexpr int R = Plan::R0;
  const int b = s / R, r = s % R;
  return lds_slot_split(lds_slot(tid + b * Plan::T), r * (M / R));
}

// Runs passes [1, NPASS-1) (the middle passes) after pass 0 has been stored:
// barrier, load, compute, barrier, store.  Leaves the last pass's input in v
// (already loaded), ready for the caller's final pass handling.
template <int M, int V, bool FWD, int P = 1, class TW>
__device__ __forceinline__ void run_middle_passes(double2* v, int tid, double2* lds, const TW& twM) {
  using Plan = FftPlan<M, V>;
  if constexpr (P < Plan::NPASS) {
    __syncthreads();
    pass_load<M, V, P>(v, tid, lds);
    if constexpr (P + 1 < Plan::NPASS) {
      __syncthreads();
      pass_compute_store<M, V, P, FWD, TW>(v, tid, lds, twM);
      run_middle_passes<M, V, FWD, P + 1, TW>(v, tid, lds, twM);
    }
  }
}

// Computes the last pass in registers (twiddles + DFT) without storing.
template <int M, int V, bool FWD, class TW>
__device__ __forceinline__ void last_pass_compute(double2* v, int tid, const TW& twM) {
  using Plan = FftPlan<M, V>;
  constexpr int P = Plan::NPASS - 1;
  constexpr int R = Plan::radix(P);
  constexpr int NS = Plan::ns(P);
  constexpr int NB = V / R;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int jb = tid + b * Plan::T;
    apply_twiddles<M, R, NS, FWD, TW>(v + b * R, jb, twM);
    Dft<R, FWD>::run(v + b * R);
  }
}

// Output index held by slot s after last_pass_compute.
template <int M, int V = 16>
__device__ __forceinline__ int last_pass_index(int tid, int s) {
  using Plan = FftPlan<M, V>;
  constexpr int P = Plan::NPASS - 1;
  constexpr int R = Plan::radix(P);
  constexpr int NS = Plan::ns(P);
  const int b = s / R, r = s % R;
  const int jb = tid + b * Plan::T;
  return (jb / NS) * NS * R + (jb & (NS - 1)) + r * NS;
}

// lds_slot(last_pass_index(tid, s)): the base (jb / NS) NS R + (jb mod NS) and
// r NS have disjoint bits.
template <int M, int V = 16>
__device__ __forceinline__ int last_pass_slot(int tid, int s) {
  using Plan = FftPlan<M, V>;
  constexpr int P = Plan::NPASS - 1;
  constexpr int R = Plan::radix(P);
  constexpr int NS = Plan::ns(P);
  const int b = s / R, r = s % R;
  const int jb = tid + b * Plan::T;
  return lds_slot_split(lds_slot((jb / NS) * NS * R + (jb & (NS - 1))), r * NS);
}

// Full FFT of the thread's V pass-0 values (forward or inverse); the result
// sits in v at last_pass_index order.
template <int M, int V, bool FWD, class TW>
__device__ __forceinline__ void fft_run(double2* v, int tid, double2* lds, const TW& twM) {
  using Plan = FftPlan<M, V>;
  if constexpr (Plan::NPASS > 1) {
    pass_compute_store<M, V, 0, FWD, TW>(v, tid, lds, twM);
    run_middle_passes<M, V, FWD, 1, TW>(v, tid, lds, twM);
  }
  last_pass_compute<M, V, FWD, TW>(v, tid, twM);
}

// fft_run for a workgroup where only some waves hold a transform: `active`
// (wave-uniform) guards the arithmetic and the LDS traffic, while every wave
// still takes each barrier of the passes (s_barrier counts all waves).
template <int M, int V, bool FWD, int P = 1, class TW>
__device__ __forceinline__ void run_middle_passes_active(double2* v, int tid, double2* lds, const TW& twM, bool active) {
  using Plan = FftPlan<M, V>;
  if constexpr (P < Plan::NPASS) {
    __syncthreads();
    if (active) pass_load<M, V, P>(v, tid, lds);
    if constexpr (P + 1 < Plan::NPASS) {
      __syncthreads();
      if (active) pass_compute_store<M, V, P, FWD, TW>(v, tid, lds, twM);
      run_middle_passes_active<M, V, FWD, P + 1, TW>(v, tid, lds, twM, active);
    }
  }
}
template <int M, int V, bool FWD, class TW>
__device__ __forceinline__ void fft_run_active(double2* v, int tid, double2* lds, const TW& twM, bool active) {
  using Plan = FftPlan<M, V>;
  if constexpr (Plan::NPASS > 1) {
    if (active) pass_compute_store<M, V, 0, FWD, TW>(v, tid, lds, twM);
    run_middle_passes_active<M, V, FWD, 1, TW>(v, tid, lds, twM, active);
  }
  if (active) last_pass_compute<M, V, FWD, TW>(v, tid, twM);
}

}  // namespace adsp
