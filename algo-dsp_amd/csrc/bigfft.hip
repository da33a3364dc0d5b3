// Device kernels of the large power-of-two FFT and the pointwise spectral
// operations of CorrelateFFT / Deconvolve / InverseFilter (see bigfft.hpp).
// Pass outputs are stored non-temporally (1; a whole pass's output, 268-537 MB
// at 2^24 points, overflows the Infinity Cache before the next pass reads it):
// CorrelateFFT 0.670 -> 0.641-0.652 ms.  2 (tools/ A/B): non-temporal pass
// inputs too (no better).
#ifndef AD_FFT_NT
#define AD_FFT_NT 1
#endif
#include "bigfft.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "ad_common.hpp"
#include "fft_device.hpp"

namespace adsp {

// Go complex128 product (a*b as (ac - bd, ad + bc), no contraction): the
// correlation's pointwise step, also fused into the inverse's first pass.
#pragma clang fp contract(off)
__device__ __forceinline__ double2 go_cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 go_cdiv(double2 n, double2 m) {
  double e, f;
  if (fabs(m.x) >= fabs(m.y)) {
    const double ratio = m.y / m.x;
    const double denom = m.x + ratio * m.y;
    e = (n.x + n.y * ratio) / denom;
    f = (n.y - n.x * ratio) / denom;
  } else {
    const double ratio = m.x / m.y;
    const double denom = m.y + ratio * m.x;
    e = (n.x * ratio + n.y) / denom;
    f = (n.y * ratio - n.x) / denom;
  }
  return make_double2(e, f);
}
__device__ __forceinline__ double go_hypot(double p, double q) {
  p = fabs(p);
  q = fabs(q);
  if (isinf(p) || isinf(q)) return INFINITY;
  if (isnan(p) || isnan(q)) return NAN;
  if (p < q) {
    const double t = p;
    p = q;
    q = t;
  }
  if (p == 0) return 0;
  q = q / p;
  return p * sqrt(1 + q * q);
}
// The pointwise step of the spectral row on one bin (see SpecOp): x the
// signal's (or the only input's) spectrum, h the kernel's; bin index k for
// the naive method's first-failing-bin report.
__device__ __forceinline__ double2 spec_op(int op, double2 x, double2 h, double eps, int64_t k,
                                           unsigned long long* bad) {
  switch (op) {
    case kSpecCorr:
      return go_cmul(x, c_conj(h));
    case kSpecNaive:
      if (go_hypot(h.x, h.y) < 1e-15) atomicMin(bad, (unsigned long long)k);
      return go_cdiv(x, h);
    case kSpecReg: {
      const double mag2 = h.x * h.x + h.y * h.y;
      return go_cdiv(go_cmul(x, c_conj(h)), make_double2(mag2 + eps, 0.0));
    }
    default: {  // kSpecInvFilt
      const double mag2 = x.x * x.x + x.y * x.y;
      return go_cdiv(c_conj(x), make_double2(mag2 + eps, 0.0));
    }
  }
}
#pragma clang fp contract(fast)  // the HIP default again for the transforms below

// The packing scales of a CorrelateFFT (FftPassArgs::amax): both signals are
// normalised before they share one transform, a' = a 2^-ea, b' = b 2^-eb with
// ea, eb = the exponents of max|a|, max|b| (clamped to [-1000, 1000] so every
// factor is a normal power of two), and the output is scaled back by
// 2^(ea + eb), applied as two factors when the sum leaves [-1000, 1000] (the
// result itself is then near the double range's ends, as the reference's is).
// All 1 when either maximum is zero or not finite.  Powers of two, so in the
// normal range the scaling is exact and the result is that of the unscaled
// transform; without it an |a| / |b| of 2^1000 made 2^e or 2^-e overflow.
struct PackScale {
  double a = 1.0, b = 1.0, o1 = 1.0, o2 = 1.0;
};
__device__ __forceinline__ PackScale pack_scale_bits(unsigned long long ba, unsigned long long bb) {
  PackScale p;
  const double ma = __longlong_as_double((long long)ba), mb = __longlong_as_double((long long)bb);
  if (!(ma > 0.0) || !(mb > 0.0) || !__builtin_isfinite(ma) || !__builtin_isfinite(mb)) return p;
  int ea = 0, eb = 0;
  (void)frexp(ma, &ea);
  (void)frexp(mb, &eb);
  ea = max(-1000, min(1000, ea));
  eb = max(-1000, min(1000, eb));
  const int e = ea + eb, e1 = e / 2;
  p.a = ldexp(1.0, -ea);
  p.b = ldexp(1.0, -eb);
  if (e >= -1000 && e <= 1000) {
    p.o1 = ldexp(1.0, e);
  } else {
    p.o1 = ldexp(1.0, e1);
    p.o2 = ldexp(1.0, e - e1);
  }
  return p;
}
__device__ __forceinline__ PackScale pack_scale(const unsigned long long* amax) {
  if (!amax) return PackScale{};
  return pack_scale_bits(amax[0], amax[1]);
}

// {max|a[0..n)|, max|b[0..m)|} as bit patterns (non-negative doubles order
// like their unsigned bit patterns; a NaN sorts above +inf and disables the
// scale) into out[0..1].  16-B loads, four in flight per thread, one partial
// per workgroup (same-address atomics serialise: one per wave over 8192 waves
// took 120-196 us for a 134 MB read); the last workgroup to finish (a counter
// at out[2], release/acquire at agent scope) reduces the partials at out[8..)
// and puts the counter back to zero for the next call, so no memset precedes
// the kernel (kAbsmaxWords words of device scratch, zeroed once).
#ifndef AD_ABSMAX_G
#define AD_ABSMAX_G 256  // workgroups per signal (<= kAbsmaxMaxGroups)
#endif
static_assert(AD_ABSMAX_G <= kAbsmaxMaxGroups, "max-abs partials");
constexpr int kAbsmaxPart = 8;  // out[kAbsmaxPart + y * gridDim.x + x]: partial of block (x, y)
__global__ __launch_bounds__(256) void k_absmax2(const double* __restrict__ a, int64_t n, const double* __restrict__ b,
                                                 int64_t m, unsigned long long* out) {
  const double* x = blockIdx.y ? b : a;
  const int64_t len = blockIdx.y ? m : n;
  unsigned long long mx = 0;
  auto acc = [&](double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(fabs(v));
    mx = u > mx ? u : mx;
  };
  const int head = ((uintptr_t)x & 15) ? 1 : 0;  // doubles are 8-B aligned
  const int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
  if (t0 == 0 && len > 0) {
    if (head) acc(x[0]);
    if ((len - head) & 1) acc(x[len - 1]);
  }
  const double2* x2 = reinterpret_cast<const double2*>(x + head);
  const int64_t n2 = len > head ? (len - head) / 2 : 0;
  int64_t i = t0;
#if AD_ABSMAX_U8  // tools/ A/B builds: eight 16-B loads in flight per thread
  for (; i + 7 * stride < n2; i += 8 * stride) {
    double2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = x2[i + u * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc(v[u].x), acc(v[u].y);
  }
#endif
  for (; i + 3 * stride < n2; i += 4 * stride) {
    const double2 v0 = x2[i], v1 = x2[i + stride], v2 = x2[i + 2 * stride], v3 = x2[i + 3 * stride];
    acc(v0.x), acc(v0.y), acc(v1.x), acc(v1.y), acc(v2.x), acc(v2.y), acc(v3.x), acc(v3.y);
  }
  for (; i < n2; i += stride) {
    const double2 v = x2[i];
    acc(v.x), acc(v.y);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long t = __shfl_xor(mx, o);
    mx = t > mx ? t : mx;
  }
  __shared__ unsigned long long wmax[4];
  __shared__ int last;
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = mx;
  __syncthreads();
  const unsigned nblk = gridDim.x * gridDim.y;
  if (threadIdx.x == 0) {
    unsigned long long m4 = wmax[0];
    for (int w = 1; w < 4; ++w) m4 = wmax[w] > m4 ? wmax[w] : m4;
    __hip_atomic_store(out + kAbsmaxPart + blockIdx.y * gridDim.x + blockIdx.x, m4, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long done =
        __hip_atomic_fetch_add(out + 2, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = done + 1 == nblk;
  }
  __syncthreads();
  if (!last) return;
  // the last workgroup: max over the partials of each signal (wave y = signal y)
  if (threadIdx.x < 128) {
    const int y = threadIdx.x >> 6, l = threadIdx.x & 63;
    unsigned long long r = 0;
    for (unsigned k = l; k < gridDim.x; k += 64) {
      const unsigned long long v =
          __hip_atomic_load(out + kAbsmaxPart + y * gridDim.x + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r = v > r ? v : r;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const unsigned long long t = __shfl_xor(r, o);
      r = t > r ? t : r;
    }
    if (l == 0) __hip_atomic_store(out + y, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) __hip_atomic_store(out + 2, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// One global Stockham pass of radix R (16 <= R <= 4096): F = BLOCK*16/R
// butterflies per workgroup.
// ---------------------------------------------------------------------------
// Pass shape.  V values per thread (FftPlan<R, V>); FW butterflies per
// workgroup (FftPlan's F, times AD_FFT_FWX).  Compile-time A/B knobs for
// tools/ builds only (the product library is built with the defaults).
#ifndef AD_FFT_V
#define AD_FFT_V 8
#endif
#ifndef AD_FFT_FWX
#define AD_FFT_FWX 2
#endif
// The real-output last pass at radix <= 256 (PassShape::SMALL_RO): 4 values per
// thread, two FftPlan tiles per workgroup (R = 128: 16 butterflies, 512 threads,
// 33 KiB of LDS).  CorrelateFFT 2 x 2^23, same box (profiles/r06_corr_ro_tile_ab.txt):
// V 8 / 2 tiles 0.4947, V 8 / 1 tile 0.4900-0.4914, V 4 / 2 tiles 0.4842-0.4854 ms
// per call; V 16 0.517-0.522.
#ifndef AD_FFT_V_RO
#define AD_FFT_V_RO 4
#endif
#ifndef AD_FFT_FWX_RO
#define AD_FFT_FWX_RO 2
#endif
#ifndef AD_FFT_PAIR
#define AD_FFT_PAIR 1  // mirror-paired tiles in the half inverse's first pass
#endif
#ifndef AD_FFT_TWC
#define AD_FFT_TWC 1  // twiddles computed in the kernel (no table loads after the data loads)
#endif
#ifndef AD_CORR_FUSED
#define AD_CORR_FUSED 1  // CorrelateFFT: forward last pass + half inverse first pass in one kernel
#endif
#ifndef AD_CORR_INV_V4
#define AD_CORR_INV_V4 1  // the fused kernel's inverse butterflies at 4 values per thread: all threads busy, 80 VGPRs (0.586 -> 0.571-0.575 ms same box)
#endif
#ifndef AD_FFT_PF
#define AD_FFT_PF 1  // plain radix-256 passes as a persistent kernel with the next tile's loads in flight
#endif
#ifndef AD_CORR_SPLIT
#define AD_CORR_SPLIT 1  // CorrelateFFT at N = 2^24: the max-abs inside the first pass (k_corr_split0)
#endif
#ifndef AD_SPLIT0_F
#define AD_SPLIT0_F 16  // k_corr_split0's columns per workgroup (8: 256 threads, 4 workgroups per CU)
#endif
#ifndef AD_PACKIN_NT
#define AD_PACKIN_NT 0
#endif
#ifndef AD_PACKIN_EXP
#define AD_PACKIN_EXP 0  // tools/ timing probes only (wrong results): 1 = mirror loads contiguous, 2 = stores contiguous
#endif
#ifndef AD_FFT_RO_VEC
#define AD_FFT_RO_VEC 1  // real-pair outputs in the lag order as 16-B stores
#endif
#ifndef AD_FFT_PF_V
#define AD_FFT_PF_V 8  // its values per thread (4: 1024-thread workgroups)
#endif
#ifndef AD_FFT_PF_F
#define AD_FFT_PF_F 16  // its butterflies per tile (PACKIN: half of them mirrors)
#endif
#ifndef AD_FFT_PF_RO
#define AD_FFT_PF_RO 0  // the last inverse pass (real outputs) persistent too: measured slower (0.551 -> 0.566-0.578 ms per call, profiles/r05_corr_pf_ro_ab.txt)
#endif
#ifndef AD_FFT_PF_RO_G
#define AD_FFT_PF_RO_G 1024  // its workgroups (R = 128: 33 KiB of LDS, four per CU)
#endif
#ifndef AD_FFT_PF_G
#define AD_FFT_PF_G 512  // its workgroups (2 per CU)
#endif
#ifndef AD_CORR_TW_EARLY
#define AD_CORR_TW_EARLY 1  // the fused kernel's twiddles from the tables, loaded ahead of its data
#endif
#ifndef AD_CORR_FUSED_PF
#define AD_CORR_FUSED_PF 0  // the fused kernel as a persistent grid with the next item's loads in flight
#endif
#ifndef AD_CORR_PF_AT
#define AD_CORR_PF_AT 1  // where it issues the next item's loads: 0 = after staging, 1 = after the forward pass
#endif
#ifndef AD_CORR_FUSED_PF_G
#define AD_CORR_FUSED_PF_G 1024  // its workgroups (4 per CU)
#endif
#ifndef AD_CORR_FUSED_NT
#define AD_CORR_FUSED_NT 256  // 2 inverse pairs per workgroup, 4 workgroups per CU (512: 0.530 -> 0.522-0.530 ms; 1024 slower)
#endif
// Pieces shared by k_fft_pass and the fused CorrelateFFT kernel below, so
// both round identically.
// Pre-twiddle of a pass (Ns > 1): v[slot s] *= W_{Ns R}^{(j mod Ns) r_s}.
// With u = W_N^{(j mod Ns) N/(Ns R)}, slot s holds r = tid + T k_s, where
// k_s = b + r0 V/R0 (pass0_index) runs over 0..V-1: w_s = u^tid (u^T)^k_s.
// Two twiddle evaluations per thread and a power recurrence in registers, not
// one per value; <= V roundings, far inside the 1e-10 parity bars.
// Split in two so a caller can evaluate the factors early (k_fft_pass_pf does
// it before its next tile's loads occupy registers); same operations either way.
template <int R, int V, bool FWD>
__device__ __forceinline__ void pretwiddle_uc(int64_t j, int64_t Ns, int64_t N, int tid, const double2* tw_lo,
                                              const double2* tw_hi, int S, double2* base_out, double2* c_out) {
  using Plan = FftPlan<R, V>;
  constexpr int T = Plan::T;
  const int64_t jm = j & (Ns - 1);
  // N, Ns and R are powers of two: shifts and an exact power-of-two scale
  // instead of a 64-bit integer division and a float64 division per call
  // (the same values: N / (Ns R) and e / N are exact either way)
  const int lgN = __builtin_ctzll((unsigned long long)N);
  const int64_t step = N >> (__builtin_ctzll((unsigned long long)Ns) + ilog2c(R));
  const int64_t mask = ((int64_t)1 << S) - 1;
  auto tw = [&](int64_t e) {
    e &= N - 1;
#if AD_FFT_TWC
    (void)mask;
    double sn, cs;
    sincospi(ldexp(-2.0 * (double)e, -lgN), &sn, &cs);  // -2 e / N, exact
    return make_double2(cs, sn);
#else
    return c_mul(tw_lo[e & mask], tw_hi[e >> S]);
#endif
  };
  double2 base = tw(jm * step * tid);  // u^tid
  const double2 cT = tw(jm * step * T);  // u^T
  *base_out = FWD ? base : c_conj(base);
  *c_out = FWD ? cT : c_conj(cT);
}
template <int R, int V>
__device__ __forceinline__ void pretwiddle_apply(double2* v, double2 base, const double2 c) {
  constexpr int R0 = FftPlan<R, V>::R0;
#pragma unroll
  for (int k = 0; k < V; ++k) {  // base = u^tid (u^T)^k
#pragma unroll
    for (int s = 0; s < V; ++s)
      if ((s / R0) + (s % R0) * (V / R0) == k) v[s] = c_mul(v[s], base);
    if (k + 1 < V) base = c_mul(base, c);
  }
}
template <int R, int V, bool FWD>
__device__ __forceinline__ void pass_pretwiddle(double2* v, int64_t j, int64_t Ns, int64_t N, int tid,
                                                const double2* tw_lo, const double2* tw_hi, int S) {
  double2 base, c;
  pretwiddle_uc<R, V, FWD>(j, Ns, N, tid, tw_lo, tw_hi, S, &base, &c);
  pretwiddle_apply<R, V>(v, base, c);
}
// The half inverse's input pieces (FftPassArgs::half): the correlation
// product X[q] = A conj(B) from the packed spectrum, A = (Z[q] + conj Z[-q]) / 2,
// B = (Z[q] - conj Z[-q]) / 2i; W_NF^-g; z = E + i O from X[g], X[g + NF/2].
__device__ __forceinline__ double2 corr_ab(double2 zk, double2 zm, double2* B) {
  *B = make_double2(0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x));
  return make_double2(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));
}
__device__ __forceinline__ double2 corr_xop(double2 zk, double2 zm) {
  double2 B;
  const double2 A = corr_ab(zk, zm, &B);
  return go_cmul(A, c_conj(B));
}
__device__ __forceinline__ double2 half_wneg(int64_t g, int64_t NF, const double2* ftw_lo, const double2* ftw_hi,
                                             int fS) {  // W_NF^-g
#if AD_FFT_TWC
  (void)ftw_lo, (void)ftw_hi, (void)fS;
  double sn, cs;
  sincospi(ldexp(2.0 * (double)g, -__builtin_ctzll((unsigned long long)NF)), &sn, &cs);  // 2 g / NF, exact
  return make_double2(cs, sn);
#else
  const int64_t fm = ((int64_t)1 << fS) - 1;
  return c_conj(c_mul(ftw_lo[g & fm], ftw_hi[g >> fS]));
#endif
}
__device__ __forceinline__ double2 half_zcomb(double2 x1, double2 x2, double2 w) {
  const double2 e = make_double2(0.5 * (x1.x + x2.x), 0.5 * (x1.y + x2.y));
  const double2 o = c_mul(make_double2(0.5 * (x1.x - x2.x), 0.5 * (x1.y - x2.y)), w);
  return make_double2(e.x - o.y, e.y + o.x);
}

// The last inverse pass's real outputs (REALOUT): element rr of butterfly jj
// of a tile of F butterflies, output index o, value val (LDS row stride MP).
template <int F>
__device__ __forceinline__ void realout_store(const FftPassArgs& a, const double2* lds_all, int MP, int jj, int rr,
                                              int64_t o, double2 val, int bt, double oscale, double oscale2,
                                              int64_t Ns, int64_t nb) {
  auto emit = [&](int64_t q, double x) {
    if (a.remap) {
      if (q < a.n_front)
        a.out_real[a.front_off + q] = x * oscale * oscale2;
      else if (q >= a.back_from)
        a.out_real[q - a.back_from] = x * oscale * oscale2;
    } else {
      a.out_real[bt * a.out_batch + q] = x * a.scale;
    }
  };
  if (AD_FFT_RO_VEC && a.remap && a.pairs && Ns >= F && nb % F == 0 && ((a.front_off + a.back_from) & 1) == 0) {
    // Real pairs into the lag order with 16-B stores.  For fixed rr the
    // tile's F butterflies give 2F consecutive reals q = 2o, 2o + 1, and
    // both region maps (q + front_off, q - back_from) shift q by amounts of
    // one parity (N is even), so whether (2o, 2o+1) lands on a 16-B slot
    // is the same for every element: `odd` = it does not, and lane jj then
    // owns the slot (2o - 1, 2o) (its left neighbour's Im and its Re); lane
    // 0 writes only its Re, lane F - 1 also its Im.  A slot whose two
    // reals do not land side by side (a region edge) is written per real.
    auto dst = [&](int64_t q) -> int64_t {
      return q < a.n_front ? a.front_off + q : (q >= a.back_from ? q - a.back_from : -1);
    };
    const bool odd = ((a.front_off + (int64_t)(((uintptr_t)a.out_real >> 3) & 1)) & 1) != 0;
    typedef double d2v __attribute__((ext_vector_type(2)));
    const double x = val.x * oscale * oscale2, y = val.y * oscale * oscale2;
    auto put2 = [&](int64_t ql, double lo, double hi) {  // reals ql, ql + 1
      const int64_t d0 = dst(ql), d1 = dst(ql + 1);
      if (d0 >= 0 && d1 == d0 + 1) {
        *reinterpret_cast<d2v*>(a.out_real + d0) = d2v{lo, hi};
      } else {
        if (d0 >= 0) a.out_real[d0] = lo;
        if (d1 >= 0) a.out_real[d1] = hi;
      }
    };
    if (!odd) {
      put2(2 * o, x, y);
    } else {
      if (jj > 0) {
        const double py = lds_all[(jj - 1) * MP + lds_slot(rr)].y * oscale * oscale2;
        put2(2 * o - 1, py, x);
      } else {
        const int64_t d0 = dst(2 * o);
        if (d0 >= 0) a.out_real[d0] = x;
      }
      if (jj == F - 1) {
        const int64_t d1 = dst(2 * o + 1);
        if (d1 >= 0) a.out_real[d1] = y;
      }
    }
  } else if (a.pairs) {
    emit(2 * o, val.x);
    emit(2 * o + 1, val.y);
  } else {
    emit(o, val.x);
  }
}

template <int R, bool RO = false>
struct PassShape {
  // the real-output last pass of a multi-pass plan (radix <= 256) has its own shape
  static constexpr bool SMALL_RO = RO && R <= 256;
  static constexpr int V = SMALL_RO ? AD_FFT_V_RO : AD_FFT_V;
  static constexpr int T = FftPlan<R, V>::T;
  static constexpr int F = FftPlan<R, V>::F * (SMALL_RO ? AD_FFT_FWX_RO : AD_FFT_FWX);
  static constexpr int BLOCK = F * T;
};
// HALF: the first inverse pass of the spectral row's half-length inverse
// (FftPassArgs::half), instantiated only where it can occur.
// PAIR (HALF only, Z = FFT(a + i b) packed, Ns = 1, not the last pass): the
// workgroup takes the butterfly tile [j0, j0 + F/2) and its Hermitian mirror
// tile {nb - j}: the four Z values a lane loads (Z[g], Z[g + NF/2] and their
// mirrors) give one element of each tile, so Z is read once instead of twice.
template <int R, bool FWD, bool REALIN, bool REALOUT, int HALF = 0, bool PAIR = false>
__global__ __launch_bounds__((PassShape<R, REALOUT>::BLOCK)) void k_fft_pass(FftPassArgs a) {
  using Sh = PassShape<R, REALOUT>;
  using Plan = FftPlan<R, Sh::V>;
  // per-butterfly LDS stride: odd when a 16-lane group stays inside one
  // transform (T >= 16), so the jj-fastest staging accesses spread over the banks
  constexpr int V = Sh::V, T = Plan::T, F = Sh::F, BLOCK = Sh::BLOCK, MP = Plan::MP + (T >= 16 ? 1 : 0);
  __shared__ __attribute__((aligned(16))) double2 lds_all[F * MP];
  __shared__ __attribute__((aligned(16))) double2 ltw[AD_FFT_TWC ? TwSplit<R>::N : 1];
  const int bt = blockIdx.y;
  const int64_t nb = a.N / R;  // butterflies
  // XCD-contiguous tiles: neighbouring butterfly tiles read neighbouring
  // runs of the same rows, so they share an L2 and DRAM pages
  const int64_t j0 = (int64_t)xcd_remap((int)blockIdx.x, (int)gridDim.x) * F;
#if AD_FFT_TWC
  const TwLds<R> twr = tw_lds_compute<R>(ltw, (int)threadIdx.x, BLOCK);
#else
  const TwGlobal twr{a.twR};
#endif

  // stage in: element r of butterfly j0 + jj is x[j0 + jj + r nb]; jj fastest
  const PackScale ps = REALIN ? pack_scale(a.amax) : PackScale{};
  // The half inverse's input (HALF): X[q] = op(A[q], B[q]) from the forward
  // spectrum Z = FFT(a + i b), A = (Z[q] + conj Z[-q]) / 2,
  // B = (Z[q] - conj Z[-q]) / 2i (HALF = 1: the correlation, op fixed; 2: any
  // op), then z[g] = E + i O with E = (X[g] + X[g + NF/2]) / 2 and
  // O = (X[g] - X[g + NF/2]) W_NF^-g / 2.  spec2 set: A and B come from two
  // separate transforms, in and spec2 (the division of Deconvolve must not
  // take B out of a transform that A dominates).
  const int64_t NF = a.NF, msk = NF - 1;
  auto xop = [&](double2 zk, double2 zm, int64_t q) {  // zk = Z[q], zm = Z[-q]
    if constexpr (HALF == 1) {
      return corr_xop(zk, zm);
    } else {
      double2 B;
      const double2 A = corr_ab(zk, zm, &B);
      return spec_op(a.op, A, B, a.eps, q, a.bad);
    }
  };
  auto xq = [&](int64_t q) {
    if (HALF == 2 && a.spec2) return spec_op(a.op, a.in[q], a.spec2[q], a.eps, q, a.bad);
    return xop(a.in[q], a.in[(NF - q) & msk], q);
  };
  auto wneg = [&](int64_t g) { return half_wneg(g, NF, a.ftw_lo, a.ftw_hi, a.fS); };
  auto zcomb = [&](double2 x1, double2 x2, double2 w) { return half_zcomb(x1, x2, w); };
  auto half_in = [&](int64_t g) { return zcomb(xq(g), xq(g + NF / 2), wneg(g)); };
  constexpr int FP = F / 2;  // PAIR: butterflies per tile
  const int64_t jp0 = PAIR ? j0 / 2 : 0;  // PAIR: tile A = [jp0, jp0 + FP)
  if constexpr (PAIR) {
    static_assert(HALF != 0 && !REALIN && !REALOUT, "PAIR: first pass of the half inverse only");
#pragma unroll
    for (int i = 0; i < V / 2; ++i) {
      const int idx = i * BLOCK + (int)threadIdx.x;
      const int jj = idx % FP, r = idx / FP;
      const int64_t j = jp0 + jj;
      double2 vA, vB;
      if (j == 0) {  // butterfly 0 is its own mirror; tile B's slot 0 takes butterfly nb/2 (also its own)
        vA = half_in((int64_t)r * nb);
        vB = half_in(nb / 2 + (int64_t)(R - 1 - r) * nb);
      } else {
        // element (j, r) of tile A and (nb - j, R - 1 - r) of tile B:
        //   g = j + r nb,  g* = NF/2 - g = (nb - j) + (R - 1 - r) nb
        const int64_t g = j + (int64_t)r * nb, gs = (nb - j) + (int64_t)(R - 1 - r) * nb;
        const double2 z1 = a.in[g], z2 = a.in[g + NF / 2];        // Z[g], Z[g + NF/2]
        const double2 z3 = a.in[gs], z4 = a.in[gs + NF / 2];      // Z[-(g + NF/2)], Z[-g]
        const double2 w = wneg(g);                                // W_NF^-g* = -conj(W_NF^-g)
        vA = zcomb(xop(z1, z4, g), xop(z2, z3, g + NF / 2), w);
        vB = zcomb(xop(z3, z2, gs), xop(z4, z1, gs + NF / 2), make_double2(-w.x, w.y));
      }
      lds_all[jj * MP + lds_slot(r)] = vA;
      lds_all[(FP + jj) * MP + lds_slot(R - 1 - r)] = vB;
    }
  } else {
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int idx = i * BLOCK + (int)threadIdx.x;
    const int jj = idx % F, r = idx / F;
    const int64_t j = j0 + jj;
    double2 v = make_double2(0.0, 0.0);
    if (j < nb) {
      const int64_t g = j + (int64_t)r * nb;
      if constexpr (REALIN) {
        if (a.pack2) {
          v.x = g < a.nr[0] ? a.xb[0][g] * ps.a : 0.0;
          v.y = g < a.nr[1] ? a.xb[1][g] * ps.b : 0.0;
        } else {
          v.x = g < a.nr[bt] ? a.xb[bt][g] : 0.0;
        }
      } else if constexpr (HALF != 0) {
        v = half_in(g);
      } else {
#if AD_FFT_NT >= 2
        typedef double d2v __attribute__((ext_vector_type(2)));
        const d2v t = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(a.in + bt * a.in_batch + g));
        v = make_double2(t.x, t.y);
#else
        v = a.in[bt * a.in_batch + g];
#endif
      }
    }
    lds_all[jj * MP + lds_slot(r)] = v;
  }
  }
  __syncthreads();

  const int f = threadIdx.x / T, tid = threadIdx.x % T;
  double2* lds = lds_all + f * MP;
  const int64_t j = j0 + f;
  double2 v[V];
#pragma unroll
  for (int s = 0; s < V; ++s) v[s] = lds[pass0_slot<R, V>(tid, s)];
  if (a.Ns > 1)  // pre-twiddle W_{Ns R}^{(j mod Ns) r} = W_N^{(j mod Ns) r N/(Ns R)}
    pass_pretwiddle<R, V, FWD>(v, j, a.Ns, a.N, tid, a.tw_lo, a.tw_hi, a.S);
  __syncthreads();
  fft_run<R, V, FWD>(v, tid, lds, twr);
  __syncthreads();
#pragma unroll
  for (int s = 0; s < V; ++s) lds[last_pass_slot<R, V>(tid, s)] = v[s];
  __syncthreads();

  // stage out: output rr of butterfly j goes to (j/Ns) Ns R + (j mod Ns) + rr Ns
  const int64_t Ns = a.Ns;
  const PackScale ops = REALOUT ? pack_scale(a.amax) : PackScale{};
  const double oscale = a.scale * ops.o1, oscale2 = ops.o2;  // powers of two: exact
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int idx = i * BLOCK + (int)threadIdx.x;
    int jj, rr;
    if (Ns == 1) {  // each butterfly's R outputs are contiguous
      rr = idx % R;
      jj = idx / R;
    } else {  // consecutive butterflies are contiguous for a fixed rr
      jj = idx % F;
      rr = idx / F;
    }
    int64_t jo = j0 + jj;
    if constexpr (PAIR) jo = jj < FP ? jp0 + jj : (jp0 + jj == FP ? nb / 2 : nb - jp0 - (jj - FP));
    if (jo >= nb) continue;
    const double2 val = lds_all[jj * MP + lds_slot(rr)];
    const int64_t o = (jo & ~(Ns - 1)) * R + (jo & (Ns - 1)) + (int64_t)rr * Ns;
    if constexpr (REALOUT) {
      realout_store<F>(a, lds_all, MP, jj, rr, o, val, bt, oscale, oscale2, Ns, nb);
    } else {
#if AD_FFT_NT  // non-temporal pass outputs (AD_FFT_NT above)
      typedef double d2v __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(d2v{val.x, val.y}, reinterpret_cast<d2v*>(a.out + bt * a.out_batch + o));
#else
      a.out[bt * a.out_batch + o] = val;
#endif
    }
  }
}

// Workgroup barrier for LDS hand-offs only: __syncthreads() is a workgroup
// release/acquire fence and waits for every outstanding global load and store
// of the wave (vmcnt(0)), which would drain the next tile's loads below.
__device__ __forceinline__ void pass_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <int M, int V, bool FWD, int P = 1, class TW>
__device__ __forceinline__ void run_middle_passes_lb(double2* v, int tid, double2* lds, const TW& twM) {
  using Plan = FftPlan<M, V>;
  if constexpr (P < Plan::NPASS) {
    pass_lds_barrier();
    pass_load<M, V, P>(v, tid, lds);
    if constexpr (P + 1 < Plan::NPASS) {
      pass_lds_barrier();
      pass_compute_store<M, V, P, FWD, TW>(v, tid, lds, twM);
      run_middle_passes_lb<M, V, FWD, P + 1, TW>(v, tid, lds, twM);
    }
  }
}
template <int M, int V, bool FWD, class TW>
__device__ __forceinline__ void fft_run_lb(double2* v, int tid, double2* lds, const TW& twM) {
  using Plan = FftPlan<M, V>;
  if constexpr (Plan::NPASS > 1) {
    pass_compute_store<M, V, 0, FWD, TW>(v, tid, lds, twM);
    run_middle_passes_lb<M, V, FWD, 1, TW>(v, tid, lds, twM);
  }
  last_pass_compute<M, V, FWD, TW>(v, tid, twM);
}

// A plain complex pass (not the first of a real-input transform, not the last
// of a real-output one, not the half inverse's first) as a persistent kernel:
// workgroup b takes tiles b, b + G, b + 2G, ... and holds the next tile's
// inputs in registers while it transforms the current one, so its loads stay
// in flight under the LDS passes (barriers wait on LDS only).  Same
// arithmetic as k_fft_pass in the same order: bit-identical results.
// Requires nb % F == 0 (whole tiles) and Ns == 1 or Ns >= F.
template <int R>
struct PfShape {  // k_fft_pass_pf: AD_FFT_PF_V values per thread, 16 butterflies per tile
  static constexpr int V = AD_FFT_PF_V;
  static constexpr int T = FftPlan<R, V>::T;
  static constexpr int F = AD_FFT_PF_F;
  static constexpr int BLOCK = F * T;
};
// PACKIN (CorrelateFFT's second forward pass after k_corr_split0, Ns = that
// pass's radix K0): the input holds each first-pass column's real
// transforms A, B in the split slot form, and butterfly j = cg K0 + k of
// this pass reads slot k of its rows, so the butterflies k and K0 - k read
// the same two slots {k, K0 - k} (A[k] and B[k]).  A tile is 8 butterflies
// k = kb .. kb+7 (kb < K0/2) and their 8 mirrors K0 - k (K0/2 for k = 0):
// each pair of loads gives z[k] = sa A + i sb B and z[K0-k] = sa conj(A) +
// i sb conj(B) (sa, sb from the first pass's max-abs partials), the packed
// first-pass output the plain form would read.
template <int R, bool FWD, bool PACKIN = false, bool REALOUT = false>
__global__ __launch_bounds__((PfShape<R>::BLOCK)) __attribute__((amdgpu_waves_per_eu(4))) void k_fft_pass_pf(
    FftPassArgs a, int tiles) {
  using Sh = PfShape<R>;
  using Plan = FftPlan<R, Sh::V>;
  constexpr int V = Sh::V, T = Plan::T, F = Sh::F, BLOCK = Sh::BLOCK, MP = Plan::MP + (T >= 16 ? 1 : 0);
  static_assert(BLOCK % R == 0, "k_fft_pass_pf: whole butterflies per store row");
  static_assert(!PACKIN || (V % 2 == 0 && F % 2 == 0), "PACKIN: load pairs, F/2 butterflies + their mirrors per tile");
  static_assert(!(PACKIN && REALOUT), "PACKIN is a forward pass, REALOUT the last inverse one");
  // REALOUT (the last pass of a real-output inverse, Ns >= F): the scales of
  // the packed pair (pack_scale of the first pass's max-abs) once per workgroup
  const PackScale ops = REALOUT ? pack_scale(a.amax) : PackScale{};
  const double oscale = a.scale * ops.o1, oscale2 = ops.o2;
  constexpr int H = F / 2;  // PACKIN: butterflies per half tile
  __shared__ __attribute__((aligned(16))) double2 lds_all[F * MP];
  __shared__ __attribute__((aligned(16))) double2 ltw[TwSplit<R>::N];
  const int64_t nb = a.N / R, Ns = a.Ns;
  const double2* in = a.in + blockIdx.y * a.in_batch;
  double2* out = a.out + blockIdx.y * a.out_batch;
  const TwLds<R> twr = tw_lds_compute<R>(ltw, (int)threadIdx.x, BLOCK);
  const int G = (int)gridDim.x;
  int tile = xcd_remap((int)blockIdx.x, G);
  typedef double d2v __attribute__((ext_vector_type(2)));  // (a double2 struct copy becomes a memcpy through scratch)
  d2v pf[V];
  // PACKIN tiles: column group cg, butterflies kb .. kb+7 and their mirrors
  const int tpg = PACKIN ? (int)(Ns / F) : 1;  // tiles per column group
  auto kmir = [&](int k) { return k == 0 ? (int)(Ns / 2) : (int)Ns - k; };
  // element (jj, r) of tile t is in[t F + jj + r nb]; idx = i BLOCK + thread
  // gives jj = thread % F, r = i BLOCK / F + thread / F: a wave-uniform base
  // per i plus one 32-bit lane offset (global loads with an SGPR base).
  // PACKIN: e = i BLOCK + thread (i < V/2), jj = e % 8, r = e / 8: slots
  // kb + jj and kmir(kb + jj) of row cg Ns + r nb.
#define AD_PF_LOAD(t, tx)                                                                         \
  {                                                                                               \
  if constexpr (PACKIN) {                                                                         \
    const int64_t cg = (t) / tpg;                                                                  \
    const int kb = H * ((t) % tpg), k = kb + (tx) % H;                                             \
    const int64_t lane = (int64_t)((tx) / H) * nb;                                                 \
    _Pragma("unroll") for (int i = 0; i < V / 2; ++i) {                                           \
      const d2v* row = reinterpret_cast<const d2v*>(in + cg * Ns + (int64_t)(i * (BLOCK / H)) * nb + lane); \
      pf[2 * i] = row[k];                                                                         \
      pf[2 * i + 1] = row[AD_PACKIN_EXP == 1 ? k + H : kmir(k)];                                   \
    }                                                                                             \
  } else {                                                                                        \
    const uint32_t lane_off = (uint32_t)(((int64_t)((tx) % F) + (int64_t)((tx) / F) * nb) * 16);   \
    _Pragma("unroll") for (int i = 0; i < V; ++i) {                                               \
      const char* base = reinterpret_cast<const char*>(in + (int64_t)(t) * F + (int64_t)(i * (BLOCK / F)) * nb); \
      pf[i] = *reinterpret_cast<const d2v*>(base + lane_off);                                     \
    }                                                                                             \
  }                                                                                               \
  }
  if (tile < tiles) AD_PF_LOAD(tile, (int)threadIdx.x)
  // PACKIN: the packing scales from the first pass's partials (every
  // workgroup reduces all of them; workgroup 0 also stores the totals at
  // amax[0..1] for the last inverse pass)
  PackScale ps{};
  if constexpr (PACKIN) {
    __shared__ unsigned long long wred[2][BLOCK / 64];
    // 16-B loads, all of a thread's in flight at once (with the first tile's):
    // one memory round trip, not one per loop trip (every workgroup starts here)
    unsigned long long ma = 0, mb = 0;
    const ulonglong2* pa = reinterpret_cast<const ulonglong2*>(a.amax_part);  // amax + 8 words: 16-B aligned
    const int n2 = a.amax_parts / 2;  // even (host)
    constexpr int U = 8;
    for (int b0 = 0; b0 < n2; b0 += U * BLOCK) {
      ulonglong2 va[U], vb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // clamped, not guarded: a repeated partial leaves the max as it is
        const int i = min(b0 + u * BLOCK + (int)threadIdx.x, n2 - 1);
        va[u] = pa[i];
        vb[u] = pa[n2 + i];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        ma = va[u].x > ma ? va[u].x : ma;
        ma = va[u].y > ma ? va[u].y : ma;
        mb = vb[u].x > mb ? vb[u].x : mb;
        mb = vb[u].y > mb ? vb[u].y : mb;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const unsigned long long ta = __shfl_xor(ma, o), tb = __shfl_xor(mb, o);
      ma = ta > ma ? ta : ma;
      mb = tb > mb ? tb : mb;
    }
    if ((threadIdx.x & 63) == 0) {
      wred[0][threadIdx.x >> 6] = ma;
      wred[1][threadIdx.x >> 6] = mb;
    }
    __syncthreads();
    ma = 0;
    mb = 0;
    for (int w = 0; w < BLOCK / 64; ++w) {
      ma = wred[0][w] > ma ? wred[0][w] : ma;
      mb = wred[1][w] > mb ? wred[1][w] : mb;
    }
    ps = pack_scale_bits(ma, mb);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      unsigned long long* tot = const_cast<unsigned long long*>(a.amax);
      tot[0] = ma;
      tot[1] = mb;
    }
  }
  for (; tile < tiles; tile += G) {
    // the thread index through an opaque copy each tile: its LDS and global
    // offsets are recomputed per tile (a few VALU ops) instead of ~30 of them
    // staying live across the loop and spilling beside the prefetch registers
    int tx;
    asm volatile("v_mov_b32 %0, %1" : "=v"(tx) : "v"((int)threadIdx.x));
    const int f = tx / T, tid = tx % T;
    double2* lds = lds_all + f * MP;
    const int64_t j0 = (int64_t)tile * F;
    const int64_t cg = PACKIN ? tile / tpg : 0;
    const int kb = PACKIN ? H * (tile % tpg) : 0;
    // butterfly of tile slot s (PACKIN: kb + s, then the mirrors)
    auto jbut = [&](int sl) -> int64_t {
      if constexpr (PACKIN) return cg * Ns + (sl < H ? kb + sl : kmir(kb + sl - H));
      return j0 + sl;
    };
    double2 twb, twc;  // pre-twiddle factors, evaluated before the next tile's loads take their registers
    if (Ns > 1) pretwiddle_uc<R, V, FWD>(jbut(f), Ns, a.N, tid, a.tw_lo, a.tw_hi, a.S, &twb, &twc);
    pass_lds_barrier();  // the previous tile's stage-out reads (and the twiddle tables) are done
    if constexpr (PACKIN) {
#pragma unroll
      for (int i = 0; i < V / 2; ++i) {
        const int e = i * BLOCK + tx, jj = e % H, r = e / H;
        const d2v A = pf[2 * i], B = pf[2 * i + 1];
        // k > 0: A = A[k], B = B[k]: z[k] = sa A + i sb B, z[K0-k] = sa conj(A) + i sb conj(B).
        // k = 0: slots 0 and K0/2 hold the real pairs (A[0], B[0]) and (A[K0/2], B[K0/2]).
        // Selects, not branches (a branch here makes the compiler drain the loads).
        const bool self = kb + jj == 0;
        const double ax = ps.a * A.x, ay = ps.a * A.y, bx = ps.b * B.x, by = ps.b * B.y;
        const double2 zA = self ? make_double2(ax, ps.b * A.y) : make_double2(ax - by, ay + bx);
        const double2 zB = self ? make_double2(ps.a * B.x, by) : make_double2(ax + by, bx - ay);
        lds_all[jj * MP + lds_slot(r)] = zA;
        lds_all[(H + jj) * MP + lds_slot(r)] = zB;
      }
    } else {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int idx = i * BLOCK + tx;
        lds_all[(idx % F) * MP + lds_slot(idx / F)] = make_double2(pf[i].x, pf[i].y);
      }
    }
    if (tile + G < tiles) AD_PF_LOAD(tile + G, tx)
    pass_lds_barrier();
    double2 v[V];
#pragma unroll
    for (int s = 0; s < V; ++s) v[s] = lds[pass0_slot<R, V>(tid, s)];
    if (Ns > 1) pretwiddle_apply<R, V>(v, twb, twc);
    pass_lds_barrier();
    fft_run_lb<R, V, FWD>(v, tid, lds, twr);
    pass_lds_barrier();
#pragma unroll
    for (int s = 0; s < V; ++s) lds[last_pass_slot<R, V>(tid, s)] = v[s];
    pass_lds_barrier();
    // output rr of butterfly j0 + jj goes to (jo & ~(Ns-1)) R + (jo & (Ns-1)) + rr Ns:
    // Ns = 1: contiguous (o = j0 R + idx); Ns >= F: the tile sits in one Ns group, so
    // o = (j0 & ~(Ns-1)) R + (j0 & (Ns-1)) + i (BLOCK/F) Ns + [jj + (thread/F) Ns]
    if constexpr (REALOUT) {  // Ns >= F (launch condition): jj = idx % F, rr = idx / F
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int idx = i * BLOCK + tx, jj = idx % F, rr = idx / F;
        const int64_t jo = j0 + jj;
        const double2 val = lds_all[jj * MP + lds_slot(rr)];
        const int64_t o = (jo & ~(Ns - 1)) * R + (jo & (Ns - 1)) + (int64_t)rr * Ns;
        realout_store<F>(a, lds_all, MP, jj, rr, o, val, (int)blockIdx.y, oscale, oscale2, Ns, nb);
      }
    } else if constexpr (PACKIN) {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int idx = i * BLOCK + tx, jj = idx % F, rr = idx / F;
        const int64_t jo = AD_PACKIN_EXP == 2 ? cg * Ns + 2 * kb + jj : jbut(jj);
        const double2 val = lds_all[jj * MP + lds_slot(rr)];
        const int64_t o = (jo & ~(Ns - 1)) * R + (jo & (Ns - 1)) + (int64_t)rr * Ns;
        // the mirror run [K0-kb-7, K0-kb] is one element off the 128-B lines: its
        // partial lines are completed by the neighbouring tile (same XCD), so
        // they are stored through the L2 (write-back merges them) unless
        // AD_PACKIN_NT (non-temporal: partial-line writes reach memory)
        if (AD_PACKIN_NT)
          __builtin_nontemporal_store(d2v{val.x, val.y}, reinterpret_cast<d2v*>(out + o));
        else
          *reinterpret_cast<d2v*>(out + o) = d2v{val.x, val.y};
      }
    } else if (Ns == 1) {
      d2v* dst = reinterpret_cast<d2v*>(out + j0 * R) + tx;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int idx = i * BLOCK + tx;
        const double2 val = lds_all[(idx / R) * MP + lds_slot(idx % R)];
        __builtin_nontemporal_store(d2v{val.x, val.y}, dst + i * BLOCK);
      }
    } else {
      const int64_t ob = (j0 & ~(Ns - 1)) * R + (j0 & (Ns - 1)), ostep = (int64_t)(BLOCK / F) * Ns;
      const uint32_t olane = (uint32_t)((tx % F) + (int64_t)(tx / F) * Ns);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int idx = i * BLOCK + tx;
        const double2 val = lds_all[(idx % F) * MP + lds_slot(idx / F)];
        __builtin_nontemporal_store(d2v{val.x, val.y}, reinterpret_cast<d2v*>(out + ob + i * ostep) + olane);
      }
    }
  }
#undef AD_PF_LOAD
}

// CorrelateFFT's first forward pass with the max-abs folded in (the "split"
// form; VERDICT r4's CorrelateFFT item: k_absmax2 read a and b, 134 MB, only
// for the packing scale).  The packed transform Z = FFT(sa a + i sb b) needs
// sa, sb before the first pass, but the pass is linear: its butterfly j (a
// column a_j[r] = a[j + r nb] of 256 samples) is computed here as two REAL
// 256-point transforms A_j = DFT(a_j), B_j = DFT(b_j), unscaled, each paired
// with its neighbour column in one complex FFT (a_j + i a_{j+1}; the
// Hermitian split A = (Z_k + conj Z_-k)/2, A' = (Z_k - conj Z_-k)/2i), so a
// and b never share a transform before the scale is known.  Real inputs give
// A_j[256 - k] = conj A_j[k]: slot k of the butterfly's 256 outputs holds
//   k = 1..127:   A_j[k]          k = 129..255: B_j[256 - k]
//   k = 0:        (A_j[0], B_j[0])   k = 128:   (A_j[128], B_j[128])   (all real)
// the same 256 complex values as before.  The workgroup's max|a|, max|b| go
// to amax[8 + blk], amax[8 + gridDim.x + blk]; the second pass
// (k_fft_pass_pf's PACKIN form) reduces them and forms
// sa A_j[k] + i sb B_j[k] = the packed pass-0 output at its load.
template <int R, int FT>
__global__ __launch_bounds__((FT * FftPlan<R, 8>::T)) void k_corr_split0(FftPassArgs a) {
  using Plan = FftPlan<R, 8>;
  constexpr int V = 8, T = Plan::T, F = FT, BLOCK = F * T, MP = Plan::MP + (T >= 16 ? 1 : 0), NP = F / 2;
  static_assert(F % 2 == 0 && BLOCK % R == 0, "k_corr_split0: column pairs of a and of b, whole output rows");
  __shared__ __attribute__((aligned(16))) double2 lds_all[F * MP];
  __shared__ __attribute__((aligned(16))) double2 ltw[TwSplit<R>::N];
  __shared__ unsigned long long wmax[2][BLOCK / 64];
  const int64_t nb = a.N / R;
  const int64_t j0 = (int64_t)xcd_remap((int)blockIdx.x, (int)gridDim.x) * F;
  const TwLds<R> twr = tw_lds_compute<R>(ltw, (int)threadIdx.x, BLOCK);
  // stage in: columns 2p, 2p + 1 of a -> FFT p (re, im), of b -> FFT F/2 + p; a
  // lane takes one column pair of one row (one 16-B LDS write); slots i < V/2
  // are a's, the rest b's
  // two 8-B loads per pair (one 16-B load where aligned measured the same:
  // profiles/r04_split_ab3.txt), all issued before the LDS writes
  unsigned long long mxa = 0, mxb = 0;
  double2 xv[V];
  const int pp = (int)threadIdx.x % NP;
  {
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int sg = i / (V / 2), r = (i % (V / 2)) * (BLOCK / NP) + (int)threadIdx.x / NP;
      const double* x = a.xb[sg];
      const int64_t nr = a.nr[sg], g = j0 + 2 * pp + (int64_t)r * nb;
      xv[i] = make_double2(g < nr ? x[g] : 0.0, g + 1 < nr ? x[g + 1] : 0.0);
    }
  }
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int sg = i / (V / 2), r = (i % (V / 2)) * (BLOCK / NP) + (int)threadIdx.x / NP;
    const unsigned long long u0 = (unsigned long long)__double_as_longlong(fabs(xv[i].x));
    const unsigned long long u1 = (unsigned long long)__double_as_longlong(fabs(xv[i].y));
    const unsigned long long u = u0 > u1 ? u0 : u1;
    if (sg == 0)
      mxa = u > mxa ? u : mxa;
    else
      mxb = u > mxb ? u : mxb;
    lds_all[(sg * (F / 2) + pp) * MP + lds_slot(r)] = xv[i];
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long ta = __shfl_xor(mxa, o), tb = __shfl_xor(mxb, o);
    mxa = ta > mxa ? ta : mxa;
    mxb = tb > mxb ? tb : mxb;
  }
  if ((threadIdx.x & 63) == 0) {
    wmax[0][threadIdx.x >> 6] = mxa;
    wmax[1][threadIdx.x >> 6] = mxb;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    unsigned long long m = 0;
    for (int w = 0; w < BLOCK / 64; ++w) m = wmax[threadIdx.x][w] > m ? wmax[threadIdx.x][w] : m;
    a.amax_part[threadIdx.x * gridDim.x + blockIdx.x] = m;
  }
  const int f = threadIdx.x / T, tid = threadIdx.x % T;
  double2* lds = lds_all + f * MP;
  double2 v[V];
#pragma unroll
  for (int s = 0; s < V; ++s) v[s] = lds[pass0_slot<R, V>(tid, s)];
  __syncthreads();
  fft_run<R, V, true>(v, tid, lds, twr);
  __syncthreads();
#pragma unroll
  for (int s = 0; s < V; ++s) lds[last_pass_slot<R, V>(tid, s)] = v[s];
  __syncthreads();
  // stage out (Ns = 1): slot k of column j0 + jj at (j0 + jj) R + k, contiguous
  auto split = [&](int fi, int k, int second) {  // DFT of FFT fi's re (second = 0) or im input at bin k
    const double2 zk = lds_all[fi * MP + lds_slot(k)], zm = lds_all[fi * MP + lds_slot((R - k) & (R - 1))];
    double2 B;
    const double2 A = corr_ab(zk, zm, &B);
    return second ? B : A;
  };
  typedef double d2v __attribute__((ext_vector_type(2)));
  d2v* dst = reinterpret_cast<d2v*>(a.out + j0 * R) + threadIdx.x;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int idx = i * BLOCK + (int)threadIdx.x;
    const int k = idx % R, jj = idx / R;
    const int fa = jj / 2, fb = F / 2 + jj / 2, c = jj & 1;
    // k < R/2: A[k] (k = 0: its pair with B[0] below); k >= R/2: B[R - k]
    // (k = R/2: its pair with A[R/2]).  Lanes k = 0, R/2 are lane 0 of their
    // wave: one short divergent step instead of a three-way split of the body.
    const bool lo = k < R / 2;
    double2 val = split(lo ? fa : fb, lo ? k : R - k, c);
    if (k == 0 || k == R / 2) {
      const double2 o = split(lo ? fb : fa, k, c);
      val = lo ? make_double2(val.x, o.x) : make_double2(o.x, val.x);
    }
    __builtin_nontemporal_store(d2v{val.x, val.y}, dst + i * BLOCK);
  }
}

// CorrelateFFT: the forward transform's last pass fused with the half
// inverse's first pass (the 2 x 268 MB round trip of the packed
// spectrum Z through HBM at N = 2^24).  Both passes have radix R; the forward
// pass has nbF = N/R butterflies (Ns = nbF: butterfly j writes
// Z[j + nbF k]), the half inverse's first pass nbH = NH/R = nbF/2 (Ns = 1:
// butterfly j' reads z[j' + nbH r] and writes its R outputs contiguously).
// z[g] needs X[g] and X[g + NH], X[q] needs Z[q] and Z[-q]: with
// g = j' + nbH r, Z[g] and Z[g + NH] are outputs r/2 and r/2 + R/2 of forward
// butterfly j' (r even) or j' + nbH (r odd), and Z[-g], Z[-(g + NH)] those of
// butterflies nbF - j' / nbH - j'.  The inverse butterfly pair {j', nbH - j'}
// (the mirror tiles of k_fft_pass's PAIR form) needs exactly the four forward
// butterflies {j', j' + nbH, nbF - j', nbH - j'} (for j' = 0: {0, nbH, nbH/2,
// 3 nbH/2}, the pair {0, nbH/2}).  A workgroup of NT threads takes
// FP = NT/128 inverse pairs (NT = 256: 2, four workgroups per CU): it loads
// the 4 FP forward butterflies' inputs (runs of FP values), runs the forward
// pass with k_fft_pass's arithmetic, keeps Z in LDS, forms z with the PAIR
// form's arithmetic, runs the 2 FP inverse butterflies (at 4 values per
// thread with AD_CORR_INV_V4: every wave busy) and stores their outputs
// contiguously.  Z never reaches memory.  The forward half is bit-identical
// to k_fft_pass; the 4-value inverse rounds differently from the 8-value
// pass (a 4.4.4.4 factoring of the radix-256 butterfly).
struct CorrFusedArgs {
  const double2* in;  // the forward transform's next-to-last pass output [N]
  double2* out;       // the half inverse's first-pass output [NH]
  int64_t N;          // forward size (NH = N/2)
  const double2* tw_lo;  // forward plan's pre-twiddle tables (AD_FFT_TWC = 0 builds)
  const double2* tw_hi;
  int S;
  const double2* htw_lo;  // W_NF tables for W_NF^-g (AD_FFT_TWC = 0 builds)
  const double2* htw_hi;
  int hS;
};
// fft_run_active with LDS-only barriers (the persistent form below keeps its
// next item's loads in flight across them).
template <int M, int V, bool FWD, int P = 1, class TW>
__device__ __forceinline__ void run_middle_passes_active_lb(double2* v, int tid, double2* lds, const TW& twM, bool active) {
  using Plan = FftPlan<M, V>;
  if constexpr (P < Plan::NPASS) {
    pass_lds_barrier();
    if (active) pass_load<M, V, P>(v, tid, lds);
    if constexpr (P + 1 < Plan::NPASS) {
      pass_lds_barrier();
      if (active) pass_compute_store<M, V, P, FWD, TW>(v, tid, lds, twM);
      run_middle_passes_active_lb<M, V, FWD, P + 1, TW>(v, tid, lds, twM, active);
    }
  }
}
template <int M, int V, bool FWD, class TW>
__device__ __forceinline__ void fft_run_active_lb(double2* v, int tid, double2* lds, const TW& twM, bool active) {
  using Plan = FftPlan<M, V>;
  if constexpr (Plan::NPASS > 1) {
    if (active) pass_compute_store<M, V, 0, FWD, TW>(v, tid, lds, twM);
    run_middle_passes_active_lb<M, V, FWD, 1, TW>(v, tid, lds, twM, active);
  }
  if (active) last_pass_compute<M, V, FWD, TW>(v, tid, twM);
}

template <int R, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 512 ? 4 : 4))) void k_corr_fwd_last_inv_first(CorrFusedArgs a) {
  constexpr int V = 8;
  using Plan = FftPlan<R, V>;
  constexpr int T = Plan::T;          // threads per butterfly
  constexpr int NBF = NT / T;         // forward butterflies per workgroup
  constexpr int FP = NBF / 4;         // inverse butterfly pairs per workgroup
  constexpr int MP = Plan::MP + (T >= 16 ? 1 : 0);
  static_assert(FP >= 1 && 2 * FP <= NBF, "fused CorrelateFFT pass shape");
  __shared__ __attribute__((aligned(16))) double2 lds_all[NBF * MP];
  __shared__ __attribute__((aligned(16))) double2 ltw[AD_FFT_TWC ? TwSplit<R>::N : 1];
  const int64_t N = a.N, NH = N / 2, nbF = N / R, nbH = nbF / 2;
  const int64_t jp0 = (int64_t)xcd_remap((int)blockIdx.x, (int)gridDim.x) * FP;
  const TwLds<R> twr = tw_lds_compute<R>(ltw, (int)threadIdx.x, NT);
  // forward butterfly of slot b = set * FP + jj (set: j', j' + nbH, nbF - j', nbH - j')
  auto fbut = [&](int b) -> int64_t {
    const int set = b / FP;
    const int64_t j = jp0 + (b % FP);
    if (set == 0) return j;
    if (set == 1) return j + nbH;
    if (set == 2) return j == 0 ? nbH / 2 : nbF - j;
    return j == 0 ? 3 * (nbH / 2) : nbH - j;
  };
  constexpr int NPAIR = FP * R / NT;  // (jj, r) pairs per thread in step 3
#if AD_CORR_TW_EARLY
  // The twiddles of steps 2 and 3 from the W_N table pair, loaded ahead of the
  // data (vmcnt retires in order: they land with it), instead of four FP64
  // sincospi per thread on the VALU.  Step 2's pre-twiddle (Ns = nbF, so
  // j mod Ns = j and N / (Ns R) = 1): u^tid and u^T with u = W_N^j; step 3's
  // W_N^-g, g = j' + r nbH.
  const int64_t tmask = ((int64_t)1 << a.S) - 1, hmask = ((int64_t)1 << a.hS) - 1;
  const int64_t jf = fbut((int)threadIdx.x / T);
  const int64_t e1 = (jf * ((int)threadIdx.x % T)) & (N - 1), e2 = (jf * T) & (N - 1);
  const double2 tl1 = a.tw_lo[e1 & tmask], th1 = a.tw_hi[e1 >> a.S];
  const double2 tl2 = a.tw_lo[e2 & tmask], th2 = a.tw_hi[e2 >> a.S];
  double2 zl[NPAIR], zh[NPAIR];
#pragma unroll
  for (int i = 0; i < NPAIR; ++i) {
    const int idx = i * NT + (int)threadIdx.x;
    const int64_t g = jp0 + idx % FP + (int64_t)(idx / FP) * nbH;
    zl[i] = a.htw_lo[g & hmask];
    zh[i] = a.htw_hi[g >> a.hS];
  }
#endif
  // 1. stage the forward butterflies' inputs: element r of slot b is in[fbut(b) + r nbF]
  static_assert(NT % NBF == 0, "staging: b = tid mod NBF for every i");
  const int sb1 = lds_slot((int)threadIdx.x / NBF);  // r = i NT / NBF + tid / NBF: disjoint bits
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int idx = i * NT + (int)threadIdx.x;
    const int b = idx % NBF, r = idx / NBF;
    lds_all[b * MP + lds_slot_split(sb1, i * (NT / NBF))] = a.in[fbut(b) + (int64_t)r * nbF];
  }
  __syncthreads();
  // 2. the forward last pass (k_fft_pass<R, true, ...> with Ns = nbF)
  const int fs = (int)threadIdx.x / T, tid = (int)threadIdx.x % T;
  double2* lds = lds_all + fs * MP;
  double2 v[V];
#pragma unroll
  for (int s = 0; s < V; ++s) v[s] = lds[pass0_slot<R, V>(tid, s)];
#if AD_CORR_TW_EARLY
  pretwiddle_apply<R, V>(v, c_mul(tl1, th1), c_mul(tl2, th2));
#else
  pass_pretwiddle<R, V, true>(v, fbut(fs), nbF, N, tid, a.tw_lo, a.tw_hi, a.S);
#endif
  __syncthreads();
  fft_run<R, V, true>(v, tid, lds, twr);
  __syncthreads();
#pragma unroll
  for (int s = 0; s < V; ++s) lds[last_pass_slot<R, V>(tid, s)] = v[s];  // Z[fbut(fs) + nbF k]
  __syncthreads();
  // 3. z for the inverse pairs (k_fft_pass's PAIR form): element (jj, r) of
  //    tile A and (jj, R-1-r) of tile B; Z of slot b, output k:
  auto zs = [&](int b, int k) { return lds_all[b * MP + lds_slot(k)]; };
  auto zq = [&](int64_t q) {  // Z[q] for the j' = 0 pair (any of its four butterflies)
    const int64_t fb = q & (nbF - 1);
    const int k = (int)(q / nbF);
    const int set = fb == 0 ? 0 : fb == nbH ? 1 : fb == nbH / 2 ? 2 : 3;
    return zs(set * FP, k);
  };
  auto half_in0 = [&](int64_t g) {  // half_in of k_fft_pass for the j' = 0 pair
    const double2 x1 = corr_xop(zq(g), zq((N - g) & (N - 1)));
    const double2 x2 = corr_xop(zq(g + NH), zq((N - g - NH) & (N - 1)));
    return half_zcomb(x1, x2, half_wneg(g, N, a.htw_lo, a.htw_hi, a.hS));
  };
  double2 vA[NPAIR], vB[NPAIR];
#pragma unroll
  for (int i = 0; i < NPAIR; ++i) {
    const int idx = i * NT + (int)threadIdx.x;
    const int jj = idx % FP, r = idx / FP;
    const int64_t j = jp0 + jj;
    if (j == 0) {
      vA[i] = half_in0((int64_t)r * nbH);
      vB[i] = half_in0(nbH / 2 + (int64_t)(R - 1 - r) * nbH);
    } else {
      const int odd = r & 1, k1 = r >> 1, k3 = (R - 1 - r) >> 1;
      // k1, k3 < R / 2: the slots of k + R / 2 are one XOR away (lds_slot_split)
      const int s1 = lds_slot(k1), s3 = lds_slot(k3);
      const double2* z13 = lds_all + (odd * FP + jj) * MP;
      const double2* z34 = lds_all + ((2 + odd) * FP + jj) * MP;
      const double2 z1 = z13[s1], z2 = z13[lds_slot_split(s1, R / 2)];  // Z[g], Z[g + NH]
      // gs = (nbH - j) + (R-1-r) nbH: forward butterfly nbF - j (r even, set 2) or nbH - j (r odd, set 3)
      const double2 z3 = z34[s3], z4 = z34[lds_slot_split(s3, R / 2)];  // Z[-(g + NH)], Z[-g]
#if AD_CORR_TW_EARLY
      const double2 w = c_conj(c_mul(zl[i], zh[i]));  // W_N^-g, g = j + r nbH
#else
      const int64_t g = j + (int64_t)r * nbH;
      const double2 w = half_wneg(g, N, a.htw_lo, a.htw_hi, a.hS);  // W_NF^-g* = -conj(W_NF^-g)
#endif
      vA[i] = half_zcomb(corr_xop(z1, z4), corr_xop(z2, z3), w);
      vB[i] = half_zcomb(corr_xop(z3, z2), corr_xop(z4, z1), make_double2(-w.x, w.y));
    }
  }
  __syncthreads();  // every Z read is done: the inverse staging reuses slots 0 .. 2 FP - 1
#pragma unroll
  for (int i = 0; i < NPAIR; ++i) {
    const int idx = i * NT + (int)threadIdx.x;
    const int jj = idx % FP, r = idx / FP;
    const int sr = lds_slot(r);  // R - 1 - r == r ^ (R - 1): one XOR away
    lds_all[jj * MP + sr] = vA[i];
    lds_all[(FP + jj) * MP + lds_slot_split(sr, R - 1)] = vB[i];
  }
  __syncthreads();
  // 4. the inverse first pass (Ns = 1: no pre-twiddle) on slots 0 .. 2 FP - 1:
  //    2 FP butterflies over all NT threads at VI values per thread
#if AD_CORR_INV_V4
  constexpr int VI = 4;
#else
  constexpr int VI = V;
#endif
  using PlanI = FftPlan<R, VI>;
  constexpr int TI = PlanI::T;
  const int fi = (int)threadIdx.x / TI, ti = (int)threadIdx.x % TI;
  double2* ldsi = lds_all + fi * MP;
  const bool act = fi < 2 * FP;  // wave-uniform (TI is a multiple of the wave or divides it)
  double2 u[VI];
  if (act) {
#pragma unroll
    for (int s = 0; s < VI; ++s) u[s] = ldsi[pass0_slot<R, VI>(ti, s)];
  }
  __syncthreads();
  fft_run_active<R, VI, false>(u, ti, ldsi, twr, act);
  __syncthreads();
  if (act) {
#pragma unroll
    for (int s = 0; s < VI; ++s) ldsi[last_pass_slot<R, VI>(ti, s)] = u[s];
  }
  __syncthreads();
  // 5. outputs: inverse butterfly jo's R values at jo R .. jo R + R - 1
#pragma unroll
  for (int i = 0; i < 2 * FP * R / NT; ++i) {
    const int idx = i * NT + (int)threadIdx.x;
    const int rr = idx % R, jj = idx / R;
    const int64_t jo = jj < FP ? jp0 + jj : (jp0 + jj == FP ? nbH / 2 : nbH - jp0 - (jj - FP));
    const double2 val = lds_all[jj * MP + lds_slot(rr)];
    typedef double d2v __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(d2v{val.x, val.y}, reinterpret_cast<d2v*>(a.out + jo * R + rr));
  }
}

// The same as a persistent grid (AD_CORR_FUSED_PF): each workgroup takes items
// (inverse pair groups) t, t + G, ... and issues the next item's loads (V
// values per thread, into registers) once its forward pass is done, so they
// stay in flight under the z formation, the inverse pass and the stores
// (LDS-only barriers).  Same arithmetic in the same order.
template <int R, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_corr_fused_pf(CorrFusedArgs a, int items) {
  constexpr bool PF = true;
  constexpr int V = 8;
  using Plan = FftPlan<R, V>;
  constexpr int T = Plan::T;          // threads per butterfly
  constexpr int NBF = NT / T;         // forward butterflies per workgroup
  constexpr int FP = NBF / 4;         // inverse butterfly pairs per workgroup
  constexpr int MP = Plan::MP + (T >= 16 ? 1 : 0);
  static_assert(FP >= 1 && 2 * FP <= NBF, "fused CorrelateFFT pass shape");
  __shared__ __attribute__((aligned(16))) double2 lds_all[NBF * MP];
  __shared__ __attribute__((aligned(16))) double2 ltw[AD_FFT_TWC ? TwSplit<R>::N : 1];
  const int64_t N = a.N, NH = N / 2, nbF = N / R, nbH = nbF / 2;
  const int G = (int)gridDim.x;
  int item = xcd_remap((int)blockIdx.x, G);
  const TwLds<R> twr = tw_lds_compute<R>(ltw, (int)threadIdx.x, NT);
  // forward butterfly of slot b = set * FP + jj (set: j', j' + nbH, nbF - j', nbH - j')
  auto fbut_of = [&](int64_t jp0, int b) -> int64_t {
    const int set = b / FP;
    const int64_t j = jp0 + (b % FP);
    if (set == 0) return j;
    if (set == 1) return j + nbH;
    if (set == 2) return j == 0 ? nbH / 2 : nbF - j;
    return j == 0 ? 3 * (nbH / 2) : nbH - j;
  };
  typedef double d2v __attribute__((ext_vector_type(2)));  // (a double2 struct copy becomes a memcpy through scratch)
  d2v pf[V];
  // element r of slot b is in[fbut(b) + r nbF], idx = i NT + thread: b = idx % NBF, r = idx / NBF
  auto load_item = [&](int it, int tx) {
    const int64_t jp0 = (int64_t)it * FP;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int idx = i * NT + tx;
      const int b = idx % NBF, r = idx / NBF;
      pf[i] = *reinterpret_cast<const d2v*>(a.in + fbut_of(jp0, b) + (int64_t)r * nbF);
    }
  };
  if (PF && item < items) load_item(item, (int)threadIdx.x);
  for (; item < items; item += G) {
    int tx;  // an opaque copy of the thread index per item (k_fft_pass_pf: fewer live registers)
    asm volatile("v_mov_b32 %0, %1" : "=v"(tx) : "v"((int)threadIdx.x));
    const int64_t jp0 = (int64_t)item * FP;
    auto fbut = [&](int b) { return fbut_of(jp0, b); };
    // 1. stage the forward butterflies' inputs
    if constexpr (PF) {
      pass_lds_barrier();  // the previous item's output reads (and the twiddle tables) are done
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int idx = i * NT + tx;
        lds_all[(idx % NBF) * MP + lds_slot(idx / NBF)] = make_double2(pf[i].x, pf[i].y);
      }
      if (AD_CORR_PF_AT == 0 && item + G < items) load_item(item + G, tx);
      pass_lds_barrier();
    } else {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int idx = i * NT + tx;
        const int b = idx % NBF, r = idx / NBF;
        lds_all[b * MP + lds_slot(r)] = a.in[fbut(b) + (int64_t)r * nbF];
      }
      __syncthreads();
    }
    // 2. the forward last pass (k_fft_pass<R, true, ...> with Ns = nbF)
    const int fs = tx / T, tid = tx % T;
    double2* lds = lds_all + fs * MP;
    double2 v[V];
#pragma unroll
    for (int s = 0; s < V; ++s) v[s] = lds[pass0_slot<R, V>(tid, s)];
    pass_pretwiddle<R, V, true>(v, fbut(fs), nbF, N, tid, a.tw_lo, a.tw_hi, a.S);
    if constexpr (PF) {
      pass_lds_barrier();
      fft_run_lb<R, V, true>(v, tid, lds, twr);
      pass_lds_barrier();
    } else {
      __syncthreads();
      fft_run<R, V, true>(v, tid, lds, twr);
      __syncthreads();
    }
#pragma unroll
    for (int s = 0; s < V; ++s) lds[last_pass_slot<R, V>(tid, s)] = v[s];  // Z[fbut(fs) + nbF k]
    if (AD_CORR_PF_AT == 1 && item + G < items) load_item(item + G, tx);  // v is dead: room for the next item
    if constexpr (PF) pass_lds_barrier(); else __syncthreads();
    // 3. z for the inverse pairs (k_fft_pass's PAIR form): element (jj, r) of
    //    tile A and (jj, R-1-r) of tile B; Z of slot b, output k:
    auto zs = [&](int b, int k) { return lds_all[b * MP + lds_slot(k)]; };
    auto zq = [&](int64_t q) {  // Z[q] for the j' = 0 pair (any of its four butterflies)
      const int64_t fb = q & (nbF - 1);
      const int k = (int)(q / nbF);
      const int set = fb == 0 ? 0 : fb == nbH ? 1 : fb == nbH / 2 ? 2 : 3;
      return zs(set * FP, k);
    };
    auto half_in0 = [&](int64_t g) {  // half_in of k_fft_pass for the j' = 0 pair
      const double2 x1 = corr_xop(zq(g), zq((N - g) & (N - 1)));
      const double2 x2 = corr_xop(zq(g + NH), zq((N - g - NH) & (N - 1)));
      return half_zcomb(x1, x2, half_wneg(g, N, a.htw_lo, a.htw_hi, a.hS));
    };
    constexpr int NPAIR = FP * R / NT;  // (jj, r) pairs per thread
    double2 vA[NPAIR], vB[NPAIR];
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) {
      const int idx = i * NT + tx;
      const int jj = idx % FP, r = idx / FP;
      const int64_t j = jp0 + jj;
      if (j == 0) {
        vA[i] = half_in0((int64_t)r * nbH);
        vB[i] = half_in0(nbH / 2 + (int64_t)(R - 1 - r) * nbH);
      } else {
        const int odd = r & 1, k1 = r >> 1, k3 = (R - 1 - r) >> 1;
        const double2 z1 = zs(odd * FP + jj, k1), z2 = zs(odd * FP + jj, k1 + R / 2);          // Z[g], Z[g + NH]
        // gs = (nbH - j) + (R-1-r) nbH: forward butterfly nbF - j (r even, set 2) or nbH - j (r odd, set 3)
        const double2 z3 = zs((2 + odd) * FP + jj, k3), z4 = zs((2 + odd) * FP + jj, k3 + R / 2);  // Z[-(g + NH)], Z[-g]
        const int64_t g = j + (int64_t)r * nbH;
        const double2 w = half_wneg(g, N, a.htw_lo, a.htw_hi, a.hS);  // W_NF^-g* = -conj(W_NF^-g)
        vA[i] = half_zcomb(corr_xop(z1, z4), corr_xop(z2, z3), w);
        vB[i] = half_zcomb(corr_xop(z3, z2), corr_xop(z4, z1), make_double2(-w.x, w.y));
      }
    }
    if constexpr (PF) pass_lds_barrier(); else __syncthreads();  // every Z read is done: the inverse staging reuses slots 0 .. 2 FP - 1
#pragma unroll
    for (int i = 0; i < NPAIR; ++i) {
      const int idx = i * NT + tx;
      const int jj = idx % FP, r = idx / FP;
      lds_all[jj * MP + lds_slot(r)] = vA[i];
      lds_all[(FP + jj) * MP + lds_slot(R - 1 - r)] = vB[i];
    }
    if constexpr (PF) pass_lds_barrier(); else __syncthreads();
    // 4. the inverse first pass (Ns = 1: no pre-twiddle) on slots 0 .. 2 FP - 1:
    //    2 FP butterflies over all NT threads at VI values per thread
#if AD_CORR_INV_V4
    constexpr int VI = 4;
#else
    constexpr int VI = V;
#endif
    using PlanI = FftPlan<R, VI>;
    constexpr int TI = PlanI::T;
    const int fi = tx / TI, ti = tx % TI;
    double2* ldsi = lds_all + fi * MP;
    const bool act = fi < 2 * FP;  // wave-uniform (TI is a multiple of the wave or divides it)
    double2 u[VI];
    if (act) {
#pragma unroll
      for (int s = 0; s < VI; ++s) u[s] = ldsi[pass0_slot<R, VI>(ti, s)];
    }
    if constexpr (PF) {
      pass_lds_barrier();
      fft_run_active_lb<R, VI, false>(u, ti, ldsi, twr, act);
      pass_lds_barrier();
    } else {
      __syncthreads();
      fft_run_active<R, VI, false>(u, ti, ldsi, twr, act);
      __syncthreads();
    }
    if (act) {
#pragma unroll
      for (int s = 0; s < VI; ++s) ldsi[last_pass_slot<R, VI>(ti, s)] = u[s];
    }
    if constexpr (PF) pass_lds_barrier(); else __syncthreads();
    // 5. outputs: inverse butterfly jo's R values at jo R .. jo R + R - 1
#pragma unroll
    for (int i = 0; i < 2 * FP * R / NT; ++i) {
      const int idx = i * NT + tx;
      const int rr = idx % R, jj = idx / R;
      const int64_t jo = jj < FP ? jp0 + jj : (jp0 + jj == FP ? nbH / 2 : nbH - jp0 - (jj - FP));
      const double2 val = lds_all[jj * MP + lds_slot(rr)];
      __builtin_nontemporal_store(d2v{val.x, val.y}, reinterpret_cast<d2v*>(a.out + jo * R + rr));
    }
  }
}

// Naive DFT for N <= 8 (one thread per output bin).
__global__ void k_dft_small(FftPassArgs a, int fwd) {
  const int k = threadIdx.x;
  const int bt = blockIdx.y;
  if (k >= a.N) return;
  double2 acc = make_double2(0.0, 0.0);
  for (int n = 0; n < a.N; ++n) {
    double2 x;
    if (a.xr) {
      const int64_t g = n;
      x = make_double2(g < a.n_real ? a.xr[bt * a.in_batch + g] : 0.0, 0.0);
    } else {
      x = a.in[bt * a.in_batch + n];
    }
    const int e = (int)(((int64_t)n * k) % a.N);
    double2 w = a.tw_lo[e];  // S covers the whole table for N <= 8
    if (!fwd) w = c_conj(w);
    acc = c_add(acc, c_mul(x, w));
  }
  if (a.out_real)
    a.out_real[bt * a.out_batch + k] = acc.x * a.scale;
  else
    a.out[bt * a.out_batch + k] = acc;
}

// ---------------------------------------------------------------------------
// Host plan
// ---------------------------------------------------------------------------
namespace {
std::vector<double2> twiddles(int64_t N, int64_t count, int64_t stride) {
  // W_N^(i*stride) = exp(-2 pi i (i*stride)/N), evaluated in long double
  std::vector<double2> t((size_t)count);
  const long double two_pi = 6.283185307179586476925286766559005768L;
  for (int64_t i = 0; i < count; ++i) {
    const int64_t e = (i * stride) % N;
    const long double ang = -two_pi * (long double)e / (long double)N;
    t[(size_t)i] = make_double2((double)cosl(ang), (double)sinl(ang));
  }
  return t;
}
double2* upload(const std::vector<double2>& v) {
  double2* p = nullptr;
  AD_HIP(hipMalloc(reinterpret_cast<void**>(&p), v.size() * sizeof(double2)));
  AD_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(double2), hipMemcpyHostToDevice));
  return p;
}

template <int R, bool FWD, bool RI, bool RO>
void go_pass(const FftPassArgs& a, int batch, hipStream_t s) {
  using Sh = PassShape<R, RO>;
  const dim3 grid((unsigned)((a.N / R + Sh::F - 1) / Sh::F), (unsigned)batch);
  if constexpr (!FWD && !RI) {
    if (a.half) {
      // mirror-paired tiles: packed spectrum, not the last pass, whole tile pairs
      const bool pair = AD_FFT_PAIR && !a.spec2 && !RO && (a.N / R) % Sh::F == 0;
      if constexpr (!RO) {
        if (pair) {
          if (a.op == kSpecCorr)
            hipLaunchKernelGGL((k_fft_pass<R, FWD, RI, RO, 1, true>), grid, dim3(Sh::BLOCK), 0, s, a);
          else
            hipLaunchKernelGGL((k_fft_pass<R, FWD, RI, RO, 2, true>), grid, dim3(Sh::BLOCK), 0, s, a);
          return;
        }
      }
      if (a.op == kSpecCorr && !a.spec2)
        hipLaunchKernelGGL((k_fft_pass<R, FWD, RI, RO, 1>), grid, dim3(Sh::BLOCK), 0, s, a);
      else
        hipLaunchKernelGGL((k_fft_pass<R, FWD, RI, RO, 2>), grid, dim3(Sh::BLOCK), 0, s, a);
      return;
    }
  }
#if AD_FFT_PF && AD_FFT_TWC && AD_FFT_NT == 1
  if constexpr (!RI && RO && !FWD && (R == 128 || R == 256)) {  // the last inverse pass, persistent
    using Pf = PfShape<R>;
    const int64_t tiles = a.N / R / Pf::F;
    if (AD_FFT_PF_RO && !a.half && (a.N / R) % Pf::F == 0 && a.Ns >= Pf::F && tiles >= 2 * AD_FFT_PF_RO_G) {
      hipLaunchKernelGGL((k_fft_pass_pf<R, false, false, true>), dim3(AD_FFT_PF_RO_G, (unsigned)batch), dim3(Pf::BLOCK),
                         0, s, a, (int)tiles);
      return;
    }
  }
  if constexpr (!RI && !RO && R == 256) {
    using Pf = PfShape<R>;
    const int64_t tiles = a.N / R / Pf::F;
    if (!a.half && (a.N / R) % Pf::F == 0 && (a.Ns == 1 || a.Ns >= Pf::F) && tiles >= 2 * AD_FFT_PF_G) {
      hipLaunchKernelGGL((k_fft_pass_pf<R, FWD>), dim3(AD_FFT_PF_G, (unsigned)batch), dim3(Pf::BLOCK), 0, s, a,
                         (int)tiles);
      return;
    }
  }
#endif
  hipLaunchKernelGGL((k_fft_pass<R, FWD, RI, RO>), grid, dim3(Sh::BLOCK), 0, s, a);
}

template <bool FWD, bool RI, bool RO>
void launch_pass_r(int R, const FftPassArgs& a, int batch, hipStream_t s) {
#define AD_PASS(RR)                          \
  case RR: {                                 \
    go_pass<RR, FWD, RI, RO>(a, batch, s);   \
    break;                                   \
  }
  switch (R) {
    AD_PASS(16)
    AD_PASS(32)
    AD_PASS(64)
    AD_PASS(128)
    AD_PASS(256)
    AD_PASS(512)
    AD_PASS(1024)
    AD_PASS(2048)
    AD_PASS(4096)
    default:
      AD_FAIL(AD_ERR_INTERNAL, "BigFft: unsupported radix");
  }
#undef AD_PASS
}

template <bool FWD>
void launch_pass(int R, bool ri, bool ro, const FftPassArgs& a, int batch, hipStream_t s) {
  if (ri && ro) return launch_pass_r<FWD, true, true>(R, a, batch, s);
  if (ri) return launch_pass_r<FWD, true, false>(R, a, batch, s);
  if (ro) return launch_pass_r<FWD, false, true>(R, a, batch, s);
  launch_pass_r<FWD, false, false>(R, a, batch, s);
}
}  // namespace

BigFft::BigFft(int64_t N) : N_(N) {
  if (!is_pow2(N) || N > ((int64_t)1 << 27)) AD_FAIL(AD_ERR_INVALID_ARGUMENT, "BigFft: size must be a power of two <= 2^27");
  int k = 0;
  while (((int64_t)1 << k) < N) ++k;
  if (k <= 3) {
    S_ = k;  // the naive DFT reads W_N^e straight from lo
  } else if (k <= 12) {
    radix_.push_back((int)N);
    S_ = (k + 1) / 2;
  } else {
    // passes of radix <= 2^maxlog = 512 (F >= 8: 128-B runs)
    constexpr int maxlog = 9;
    const int np = (k + maxlog - 1) / maxlog;
    const int base = k / np, extra = k % np;
    for (int p = 0; p < np; ++p) radix_.push_back(1 << (base + (p < extra ? 1 : 0)));
    S_ = (k + 1) / 2;
  }
  const int64_t nlo = (int64_t)1 << S_;
  tw_lo_ = upload(twiddles(N, nlo, 1));
  tw_hi_ = upload(twiddles(N, std::max<int64_t>(1, N >> S_), nlo));
  for (int R : radix_) twR_.push_back(upload(twiddles(R, R, 1)));
}

BigFft::~BigFft() {
  for (double2* p : twR_) (void)hipFree(p);
  if (tw_lo_) (void)hipFree(tw_lo_);
  if (tw_hi_) (void)hipFree(tw_hi_);
}

void BigFft::run(bool forward, const double2* in, const double* xr, int64_t n_real, int64_t in_batch, double2* out,
                 double* out_real, int64_t out_batch, double scale, int batch, double2* scratch,
                 hipStream_t s) const {
  FftPassArgs a{};
  a.N = N_;
  a.tw_lo = tw_lo_;
  a.tw_hi = tw_hi_;
  a.S = S_;
  a.scale = scale;
  for (int b = 0; b < 2; ++b) {
    a.xb[b] = xr ? xr + b * in_batch : nullptr;
    a.nr[b] = n_real;
  }
  run_passes(forward, a, in, xr, in_batch, out, out_real, out_batch, batch, scratch, s);
}

// The split first pass (k_corr_split0 + k_fft_pass_pf PACKIN) replaces the
// max-abs kernel when the forward plan is 256 x 256 x 256 (N = 2^24) and the
// correlation takes the fused path.
bool BigFft::corr_split(const BigFft& half) const {
  return AD_CORR_SPLIT && AD_CORR_FUSED && AD_FFT_PF && radix_.size() == 3 && radix_[0] == 256 &&
         radix_[1] == 256 && radix_[2] == 256 && !half.radix_.empty() && half.radix_.front() == 256 &&
         half.radix_.size() >= 2 && N_ / 256 / AD_SPLIT0_F <= kAbsmaxMaxGroups &&
         N_ / 256 / PfShape<256>::F >= 2 * AD_FFT_PF_G;
}

void BigFft::correlate_half(const BigFft& half, const double* a_, int64_t n, const double* b_, int64_t m,
                            double2* spec, double* out, double2* scratch, unsigned long long* amax,
                            hipStream_t s) const {
  if (!corr_split(half)) {  // the split first pass takes the max-abs itself
    const int64_t mx = std::max(n, m);
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(AD_ABSMAX_G, (mx / 2 + 1023) / 1024));
    hipLaunchKernelGGL(k_absmax2, dim3(gx, 2), dim3(256), 0, s, a_, n, b_, m, amax);
    AD_HIP(hipGetLastError());
  }
  // lags 0..n-1 from the front, -(m-1)..-1 from the back (correlate.go:165-171)
  spectral_half(half, kSpecCorr, 0.0, nullptr, true, a_, n, b_, m, n, m - 1, N_ - m + 1, spec, out, scratch, s, amax);
}

void BigFft::spectral_half(const BigFft& half, int op, double eps, unsigned long long* bad, bool pack,
                           const double* a_, int64_t n, const double* b_, int64_t m, int64_t n_front,
                           int64_t front_off, int64_t back_from, double2* spec, double* out, double2* scratch,
                           hipStream_t s, const unsigned long long* amax) const {
  FftPassArgs a{};
  a.N = N_;
  a.tw_lo = tw_lo_;
  a.tw_hi = tw_hi_;
  a.S = S_;
  a.scale = 1.0;
  a.xb[0] = a_;
  a.nr[0] = n;
  a.xb[1] = b_;
  a.nr[1] = m;
  // The correlation's forward last pass and half inverse's first pass fused
  // (k_corr_fwd_last_inv_first): both radix 256, three passes each side.
  const int P = (int)radix_.size(), PH = (int)half.radix_.size();
  const bool fused = AD_CORR_FUSED && pack && op == kSpecCorr && P >= 2 && PH >= 2 && radix_.back() == 256 &&
                     half.radix_.front() == 256 && N_ / 256 >= 16;
  const double2* fused_out = nullptr;
  if (fused) {
    a.pack2 = 1;
    a.amax = amax;
    const double2* mid = nullptr;
    if (amax && corr_split(half)) {
      // the max-abs folded into the first pass (k_corr_split0), the packing
      // at the second pass's load (k_fft_pass_pf PACKIN); the rest as below
      FftPassArgs p0 = a;
      p0.Ns = 1;
      p0.twR = twR_[0];
      p0.out = scratch;
      p0.amax_part = const_cast<unsigned long long*>(amax) + 8;  // the caller's scratch
      constexpr int FT = AD_SPLIT0_F;
      const int nblk = (int)(N_ / 256 / FT);
      hipLaunchKernelGGL((k_corr_split0<256, FT>), dim3((unsigned)nblk), dim3(FT * FftPlan<256, 8>::T), 0, s, p0);
      AD_HIP(hipGetLastError());
      FftPassArgs p1 = a;
      p1.pack2 = 0;
      p1.in = scratch;
      p1.in_batch = N_;
      p1.out = scratch + N_;
      p1.out_batch = N_;
      p1.Ns = 256;
      p1.twR = twR_[1];
      p1.amax_part = const_cast<unsigned long long*>(amax) + 8;
      p1.amax_parts = nblk;
      const int tiles = (int)(N_ / 256 / PfShape<256>::F);
      hipLaunchKernelGGL((k_fft_pass_pf<256, true, true>), dim3(AD_FFT_PF_G), dim3(PfShape<256>::BLOCK), 0, s, p1,
                         tiles);
      AD_HIP(hipGetLastError());
      mid = scratch + N_;
    } else {
      mid = run_passes(true, a, nullptr, a_, 0, nullptr, nullptr, N_, 1, scratch, s, 0, P - 1);
    }
    CorrFusedArgs f{};
    f.in = mid;
    // the half plan's first scratch half (a consumed forward pass output) unless
    // the forward part's result sits there (two-pass plans): then past it
    f.out = mid == scratch ? scratch + N_ : scratch;
    f.N = N_;
    f.tw_lo = tw_lo_;
    f.tw_hi = tw_hi_;
    f.S = S_;
    f.htw_lo = tw_lo_;
    f.htw_hi = tw_hi_;
    f.hS = S_;

    constexpr int NT = AD_CORR_FUSED_NT;  // threads per workgroup (4 inverse pairs per 512)
    const int items = (int)(N_ / 256 / 2 / 2 / (NT / FftPlan<256, 8>::T / 4));
    if (AD_CORR_FUSED_PF)
      hipLaunchKernelGGL((k_corr_fused_pf<256, NT>), dim3(std::min(items, AD_CORR_FUSED_PF_G)), dim3(NT), 0, s,
                         f, items);
    else
      hipLaunchKernelGGL((k_corr_fwd_last_inv_first<256, NT>), dim3(items), dim3(NT), 0, s, f);
    fused_out = f.out;
    AD_HIP(hipGetLastError());
  } else if (pack) {
    a.pack2 = 1;  // Z = FFT(a + i b)
    a.amax = amax;
    run_passes(true, a, nullptr, a_, 0, spec, nullptr, N_, 1, scratch, s);
  } else {  // FFT(a) and FFT(b) as a batch of two real inputs: spec [2][N]
    run_passes(true, a, nullptr, a_, 0, spec, nullptr, N_, 2, scratch, s);
  }
  FftPassArgs i{};
  i.N = half.N_;
  i.tw_lo = half.tw_lo_;
  i.tw_hi = half.tw_hi_;
  i.S = half.S_;
  i.scale = 1.0 / (double)half.N_;
  i.half = 1;
  i.NF = N_;
  i.ftw_lo = tw_lo_;
  i.ftw_hi = tw_hi_;
  i.fS = S_;
  i.spec2 = pack ? nullptr : spec + N_;
  i.op = op;
  i.eps = eps;
  i.bad = bad;
  i.remap = 1;
  i.amax = pack ? amax : nullptr;
  i.n_front = n_front;
  i.front_off = front_off;
  i.back_from = back_from;
  if (fused)  // passes 1 .. of the half inverse, from the fused pass's output
    half.run_passes(false, i, fused_out, nullptr, half.N_, nullptr, out, 0, 1, scratch, s, 1);
  else
    half.run_passes(false, i, spec, nullptr, half.N_, nullptr, out, 0, 1, scratch, s);
}

const double2* BigFft::run_passes(bool forward, FftPassArgs a, const double2* in, const double* xr, int64_t in_batch,
                                  double2* out, double* out_real, int64_t out_batch, int batch, double2* scratch,
                                  hipStream_t s, int p_begin, int p_end) const {
  const int64_t n_real = a.nr[0];
  const int pack2 = a.pack2, halfz = a.half;  // first / last pass only
  if (radix_.empty()) {  // N <= 8 (no fused edges: callers check fused_ok())
    a.in = in;
    a.xr = xr;
    a.n_real = n_real;
    a.in_batch = in_batch;
    a.out = out;
    a.out_real = out_real;
    a.out_batch = out_batch;
    hipLaunchKernelGGL(k_dft_small, dim3(1, (unsigned)batch), dim3(64), 0, s, a, forward ? 1 : 0);
    AD_HIP(hipGetLastError());
    return out;
  }
  // pass p writes the final destination when p is last, else one of two
  // scratch halves (pass p-1's output is pass p's input).  [p_begin, p_end):
  // a part of the plan (p_begin > 0: `in` is pass p_begin - 1's output; the
  // result of a part ending early stays in its scratch half, returned).
  const int P = (int)radix_.size();
  const int pe = p_end < 0 ? P : p_end;
  double2* half[2] = {scratch, scratch + N_ * batch};
  int64_t Ns = 1;
  for (int p = 0; p < p_begin; ++p) Ns *= radix_[(size_t)p];
  const double2* cur = in;
  for (int p = p_begin; p < pe; ++p) {
    const int R = radix_[(size_t)p];
    const bool first = p == 0, last = p == P - 1;
    a.in = first ? in : cur;
    a.pack2 = first ? pack2 : 0;
    a.half = first ? halfz : 0;
    a.pairs = last ? halfz : 0;
    a.xr = first ? xr : nullptr;
    a.n_real = n_real;
    a.in_batch = first ? in_batch : N_;
    a.Ns = Ns;
    a.twR = twR_[(size_t)p];
    double2* dst = last ? out : half[p & 1];
    a.out = dst;
    a.out_real = last ? out_real : nullptr;
    a.out_batch = last ? out_batch : N_;
    const bool ri = first && xr != nullptr;
    const bool ro = last && out_real != nullptr;
    if (forward)
      launch_pass<true>(R, ri, ro, a, batch, s);
    else
      launch_pass<false>(R, ri, ro, a, batch, s);
    AD_HIP(hipGetLastError());
    cur = dst;
    Ns *= R;
  }
  return cur;
}

// ---------------------------------------------------------------------------
// Pointwise spectral operations, restated in Go complex128 arithmetic:
// products as (ac - bd, ad + bc), quotients by the Go runtime's
// complex128div (Smith's algorithm), magnitudes by math.Hypot.
// ---------------------------------------------------------------------------
#pragma clang fp contract(off)
__global__ __launch_bounds__(256) void k_spec_op(int op, double2* __restrict__ a, const double2* __restrict__ b,
                                                 int64_t n, double eps, unsigned long long* bad) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  a[i] = spec_op(op, a[i], b ? b[i] : make_double2(0.0, 0.0), eps, i, bad);
}

void launch_spec_op(int op, double2* a, const double2* b, int64_t n, double eps, unsigned long long* bad,
                    hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_spec_op, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, op, a, b, n, eps, bad);
  AD_HIP(hipGetLastError());
}

}  // namespace adsp
