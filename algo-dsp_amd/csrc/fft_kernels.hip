// Window real-FFT (K1) and inverse real-FFT + overlap-save store (K3) kernels
// of the UPOLS convolution engine (see conv_kernels.hip for the data flow).
//
// K1: P[c][g] = FFT_M(z), z[m] = x[gL + 2m] + i x[gL + 2m + 1] for m < M/2 and
//     z[m] = 0 above: the packed half-length complex FFT of input block g
//     zero padded to N = 2L (M = L).  The window spectrum overlap-save needs,
//     the packed FFT of x[(g-1)L .. (g+1)L), is Zr[g][k] = P[g-1][k] +
//     (-1)^k P[g][k] (a shift by M/2 in an M-point FFT is a factor (-1)^k),
//     which k_fdl_mac forms on load from consecutive rows of its stream and
//     then separates into the real spectrum
//     X[k] = (Zr[k] + conj Zr[M-k])/2 - i W_2M^k (Zr[k] - conj Zr[M-k])/2.
//     One transform per input block (not per output block): a call of n
//     samples runs ceil(n/L) K1 items, the convolution tail none, and no
//     input history is kept between streaming calls (the previous block's P
//     is in the ring).
// K3: y[c][jL .. (j+1)L) = last L samples of irFFT_N(Y[c][j]); the input is
//     the half-length spectrum Z already folded by k_fdl_mac's epilogue, so
//     K3 is a plain inverse complex FFT + store of the upper half.
// The reference's equivalents are the FFT calls inside
// StreamingOverlapSaveT.processBlockCore (dsp/conv/streaming_overlap_save.go:100-133)
// and partStageT.process (dsp/conv/partitioned.go:134-183), which run a
// complex FFT of real data (2x the work) through algo-fft.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "conv_kernels.hpp"
#include "fft_device.hpp"

namespace adsp {

__device__ __forceinline__ double2 fetch_pair(const double* xc, int64_t t, int64_t n, bool aligned) {
  if (t + 1 < n && aligned) return *reinterpret_cast<const double2*>(xc + t);
  return make_double2(t < n ? xc[t] : 0.0, t + 1 < n ? xc[t + 1] : 0.0);
}

// Inverse store: the upper half of the time window (m >= M/2) to y.
template <int M, int V>
__device__ __forceinline__ void irfft_store_out(const double2* v, int tid, double* yc, int64_t ob, int64_t out_len,
                                                bool aligned, bool acc) {
#pragma unroll
  for (int s = 0; s < V; ++s) {
    const int m = last_pass_index<M, V>(tid, s);
    if (m < M / 2) continue;
    const int64_t o = ob + 2 * m;
    if (o + 1 < out_len && aligned) {
      double2 r = v[s];
      if (acc) {
        const double2 q = *reinterpret_cast<const double2*>(yc + o);
        r = make_double2(q.x + r.x, q.y + r.y);
      }
      *reinterpret_cast<double2*>(yc + o) = r;
    } else {
      if (o < out_len) yc[o] = acc ? yc[o] + v[s].x : v[s].x;
      if (o + 1 < out_len) yc[o + 1] = acc ? yc[o + 1] + v[s].y : v[s].y;
    }
  }
}

// ---------------------------------------------------------------------------
// One-shot forms (M <= 1024): F = BLOCK/T FFTs per workgroup, one
// (channel, block) item each.
// ---------------------------------------------------------------------------
// StreamGate (conv_kernels.hpp): K1's wait for the host's go word.  Thread 0
// polls (system-scope acquire loads of mapped host memory, s_sleep between
// polls) until go == seq, go == kGateAbort or the timeout; it records the
// decision for K2 / K3 (gate) and the host (k1_state).  Returns false when
// the workgroup must not run.
__device__ __forceinline__ bool gate_wait(const StreamGate& g) {
  if (!g.go) return true;
  __shared__ int ok;
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int run = 0;
    for (;;) {
      const uint64_t v = __hip_atomic_load(g.go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v == g.seq) {
        run = 1;
        break;
      }
      if (v == kGateAbort || __builtin_amdgcn_s_memrealtime() - t0 > g.timeout) break;
      __builtin_amdgcn_s_sleep(4);
    }
    __hip_atomic_store(g.gate, run ? g.seq : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(g.k1_state, run ? g.seq : (g.seq | kGateSkipped), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    ok = run;
  }
  __syncthreads();
  return ok != 0;
}
// K2 / K3 of a gated chain: did its K1 run?  (K1 finished before this launch
// started: stream order.)
__device__ __forceinline__ bool gate_open(const StreamGate& g) {
  return !g.gate || __hip_atomic_load(g.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g.seq;
}
// K3 of a gated chain: every thread's output stores are complete and visible
// system-wide, then one lane publishes seq.
__device__ __forceinline__ void gate_done(const StreamGate& g) {
  if (!g.done) return;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(g.done, g.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int M, int V>
__global__ __launch_bounds__((FftPlan<M, V>::BLOCK)) void k_window_rfft(RfftArgs a) {
  using Plan = FftPlan<M, V>;
  constexpr int T = Plan::T;
  constexpr int L = M;
  __shared__ __attribute__((aligned(16))) double2 lds_all[Plan::F * Plan::MP];
  const int f = threadIdx.x / T;
  const int tid = threadIdx.x % T;
  const int64_t e = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * a.per_wg + f;
  const bool active = f < a.per_wg && e < (int64_t)a.channels * a.jc;
  const int c = active ? (int)(e / a.jc) : 0;
  const int j = active ? (int)(e % a.jc) : 0;
  double2* lds = lds_all + f * Plan::MP;
  const double* xc = a.x + (int64_t)c * a.x_stride;
  const int64_t t0 = a.s0 + (int64_t)j * L;  // first sample of block j

  double2 v[V];
#pragma unroll
  for (int s = 0; s < V; ++s) {
    const int m = pass0_index<M, V>(tid, s);
    v[s] = (active && m < M / 2) ? fetch_pair(xc, t0 + 2 * m, a.n, a.aligned) : make_double2(0, 0);
  }
  fft_run<M, V, true>(v, tid, lds, TwGlobal{a.twM});
  if (!active) return;
  double2* Xo = a.X + (int64_t)c * a.x_ch_stride + (int64_t)((a.slot0 + j) % a.Q) * a.MS;
#pragma unroll
  for (int s = 0; s < V; ++s) Xo[xrow_pos(last_pass_index<M, V>(tid, s), M)] = v[s];
}

template <int M, int V>
__global__ __launch_bounds__((FftPlan<M, V>::BLOCK)) void k_irfft_store(IrfftArgs a) {
  using Plan = FftPlan<M, V>;
  constexpr int T = Plan::T;
  constexpr int L = M;
  __shared__ __attribute__((aligned(16))) double2 lds_all[Plan::F * Plan::MP];
  const int f = threadIdx.x / T;
  const int tid = threadIdx.x % T;
  const int64_t e = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * Plan::F + f;
  const bool active = e < (int64_t)a.channels * a.jc;
  const int c = active ? (int)(e / a.jc) : 0;
  const int j = active ? (int)(e % a.jc) : 0;
  double2* lds = lds_all + f * Plan::MP;
  const double2* Zb = a.Y + (int64_t)c * a.y_ch_stride + (int64_t)j * a.MS;
  double2 v[V];
#pragma unroll
  for (int s = 0; s < V; ++s) {
    const int k = pass0_index<M, V>(tid, s);
    v[s] = active ? Zb[zrow_pos(k, M)] : make_double2(0.0, 0.0);  // wave-lane row order
  }
  fft_run<M, V, false>(v, tid, lds, TwGlobal{a.twM});
  if (!active) return;
  irfft_store_out<M, V>(v, tid, a.out + (int64_t)c * a.out_stride, a.o0 + (int64_t)j * L - M, a.out_len, a.aligned,
                        a.accumulate);
}

// ---------------------------------------------------------------------------
// Split forms (M >= 2048): one item per workgroup, the M-point transform done
// as two M/2-point LDS transforms plus one radix-2 step in registers
// (decimation in time for K1, in frequency-index parity for K3):
//   K1: Zr[k] = E[k] + W_M^k O[k], Zr[k+M/2] = E[k] - W_M^k O[k],
//       E = FFT(z[2m]), O = FFT(z[2m+1]), z[m] = x[2m] + i x[2m+1];
//   K3: z[M/2+m] = A[m] - W_M^-m B[m] (only the upper half is kept),
//       A = IFFT(Z[2k]), B = IFFT(Z[2k+1]); k_fdl_mac stores Z rows in
//       wave-lane order with even and odd bins in separate 256-B runs
//       (zrow_pos), so A and B are two whole-line load streams.
// Each thread's E/O inputs are 32 contiguous bytes, and its outputs of
// both halves are the same last-pass indices, so the radix-2 step needs no
// exchange.  The LDS image is that of an M/2 transform (69.6 KiB at M = 8192),
// so two workgroups share a CU and one's HBM phase hides under the other's
// LDS/VALU phase: a workgroup barriers only with itself.  Twiddles live in LDS
// (no global load between the loads and stores of an item).
// K1 stores the packed block spectrum P (M values); k_fdl_mac forms the
// window spectrum Zr from two consecutive P rows and separates it into the
// real-signal spectrum on load (Zr[k] and Zr[M-k] sit in partner lanes of
// its pair waves).  Half of K1's pass-0 inputs are the block's zero padding.
// ---------------------------------------------------------------------------
// Z[M/2] of output block j of channel c (MidBin; K2's middle-bin wave, in one
// wave here): lane p takes partition p (and p + 64, ...), forms the window
// spectrum's middle bin from two block-spectrum rows, separates it and the
// partition's H the way K2 does for a self-mirrored bin (u = v), multiplies,
// and the wave sums the products (fixed xor-tree order, so deterministic);
// then K2's Z fold.  Every lane returns the value.
// Split in two so that the loads of the first partitions (p = lane) go out
// ahead of the item's Z loads: mid_bin_issue loads them, mid_bin_z (after
// the Z loads are issued) waits for those alone -- vmcnt retires in order --
// and finishes; partitions p >= 64 (P > 64) are loaded and summed there.
struct MidLoads {
  double2 pp, pc, h;  // P[g-1], P[g], H[p] of partition p = lane (zeros past P)
};
template <int M>
struct MidRows {
  const double2* Xc;
  const double2* Hc;
  int64_t G;     // logical block of this output
  int64_t gend;  // last logical block holding input
  int Q, P, MS;
  __device__ __forceinline__ MidRows(const IrfftArgs& a, int c, int j)
      : G(a.mid.g0 + j), gend(a.mid.gend), Q(a.mid.Q), P(a.mid.P), MS(a.MS) {
    Xc = a.mid.X + (int64_t)c * a.mid.x_ch_stride + xrow_pos(M / 2, M);
    const int ir = a.mid.ir_index ? a.mid.ir_index[c] : (c % a.mid.n_ir);
    Hc = a.mid.H + (int64_t)ir * a.mid.h_ir_stride + xrow_pos(M / 2, M);
  }
  __device__ __forceinline__ double2 row(int64_t g) const {
    const int64_t r = (g < 0 || g > gend) ? Q : g % Q;
    return Xc[r * MS];
  }
  __device__ __forceinline__ MidLoads load(int p) const {
    if (p >= P) return MidLoads{make_double2(0, 0), make_double2(0, 0), make_double2(0, 0)};
    const int64_t g = G - p;
    return MidLoads{row(g - 1), row(g), Hc[(int64_t)p * MS]};
  }
};
template <int M>
__device__ __forceinline__ MidLoads mid_bin_issue(const IrfftArgs& a, int c, int j) {
  return MidRows<M>(a, c, j).load(threadIdx.x & 63);
}
template <int M>
__device__ double2 mid_bin_z(const IrfftArgs& a, int c, int j, MidLoads first) {
  const int lane = threadIdx.x & 63;
  const double2 tu = a.twN[M / 2];  // W_2M^(M/2), as K2's unpack
  const MidRows<M> rows(a, c, j);
  // separation of a self-mirrored bin: X' = (fma(W.x, 2a.y, 2a.x), W.y 2a.y)
  auto unpack = [&](double2 v) {
    const double sx = v.x + v.x, sy = v.y + v.y;
    return make_double2(fma(tu.x, sy, sx), tu.y * sy);
  };
  double2 t = make_double2(0.0, 0.0);
  for (int p = lane; p < rows.P; p += 64) {
    const MidLoads ld = p == lane ? first : rows.load(p);
    // Zr = P[g-1] + (-1)^(M/2) P[g], M/2 even
    const double2 x = unpack(make_double2(ld.pp.x + ld.pc.x, ld.pp.y + ld.pc.y));
    const double2 h = unpack(ld.h);
    t.x = fma(x.x, h.x, t.x);
    t.x = fma(-x.y, h.y, t.x);
    t.y = fma(x.x, h.y, t.y);
    t.y = fma(x.y, h.x, t.y);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    t.x += __shfl_xor(t.x, o);
    t.y += __shfl_xor(t.y, o);
  }
  // K2's fold for u = v = Y: Z = (S sx - t.x sy, -t.y sy), t = conj(W) S
  const double S = 0.125 / (double)M;
  const double2 te = make_double2(tu.x * S, -tu.y * S);
  const double sx = t.x + t.x, sy = t.y + t.y;
  return make_double2(fma(-te.x, sy, sx * S), -te.y * sy);
}

template <int M, int VV = 8>
struct SplitPlan {
  static constexpr int M2 = M / 2;
  static constexpr int V = VV;
  using Sub = FftPlan<M2, V>;
  static constexpr int T = Sub::T;  // threads per workgroup
  static constexpr int LDS = Sub::MP + TwSplit<M2>::N + TwSplit<M>::N;  // double2 elements
};

#ifndef AD_K1_V
#define AD_K1_V 8  // K1's values per thread in the split transforms (16: 256-lane workgroups, 2 waves/SIMD)
#endif
#ifndef AD_K3_V
#define AD_K3_V 8  // K3's (k_irfft_store_split)
#endif
template <int M, int VV = AD_K1_V>
__global__ __launch_bounds__((SplitPlan<M, VV>::T)) __attribute__((amdgpu_waves_per_eu(32 / VV))) void k_window_rfft_split(RfftArgs a) {
  using SP = SplitPlan<M, VV>;
  constexpr int M2 = SP::M2, V = SP::V, T = SP::T, L = M;
  __shared__ __attribute__((aligned(16))) double2 lds[SP::LDS];
  const int tid = threadIdx.x;
  if (!gate_wait(a.sg)) return;
  int c, j;
  if (a.ord_R > 0) {  // newest-last for K2's first steps (RfftArgs::ord_R)
    const int per = a.channels * (a.ord_ny + 1), b = blockIdx.x;
    const int t = a.ord_R - 1 - b / per, k = b % per;
    c = __builtin_amdgcn_readfirstlane(k % a.channels);
    j = __builtin_amdgcn_readfirstlane((k / a.channels) * a.ord_R - a.ord_pc + t);
    if (j < 0 || j >= a.jc) return;
  } else {
    const int e = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));  // uniform: SGPRs
    c = __builtin_amdgcn_readfirstlane(e / a.jc);
    j = __builtin_amdgcn_readfirstlane(e - c * a.jc);
  }
  const double* xc = a.x + (int64_t)c * a.x_stride;
  const int64_t t0 = a.s0 + (int64_t)j * L;  // first sample of block j
  // E[m] = z[2m], O[m] = z[2m+1] hold samples 4m.. of the block; the upper
  // half of the padded block is zero, i.e. pass-0 slots s with
  // s mod R0 >= R0/2 (pass0_index >= M2/2), known at compile time.
  constexpr int R0 = FftPlan<M2, V>::R0;
  double2 ev[V], ov[V];
  if (a.aligned && t0 + L <= a.n) {  // wave-uniform fast path
    // E's inputs first: its transform starts while O's are still in flight
#pragma unroll
    for (int s = 0; s < V; ++s)
      ev[s] = (s % R0 < R0 / 2) ? *reinterpret_cast<const double2*>(xc + t0 + 4 * pass0_index<M2, V>(tid, s))
                                : make_double2(0.0, 0.0);
#pragma unroll
    for (int s = 0; s < V; ++s)
      ov[s] = (s % R0 < R0 / 2) ? *reinterpret_cast<const double2*>(xc + t0 + 4 * pass0_index<M2, V>(tid, s) + 2)
                                : make_double2(0.0, 0.0);
  } else {
#pragma unroll
    for (int s = 0; s < V; ++s) {
      const int64_t t = t0 + 4 * pass0_index<M2, V>(tid, s);
      const bool live = s % R0 < R0 / 2;
      ev[s] = live ? fetch_pair(xc, t, a.n, a.aligned) : make_double2(0.0, 0.0);
      ov[s] = live ? fetch_pair(xc, t + 2, a.n, a.aligned) : make_double2(0.0, 0.0);
    }
  }
  const TwLds<M2> twS = tw_lds_compute<M2>(lds + FftPlan<M2, V>::MP, tid, T);
  const TwLds<M> twC = tw_lds_compute<M>(lds + FftPlan<M2, V>::MP + TwSplit<M2>::N, tid, T);
  __syncthreads();  // twiddle tables
  fft_run<M2, V, true>(ev, tid, lds, twS);
  __syncthreads();  // E's last LDS reads are done
  fft_run<M2, V, true>(ov, tid, lds, twS);
  double2* Xo = a.X + (int64_t)c * a.x_ch_stride + (int64_t)((a.slot0 + j) % a.Q) * a.MS;
#pragma unroll
  for (int s = 0; s < V; ++s) {
    const int k = last_pass_index<M2, V>(tid, s);
    const double2 wo = c_mul(twC(k), ov[s]);
    Xo[k] = c_add(ev[s], wo);  // k < M/2: xrow_pos(k) = k
    Xo[xrow_pos(k + M2, M)] = c_sub(ev[s], wo);
  }
}

// NT: non-temporal Z loads and output stores (large launches, see k3_nt).
template <int M, bool NT, int VV = AD_K3_V>
__global__ __launch_bounds__((SplitPlan<M, VV>::T)) __attribute__((amdgpu_waves_per_eu(32 / VV))) void k_irfft_store_split(IrfftArgs a) {
  using SP = SplitPlan<M, VV>;
  constexpr int M2 = SP::M2, V = SP::V, T = SP::T, L = M;
  __shared__ __attribute__((aligned(16))) double2 lds[SP::LDS];
  const int tid = threadIdx.x;
  if (!gate_open(a.sg)) return;
  // item indices and row bases are wave-uniform: keep them in SGPRs (VGPR
  // copies of 64-bit bases spilled to scratch at the 128-VGPR cap)
  int c, j;
  if (a.ord_R > 0) {  // newest first (IrfftArgs::ord_R)
    const int per = a.channels * a.ord_ny, b = blockIdx.x;
    const int t = a.ord_R - 1 - b / per, k = b % per;
    c = __builtin_amdgcn_readfirstlane(k % a.channels);
    j = __builtin_amdgcn_readfirstlane((k / a.channels) * a.ord_R + t);
    if (j >= a.jc) return;
  } else {
    const int e = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
    c = __builtin_amdgcn_readfirstlane(e / a.jc);
    j = __builtin_amdgcn_readfirstlane(e - c * a.jc);
  }
  const double2* Zb = a.Y + (int64_t)c * a.y_ch_stride + (int64_t)j * a.MS;
  double2 av[V], bv[V];
  // wave 0: the middle bin's first partition loads, ahead of the Z loads
  const bool mid = a.mid.on && tid < 64;
  MidLoads ml{};
  if (mid) ml = mid_bin_issue<M>(a, c, j);
  // all of A (even bins), then all of B (odd bins): zrow_pos keeps each
  // stream in whole lines, so A's transform starts while B is in flight
#pragma unroll
  for (int s = 0; s < V; ++s)
    av[s] = ld2<NT>(Zb + zrow_pos(2 * pass0_index<M2, V>(tid, s), M));
  __builtin_amdgcn_sched_barrier(0);  // keep B's loads behind A's
#pragma unroll
  for (int s = 0; s < V; ++s)
    bv[s] = ld2<NT>(Zb + zrow_pos(2 * pass0_index<M2, V>(tid, s) + 1, M));
  // bin M/2 = 2k at k = M2/2: thread 0, pass-0 slot R0/2
  if (mid) {
    const double2 z = mid_bin_z<M>(a, c, j, ml);
    if (tid == 0) av[FftPlan<M2, V>::R0 / 2] = z;
  }
  const TwLds<M2> twS = tw_lds_compute<M2>(lds + FftPlan<M2, V>::MP, tid, T);
  const TwLds<M> twC = tw_lds_compute<M>(lds + FftPlan<M2, V>::MP + TwSplit<M2>::N, tid, T);
  __syncthreads();  // twiddle tables
  fft_run<M2, V, false>(av, tid, lds, twS);
  __syncthreads();
  fft_run<M2, V, false>(bv, tid, lds, twS);
  const int64_t ob = a.o0 + (int64_t)j * L;  // output of time index M/2 + m is at ob + 2m
  double* yb = a.out + (int64_t)c * a.out_stride + ob;
#pragma unroll
  for (int s = 0; s < V; ++s) {
    const int m = last_pass_index<M2, V>(tid, s);
    av[s] = c_sub(av[s], c_mul(c_conj(twC(m)), bv[s]));
  }
  if (a.aligned && ob + 2 * M2 <= a.out_len) {  // wave-uniform fast paths
    if (!a.accumulate) {
#pragma unroll
      for (int s = 0; s < V; ++s)
        st2<NT>(reinterpret_cast<double2*>(yb + 2 * last_pass_index<M2, V>(tid, s)), av[s]);
    } else {
#pragma unroll
      for (int s = 0; s < V; ++s) {
        double2* p = reinterpret_cast<double2*>(yb + 2 * last_pass_index<M2, V>(tid, s));
        const double2 q = *p;
        *p = make_double2(q.x + av[s].x, q.y + av[s].y);
      }
    }
  } else {
    const int64_t left = a.out_len - ob;  // valid outputs from yb on
#pragma unroll
    for (int s = 0; s < V; ++s) {
      const int o = 2 * last_pass_index<M2, V>(tid, s);
      if (o < left) yb[o] = a.accumulate ? yb[o] + av[s].x : av[s].x;
      if (o + 1 < left) yb[o + 1] = a.accumulate ? yb[o + 1] + av[s].y : av[s].y;
    }
  }
  gate_done(a.sg);
}

#ifndef AD_K3MIX_AB
#define AD_K3MIX_AB 0
#endif  // tools/ A/B builds only
// K3 with the stereo mixdown fused (Upols::run with a MixOut,
// ad_conv_multi_process_device_mix).  One workgroup per (output block j,
// side s): it runs the split inverse transform above for every channel of the
// group on side s (local channel c with (mix_parity + c) & 1 == s, i.e. global
// index parity s), in increasing c, and sums the channels' output blocks in
// registers; only the mix block is stored.  The per-channel outputs never
// reach memory (k_mixdown re-read the 8 channel rows and wrote
// the 2 mix rows, 1.35 GB per shard step, and K3 wrote 8 rows where 2 are
// needed).  Registers: the accumulator's 32 VGPRs do not fit beside both
// halves A and B at the kernel's 128-VGPR cap (two workgroups per CU; 88
// VGPRs of spills when A and B were both live), so A is added into the
// accumulator as soon as its transform is done and B's loads are issued after
// that, and each channel enters the mix as (acc + A) - W^-m B instead of
// acc + (A - W^-m B): the same terms, rounded in another order (the mix agrees
// with k_mixdown over the per-channel outputs to rounding, and is exactly
// the per-channel output for a side with one channel).  The other workgroup
// on the CU hides B's load wait.
template <int M, bool NT, int VV>
__global__ __launch_bounds__((SplitPlan<M, VV>::T)) __attribute__((amdgpu_waves_per_eu(32 / VV))) void k_irfft_mix_split(IrfftArgs a) {
  using SP = SplitPlan<M, VV>;
  constexpr int M2 = SP::M2, V = SP::V, T = SP::T, L = M;
  __shared__ __attribute__((aligned(16))) double2 lds[SP::LDS];
  const int tid = threadIdx.x;
  const int e = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x));
  const int j = __builtin_amdgcn_readfirstlane(e >> 1);
  const int side = __builtin_amdgcn_readfirstlane(e & 1);
  const int c0 = (side ^ a.mix_parity) & 1;  // first local channel of this side
  const TwLds<M2> twS = tw_lds_compute<M2>(lds + FftPlan<M2, V>::MP, tid, T);
  const TwLds<M> twC = tw_lds_compute<M>(lds + FftPlan<M2, V>::MP + TwSplit<M2>::N, tid, T);
  double2 acc[V];
#pragma unroll
  for (int s = 0; s < V; ++s) acc[s] = make_double2(0.0, 0.0);
  for (int c = c0; c < a.channels; c += 2) {
    // an opaque copy of tid per channel: the index arithmetic below is redone
    // each iteration instead of being hoisted out of the loop into ~24 live
    // VGPRs (that hoisting spilled at the 128-VGPR cap)
    int t = tid;
    asm volatile("" : "+v"(t));
    const double2* Zb = a.Y + (int64_t)c * a.y_ch_stride + (int64_t)j * a.MS;
    double2 av[V], bv[V];
    const bool mid = a.mid.on && tid < 64;
    MidLoads ml{};
    if (mid) ml = mid_bin_issue<M>(a, c, j);
#pragma unroll
    for (int s = 0; s < V; ++s) av[s] = ld2<NT>(Zb + zrow_pos(2 * pass0_index<M2, V>(t, s), M));
    if (mid) {
      const double2 z = mid_bin_z<M>(a, c, j, ml);
      if (tid == 0) av[FftPlan<M2, V>::R0 / 2] = z;
    }
#if AD_K3MIX_AB  // tools/ A/B builds: B's loads ahead of A's transform (spills)
#pragma unroll
    for (int s = 0; s < V; ++s) bv[s] = ld2<NT>(Zb + zrow_pos(2 * pass0_index<M2, V>(t, s) + 1, M));
#endif
    __syncthreads();  // twiddle tables (first channel) / the previous channel's last LDS reads
    fft_run<M2, V, false>(av, t, lds, twS);
#pragma unroll
    for (int s = 0; s < V; ++s) acc[s] = c_add(acc[s], av[s]);
#if !AD_K3MIX_AB
    __builtin_amdgcn_sched_barrier(0);  // B's loads stay behind A's transform (registers)
#pragma unroll
    for (int s = 0; s < V; ++s) bv[s] = ld2<NT>(Zb + zrow_pos(2 * pass0_index<M2, V>(t, s) + 1, M));
#endif
    __syncthreads();
    fft_run<M2, V, false>(bv, t, lds, twS);
#pragma unroll
    for (int s = 0; s < V; ++s) acc[s] = c_sub(acc[s], c_mul(c_conj(twC(last_pass_index<M2, V>(t, s))), bv[s]));
  }
  const int64_t ob = a.o0 + (int64_t)j * L;  // output of time index M/2 + m is at ob + 2m
  double* yb = a.out + (int64_t)side * a.out_stride + ob;
  if (a.aligned && ob + 2 * M2 <= a.out_len) {
#pragma unroll
    for (int s = 0; s < V; ++s) st2<NT>(reinterpret_cast<double2*>(yb + 2 * last_pass_index<M2, V>(tid, s)), acc[s]);
  } else {
    const int64_t left = a.out_len - ob;
#pragma unroll
    for (int s = 0; s < V; ++s) {
      const int o = 2 * last_pass_index<M2, V>(tid, s);
      if (o < left) yb[o] = acc[s].x;
      if (o + 1 < left) yb[o + 1] = acc[s].y;
    }
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
namespace {

// K3 for launches of two or more resident rounds (>= 1024 items):
// non-temporal Z loads and output stores (both streams are touched once; A/B
// on one box: step -1 ... -2.6 %, K3 187 -> 152-157 us, part of which
// reappears in the next kernel as deferred write-back).  Small launches (a
// streaming block, a host-pipeline segment) keep the cached path: their Z
// rows were just written by K2 and their output is read back right after.
bool k3_nt(int64_t items) { return items >= 1024; }

template <int M, int V>
void rfft_go(const RfftArgs& a, hipStream_t s) {
  using Plan = FftPlan<M, V>;
  const int64_t items = (int64_t)a.channels * a.jc;
  // Full F windows per workgroup once the launch fills the chip; a small
  // launch (a low-latency stage's few blocks, often read from mapped host
  // memory) spreads its windows over up to 256 workgroups instead.
  RfftArgs b = a;
  b.per_wg = (int)std::min<int64_t>(Plan::F, std::max<int64_t>(1, (items + 255) / 256));
  timed_launch(k_window_rfft<M, V>, dim3((unsigned)((items + b.per_wg - 1) / b.per_wg)), dim3(Plan::BLOCK), s, b);
}
template <int M>
void rfft_split_go(const RfftArgs& a, hipStream_t s) {
  const int64_t items = a.ord_R > 0 ? (int64_t)a.channels * (a.ord_ny + 1) * a.ord_R : (int64_t)a.channels * a.jc;
  const dim3 g((unsigned)items), b(SplitPlan<M, AD_K1_V>::T);
  timed_launch(k_window_rfft_split<M>, g, b, s, a);
}
template <int M, int V>
void irfft_go(const IrfftArgs& a, hipStream_t s) {
  using Plan = FftPlan<M, V>;
  const int64_t items = (int64_t)a.channels * a.jc;
  timed_launch(k_irfft_store<M, V>, dim3((unsigned)((items + Plan::F - 1) / Plan::F)), dim3(Plan::BLOCK), s, a);
}
template <int M>
void irfft_split_go(const IrfftArgs& a, hipStream_t s) {
  const int64_t items = a.ord_R > 0 ? (int64_t)a.channels * a.ord_ny * a.ord_R : (int64_t)a.channels * a.jc;
  const dim3 g((unsigned)items), b(SplitPlan<M, AD_K3_V>::T);
  if (k3_nt(items))
    timed_launch(k_irfft_store_split<M, true>, g, b, s, a);
  else
    timed_launch(k_irfft_store_split<M, false>, g, b, s, a);
}

#ifndef AD_K3MIX_V
#define AD_K3MIX_V 16  // same-box A/B (tools/shard_ab.sh): shard 62.9 (V = 8) -> 64.9-65.0 Gsamples/s, K3 599 -> 531 us
#endif
template <int M>
void irfft_mix_go(const IrfftArgs& a, hipStream_t s) {
  const dim3 g((unsigned)(2 * a.jc)), b(SplitPlan<M, AD_K3MIX_V>::T);
  if (k3_nt((int64_t)a.channels * a.jc))
    timed_launch(k_irfft_mix_split<M, true, AD_K3MIX_V>, g, b, s, a);
  else
    timed_launch(k_irfft_mix_split<M, false, AD_K3MIX_V>, g, b, s, a);
}

}  // namespace

bool launch_irfft_mix(int M, const IrfftArgs& a, hipStream_t s) {
  if (a.jc <= 0) return true;
  switch (M) {
    case 2048: irfft_mix_go<2048>(a, s); return true;
    case 4096: irfft_mix_go<4096>(a, s); return true;
    case 8192: irfft_mix_go<8192>(a, s); return true;
    default: return false;
  }
}

bool launch_window_rfft(int M, const RfftArgs& a, hipStream_t s) {
  if (a.channels <= 0 || a.jc <= 0) return true;
  switch (M) {
    case 16: rfft_go<16, 16>(a, s); return true;
    case 32: rfft_go<32, 16>(a, s); return true;
    case 64: rfft_go<64, 16>(a, s); return true;
    case 128: rfft_go<128, 16>(a, s); return true;
    case 256: rfft_go<256, 16>(a, s); return true;
    case 512: rfft_go<512, 16>(a, s); return true;
    case 1024: rfft_go<1024, 16>(a, s); return true;
    case 2048: rfft_split_go<2048>(a, s); return true;
    case 4096: rfft_split_go<4096>(a, s); return true;
    case 8192: rfft_split_go<8192>(a, s); return true;
    default: return false;
  }
}

bool launch_irfft_store(int M, const IrfftArgs& a, hipStream_t s) {
  if (a.channels <= 0 || a.jc <= 0) return true;
  switch (M) {
    case 16: irfft_go<16, 16>(a, s); return true;
    case 32: irfft_go<32, 16>(a, s); return true;
    case 64: irfft_go<64, 16>(a, s); return true;
    case 128: irfft_go<128, 16>(a, s); return true;
    case 256: irfft_go<256, 16>(a, s); return true;
    case 512: irfft_go<512, 16>(a, s); return true;
    case 1024: irfft_go<1024, 16>(a, s); return true;
    case 2048: irfft_split_go<2048>(a, s); return true;
    case 4096: irfft_split_go<4096>(a, s); return true;
    case 8192: irfft_split_go<8192>(a, s); return true;
    default: return false;
  }
}

}  // namespace adsp
