// HIP kernels of the uniformly partitioned overlap-save (UPOLS) convolution
// engine and the time-domain convolution forms, hand-written for gfx950.
//
// Reference behaviour being accelerated (all paths compute the linear
// convolution y[t] = sum_k h[k] x[t-k] of the reference):
//   StreamingOverlapSaveT.processBlockCore  dsp/conv/streaming_overlap_save.go:100-133
//   StreamingOverlapAddT.processBlockCore   dsp/conv/streaming_overlap_add.go:98-133
//   OverlapSave.Process                     dsp/conv/overlap_save.go:126-254
//   OverlapAdd.Process                      dsp/conv/overlap_add.go:108-164
//   PartitionedConvolutionT.ProcessBlock    dsp/conv/partitioned.go:348-396
//   DirectTo / directToSIMD                 dsp/conv/conv.go:97-154
//
// UPOLS data flow for hop L (= M, a power of two), real FFT size N = 2L:
//   K1 k_window_rfft : X[c][g] = rFFT_N( x[(g-1)L .. (g+1)L) )   -> M+1 bins
//   K2 k_fdl_mac     : Y[c][j] = sum_p X[c][j-p] * H[ir(c)][p]   (per bin),
//                      folded to the half-length spectrum Z[c][j] (M bins)
//   K3 k_irfft_store : y[c][jL .. (j+1)L) = last L of irFFT_N(Y[c][j])
// K1/K3 live in fft_kernels.hip, K2 and the time-domain forms here.
// H[p] = rFFT_N( h[pL .. (p+1)L) zero-padded ) is built by K1 at create time.
// X lives in a per-channel ring of Q blocks (frequency-domain delay line); the
// bins dimension is padded to MS = M + 8 complex128 so every row starts on a
// 128-byte line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "conv_kernels.hpp"
#include "fft_device.hpp"

namespace adsp {

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

// ---------------------------------------------------------------------------
// K2: frequency-domain delay-line multiply-accumulate.
//   Y[c][j][k] = sum_{p<P} X[c][g0+j-p][k] * H[ir(c)][p][k]
// One lane per bin k; a wave owns 64 consecutive bins of one channel and a
// run of R output blocks.  PC partitions' spectra sit in VGPRs; the X stream
// is read once per run and every X value feeds PC rotating accumulators whose
// slots are compile-time indices (the unrolled u/q loops), so the kernel
// reads each spectrum once and writes each output once.  P > PC is handled
// by sweeping partition chunks, read-modify-writing Y.
//
// Blocks with logical index < 0 (before the stream/signal start) read the
// ring's zero row, so an offline call needs no memset.  The warm-up group
// (the PC-1 spectra before the run) issues only the products that reach
// outputs of the run: every FMA issued is a useful one.
// 1-D grid, XCD-remapped so the runs of one bin group (which re-read each
// other's warm-up rows) share an L2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cmac(double2& s, const double2 x, const double2 h) {
  s.x = fma(x.x, h.x, s.x);
  s.x = fma(-x.y, h.y, s.x);
  s.y = fma(x.x, h.y, s.y);
  s.y = fma(x.y, h.x, s.y);
}

// Loads xg[U0..U1) of a group of PC consecutive spectra whose first logical
// index is lx0 (ring slot s0).  Branch-free: spectra before the signal start
// (logical index < 0) read the ring's zero row (slot Q), and spectra past the
// run read stale ring rows whose products only reach outputs that are never
// stored, so every load is a plain, hoistable global load.
template <int PC, int U0, int U1>
__device__ __forceinline__ void load_span(double2 (&xg)[PC], const double2* __restrict__ Xc, int Q, int MS,
                                          int64_t lx0, int s0) {
#pragma unroll
  for (int u = U0; u < U1; ++u) {
    int sl = s0 + u;
    if (sl >= Q) sl -= Q;
    const int row = (lx0 + u >= 0) ? sl : Q;
    xg[u] = Xc[(int64_t)row * MS];
  }
}

// Warm-up products: X[j0-PC+u] only reaches outputs >= j0 through q >= PC-u.
template <int PC, int U>
struct MacWarm {
  template <int Q = PC - U>
  __device__ static __forceinline__ void macs(double2 (&acc)[PC], const double2 (&h)[PC], const double2 x) {
    if constexpr (Q < PC) {
      cmac(acc[(U + Q) % PC], x, h[Q]);
      macs<Q + 1>(acc, h, x);
    }
  }
  __device__ static __forceinline__ void run(double2 (&acc)[PC], const double2 (&h)[PC], const double2 (&xg)[PC]) {
    if constexpr (U < PC) {
      macs(acc, h, xg[U]);
      MacWarm<PC, U + 1>::run(acc, h, xg);
    }
  }
};

// Epilogue of one output spectrum of one lane: turns the product spectrum Y
// into the half-length complex spectrum Z that the inverse real FFT starts
// from, Z[m] = (Y[m] + conj Y[M-m] + i (Y[m] - conj Y[M-m]) W_2M^-m) / 2M,
// and stores (or accumulates, for partition chunks after the first) it.
// Lanes l and l+32 of a pair wave hold mirror bins, so the partner value is
// one cross-lane swap away; the mirror-free middle bin M/2 has its own wave.
struct ZEpilogue {
  double2* zc;     // Z row base of this lane's output index (nullptr: no output)
  double2 tw;      // conj(W_2M^m) * (0.5 / M)
  bool paired;     // pair wave (partner in lane ^ 32) vs the self-paired middle bin
  int MS;
  __device__ __forceinline__ void store(const double2 y, int64_t j, bool first) const {
    double2 p;
    if (paired) {
      p.x = __shfl_xor(y.x, 32);
      p.y = __shfl_xor(y.y, 32);
    } else {
      p = y;
    }
    if (!zc) return;
    const double2 fe = make_double2(y.x + p.x, y.y - p.y);  // Y + conj(P)
    const double2 d = make_double2(y.x - p.x, y.y + p.y);   // Y - conj(P)
    const double2 fo = c_mul(d, tw);
    const double2 z = make_double2(fe.x * tw_scale - fo.y, fe.y * tw_scale + fo.x);
    double2* zp = zc + j * MS;
    if (first) {
      *zp = z;
    } else {
      const double2 o = *zp;
      *zp = make_double2(o.x + z.x, o.y + z.y);
    }
  }
  double tw_scale;  // 0.5 / M (applied to fe; tw already carries it for fo)
};

// Iterations U..UE-1 of a run group: PC products per spectrum into the
// rotating accumulators, then the finished output (slot U) is stored.
template <int PC, int U, int UE>
struct MacSpan {
  template <int Q = 0>
  __device__ static __forceinline__ void macs(double2 (&acc)[PC], const double2 (&h)[PC], const double2 x) {
    if constexpr (Q < PC) {
      cmac(acc[(U + Q) % PC], x, h[Q]);
      macs<Q + 1>(acc, h, x);
    }
  }
  __device__ static __forceinline__ void run(double2 (&acc)[PC], const double2 (&h)[PC], const double2 (&xg)[PC],
                                             const ZEpilogue& epi, int i, int j1, bool first) {
    if constexpr (U < UE) {
      macs(acc, h, xg[U]);
      if (i + U < j1) epi.store(acc[U], i + U, first);  // wave-uniform
      acc[U] = make_double2(0.0, 0.0);
      MacSpan<PC, U + 1, UE>::run(acc, h, xg, epi, i, j1, first);
    }
  }
};

template <int PC>
__global__ __launch_bounds__(64) void k_fdl_mac(MacArgs a) {
  const int lg = xcd_remap(blockIdx.x, gridDim.x);
  const int ry = lg % a.ny;
  const int t = lg / a.ny;
  const int bx = t % a.nx;
  const int c = t / a.nx;
  const int lane = threadIdx.x;
  // bin of this lane: pair waves cover [0, M/2) in lanes 0-31 and the mirror
  // bins (M/2, M] in lanes 32-63; the last wave carries the middle bin M/2.
  const bool paired = bx < a.M / 64;
  int k;
  if (paired) {
    k = (lane < 32) ? bx * 32 + lane : a.M - (bx * 32 + lane - 32);
  } else {
    if (lane != 0) return;
    k = a.M / 2;
  }
  const int j0 = ry * a.R;
  const int j1 = min(j0 + a.R, a.jc);
  const int ir = a.ir_index ? a.ir_index[c] : (c % a.n_ir);
  const double2* Hc = a.H + (int64_t)ir * a.h_ir_stride + k;
  const double2* Xc = a.X + (int64_t)c * a.x_ch_stride + k;
  ZEpilogue epi;
  epi.paired = paired;
  epi.MS = a.MS;
  epi.tw_scale = 0.5 / (double)a.M;
  if (k < a.M) {
    epi.zc = a.Y + (int64_t)c * a.y_ch_stride + k;
    epi.tw = c_scale(c_conj(a.twN[k]), epi.tw_scale);
  } else {
    epi.zc = nullptr;  // the Nyquist lane only feeds its partner (bin 0)
    epi.tw = make_double2(0.0, 0.0);
  }

  for (int p0 = 0; p0 < a.P; p0 += PC) {
    double2 h[PC];
#pragma unroll
    for (int q = 0; q < PC; ++q) h[q] = (p0 + q < a.P) ? Hc[(int64_t)(p0 + q) * a.MS] : make_double2(0.0, 0.0);
    double2 acc[PC];
#pragma unroll
    for (int q = 0; q < PC; ++q) acc[q] = make_double2(0.0, 0.0);

    constexpr int HH = PC / 2 > 0 ? PC / 2 : 1;
    double2 xg[PC];
    // --- warm-up group: spectra j0-PC .. j0-1 (slot u = 0 feeds nothing)
    int64_t lx = a.g0 + j0 - PC - p0;
    int sl = (int)(((lx % a.Q) + a.Q) % a.Q);
    load_span<PC, 1, PC>(xg, Xc, a.Q, a.MS, lx, sl);
    MacWarm<PC, 1>::run(acc, h, xg);
    lx += PC;
    sl += PC;
    if (sl >= a.Q) sl -= a.Q;
    // --- run groups, software pipelined: the second half of a group is
    // loaded when the group starts, the next group's first half while the
    // second half computes.
    load_span<PC, 0, HH>(xg, Xc, a.Q, a.MS, lx, sl);
    for (int i = j0; i < j1; i += PC) {
      load_span<PC, HH, PC>(xg, Xc, a.Q, a.MS, lx, sl);
      MacSpan<PC, 0, HH>::run(acc, h, xg, epi, i, j1, p0 == 0);
      lx += PC;
      sl += PC;
      if (sl >= a.Q) sl -= a.Q;
      if (i + PC < j1) load_span<PC, 0, HH>(xg, Xc, a.Q, a.MS, lx, sl);
      MacSpan<PC, HH, PC>::run(acc, h, xg, epi, i, j1, p0 == 0);
    }
  }
}

// ---------------------------------------------------------------------------
// Direct convolution, bit-exact with conv.DirectTo (conv.go:97-154):
// each dst[k] accumulates a[i]*b[k-i] in increasing i with a rounded product
// and a rounded add (vecmath.ScaleBlock then AddBlockInPlace, no FMA).
// Output-stationary: one lane per output sample, so no atomics are needed and
// the accumulation order is exactly the reference's.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_direct(const double* __restrict__ a, int64_t n, const double* __restrict__ b,
                                                int64_t m, double* __restrict__ dst) {
#pragma clang fp contract(off)
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n + m - 1) return;
  const int64_t lo = k - m + 1 > 0 ? k - m + 1 : 0;
  const int64_t hi = k < n - 1 ? k : n - 1;
  double acc = 0.0;
  for (int64_t i = lo; i <= hi; ++i) {
    const double t = b[k - i] * a[i];
    acc = acc + t;
  }
  dst[k] = acc;
}

// conv.DirectCircularTo (conv.go:176-189): dst[(i+j)%n] += a[i]*b[j], i outer.
// For output k the terms arrive in increasing i with j = (k - i) mod n.
__global__ __launch_bounds__(256) void k_direct_circular(const double* __restrict__ a, const double* __restrict__ b,
                                                         int64_t n, double* __restrict__ dst) {
#pragma clang fp contract(off)
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  double acc = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    int64_t jj = k - i;
    if (jj < 0) jj += n;
    const double t = a[i] * b[jj];
    acc = acc + t;
  }
  dst[k] = acc;
}

// Streaming time-domain convolution for hop sizes too small for the FFT
// path: buf = [history (K-1) | new block (B)], y[i] = sum_k h[k] buf[K-1+i-k].
__global__ __launch_bounds__(256) void k_stream_direct(const double* __restrict__ h, int64_t K,
                                                       const double* __restrict__ buf, int64_t B,
                                                       double* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= B) return;
  const double* xp = buf + (K - 1) + i;
  double acc = 0.0;
  for (int64_t k = 0; k < K; ++k) acc = fma(h[k], xp[-k], acc);
  y[i] = acc;
}

// Stereo mixdown: mix[0][t] = sum over even channels, mix[1][t] = odd channels.
__global__ __launch_bounds__(256) void k_mixdown(const double* __restrict__ ch, int channels, int64_t stride,
                                                 int64_t len, double* __restrict__ mix) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= len) return;
  double l = 0.0, r = 0.0;
  for (int c = 0; c < channels; c += 2) l += ch[(int64_t)c * stride + t];
  for (int c = 1; c < channels; c += 2) r += ch[(int64_t)c * stride + t];
  mix[t] = l;
  mix[len + t] = r;
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
bool launch_fdl_mac(int PC, const MacArgs& in, int channels, hipStream_t s) {
  if (channels <= 0 || in.jc <= 0) return true;
  MacArgs a = in;
  if (a.M < 64) return false;  // pair waves need M/2 >= 32 bins
  a.nx = a.M / 64 + 1;         // pair waves + the middle-bin wave
  a.ny = (a.jc + a.R - 1) / a.R;
  dim3 grid((unsigned)((int64_t)channels * a.nx * a.ny));
  switch (PC) {
    case 1: hipLaunchKernelGGL(k_fdl_mac<1>, grid, dim3(64), 0, s, a); break;
    case 2: hipLaunchKernelGGL(k_fdl_mac<2>, grid, dim3(64), 0, s, a); break;
    case 4: hipLaunchKernelGGL(k_fdl_mac<4>, grid, dim3(64), 0, s, a); break;
    case 8: hipLaunchKernelGGL(k_fdl_mac<8>, grid, dim3(64), 0, s, a); break;
    case 16: hipLaunchKernelGGL(k_fdl_mac<16>, grid, dim3(64), 0, s, a); break;
    case 32: hipLaunchKernelGGL(k_fdl_mac<32>, grid, dim3(64), 0, s, a); break;
    default: return false;
  }
  return true;
}

void launch_direct(const double* a, int64_t n, const double* b, int64_t m, double* dst, hipStream_t s) {
  const int64_t out = n + m - 1;
  hipLaunchKernelGGL(k_direct, dim3((unsigned)((out + 255) / 256)), dim3(256), 0, s, a, n, b, m, dst);
}

void launch_direct_circular(const double* a, const double* b, int64_t n, double* dst, hipStream_t s) {
  hipLaunchKernelGGL(k_direct_circular, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, b, n, dst);
}

void launch_stream_direct(const double* h, int64_t K, const double* buf, int64_t B, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_stream_direct, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, h, K, buf, B, y);
}

void launch_mixdown(const double* ch, int channels, int64_t stride, int64_t len, double* mix, hipStream_t s) {
  hipLaunchKernelGGL(k_mixdown, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, s, ch, channels, stride, len, mix);
}

}  // namespace adsp
