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
//   K2 k_fdl_mac     : Y[c][j] = sum_p X[c][j-p] * H[ir(c)][p]   (per bin)
//   K3 k_irfft_store : y[c][jL .. (j+1)L) = last L of irFFT_N(Y[c][j])
// H[p] = rFFT_N( h[pL .. (p+1)L) zero-padded ) is built by K1 at create time.
// X lives in a per-channel ring of Q blocks (frequency-domain delay line); the
// bins dimension is padded to MS = M + 8 complex128 so every row starts on a
// 128-byte line.
#include <hip/hip_runtime.h>

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
// K1: forward real FFT of one overlap-save window per (channel, block).
// ---------------------------------------------------------------------------
template <int M>
__global__ __launch_bounds__(FftPlan<M>::BLOCK) void k_window_rfft(RfftArgs a) {
  using Plan = FftPlan<M>;
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

  const double* xc = a.x + (int64_t)c * a.x_stride;
  const double* hc = a.xhist ? a.xhist + (int64_t)c * a.hist_stride : nullptr;
  const int64_t t0 = a.s0 + (int64_t)j * L - L;  // first sample of the 2L window

  double2 v[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int m = pass0_index<M>(tid, s);
    const int64_t t = t0 + 2 * m;
    double2 z;
    if (active && t >= 0 && t + 1 < a.n && a.aligned) {
      z = *reinterpret_cast<const double2*>(xc + t);
    } else if (!active) {
      z = make_double2(0.0, 0.0);
    } else {
      double r0, r1;
      r0 = (t < 0) ? (hc ? hc[L + t] : 0.0) : (t < a.n ? xc[t] : 0.0);
      r1 = (t + 1 < 0) ? (hc ? hc[L + t + 1] : 0.0) : (t + 1 < a.n ? xc[t + 1] : 0.0);
      z = make_double2(r0, r1);
    }
    v[s] = z;
  }

  if constexpr (Plan::NPASS > 1) {
    pass_compute_store<M, 0, true>(v, tid, lds, a.twM);
    run_middle_passes<M, true>(v, tid, lds, a.twM);
  }
  last_pass_compute<M, true>(v, tid, a.twM);

  // Exchange through LDS so each thread sees Z[k] and Z[M-k].
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 16; ++s) lds[lds_pad(last_pass_index<M>(tid, s))] = v[s];
  __syncthreads();
  if (!active) return;

  double2* Xo = a.X + (int64_t)c * a.x_ch_stride + (int64_t)((a.slot0 + j) % a.Q) * a.MS;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int k = tid + q * T;
    const double2 A = lds[lds_pad(k)];
    if (k == 0) {
      Xo[0] = make_double2(A.x + A.y, 0.0);
      Xo[M] = make_double2(A.x - A.y, 0.0);
    } else {
      const double2 B = c_conj(lds[lds_pad(M - k)]);
      const double2 fe = c_scale(c_add(A, B), 0.5);
      const double2 d = c_sub(A, B);
      const double2 fo = make_double2(0.5 * d.y, -0.5 * d.x);  // -i*(A-B)/2
      Xo[k] = c_add(fe, c_mul(a.twN[k], fo));
    }
  }
}

// ---------------------------------------------------------------------------
// K3: inverse real FFT of Y[c][j], keep the last L samples (overlap-save
// discard of the first N-L circular outputs), store to y.
// ---------------------------------------------------------------------------
template <int M>
__global__ __launch_bounds__(FftPlan<M>::BLOCK) void k_irfft_store(IrfftArgs a) {
  using Plan = FftPlan<M>;
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

  const double2* Yb = a.Y + (int64_t)c * a.y_ch_stride + (int64_t)j * a.MS;
  const double sc = 0.5 / (double)M;
  double2 v[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int m = pass0_index<M>(tid, s);
    double2 z = make_double2(0.0, 0.0);
    if (active) {
      const double2 A = Yb[m];
      const double2 B = c_conj(Yb[M - m]);
      const double2 fe = c_add(A, B);
      const double2 fo = c_mul(c_sub(A, B), c_conj(a.twN[m]));
      // Z = (fe + i*fo) / (2M)
      z = make_double2((fe.x - fo.y) * sc, (fe.y + fo.x) * sc);
    }
    v[s] = z;
  }

  if constexpr (Plan::NPASS > 1) {
    pass_compute_store<M, 0, false>(v, tid, lds, a.twM);
    run_middle_passes<M, false>(v, tid, lds, a.twM);
  }
  last_pass_compute<M, false>(v, tid, a.twM);
  if (!active) return;

  double* yc = a.out + (int64_t)c * a.out_stride;
  const int64_t ob = a.o0 + (int64_t)j * L - M;  // sample of window index 0 minus L
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int m = last_pass_index<M>(tid, s);
    if (m < M / 2) continue;
    const int64_t o = ob + 2 * m;
    if (o + 1 < a.out_len && a.aligned) {
      *reinterpret_cast<double2*>(yc + o) = v[s];
    } else {
      if (o < a.out_len) yc[o] = v[s].x;
      if (o + 1 < a.out_len) yc[o + 1] = v[s].y;
    }
  }
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
// Blocks with logical index < 0 (before the stream/signal start) read as
// zeros without touching memory, so an offline call needs no memset.  The
// warm-up group (the PC-1 spectra before the run) issues only the products
// that reach outputs of the run: every FMA issued is a useful one.
// 1-D grid, XCD-remapped so the runs of one bin group (which re-read each
// other's warm-up rows) share an L2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cmac(double2& s, const double2 x, const double2 h) {
  s.x = fma(x.x, h.x, s.x);
  s.x = fma(-x.y, h.y, s.x);
  s.y = fma(x.x, h.y, s.y);
  s.y = fma(x.y, h.x, s.y);
}

// Ring cursor over the X spectra of one lane's bin (wave-uniform state).
struct MacCursor {
  int64_t lx;  // logical spectrum index (< 0: before the signal, reads zero)
  int slot;    // ring slot of lx
  int Q;
  __device__ __forceinline__ double2 load(const double2* Xc, int MS) const {
    return (lx >= 0) ? Xc[(int64_t)slot * MS] : make_double2(0.0, 0.0);
  }
  __device__ __forceinline__ void advance() {
    ++lx;
    slot = (slot + 1 == Q) ? 0 : slot + 1;
  }
};

// Compile-time unrolled iteration bodies: template recursion keeps every
// accumulator / H index a constant so the arrays stay in VGPRs.
template <int PC, int U>
struct MacWarm {
  template <int Q = PC - U>
  __device__ static __forceinline__ void macs(double2 (&acc)[PC], const double2 (&h)[PC], const double2 x) {
    if constexpr (Q < PC) {
      cmac(acc[(U + Q) % PC], x, h[Q]);
      macs<Q + 1>(acc, h, x);
    }
  }
  __device__ static __forceinline__ void run(double2 (&acc)[PC], const double2 (&h)[PC], const double2* Xc, int MS,
                                             MacCursor& cur) {
    if constexpr (U < PC) {
      const double2 x = cur.load(Xc, MS);
      macs(acc, h, x);
      cur.advance();
      MacWarm<PC, U + 1>::run(acc, h, Xc, MS, cur);
    }
  }
};

template <int PC, int U>
struct MacMain {
  template <int Q = 0>
  __device__ static __forceinline__ void macs(double2 (&acc)[PC], const double2 (&h)[PC], const double2 x) {
    if constexpr (Q < PC) {
      cmac(acc[(U + Q) % PC], x, h[Q]);
      macs<Q + 1>(acc, h, x);
    }
  }
  __device__ static __forceinline__ void run(double2 (&acc)[PC], const double2 (&h)[PC], const double2* Xc,
                                             double2* Yc, int MS, MacCursor& cur, int i, int j1, bool first) {
    if constexpr (U < PC) {
      if (i + U >= j1) return;  // wave-uniform
      const double2 x = cur.load(Xc, MS);
      macs(acc, h, x);
      double2* yp = Yc + (int64_t)(i + U) * MS;
      if (first) {
        *yp = acc[U];
      } else {
        const double2 o = *yp;
        *yp = make_double2(o.x + acc[U].x, o.y + acc[U].y);
      }
      acc[U] = make_double2(0.0, 0.0);
      cur.advance();
      MacMain<PC, U + 1>::run(acc, h, Xc, Yc, MS, cur, i, j1, first);
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
  const int k = bx * 64 + threadIdx.x;
  if (k > a.M) return;
  const int j0 = ry * a.R;
  const int j1 = min(j0 + a.R, a.jc);
  const int ir = a.ir_index ? a.ir_index[c] : (c % a.n_ir);
  const double2* Hc = a.H + (int64_t)ir * a.h_ir_stride + k;
  const double2* Xc = a.X + (int64_t)c * a.x_ch_stride + k;
  double2* Yc = a.Y + (int64_t)c * a.y_ch_stride + k;

  for (int p0 = 0; p0 < a.P; p0 += PC) {
    double2 h[PC];
#pragma unroll
    for (int q = 0; q < PC; ++q) h[q] = (p0 + q < a.P) ? Hc[(int64_t)(p0 + q) * a.MS] : make_double2(0.0, 0.0);
    double2 acc[PC];
#pragma unroll
    for (int q = 0; q < PC; ++q) acc[q] = make_double2(0.0, 0.0);

    // logical spectrum index of iteration u of the warm-up group (u = 0..PC-1)
    MacCursor cur;
    cur.lx = a.g0 + j0 - PC - p0;
    cur.slot = (int)(((cur.lx % a.Q) + a.Q) % a.Q);
    cur.Q = a.Q;
    // --- warm-up: X[j0-PC+u] only feeds outputs >= j0 through q >= PC-u
    cur.advance();
    MacWarm<PC, 1>::run(acc, h, Xc, a.MS, cur);
    // --- run: outputs j0 .. j1-1, slot (o - j0) % PC
    for (int i = j0; i < j1; i += PC) {
      MacMain<PC, 0>::run(acc, h, Xc, Yc, a.MS, cur, i, j1, p0 == 0);
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
template <int M>
static void launch_rfft_m(const RfftArgs& a, hipStream_t s) {
  using Plan = FftPlan<M>;
  const int64_t ffts = (int64_t)a.channels * a.jc;
  const int64_t grid = (ffts + Plan::F - 1) / Plan::F;
  hipLaunchKernelGGL(k_window_rfft<M>, dim3((unsigned)grid), dim3(Plan::BLOCK), 0, s, a);
}
template <int M>
static void launch_irfft_m(const IrfftArgs& a, hipStream_t s) {
  using Plan = FftPlan<M>;
  const int64_t ffts = (int64_t)a.channels * a.jc;
  const int64_t grid = (ffts + Plan::F - 1) / Plan::F;
  hipLaunchKernelGGL(k_irfft_store<M>, dim3((unsigned)grid), dim3(Plan::BLOCK), 0, s, a);
}

#define AD_DISPATCH_M(M_, FN, ...) \
  switch (M_) {                    \
    case 16: FN<16>(__VA_ARGS__); break;     \
    case 32: FN<32>(__VA_ARGS__); break;     \
    case 64: FN<64>(__VA_ARGS__); break;     \
    case 128: FN<128>(__VA_ARGS__); break;   \
    case 256: FN<256>(__VA_ARGS__); break;   \
    case 512: FN<512>(__VA_ARGS__); break;   \
    case 1024: FN<1024>(__VA_ARGS__); break; \
    case 2048: FN<2048>(__VA_ARGS__); break; \
    case 4096: FN<4096>(__VA_ARGS__); break; \
    case 8192: FN<8192>(__VA_ARGS__); break; \
    default: return false;                   \
  }

bool launch_window_rfft(int M, const RfftArgs& a, hipStream_t s) {
  if (a.channels <= 0 || a.jc <= 0) return true;
  AD_DISPATCH_M(M, launch_rfft_m, a, s);
  return true;
}

bool launch_irfft_store(int M, const IrfftArgs& a, hipStream_t s) {
  if (a.channels <= 0 || a.jc <= 0) return true;
  AD_DISPATCH_M(M, launch_irfft_m, a, s);
  return true;
}

bool launch_fdl_mac(int PC, const MacArgs& in, int channels, hipStream_t s) {
  if (channels <= 0 || in.jc <= 0) return true;
  MacArgs a = in;
  a.nx = (a.M + 1 + 63) / 64;
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
