// Window real-FFT (K1) and inverse real-FFT + overlap-save store (K3) kernels
// of the UPOLS convolution engine (see conv_kernels.hip for the data flow).
//
// K1: X[c][g] = rFFT_N(x[(g-1)L .. (g+1)L)), N = 2L, M = L complex points,
//     via the half-length complex FFT of z[m] = x[2m] + i x[2m+1] and the
//     usual split into even/odd spectra (M+1 bins stored, DC and Nyquist real).
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

// Workgroups are dealt round-robin over the 8 XCDs (b % 8 share one L2).
// Remap the hardware index so each XCD owns a contiguous run of logical
// indices: neighbouring blocks (which share input samples) then run on the
// same XCD at about the same time.  Bijective for any grid size; a different
// placement changes speed only, never results.
__device__ __forceinline__ int xcd_remap_fft(int b, int G) {
  const int xcd = b & 7, r = b >> 3;
  const int q = G >> 3, rem = G & 7;
  return (xcd < rem) ? xcd * (q + 1) + r : rem * (q + 1) + (xcd - rem) * q + r;
}

__device__ __forceinline__ double2 fetch_pair(const double* xc, const double* hc, int64_t t, int64_t n, int L,
                                              bool aligned) {
  if (t >= 0 && t + 1 < n && aligned) return *reinterpret_cast<const double2*>(xc + t);
  const double r0 = (t < 0) ? (hc ? hc[L + t] : 0.0) : (t < n ? xc[t] : 0.0);
  const double r1 = (t + 1 < 0) ? (hc ? hc[L + t + 1] : 0.0) : (t + 1 < n ? xc[t + 1] : 0.0);
  return make_double2(r0, r1);
}

// Full FFT of the thread's V pass-0 values (forward or inverse).
template <int M, int V, bool FWD>
__device__ __forceinline__ void fft_run(double2* v, int tid, double2* lds, const double2* __restrict__ twM) {
  using Plan = FftPlan<M, V>;
  if constexpr (Plan::NPASS > 1) {
    pass_compute_store<M, V, 0, FWD>(v, tid, lds, twM);
    run_middle_passes<M, V, FWD>(v, tid, lds, twM);
  }
  last_pass_compute<M, V, FWD>(v, tid, twM);
}

// Forward post-processing: Z (in registers, last-pass order) -> X[0..M] in Xo.
template <int M, int V>
__device__ __forceinline__ void rfft_post_store(double2* v, int tid, double2* lds, double2* Xo,
                                                const double2* __restrict__ twN, bool active) {
  using Plan = FftPlan<M, V>;
  __syncthreads();
#pragma unroll
  for (int s = 0; s < V; ++s) lds[lds_pad(last_pass_index<M, V>(tid, s))] = v[s];
  __syncthreads();
  if (!active) return;
#pragma unroll
  for (int q = 0; q < V; ++q) {
    const int k = tid + q * Plan::T;
    const double2 A = lds[lds_pad(k)];
    if (k == 0) {
      Xo[0] = make_double2(A.x + A.y, 0.0);
      Xo[M] = make_double2(A.x - A.y, 0.0);
    } else {
      const double2 B = c_conj(lds[lds_pad(M - k)]);
      const double2 fe = c_scale(c_add(A, B), 0.5);
      const double2 d = c_sub(A, B);
      const double2 fo = make_double2(0.5 * d.y, -0.5 * d.x);  // -i*(A-B)/2
      Xo[k] = c_add(fe, c_mul(twN[k], fo));
    }
  }
}

// Inverse store: the upper half of the time window (m >= M/2) to y.
template <int M, int V>
__device__ __forceinline__ void irfft_store_out(const double2* v, int tid, double* yc, int64_t ob, int64_t out_len,
                                                bool aligned) {
#pragma unroll
  for (int s = 0; s < V; ++s) {
    const int m = last_pass_index<M, V>(tid, s);
    if (m < M / 2) continue;
    const int64_t o = ob + 2 * m;
    if (o + 1 < out_len && aligned) {
      *reinterpret_cast<double2*>(yc + o) = v[s];
    } else {
      if (o < out_len) yc[o] = v[s].x;
      if (o + 1 < out_len) yc[o + 1] = v[s].y;
    }
  }
}

// ---------------------------------------------------------------------------
// One-shot forms: F = BLOCK/T FFTs per workgroup, one (channel, block) each.
// ---------------------------------------------------------------------------
template <int M, int V>
__global__ __launch_bounds__((FftPlan<M, V>::BLOCK)) void k_window_rfft(RfftArgs a) {
  using Plan = FftPlan<M, V>;
  constexpr int T = Plan::T;
  constexpr int L = M;
  __shared__ __attribute__((aligned(16))) double2 lds_all[Plan::F * Plan::MP];
  const int f = threadIdx.x / T;
  const int tid = threadIdx.x % T;
  const int64_t e = (int64_t)xcd_remap_fft(blockIdx.x, gridDim.x) * Plan::F + f;
  const bool active = e < (int64_t)a.channels * a.jc;
  const int c = active ? (int)(e / a.jc) : 0;
  const int j = active ? (int)(e % a.jc) : 0;
  double2* lds = lds_all + f * Plan::MP;
  const double* xc = a.x + (int64_t)c * a.x_stride;
  const double* hc = a.xhist ? a.xhist + (int64_t)c * a.hist_stride : nullptr;
  const int64_t t0 = a.s0 + (int64_t)j * L - L;  // first sample of the 2L window

  double2 v[V];
#pragma unroll
  for (int s = 0; s < V; ++s)
    v[s] = active ? fetch_pair(xc, hc, t0 + 2 * pass0_index<M, V>(tid, s), a.n, L, a.aligned) : make_double2(0, 0);
  fft_run<M, V, true>(v, tid, lds, a.twM);
  double2* Xo = a.X + (int64_t)c * a.x_ch_stride + (int64_t)((a.slot0 + j) % a.Q) * a.MS;
  rfft_post_store<M, V>(v, tid, lds, Xo, a.twN, active);
}

template <int M, int V>
__global__ __launch_bounds__((FftPlan<M, V>::BLOCK)) void k_irfft_store(IrfftArgs a) {
  using Plan = FftPlan<M, V>;
  constexpr int T = Plan::T;
  constexpr int L = M;
  __shared__ __attribute__((aligned(16))) double2 lds_all[Plan::F * Plan::MP];
  const int f = threadIdx.x / T;
  const int tid = threadIdx.x % T;
  const int64_t e = (int64_t)xcd_remap_fft(blockIdx.x, gridDim.x) * Plan::F + f;
  const bool active = e < (int64_t)a.channels * a.jc;
  const int c = active ? (int)(e / a.jc) : 0;
  const int j = active ? (int)(e % a.jc) : 0;
  double2* lds = lds_all + f * Plan::MP;
  const double2* Zb = a.Y + (int64_t)c * a.y_ch_stride + (int64_t)j * a.MS;
  double2 v[V];
#pragma unroll
  for (int s = 0; s < V; ++s) v[s] = active ? Zb[pass0_index<M, V>(tid, s)] : make_double2(0.0, 0.0);
  fft_run<M, V, false>(v, tid, lds, a.twM);
  if (!active) return;
  irfft_store_out<M, V>(v, tid, a.out + (int64_t)c * a.out_stride, a.o0 + (int64_t)j * L - M, a.out_len, a.aligned);
}

// ---------------------------------------------------------------------------
// Persistent forms for one FFT per workgroup (M >= 2048 at V = 8).
// Each workgroup walks a contiguous range of (channel, block) items, so:
//  * K1 reads every input sample once: the upper half of window j is the
//    lower half of window j+1 and sits in the SAME thread's pass-0 slots
//    (slot (b, r+R0/2) of block j == slot (b, r) of block j+1), so it is
//    carried in registers, and the next block's upper half is prefetched
//    into registers while the current FFT runs;
//  * K3 prefetches the next block's Z while the current block transforms.
// With 1-2 FFT workgroups resident per CU (LDS-bound), this overlap of the
// HBM stream with the LDS/VALU phases is what keeps the kernels HBM-bound.
// ---------------------------------------------------------------------------
template <int M, int V>
__global__ __launch_bounds__((FftPlan<M, V>::BLOCK)) void k_window_rfft_p(RfftArgs a) {
  using Plan = FftPlan<M, V>;
  static_assert(Plan::F == 1, "persistent K1 needs one FFT per workgroup");
  constexpr int L = M;
  constexpr int R0 = Plan::R0;
  constexpr int HALF = R0 / 2;
  constexpr int NB = V / R0;
  constexpr int H = V / 2;
  __shared__ __attribute__((aligned(16))) double2 lds[Plan::MP];
  const int tid = threadIdx.x;
  const int64_t total = (int64_t)a.channels * a.jc;
  const int64_t e0 = total * blockIdx.x / gridDim.x;
  const int64_t e1 = total * (blockIdx.x + 1) / gridDim.x;

  double2 lo[H];  // raw lower half of the next window (= this window's upper half)
  double2 nx[H];  // raw upper half of the next window (prefetched)
  int c = (int)(e0 / a.jc);
  int j = (int)(e0 % a.jc) - 1;
  for (int64_t e = e0; e < e1; ++e) {
    if (++j == a.jc) {
      j = 0;
      ++c;
    }
    const double* xc = a.x + (int64_t)c * a.x_stride;
    const double* hc = a.xhist ? a.xhist + (int64_t)c * a.hist_stride : nullptr;
    const int64_t t0 = a.s0 + (int64_t)j * L - L;
    double2 v[V];
    if (e == e0 || j == 0) {
      if (a.aligned && t0 >= 0 && t0 + 2 * L <= a.n) {  // wave-uniform fast path
#pragma unroll
        for (int s = 0; s < V; ++s)
          v[s] = *reinterpret_cast<const double2*>(xc + t0 + 2 * pass0_index<M, V>(tid, s));
      } else {
#pragma unroll
        for (int s = 0; s < V; ++s)
          v[s] = fetch_pair(xc, hc, t0 + 2 * pass0_index<M, V>(tid, s), a.n, L, a.aligned);
      }
    } else {
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < HALF; ++r) {
          v[b * R0 + r] = lo[b * HALF + r];
          v[b * R0 + r + HALF] = nx[b * HALF + r];
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int r = 0; r < HALF; ++r) lo[b * HALF + r] = v[b * R0 + r + HALF];
    if (e + 1 < e1 && j + 1 < a.jc) {
      if (a.aligned && t0 + L >= 0 && t0 + 3 * L <= a.n) {  // wave-uniform fast path
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int r = 0; r < HALF; ++r)
            nx[b * HALF + r] =
                *reinterpret_cast<const double2*>(xc + t0 + L + 2 * pass0_index<M, V>(tid, b * R0 + r + HALF));
      } else {
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int r = 0; r < HALF; ++r)
            nx[b * HALF + r] =
                fetch_pair(xc, hc, t0 + L + 2 * pass0_index<M, V>(tid, b * R0 + r + HALF), a.n, L, a.aligned);
      }
    }
    if (e > e0) __syncthreads();  // the previous item's LDS reads are done
    // Opaque copy of tid: keeps the ~80 loop-invariant LDS/twiddle addresses
    // from being hoisted out of the item loop and pinned in VGPRs for its
    // whole length (they are cheap to recompute per item).
    int tid_i = tid;
    asm volatile("" : "+v"(tid_i));
    fft_run<M, V, true>(v, tid_i, lds, a.twM);
    double2* Xo = a.X + (int64_t)c * a.x_ch_stride + (int64_t)((a.slot0 + j) % a.Q) * a.MS;
    rfft_post_store<M, V>(v, tid_i, lds, Xo, a.twN, true);
  }
}

template <int M, int V>
__global__ __launch_bounds__((FftPlan<M, V>::BLOCK)) void k_irfft_store_p(IrfftArgs a) {
  using Plan = FftPlan<M, V>;
  static_assert(Plan::F == 1, "persistent K3 needs one FFT per workgroup");
  constexpr int L = M;
  __shared__ __attribute__((aligned(16))) double2 lds[Plan::MP];
  const int tid = threadIdx.x;
  const int64_t total = (int64_t)a.channels * a.jc;
  const int64_t e0 = total * blockIdx.x / gridDim.x;
  const int64_t e1 = total * (blockIdx.x + 1) / gridDim.x;
  if (e0 >= e1) return;

  double2 nz[V];  // Z of the next item (prefetched)
  int c = (int)(e0 / a.jc);
  int j = (int)(e0 % a.jc);
  {
    const double2* Zb = a.Y + (int64_t)c * a.y_ch_stride + (int64_t)j * a.MS;
#pragma unroll
    for (int s = 0; s < V; ++s) nz[s] = Zb[pass0_index<M, V>(tid, s)];
  }
  for (int64_t e = e0; e < e1; ++e) {
    double2 v[V];
#pragma unroll
    for (int s = 0; s < V; ++s) v[s] = nz[s];
    int cn = c, jn = j + 1;
    if (jn == a.jc) {
      jn = 0;
      ++cn;
    }
    if (e + 1 < e1) {
      const double2* Zn = a.Y + (int64_t)cn * a.y_ch_stride + (int64_t)jn * a.MS;
#pragma unroll
      for (int s = 0; s < V; ++s) nz[s] = Zn[pass0_index<M, V>(tid, s)];
    }
    if (e > e0) __syncthreads();  // the previous item's LDS reads are done
    int tid_i = tid;  // opaque per item (see k_window_rfft_p)
    asm volatile("" : "+v"(tid_i));
    fft_run<M, V, false>(v, tid_i, lds, a.twM);
    irfft_store_out<M, V>(v, tid_i, a.out + (int64_t)c * a.out_stride, a.o0 + (int64_t)j * L - M, a.out_len,
                          a.aligned);
    c = cn;
    j = jn;
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
namespace {

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

// Persistent grid: as many FFT workgroups as the CUs hold at once (LDS-bound).
int persistent_grid(int64_t items, int lds_bytes) {
  static int cus[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  int per_cu = std::max(1, (160 * 1024) / lds_bytes);
  per_cu = std::max(1, env_int("AD_P_WG_PER_CU", per_cu));
  return (int)std::min<int64_t>(items, (int64_t)cus[dev] * per_cu);
}

// FFT shape per size: values per thread and persistence (env overrides for A/B runs).
bool persistent_for(int M) { return M >= 2048 && env_int("AD_PERSISTENT", 1) != 0; }
int v_for(int M) {
  if (M < 2048) return 16;
  return env_int("AD_FFT_V", 8) == 16 ? 16 : 8;
}

template <int M, int V>
void rfft_go(const RfftArgs& a, hipStream_t s, bool persistent) {
  using Plan = FftPlan<M, V>;
  const int64_t items = (int64_t)a.channels * a.jc;
  if constexpr (Plan::F == 1) {
    if (persistent) {
      hipLaunchKernelGGL((k_window_rfft_p<M, V>), dim3((unsigned)persistent_grid(items, Plan::MP * 16)),
                         dim3(Plan::BLOCK), 0, s, a);
      return;
    }
  }
  hipLaunchKernelGGL((k_window_rfft<M, V>), dim3((unsigned)((items + Plan::F - 1) / Plan::F)), dim3(Plan::BLOCK), 0,
                     s, a);
}

template <int M, int V>
void irfft_go(const IrfftArgs& a, hipStream_t s, bool persistent) {
  using Plan = FftPlan<M, V>;
  const int64_t items = (int64_t)a.channels * a.jc;
  if constexpr (Plan::F == 1) {
    if (persistent) {
      hipLaunchKernelGGL((k_irfft_store_p<M, V>), dim3((unsigned)persistent_grid(items, Plan::MP * 16)),
                         dim3(Plan::BLOCK), 0, s, a);
      return;
    }
  }
  hipLaunchKernelGGL((k_irfft_store<M, V>), dim3((unsigned)((items + Plan::F - 1) / Plan::F)), dim3(Plan::BLOCK), 0,
                     s, a);
}

template <template <int, int> class Go, class A>
bool dispatch(int M, const A& a, hipStream_t s) {
  const bool p = persistent_for(M);
  const int V = v_for(M);
  switch (M) {
    case 16: Go<16, 16>::run(a, s, false); return true;
    case 32: Go<32, 16>::run(a, s, false); return true;
    case 64: Go<64, 16>::run(a, s, false); return true;
    case 128: Go<128, 16>::run(a, s, false); return true;
    case 256: Go<256, 16>::run(a, s, false); return true;
    case 512: Go<512, 16>::run(a, s, false); return true;
    case 1024: Go<1024, 16>::run(a, s, false); return true;
    case 2048: V == 8 ? Go<2048, 8>::run(a, s, p) : Go<2048, 16>::run(a, s, false); return true;
    case 4096: V == 8 ? Go<4096, 8>::run(a, s, p) : Go<4096, 16>::run(a, s, p); return true;
    case 8192: V == 8 ? Go<8192, 8>::run(a, s, p) : Go<8192, 16>::run(a, s, false); return true;
    default: return false;
  }
}

template <int M, int V>
struct RfftGo {
  static void run(const RfftArgs& a, hipStream_t s, bool p) { rfft_go<M, V>(a, s, p); }
};
template <int M, int V>
struct IrfftGo {
  static void run(const IrfftArgs& a, hipStream_t s, bool p) { irfft_go<M, V>(a, s, p); }
};

}  // namespace

bool launch_window_rfft(int M, const RfftArgs& a, hipStream_t s) {
  if (a.channels <= 0 || a.jc <= 0) return true;
  return dispatch<RfftGo>(M, a, s);
}

bool launch_irfft_store(int M, const IrfftArgs& a, hipStream_t s) {
  if (a.channels <= 0 || a.jc <= 0) return true;
  return dispatch<IrfftGo>(M, a, s);
}

}  // namespace adsp
