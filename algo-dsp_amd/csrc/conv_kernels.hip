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
//   K1 k_window_rfft : Zr[c][g] = packed FFT_M of x[(g-1)L .. (g+1)L)  (M values)
//   K2 k_fdl_mac     : X = separate(Zr) (bins 0..M, on load),
//                      Y[c][j] = sum_p X[c][j-p] * H[ir(c)][p]   (per bin),
//                      folded to the half-length spectrum Z[c][j] (M bins)
//   K3 k_irfft_store : y[c][jL .. (j+1)L) = last L of irFFT_N(Y[c][j])
// K1/K3 live in fft_kernels.hip, K2 and the time-domain forms here.
// H[p] (packed spectra of h[pL .. (p+1)L) zero-padded) is built by K1 at
// create time and separated like X.
// X lives in a per-channel ring of Q blocks (frequency-domain delay line); the
// bins dimension is padded to MS = M + 8 complex128 so every row starts on a
// 128-byte line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "blocked_dot.hpp"
#include "conv_kernels.hpp"
#include "fft_device.hpp"

namespace adsp {

// ---------------------------------------------------------------------------
// K2: frequency-domain delay-line multiply-accumulate.
//   Y[c][j][k] = sum_{p<P} X[c][g0+j-p][k] * H[ir(c)][p][k]
// Bin-stationary: a lane owns one bin k for a run of R output blocks, keeps
// PC partitions' spectra in VGPRs and feeds every X value it loads into PC
// rotating accumulators whose slots are compile-time indices (unrolled u/q
// loops), so X is read once per run and every output written once.
//
// Wave layout (NH = 2, P > 1): lane = ph*32 + mi*16 + l.
//   ph  partition half: lanes 32-63 take partitions [PC, 2PC) of the chunk,
//       reading the X stream PC rows earlier; the halves' sums meet in one
//       v_permlane32_swap before the store (only ph = 0 stores);
//   mi  mirror: bins 16bx + l (mi = 0) and M - (16bx + l) (mi = 1), so the
//       conj(Zr[M-k]) that separates K1's packed spectrum, and the Y[M-m]
//       that folds the output for K3, are one v_permlane16_swap away.
// Halving the partitions per lane halves the VGPRs (h, accumulators and the
// X group), which doubles the waves per SIMD and the loads in flight: K2 is
// bound by HBM latency x loads in flight, not by its FP64 FMAs.
// NH = 1 (P = 1): lane = mi*32 + l, 32 bin pairs per wave.
// The last wave (bx = M/(32/NH*2)) carries the self-mirrored middle bin M/2.
// P > NH*PC is handled by one launch per partition chunk, the later ones
// read-modify-writing Z (FIRST = false).
//
// Blocks with logical index < 0 (before the stream/signal start) read the
// ring's zero row, so an offline call needs no memset.  The warm-up group
// (the PC-1 spectra before the run) issues only the products that reach
// outputs of the run.
// 1-D grid, XCD-remapped so the runs of one bin group (which re-read each
// other's warm-up rows) share an L2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void cmac(double2& s, const double2 x, const double2 h) {
  s.x = fma(x.x, h.x, s.x);
  s.x = fma(-x.y, h.y, s.x);
  s.y = fma(x.x, h.y, s.y);
  s.y = fma(x.y, h.x, s.y);
}

// Ring-slot walker over this lane's block-spectrum stream.  Branch-free:
// blocks before the signal start (logical index < 0) and after its last
// input block (> gend) read the ring's zero row (slot Q), so every load is a
// plain global load.
struct XStream {
  const double2* Xc;
  int Q, MS;
  int64_t lx;    // logical index of row 0 of the current group (wave-uniform, ph = 0)
  int64_t gend;  // last logical block holding input
  int sl;        // its ring slot (wave-uniform)
  int dph;       // row offset of the ph = 1 half (-PC)
  bool ph;
  __device__ __forceinline__ int slot(int off) const {  // wave-uniform
    int s = sl + off;
    if (s >= Q) s -= Q;
    if (s < 0) s += Q;
    const int64_t g = lx + off;
    return (g >= 0 && g <= gend) ? s : Q;
  }
  __device__ __forceinline__ double2 load(int off) const {  // row lx + off (+ dph for ph = 1)
    const int r0 = slot(off), r1 = slot(off + dph);
    const int row = ph ? r1 : r0;
    return Xc[(int64_t)row * MS];
  }
  template <int PC>
  __device__ __forceinline__ void advance() {
    lx += PC;
    sl += PC;
    if (sl >= Q) sl -= Q;
  }
};

// Lane-pair exchange with v_permlane{32,16}_swap (no LDS round trip; all 64
// lanes active).  For a lane pair (lower, upper) = (bit clear, bit set) of
// lane bit 5 (B32) or bit 4, xpair returns u, v with
//   lower lane: u = own value, v = partner's;  upper lane: u = partner's, v = own.
// Consumers use only u + v, u - v and a per-lane sign s = +1 (lower) / -1
// (upper) folded into constants, so no select is needed after the swap.
template <bool B32>
__device__ __forceinline__ void xpair(double a, double& u, double& v) {
  const int lo = __double2loint(a), hi = __double2hiint(a);
  if constexpr (B32) {
    const auto r = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto t = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    u = __hiloint2double(t[0], r[0]);
    v = __hiloint2double(t[1], r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto t = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    u = __hiloint2double(t[0], r[0]);
    v = __hiloint2double(t[1], r[1]);
  }
  asm volatile("" : "+v"(u), "+v"(v));  // materialise here: keeps the swap's temporaries short-lived
}
template <bool B32>
__device__ __forceinline__ void xpair(double2 a, double2& u, double2& v) {
  xpair<B32>(a.x, u.x, v.x);
  xpair<B32>(a.y, u.y, v.y);
}

// The window spectrum of output block g from K1's block spectra:
// Zr[g][k] = P[g-1][k] + (-1)^k P[g][k] (fft_kernels.hip).  A lane walks its
// stream in block order; the previous row's value waits in a per-lane LDS
// cell (not in VGPRs: K2 at PC = 16 sits at its register cap), and (-1)^k is
// a sign bit on the high dword (k's parity is the lane's: mirror partners
// M-k share it, the middle bin M/2 is even).
// v * (+1 or -1) as a sign-bit flip of the high dword (m = 0 or 0x80000000):
// exact, and one 32-bit mask per lane instead of a double or a pre-signed
// copy of each constant.
__device__ __forceinline__ double flip(double v, int m) {
  return __hiloint2double(__double2hiint(v) ^ m, __double2loint(v));
}

struct BlockPair {
  double2 prev;  // this lane's P[g-1]
  int smask;     // 0 or 0x80000000
  __device__ __forceinline__ double2 next(const double2 cur) {
    const double2 z = make_double2(prev.x + flip(cur.x, smask), prev.y + flip(cur.y, smask));
    prev = cur;
    return z;
  }
};

// Separation of the window's packed spectrum Zr into the real-signal spectrum (x2):
//   X'[k] = (A + B) - i W_2M^k (A - B),  A = Zr[k], B = conj Zr[M-k]   (= 2 X[k])
// with A, conj(B) the mirror pair (u, v) of xpair:
//   X'.x = (u.x + v.x) + W.x (u.y + v.y) + s W.y (u.x - v.x)
//   X'.y = s (u.y - v.y) + W.y (u.y + v.y) - s W.x (u.x - v.x)
// The middle-bin wave holds M/2 in every lane, so its "mirror" lane holds the
// same bin and the formula needs no special case.  The factor 2 of X' and of
// H' is taken out in the Z epilogue's scale.
template <int NH>
struct Unpack {
  double2 tw;  // W_2M^k (k = M: -1)
  int m;       // sign of s: 0 lower mirror lane (+1), 0x80000000 upper (-1)
  __device__ __forceinline__ double2 operator()(const double2 a) const {
    double2 u, v;
    xpair<NH == 1>(a, u, v);
    const double sx = u.x + v.x, sy = u.y + v.y;
    const double sdx = flip(u.x - v.x, m), sdy = flip(u.y - v.y, m);  // s (u - v), exact
    return make_double2(fma(tw.y, sdx, fma(tw.x, sy, sx)), fma(-tw.x, sdx, fma(tw.y, sy, sdy)));
  }
};

// Epilogue of one output spectrum of one lane: adds the other partition
// half's sum (NH = 2), then turns the product spectrum Y into the
// half-length complex spectrum Z that the inverse real FFT starts from,
// Z[m] = (Y[m] + conj Y[M-m] + i (Y[m] - conj Y[M-m]) W_2M^-m) / 2M
// (Y here is 4x the product spectrum: see Unpack), and stores (or
// accumulates, for partition chunks after the first) it.  With (u, v) the
// mirror pair of Y, t = conj(W_2M^m) * S and S = 1/8M:
//   Z.x = (u.x + v.x) S - s t.y (u.x - v.x) - t.x (u.y + v.y)
//   Z.y = s S (u.y - v.y) + s t.x (u.x - v.x) - t.y (u.y + v.y)
template <int NH>
struct ZEpilogue {
  double2* zb;      // Z row 0 of the channel (wave-uniform)
  unsigned zo;      // this lane's bin position in a row (bin M: the row's padding column M);
                    // a 32-bit lane offset from a uniform row base keeps the store
                    // address out of a 64-bit VGPR pair
  int64_t jstride;  // MS
  double2 tw;       // t = conj(W_2M^m) * S
  double S;         // 1/8M (wave-uniform)
  int m;            // sign of s (see Unpack)
  // Unconditional (branch-free) store: rows past the run land in the spare
  // rows after jc_max (or in rows >= jc that K3 never reads), so the wave's
  // vmcnt bookkeeping stays exact across the group loop.  Lanes that carry
  // the same bin (the two partition halves; every lane of the middle-bin
  // wave) hold bit-identical z (a + b == b + a) and store it to the same
  // address in the same instruction; bin M stores into padding column M.
  template <bool FIRST>
  __device__ __forceinline__ void store(double2 y, int64_t j) const {

    if constexpr (NH == 2) {
      double2 a, b;
      xpair<true>(y, a, b);
      y = make_double2(a.x + b.x, a.y + b.y);
    }
    double2 u, v;
    xpair<NH == 1>(y, u, v);
    const double sx = u.x + v.x, sy = u.y + v.y;
    const double sdx = flip(u.x - v.x, m), sdy = flip(u.y - v.y, m);  // s (u - v), exact
    const double2 z = make_double2(fma(-tw.x, sy, fma(-tw.y, sdx, sx * S)), fma(-tw.y, sy, fma(tw.x, sdx, S * sdy)));
    double2* zp = (zb + j * jstride) + zo;
    if constexpr (FIRST) {
#ifdef AD_K2_NT  // tools/ A/B builds only
      typedef double d2v __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(d2v{z.x, z.y}, reinterpret_cast<d2v*>(zp));
#else
      *zp = z;
#endif
    } else {
      const double2 o = *zp;
      *zp = make_double2(o.x + z.x, o.y + z.y);
    }
  }
};

// Row U of a group of PC rows: the X value prefetched D rows earlier is
// separated and fed to the rotating accumulators, and row U + D is
// prefetched into the freed ring entry (xb[U % D]; PC % D == 0 keeps the
// index compile-time across groups).  WARM: the group before the run, whose
// row U only reaches outputs of the run through partitions q >= PC - U.
// Otherwise the finished output (slot U) is stored (outputs past the run
// land in rows nobody reads; see ZEpilogue).
template <int PC, int D, int U, bool WARM>
struct Row {
  template <int Q>
  __device__ static __forceinline__ void macs(double2 (&acc)[PC], const double2 (&h)[PC], const double2 x) {
    if constexpr (Q < PC) {
      cmac(acc[(U + Q) % PC], x, h[Q]);
      macs<Q + 1>(acc, h, x);
    }
  }
  template <bool FIRST, class UP, class EPI>
  __device__ static __forceinline__ void run(double2 (&acc)[PC], const double2 (&h)[PC], double2 (&xb)[D],
                                             const XStream& st, BlockPair& bp, const UP& up, const EPI& epi,
                                             int i) {
    if constexpr (U < PC) {
      const double2 x = up(bp.next(xb[U % D]));
      xb[U % D] = st.load(U + D);
      if constexpr (WARM) {
        macs<PC - U>(acc, h, x);
      } else {
        macs<0>(acc, h, x);
        epi.template store<FIRST>(acc[U], i + U);
        acc[U] = make_double2(0.0, 0.0);
      }
      __builtin_amdgcn_sched_barrier(0);
      Row<PC, D, U + 1, WARM>::template run<FIRST>(acc, h, xb, st, bp, up, epi, i);
    }
  }
};

// Occupancy target (waves per SIMD): the scheduler otherwise hoists loads
// for ILP at the cost of occupancy, and K2 wants loads in flight per CU.
template <int PC, int NH>
struct MacOcc {
  static constexpr int W = PC <= 4 ? 4 : (PC == 8 ? 3 : 2);
};
// X prefetch depth DQ (rows in flight per lane, <= PC so the ring index stays
// compile-time across groups).
template <int PC, int NH, bool FIRST, int DQ>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MacOcc<PC, NH>::W))) void k_fdl_mac(MacArgs a) {
  constexpr int BW = 32 / NH;  // bin pairs per wave
  const int lg = xcd_remap(blockIdx.x, gridDim.x);
  // neighbouring waves: consecutive runs of one bin group (they re-read each
  // other's warm-up rows)
  const int ry = lg % a.ny;
  const int bx = (lg / a.ny) % a.nx;
  const int c = lg / a.ny / a.nx;
  const int lane = threadIdx.x;
  const bool ph = NH == 2 && lane >= 32;
  const bool mi = NH == 2 ? ((lane >> 4) & 1) : (lane >> 5);
  const int l = lane & (BW - 1);
  // pair waves: bins [0, M/2) (mi = 0) and their mirrors (M/2, M] (mi = 1);
  // the last wave: the middle bin M/2 in every lane, stored by lane 0.
  const bool paired = bx < a.M / (2 * BW);
  const int k = paired ? (mi ? a.M - (bx * BW + l) : bx * BW + l) : a.M / 2;
  const int j0 = ry * a.R;
  const int j1 = min(j0 + a.R, a.jc);
  const int ir = a.ir_index ? a.ir_index[c] : (c % a.n_ir);
  const int kz = k & (a.M - 1);  // raw spectrum index: bin M reads Zr[0]
  const double2* Hc = a.H + (int64_t)ir * a.h_ir_stride + xrow_pos(kz, a.M);
  const double2* Xc = a.X + (int64_t)c * a.x_ch_stride + xrow_pos(kz, a.M);
  Unpack<NH> up;
  up.m = mi ? (int)0x80000000u : 0;
  up.tw = (k < a.M) ? a.twN[k] : make_double2(-1.0, 0.0);
  ZEpilogue<NH> epi;
  epi.S = 0.125 / (double)a.M;
  epi.m = up.m;
  // Z rows in wave-lane order (zrow_pos): one aligned 1-KiB run per wave row.
  const int zpos = zrow_pos(k, a.M);
  epi.zb = a.Y + (int64_t)c * a.y_ch_stride;
  epi.zo = (unsigned)zpos;
  epi.jstride = a.MS;
  epi.tw = (k < a.M) ? c_scale(c_conj(a.twN[k]), epi.S) : make_double2(0.0, 0.0);

  {
    const int pb = a.p0 + (ph ? PC : 0);  // this lane's first partition
    double2 h[PC];
#pragma unroll
    for (int q = 0; q < PC; ++q) h[q] = Hc[(int64_t)min(pb + q, a.P - 1) * a.MS];
#pragma unroll
    for (int q = 0; q < PC; ++q) {
      h[q] = up(h[q]);
      if (pb + q >= a.P) h[q] = make_double2(0.0, 0.0);
      __builtin_amdgcn_sched_barrier(0);
    }
    double2 acc[PC];
#pragma unroll
    for (int q = 0; q < PC; ++q) acc[q] = make_double2(0.0, 0.0);

    constexpr int D = DQ < PC ? DQ : PC;
    XStream st;
    st.Xc = Xc;
    st.Q = a.Q;
    st.MS = a.MS;
    st.lx = a.g0 + j0 - PC - a.p0;  // row 0 of the warm-up group (only the first row's P[g-1]), ph = 0
    st.gend = a.gend;
    st.sl = (int)(((st.lx % a.Q) + a.Q) % a.Q);
    st.dph = -PC;
    st.ph = ph;
    BlockPair bp;
    bp.smask = (kz & 1) ? (int)0x80000000u : 0;
    bp.prev = st.load(0);
    double2 xb[D];
#pragma unroll
    for (int d = 1; d <= D; ++d) xb[d % D] = st.load(d);
    Row<PC, D, 1, true>::template run<FIRST>(acc, h, xb, st, bp, up, epi, j0);
    st.advance<PC>();
    for (int i = j0; i < j1; i += PC) {
      Row<PC, D, 0, false>::template run<FIRST>(acc, h, xb, st, bp, up, epi, i);
      st.advance<PC>();
    }
  }
}

// ---------------------------------------------------------------------------
// K2 with the X stream staged through LDS by LDS-DMA (global_load_lds_dwordx4):
// the same bin-stationary MAC as k_fdl_mac, but the prefetched X rows sit in
// a per-wave LDS ring of DL rows (1 KiB each) instead of VGPRs.  At PC = 16
// the h and accumulator registers (128 VGPRs) leave room for only 4 rows in
// registers at 2 waves/SIMD, i.e. 8 KiB in flight per SIMD, which at HBM
// latency caps K2 near 4.5 TB/s; the LDS ring keeps DL rows in flight per
// wave at no VGPR cost.
//
// The DMAs are inline asm (hipcc would drain every LDS-DMA with vmcnt(0)
// before the first LDS read), so their completion is counted here.  The
// vector-memory counter retires in issue order on gfx9; per row the issue
// order is: [wait row U] [ds_read row U] [DMA row U + DL] [store output U]:
//   warm-up group:        DL - 1 operations follow row U's DMA
//   first output group:   DL - 1 + min(U, DL)
//   steady state:         2 DL - 1
// (more operations in flight than counted only makes a wait conservative).
// Rows past the run (logical index > lend) read the ring's zero row, so the
// tail prefetch is L2 hits instead of HBM rows.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;

struct XRing {
  const double2* Xc;
  int Q, MS;
  int64_t lx;    // logical index of row 0 of the current group (ph = 0)
  int64_t lend;  // last logical row any output of the run needs (ph = 0)
  int sl;        // ring slot of lx
  int dph;       // row offset of the ph = 1 half (-PC)
  bool ph;
  __device__ __forceinline__ int slot(int off) const {  // wave-uniform
    int s = sl + off;
    if (s >= Q) s -= Q;
    if (s < 0) s += Q;
    const int64_t g = lx + off;
    return (g >= 0 && g <= lend) ? s : Q;
  }
  __device__ __forceinline__ double2 load(int off) const {  // plain load of row lx + off (+ dph)
    const int r0 = slot(off), r1 = slot(off + dph);
    return Xc[(int64_t)(ph ? r1 : r0) * MS];
  }
  // DMA row lx + off (+ dph for ph = 1) into LDS at byte address lds (+16 B per lane).
  __device__ __forceinline__ void issue(int off, unsigned lds) const {
    const int r0 = slot(off), r1 = slot(off + dph);
    const int row = ph ? r1 : r0;
    const double2* p = Xc + (int64_t)row * MS;
    unsigned keep;
    asm volatile(
        // nt: the X rows are streamed once per run (K2 250 -> 230 us at the
        // bench config; K3 after it +12 us, the whole step unchanged to +2 %)
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(p), "s"(lds)
        : "memory");
  }
  template <int PC>
  __device__ __forceinline__ void advance() {
    lx += PC;
    sl += PC;
    if (sl >= Q) sl -= Q;
  }
};

template <int DL>
__device__ __forceinline__ unsigned ring_addr(const double2* ring, int slot) {
  return (unsigned)(uintptr_t)(lds_void_t*)(ring + slot * 64);
}

// GRP: 0 warm-up group, 1 first output group, 2 steady state.
template <int PC, int DL, int U, int GRP>
struct RowL {
  template <int Q>
  __device__ static __forceinline__ void macs(double2 (&acc)[PC], const double2 (&h)[PC], const double2 x) {
    if constexpr (Q < PC) {
      cmac(acc[(U + Q) % PC], x, h[Q]);
      macs<Q + 1>(acc, h, x);
    }
  }
  static constexpr int wait_count() {
    return GRP == 0 ? DL - 1 : (GRP == 1 ? DL - 1 + (U < DL ? U : DL) : 2 * DL - 1);
  }
  template <bool FIRST, class UP, class EPI>
  __device__ static __forceinline__ void run(double2 (&acc)[PC], const double2 (&h)[PC], double2* ring,
                                             const XRing& st, BlockPair& bp, const UP& up, const EPI& epi,
                                             int i) {
    if constexpr (U < PC) {
      constexpr int S = U % DL;
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(wait_count()) : "memory");
      const double2 xr = ring[S * 64 + threadIdx.x];
      // the fake operand holds the DMA that refills slot S behind this read
      asm volatile("" ::"v"(xr.x), "v"(xr.y));
      st.issue(U + DL, ring_addr<DL>(ring, S));
      const double2 x = up(bp.next(xr));
      if constexpr (GRP == 0) {
        macs<PC - U>(acc, h, x);
      } else {
        macs<0>(acc, h, x);
        epi.template store<FIRST>(acc[U], i + U);
        acc[U] = make_double2(0.0, 0.0);
      }
      __builtin_amdgcn_sched_barrier(0);
      RowL<PC, DL, U + 1, GRP>::template run<FIRST>(acc, h, ring, st, bp, up, epi, i);
    }
  }
};

// Occupancy target of the LDS-ring variant: no X registers, so PC = 16 fits 3 waves.
template <int PC, int NH>
struct MacOccL {
  static constexpr int W = PC <= 8 ? 4 : 3;
};
template <int PC, int NH, bool FIRST, int DL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MacOccL<PC, NH>::W))) void k_fdl_mac_lds(MacArgs a) {
  static_assert(DL <= 16 && PC % DL == 0, "ring depth: slots must repeat every group");
  __shared__ double2 ring[DL * 64];
  constexpr int BW = 32 / NH;
  const int lg = xcd_remap(blockIdx.x, gridDim.x);
  // neighbouring waves: consecutive runs of one bin group (they re-read each
  // other's warm-up rows)
  const int ry = lg % a.ny;
  const int bx = (lg / a.ny) % a.nx;
  const int c = lg / a.ny / a.nx;
  const int lane = threadIdx.x;
  const bool ph = NH == 2 && lane >= 32;
  const bool mi = NH == 2 ? ((lane >> 4) & 1) : (lane >> 5);
  const int l = lane & (BW - 1);
  const bool paired = bx < a.M / (2 * BW);
  const int k = paired ? (mi ? a.M - (bx * BW + l) : bx * BW + l) : a.M / 2;
  const int j0 = ry * a.R;
  const int j1 = min(j0 + a.R, a.jc);
  const int ir = a.ir_index ? a.ir_index[c] : (c % a.n_ir);
  const int kz = k & (a.M - 1);
  const double2* Hc = a.H + (int64_t)ir * a.h_ir_stride + xrow_pos(kz, a.M);
  const double2* Xc = a.X + (int64_t)c * a.x_ch_stride + xrow_pos(kz, a.M);
  Unpack<NH> up;
  up.m = mi ? (int)0x80000000u : 0;
  up.tw = (k < a.M) ? a.twN[k] : make_double2(-1.0, 0.0);
  ZEpilogue<NH> epi;
  epi.S = 0.125 / (double)a.M;
  epi.m = up.m;
  const int zpos = zrow_pos(k, a.M);
  epi.zb = a.Y + (int64_t)c * a.y_ch_stride;
  epi.zo = (unsigned)zpos;
  epi.jstride = a.MS;
  epi.tw = (k < a.M) ? c_scale(c_conj(a.twN[k]), epi.S) : make_double2(0.0, 0.0);

  XRing st;
  st.Xc = Xc;
  st.Q = a.Q;
  st.MS = a.MS;
  st.lx = a.g0 + j0 - PC - a.p0;
  st.lend = min((int64_t)(a.g0 + j1 - 1 - a.p0), a.gend);
  st.sl = (int)(((st.lx % a.Q) + a.Q) % a.Q);
  st.dph = -PC;
  st.ph = ph;
  // P[g-1] of the first row the run consumes, ahead of the ring DMAs (vmcnt
  // retires in order, so the counted waits below stay conservative)
  BlockPair bp;
  bp.smask = (kz & 1) ? (int)0x80000000u : 0;
  bp.prev = st.load(0);
  // ring prologue first: its DMAs overlap the H loads
#pragma unroll
  for (int d = 1; d <= DL; ++d) st.issue(d, ring_addr<DL>(ring, d % DL));

  const int pb = a.p0 + (ph ? PC : 0);
  double2 h[PC];
  // all PC loads in flight at once, then separated one by one
#pragma unroll
  for (int q = 0; q < PC; ++q) h[q] = Hc[(int64_t)min(pb + q, a.P - 1) * a.MS];
#pragma unroll
  for (int q = 0; q < PC; ++q) {
    h[q] = up(h[q]);
    if (pb + q >= a.P) h[q] = make_double2(0.0, 0.0);
    __builtin_amdgcn_sched_barrier(0);
  }
  double2 acc[PC];
#pragma unroll
  for (int q = 0; q < PC; ++q) acc[q] = make_double2(0.0, 0.0);

  RowL<PC, DL, 1, 0>::template run<FIRST>(acc, h, ring, st, bp, up, epi, j0);
  st.advance<PC>();
  if (j0 < j1) {
    RowL<PC, DL, 0, 1>::template run<FIRST>(acc, h, ring, st, bp, up, epi, j0);
    st.advance<PC>();
  }
  for (int i = j0 + PC; i < j1; i += PC) {
    RowL<PC, DL, 0, 2>::template run<FIRST>(acc, h, ring, st, bp, up, epi, i);
    st.advance<PC>();
  }
  // drain the tail DMAs before the wave (and its LDS) retires
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// K2 for calls of one or two output blocks per channel (a streaming block, a
// partitioned stage firing once): one wave per (channel, output block, bin
// group), all P partitions in one launch.  The run-based kernels above keep
// PC partitions of H in VGPRs to reuse them over a run of R outputs; with a
// single output there is no reuse, so this form streams H and X rows
// instead: no H registers, no rotating accumulators, so many more waves (and
// loads) per SIMD, and no second launch with a Z read-modify-write when
// P > 16.  Bit-identical to k_fdl_mac_lds: the same products in the same
// order -- per chunk of PC partitions p descending, each chunk folded to Z,
// the chunks' Z summed in launch order -- so a call gives the same outputs
// whichever form ran.
// ---------------------------------------------------------------------------
template <int PC>
__global__ __launch_bounds__(256) void k_fdl_mac_row(MacArgs a) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= a.ny) return;  // ny = waves in this launch (set by the launcher)
  // a pre-enqueued chain whose K1 did not run (StreamGate)
  if (a.sg.gate && __hip_atomic_load(a.sg.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != a.sg.seq) return;
  const int lane = threadIdx.x & 63;
  const int bx = w % a.nx;
  const int t = w / a.nx;
  const int j = t % a.jc;
  const int c = t / a.jc;
  const bool mi = lane >> 5;
  const int l = lane & 31;
  const bool paired = bx < a.M / 64;
  const int k = paired ? (mi ? a.M - (bx * 32 + l) : bx * 32 + l) : a.M / 2;
  const int ir = a.ir_index ? a.ir_index[c] : (c % a.n_ir);
  const int kz = k & (a.M - 1);
  const double2* Hc = a.H + (int64_t)ir * a.h_ir_stride + xrow_pos(kz, a.M);
  const double2* Xc = a.X + (int64_t)c * a.x_ch_stride + xrow_pos(kz, a.M);
  Unpack<1> up;
  up.m = mi ? (int)0x80000000u : 0;
  up.tw = (k < a.M) ? a.twN[k] : make_double2(-1.0, 0.0);
  ZEpilogue<1> epi;
  epi.S = 0.125 / (double)a.M;
  epi.m = up.m;
  epi.zb = a.Y + (int64_t)c * a.y_ch_stride;
  epi.zo = (unsigned)zrow_pos(k, a.M);
  epi.jstride = a.MS;
  epi.tw = (k < a.M) ? c_scale(c_conj(a.twN[k]), epi.S) : make_double2(0.0, 0.0);
  const int smask = (kz & 1) ? (int)0x80000000u : 0;
  const int64_t G = a.g0 + j;  // logical block of this output
  auto row = [&](int64_t g) {  // block-spectrum row of logical block g (zero row outside the signal)
    const int64_t r = (g < 0 || g > a.gend) ? a.Q : g % a.Q;
    return Xc[r * a.MS];
  };
  double2 zt = make_double2(0.0, 0.0);
  for (int p0 = 0; p0 < a.P; p0 += PC) {
    double2 xr[PC + 1], h[PC];
    // rows G - p0 - PC .. G - p0 (oldest first) and H[p0 .. p0 + PC)
#pragma unroll
    for (int u = 0; u <= PC; ++u) xr[u] = row(G - p0 - PC + u);
#pragma unroll
    for (int q = 0; q < PC; ++q) h[q] = Hc[(int64_t)min(p0 + q, a.P - 1) * a.MS];
    double2 acc = make_double2(0.0, 0.0);
#pragma unroll
    for (int u = 1; u <= PC; ++u) {  // window G - p, p = p0 + PC - u (descending)
      const double2 pp = xr[u - 1], pc = xr[u];
      const double2 x = up(make_double2(pp.x + flip(pc.x, smask), pp.y + flip(pc.y, smask)));
      const int q = PC - u;
      double2 hq = up(h[q]);
      if (p0 + q >= a.P) hq = make_double2(0.0, 0.0);
      cmac(acc, x, hq);
    }
    // the epilogue's fold, summed over the chunks as the RMW launches do
    double2 u2, v2;
    xpair<true>(acc, u2, v2);
    const double sx = u2.x + v2.x, sy = u2.y + v2.y;
    const double sdx = flip(u2.x - v2.x, epi.m), sdy = flip(u2.y - v2.y, epi.m);
    const double2 z = make_double2(fma(-epi.tw.x, sy, fma(-epi.tw.y, sdx, sx * epi.S)),
                                   fma(-epi.tw.y, sy, fma(epi.tw.x, sdx, epi.S * sdy)));
    zt = p0 == 0 ? z : make_double2(zt.x + z.x, zt.y + z.y);
  }
  epi.zb[(int64_t)j * epi.jstride + epi.zo] = zt;
}

// ---------------------------------------------------------------------------
// Direct convolution, bit-exact with conv.DirectTo (conv.go:97-154):
// each dst[k] accumulates a[i]*b[k-i] in increasing i with a rounded product
// and a rounded add (vecmath.ScaleBlock then AddBlockInPlace, no FMA).
// Output-stationary: one lane per output sample, so no atomics are needed and
// the accumulation order is exactly the reference's.
// ---------------------------------------------------------------------------
constexpr int DC = 1024;  // taps per chunk

// Tap-stationary register-blocked form.  The sum for output k
// is read the other way round: y[k] = sum over j = m-1 down to 0 of
// b[j] * a[k-j], which is the same increasing-i order.  b[j] is wave-uniform
// (scalar loads) and a lane owns R consecutive outputs, so its inputs
// a[k-j .. k-j+R-1] slide by one per term (blocked_dot.hpp: one R-wide LDS
// read per R*R products).  Unlike the input-stationary form every lane of a
// wave takes every term, except at the two ends of the signal where a lane
// meets a[i] outside [0, n) stored as zero: b[j] * 0 = +-0 leaves the sum
// unchanged unless b[j] is not finite, so a tap chunk holding a non-finite
// tap takes the per-lane bounds-checked loop.  Taps are walked in chunks of
// DC; the input window one chunk meets is 256 R + DC - 1 samples in LDS.
template <int R>
__global__ __launch_bounds__(256) void k_direct_reg(const double* __restrict__ a, int64_t n,
                                                    const double* __restrict__ b, int64_t m,
                                                    double* __restrict__ dst) {
#pragma clang fp contract(off)
  constexpr int DT = 256 * R;
  __shared__ __attribute__((aligned(32))) double win[DT + DC + 8];
  const int t = threadIdx.x;
  const int64_t k0 = (int64_t)blockIdx.x * DT;
  const int64_t out = n + m - 1;
  // taps reaching this tile: k - j in [0, n) for some k in [k0, k0 + DT)
  const int64_t jtop = m - 1 < k0 + DT - 1 ? m - 1 : k0 + DT - 1;
  const int64_t jbot = k0 - n + 1 > 0 ? k0 - n + 1 : 0;
  double acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0;
  for (int64_t jhi = jtop; jhi >= jbot; jhi -= DC) {
    const int cj = (int)(jhi - jbot + 1 < DC ? jhi - jbot + 1 : DC);
    const int64_t g0 = k0 - jhi;  // win[1 + v] = a[g0 + v]
    __syncthreads();
    int bad = 0;
    for (int u = t; u < cj; u += 256) bad |= !__builtin_isfinite(b[jhi - u]);
    for (int v = t; v < DT + cj - 1; v += 256) {
      const int64_t g = g0 + v;
      win[1 + v] = (g >= 0 && g < n) ? a[g] : 0.0;
    }
    bad = __syncthreads_or(bad);
    const double* wt = win + 1 + t * R;  // term u (j = jhi - u) of output r: wt[u + r]
    if (!bad) {
      blocked_dot<R, -1>(b + jhi, wt, cj, acc);
    } else {
      for (int u = 0; u < cj; ++u) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int64_t i = g0 + t * R + r + u;
          if (i >= 0 && i < n) {
            const double p = b[jhi - u] * wt[u + r];
            acc[r] = acc[r] + p;
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t k = k0 + t * R + r;
    if (k < out) dst[k] = acc[r];
  }
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

// Streaming block staging: host-mapped (zero-copy) <-> device buffer.  One
// workgroup reading 32 KiB over PCIe is bound by the few requests one CU
// keeps in flight (K1 alone took 16.5 us per 4096-sample block); a grid of
// one double per lane spreads the block over many CUs.
__global__ __launch_bounds__(64) void k_copy_f64(const double* __restrict__ src, double* __restrict__ dst,
                                                 int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// Stereo mixdown of a channel group: mix[0][t] (L) sums the channels of even
// global index, mix[mix_stride + t] (R) the odd ones; channel c of the group
// has global index first + c, so only first's parity matters.
__global__ __launch_bounds__(256) void k_mixdown(const double* __restrict__ ch, int channels, int64_t stride,
                                                 int64_t len, double* __restrict__ mix, int64_t mix_stride,
                                                 int first_parity) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= len) return;
  double e = 0.0, o = 0.0;  // group-local even / odd channels
  for (int c = 0; c < channels; c += 2) e += ch[(int64_t)c * stride + t];
  for (int c = 1; c < channels; c += 2) o += ch[(int64_t)c * stride + t];
  mix[t] = first_parity ? o : e;
  mix[mix_stride + t] = first_parity ? e : o;
}

// Column shift with zero fill (accumulator / FIFO compaction of the
// multichannel partitioned engine).
__global__ __launch_bounds__(256) void k_shift_cols(const double* __restrict__ src, int64_t src_stride,
                                                    double* __restrict__ dst, int64_t dst_stride, int64_t ncopy,
                                                    int64_t ncols) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  if (j >= ncols) return;
  dst[(int64_t)c * dst_stride + j] = j < ncopy ? src[(int64_t)c * src_stride + j] : 0.0;
}

// Emit of the partitioned convolution / ConvolutionReverb mix
// (reverb/convolution.go:60-85: block[i] = dry*block[i] + wet*reverbOut[i]).
// Optionally also appends the input block to the engine's input FIFO (one
// launch for a call's I/O).
__global__ __launch_bounds__(256) void k_pc_emit(const double* in, int64_t in_stride, double* out,
                                                 int64_t out_stride, const double* __restrict__ acc,
                                                 int64_t acc_stride, int64_t off, int64_t first, int64_t n, int mix,
                                                 double wet, double dry, double* append_to, int64_t append_stride,
                                                 int emit, int64_t row2) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  if (i >= n) return;
  if (append_to) append_to[(int64_t)c * append_stride + i] = in[(int64_t)c * in_stride + i];
  if (!emit) return;
  double r = 0.0;
  if (i >= first) {
    const int64_t q = (int64_t)c * acc_stride + off + i;
    r = acc[q];
    if (row2) r = r + acc[row2 + q];  // the side-stream stages' accumulator row
  }
  if (mix) {
    const double x = in[(int64_t)c * in_stride + i];
    const double a = dry * x;
    const double b = wet * r;
    out[(int64_t)c * out_stride + i] = a + b;
  } else {
    out[(int64_t)c * out_stride + i] = r;
  }
}

// The emit + FIFO append of a pre-enqueued low-latency call (NupolsDev,
// one channel, n <= 256: one workgroup).  Thread 0 waits for the host's go
// word like the streaming chains' K1 (StreamGate: system-scope acquire loads
// of mapped memory, s_sleep between polls, give up at the timeout or at
// kGateAbort) and reports its decision in k1_state; when it runs, the
// workgroup does k_pc_emit's work and then publishes seq in `done` after its
// stores are visible system-wide.
__global__ __launch_bounds__(256) void k_pc_emit_gated(const double* in, double* out, const double* __restrict__ acc,
                                                       int64_t off, int64_t first, int64_t n, int mix, double wet,
                                                       double dry, double* append_to, StreamGate g) {
#pragma clang fp contract(off)
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
      __builtin_amdgcn_s_sleep(2);
    }
    __hip_atomic_store(g.k1_state, run ? g.seq : (g.seq | kGateSkipped), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    ok = run;
  }
  __syncthreads();
  if (!ok) return;
  const int64_t i = threadIdx.x;
  if (i < n) {
    const double x = in[i];
    append_to[i] = x;
    const double r = i >= first ? acc[off + i] : 0.0;
    if (mix) {
      const double a = dry * x;
      const double b = wet * r;
      out[i] = a + b;
    } else {
      out[i] = r;
    }
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(g.done, g.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
LaunchTiming& launch_timing() {
  static thread_local LaunchTiming t;
  return t;
}

namespace {
// PC < 8: the register-prefetch form (4 rows in flight per lane); PC >= 8: the
// LDS-DMA ring of 8 rows per wave (its h and accumulator registers leave no
// room for a register ring at PC = 16).
template <int PC>
void mac_go(const MacArgs& a, dim3 grid, hipStream_t s) {
  MacArgs c = a;
  for (c.p0 = 0; c.p0 < a.P; c.p0 += PC) {
    if constexpr (PC >= 8) {
      if (c.p0 == 0)
        timed_launch(k_fdl_mac_lds<PC, 1, true, 8>, grid, dim3(64), s, c);
      else
        timed_launch(k_fdl_mac_lds<PC, 1, false, 8>, grid, dim3(64), s, c);
    } else {
      if (c.p0 == 0)
        timed_launch(k_fdl_mac<PC, 1, true, 4>, grid, dim3(64), s, c);
      else
        timed_launch(k_fdl_mac<PC, 1, false, 4>, grid, dim3(64), s, c);
    }
  }
}
}  // namespace

// Resident waves per SIMD of the K2 variant that launch_fdl_mac will pick.
int mac_waves_per_simd(int PC, int NH) {
  if (PC >= 8) return PC <= 8 ? 4 : 3;    // MacOccL (VGPR-bound; the 8-row ring is 8 KiB per wave)
  return PC <= 4 ? 4 : (PC == 8 ? 3 : 2);  // MacOcc
}

int device_cus() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    return cus;
  }();
  return n;
}

void mac_run_geometry(int PC, int NH, int M, int mid_in_k3, int channels, int jc, int R_req, int* R_out,
                      int* ny_out) {
  const int BW = 32 / NH;
  const int nx = M / (2 * BW) + (mid_in_k3 ? 0 : 1);
  int R = R_req;
  if (R <= 0) {
    // Auto run length: the fewest runs that still fill every SIMD to its
    // resident-wave limit in ONE round.  A second, partial round leaves a
    // tail of idle SIMDs, and longer runs re-read fewer warm-up rows and H
    // spectra (stereo 2 x 2064 blocks at M = 8192: R = 192, 2838 waves,
    // K2 237 us vs 285 us at R = 64).
    const int64_t slots = (int64_t)mac_waves_per_simd(PC, NH) * 4 * device_cus();
    const int64_t per_run = (int64_t)channels * nx;
    int64_t ny = std::max<int64_t>(1, slots / per_run);
    ny = std::min<int64_t>(ny, (jc + 31) / 32);  // runs of at least 32 blocks
    ny = std::max<int64_t>(ny, 1);
    R = (int)((jc + ny - 1) / ny);
  }
  // runs must be whole groups of PC (<= 16) outputs so the overshoot of a run
  // never lands in the next run's rows
  if (jc > R) R = (R + 15) / 16 * 16;
  *R_out = R;
  *ny_out = (jc + R - 1) / R;
}

bool launch_fdl_mac(int PC, int NH, const MacArgs& in, int channels, hipStream_t s) {
  if (channels <= 0 || in.jc <= 0) return true;
  if (NH != 1) return false;  // one lane holds all of a chunk's partitions
  MacArgs a = in;
  if (a.M < 64) return false;  // a pair wave needs M/2 >= 32 bins
  a.nx = a.M / 64 + (a.mid_in_k3 ? 0 : 1);  // pair waves (+ the middle-bin wave)
  if (a.jc <= 2) {  // one or two outputs per channel: the row form (no H reuse to exploit)
    const int64_t waves = (int64_t)channels * a.nx * a.jc;
    a.ny = (int)waves;
    const dim3 grid((unsigned)((waves + 3) / 4)), blk(256);
    switch (PC) {
      case 1: timed_launch(k_fdl_mac_row<1>, grid, blk, s, a); return true;
      case 2: timed_launch(k_fdl_mac_row<2>, grid, blk, s, a); return true;
      case 4: timed_launch(k_fdl_mac_row<4>, grid, blk, s, a); return true;
      case 8: timed_launch(k_fdl_mac_row<8>, grid, blk, s, a); return true;
      case 16: timed_launch(k_fdl_mac_row<16>, grid, blk, s, a); return true;
      default: return false;
    }
  }
  mac_run_geometry(PC, 1, a.M, a.mid_in_k3, channels, a.jc, a.R, &a.R, &a.ny);
  const dim3 grid((unsigned)((int64_t)channels * a.nx * a.ny));
  switch (PC) {
    case 1: mac_go<1>(a, grid, s); break;
    case 2: mac_go<2>(a, grid, s); break;
    case 4: mac_go<4>(a, grid, s); break;
    case 8: mac_go<8>(a, grid, s); break;
    case 16: mac_go<16>(a, grid, s); break;
    default: return false;
  }
  return true;
}

void launch_direct(const double* a, int64_t n, const double* b, int64_t m, double* dst, hipStream_t s) {
  const int64_t out = n + m - 1;
  // R = 4 outputs per lane once that still gives >= 2 workgroups per CU
  const int R = out >= 512 * 1024 ? 4 : out >= 512 * 512 ? 2 : 1;
  switch (R) {
    case 4:
      hipLaunchKernelGGL(k_direct_reg<4>, dim3((unsigned)((out + 1023) / 1024)), dim3(256), 0, s, a, n, b, m, dst);
      break;
    case 2:
      hipLaunchKernelGGL(k_direct_reg<2>, dim3((unsigned)((out + 511) / 512)), dim3(256), 0, s, a, n, b, m, dst);
      break;
    default:
      hipLaunchKernelGGL(k_direct_reg<1>, dim3((unsigned)((out + 255) / 256)), dim3(256), 0, s, a, n, b, m, dst);
      break;
  }
}

void launch_direct_circular(const double* a, const double* b, int64_t n, double* dst, hipStream_t s) {
  hipLaunchKernelGGL(k_direct_circular, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, b, n, dst);
}

void launch_stream_direct(const double* h, int64_t K, const double* buf, int64_t B, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_stream_direct, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, h, K, buf, B, y);
}

void launch_copy_f64(const double* src, double* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_copy_f64, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, src, dst, n);
}

void launch_mixdown(const double* ch, int channels, int64_t stride, int64_t len, double* mix, int64_t mix_stride,
                    int first_parity, hipStream_t s) {
  hipLaunchKernelGGL(k_mixdown, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, s, ch, channels, stride, len, mix,
                     mix_stride, first_parity & 1);
}

void launch_shift_cols(const double* src, int64_t src_stride, double* dst, int64_t dst_stride, int channels,
                       int64_t ncopy, int64_t ncols, hipStream_t s) {
  if (channels <= 0 || ncols <= 0) return;
  hipLaunchKernelGGL(k_shift_cols, dim3((unsigned)((ncols + 255) / 256), (unsigned)channels), dim3(256), 0, s, src,
                     src_stride, dst, dst_stride, ncopy, ncols);
}

void launch_pc_emit(const double* in, int64_t in_stride, double* out, int64_t out_stride, const double* acc,
                    int64_t acc_stride, int64_t off, int64_t first, int64_t n, int channels, int mix, double wet,
                    double dry, hipStream_t s, double* append_to, int64_t append_stride, bool emit, int64_t row2) {
  if (channels <= 0 || n <= 0) return;
  hipLaunchKernelGGL(k_pc_emit, dim3((unsigned)((n + 255) / 256), (unsigned)channels), dim3(256), 0, s, in, in_stride,
                     out, out_stride, acc, acc_stride, off, first, n, mix, wet, dry, append_to, append_stride,
                     emit ? 1 : 0, row2);
}

void launch_pc_emit_gated(const double* in, double* out, const double* acc, int64_t off, int64_t first, int64_t n,
                          int mix, double wet, double dry, double* append_to, const StreamGate& g, hipStream_t s) {
  hipLaunchKernelGGL(k_pc_emit_gated, dim3(1), dim3(256), 0, s, in, out, acc, off, first, n, mix, wet, dry, append_to,
                     g);
}

// ---------------------------------------------------------------------------
// Fused small partitioned stage (NupolsDev; PartitionedConvolutionT stages of
// two partitions, partitioned.go:134-183).  Stateless per block: the
// frequency-domain delay line of two partitions is replaced by transforming
// the previous window again, so every (block, channel) is independent and a
// call of any length is one launch per stage.
//   y[t] (t in [d, d+p)) = IFFT_N( FFT_N(x[d-p, d+p)) . H0 + FFT_N(x[d-2p, d)) . H1 )[p + t - d]
// Radix-2 Stockham passes in LDS (natural order in and out), 256 threads.
// ---------------------------------------------------------------------------
namespace {

// Twiddles W_N^e read from the W_2048 table (e << (11 - log2 N)).
struct TwStrided {
  const double2* __restrict__ t;
  int sh;
  __device__ __forceinline__ double2 operator()(int e) const { return t[e << sh]; }
};

// Register FFTs (FftPlan<N, 16>: T = N/16 threads per transform, radix-16
// passes through LDS): lanes [0, T) transform the previous window, lanes
// [T, 2T) the current one, concurrently; a 256-thread block repeats the two
// groups (duplicate lanes compute and store identical values) so every lane
// reaches the same barriers.  The products meet in LDS, one group inverts.
template <int N>
__device__ __forceinline__ void pc_small_body(const PcSmallArgs& a, int blk, int c, double2* lds) {
  using Plan = FftPlan<N, 16>;
  constexpr int T = Plan::T, P = N / 2, MP = Plan::MP;
  const int tid = threadIdx.x;
  const int lt = tid % T;
  const int g = (tid / T) & 1;
  const bool lead = tid < 2 * T;  // the lanes whose results are kept
  const int64_t d = a.d0 + (int64_t)blk * P;
  const double* xc = a.xin + (int64_t)c * a.xstride;
  const TwStrided tw{a.tw, 11 - ilog2c(N)};
  const int64_t w0 = d - 2 * P + (int64_t)g * P;  // window start: x[d-2p, d) (g = 0), x[d-p, d+p) (g = 1)
  double2 v[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int64_t t = w0 + pass0_index<N, 16>(lt, s);
    v[s] = make_double2(t < 0 ? 0.0 : xc[t - a.xbase], 0.0);
  }
  double2* img = lds + g * MP;
  fft_run<N, 16, true>(v, lt, img, tw);
  // spectra products: g = 0 with the second partition H1, g = 1 with H0
  const double2* Hg = a.H + (g ? 0 : N);
#pragma unroll
  for (int s = 0; s < 16; ++s) v[s] = c_mul(v[s], Hg[last_pass_index<N, 16>(lt, s)]);
  __syncthreads();  // both transforms' last LDS reads are done
  if (g == 0) {
#pragma unroll
    for (int s = 0; s < 16; ++s) lds[last_pass_index<N, 16>(lt, s)] = v[s];
  }
  __syncthreads();
  if (g == 1) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = last_pass_index<N, 16>(lt, s);
      lds[MP + k] = c_add(lds[k], v[s]);
    }
  }
  __syncthreads();
  // inverse transform of Y (both groups run it on the same data)
#pragma unroll
  for (int s = 0; s < 16; ++s) v[s] = lds[MP + pass0_index<N, 16>(lt, s)];
  __syncthreads();
  fft_run<N, 16, false>(v, lt, lds + g * MP, tw);
  if (!lead || g != 1) return;
  double* out = a.acc + (int64_t)c * a.acc_stride + a.acc_off + (int64_t)blk * P;
  constexpr double inv = 1.0 / N;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int m = last_pass_index<N, 16>(lt, s);
    if (m >= P) out[m - P] += v[s].x * inv;
  }
}

template <int N>
__global__ __launch_bounds__(256) void k_pc_small(PcSmallArgs a) {
  __shared__ __attribute__((aligned(16))) double2 lds[2 * FftPlan<N, 16>::MP];
  pc_small_body<N>(a, blockIdx.x, blockIdx.y, lds);
}

__global__ __launch_bounds__(256) void k_pc_small_multi(PcSmallMulti m) {
  __shared__ __attribute__((aligned(16))) double2 lds[2 * FftPlan<2048, 16>::MP];
  int k = 0;
  while (k + 1 < m.nst && (int)blockIdx.x >= m.first[k + 1]) ++k;
  const int blk = blockIdx.x - m.first[k];
  switch (m.N[k]) {
    case 128: pc_small_body<128>(m.st[k], blk, blockIdx.y, lds); break;
    case 256: pc_small_body<256>(m.st[k], blk, blockIdx.y, lds); break;
    case 512: pc_small_body<512>(m.st[k], blk, blockIdx.y, lds); break;
    case 1024: pc_small_body<1024>(m.st[k], blk, blockIdx.y, lds); break;
    default: pc_small_body<2048>(m.st[k], blk, blockIdx.y, lds); break;
  }
}

template <int N>
void pc_small_go(const PcSmallArgs& a, int channels, hipStream_t s) {
  hipLaunchKernelGGL((k_pc_small<N>), dim3((unsigned)a.nb, (unsigned)channels), dim3(256), 0, s, a);
}

}  // namespace

void launch_pc_small_multi(const PcSmallMulti& m, int channels, hipStream_t s) {
  if (m.nst <= 0 || channels <= 0 || m.first[m.nst] <= 0) return;
  hipLaunchKernelGGL(k_pc_small_multi, dim3((unsigned)m.first[m.nst], (unsigned)channels), dim3(256), 0, s, m);
}

bool launch_pc_small(int N, const PcSmallArgs& a, int channels, hipStream_t s) {
  if (a.nb <= 0 || channels <= 0) return true;
  switch (N) {
    case 128: pc_small_go<128>(a, channels, s); return true;
    case 256: pc_small_go<256>(a, channels, s); return true;
    case 512: pc_small_go<512>(a, channels, s); return true;
    case 1024: pc_small_go<1024>(a, channels, s); return true;
    case 2048: pc_small_go<2048>(a, channels, s); return true;
    default: return false;
  }
}

}  // namespace adsp
