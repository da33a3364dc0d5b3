// K_lanes: the bit-exact biquad cascade of an EQ-only effect chain (and of
// biquad.Chain over many channels) with the cascade's sections across lanes.
//
// Reference: biquad.Chain.ProcessBlock (dsp/filter/biquad/chain.go:59-70),
// Section.ProcessSample (section.go:47-53), DF-II-T:
//   y = b0 x + d0;  d0 = b1 x - a1 y + d1;  d1 = b2 x - a2 y
// with the chain gain as section 0's pre-gain (dsp_kernels.hpp kSecStride).
// Every value below is formed by the same IEEE operations in the same order
// as eq_section_step (fx_staged.hip) and the oracle, contraction off.
//
// Why lanes: a section's recurrence d0 -> y -> a1 y -> (b1 x - a1 y) -> + d1
// is four dependent FP64 operations per sample (~52 clocks,
// tools/biquad_latency.hip), so a channel's cascade can take one sample per
// section chain only if its sections run concurrently on different samples.
// The per-section pipeline (k_fx_eq_sec) gives each section a workgroup and
// hands samples over through LDS rings, an I/O wave and barriers; the section
// wave then spends ~80 clocks per sample, the LDS and memory traffic beside
// it being the difference.  Here the hand-over is a lane
// shift instead:
//   - row r of a wave (lanes 16 r .. 16 r + 15) is one channel, lane 16 r + k
//     its section k (nsec <= 16; lanes past nsec idle);
//   - at step s lane k filters sample s - k: its input is lane k - 1's output
//     of step s - 1, moved by one DPP row shift (row_shr:1), and lane 0 of the
//     row, which has no source lane in the shift, keeps the DPP's old operand,
//     the input sample (read from LDS, where it was staged a block ahead);
//   - every lane writes its output to an LDS row per step; once per block of
//     kLnB steps the row's 16 lanes store the last section's kLnB outputs
//     (two 128-B runs).
// So the step has no barrier and no hand-over beyond one DPP pair, and the
// loop-carried path is the section's own four-operation chain.  A wave holds
// four channels; lanes are cheap here (the EQ of 256 channels is 64 waves on
// a 1024-SIMD chip), latency is not.
//
// Memory: each block's input samples (kLnB per channel) are moved into an
// LDS slot by LDS-DMA (global_load_lds_dword: four 64-B runs per channel),
// kLnD blocks ahead, and the outputs stored with inline-asm stores; neither
// has a VGPR destination, so nothing can read a register whose load is still
// in flight, and the vector-memory counter is counted here (hipcc drains it
// to 0 before the first LDS read behind a DMA).  Per block the issue order is
//   [wait DMA(b)] [DMA(b+1+D)] [steps] [stores(b)]
// and vmcnt retires in issue order.  Every block issues exactly four DMAs and
// two stores per lane (samples past the signal re-read its last one; outputs
// outside [0, n) and the rows of a partial last wave go to a per-lane dump
// slot), so the counts are exact.  In place: a sample's DMA is issued blocks
// before its output is stored.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dsp_kernels.hpp"

namespace adsp {

namespace {

constexpr int kLnB = 64;             // steps per block
constexpr int kLnD = 2;              // blocks of DMAs in flight beyond the current one
constexpr int kLnSlots = kLnD + 2;   // LDS input slots (the current block, D ahead, one being refilled)
constexpr int kLnRows = 4;           // channels per wave (one per 16-lane DPP row)
constexpr int kLnDma = kLnB / 8;     // DMAs per block: 8 samples (64 B) per row each
constexpr int kLnSt = kLnB / 16;     // output stores per block and lane
static_assert(64 * kLnSt <= kFxEqLaneDump, "one dump slot per lane and store");
constexpr int kLnSlotB = kLnB * kLnRows * 8;  // bytes per slot

__device__ __forceinline__ double row_shr1(double src, double old) {
  // lanes 1..15 of each row: src of the lane below; lane 0: old (no source lane)
  const long long s = __double_as_longlong(src), o = __double_as_longlong(old);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)s, 0x111, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(s >> 32), 0x111, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

typedef __attribute__((address_space(3))) void lds_void_t;
__device__ __forceinline__ unsigned lds_addr(const void* p) { return (unsigned)(uintptr_t)(lds_void_t*)p; }

// 4 B per lane into LDS at m0 + 4 lane (the row's 16 lanes: one 64-B run)
__device__ __forceinline__ void dma4(const void* g, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds)
               : "memory");
}
__device__ __forceinline__ void gstore(double* p, double v) {
  asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// One block of kLnB steps.  The step is software-pipelined by hand: the
// next step's input (the DPP of this step's output) and its three input
// products are formed while this step's output runs down its chain
// yy -> q4 yy -> (q2 v - q4 yy) -> + d1 -> d0, so that in the wave's in-order
// issue the loop-carried path is that chain alone (4 dependent operations)
// and everything else fills its latency.  sched_barrier pins the order (the
// scheduler's model interleaved the steps less well: 96 clocks per step).
#define AD_LN_SB __builtin_amdgcn_sched_barrier(0)
template <bool MASK, bool G1>
__device__ __forceinline__ void lane_steps(const double (&q)[kSecStride], double g0, double& d0, double& d1, double& y,
                                           const double* xb, double* yl, int lane, int64_t tk, int64_t n) {
#pragma clang fp contract(off)
  double xv[kLnB];
#pragma unroll
  for (int i = 0; i < kLnB; ++i) xv[i] = xb[(i >> 3) * (kLnRows * 8) + (i & 7)];  // the row's input (broadcast read)
  // lane 0 takes x * pre_gain (section 0; G1), lanes k > 0 the output of lane k - 1 one step ago
  auto input = [&](double yprev, int i) {
    double v = row_shr1(yprev, G1 ? xv[i] * g0 : xv[i]);
    if (!G1) v = v * q[0];  // G1: x * 1.0 == x on the other sections
    return v;
  };
  double v = input(y, 0);
  double t1 = q[1] * v, t2 = q[2] * v, t3 = q[3] * v;
  AD_LN_SB;
#pragma unroll
  for (int i = 0; i < kLnB; ++i) {
    const double yy = t1 + d0;  // y = b0 x + d0
    AD_LN_SB;
    const double t4 = q[4] * yy;
    AD_LN_SB;
    double vn = 0.0;
    if (i + 1 < kLnB) vn = input(yy, i + 1);
    AD_LN_SB;
    const double t5 = q[5] * yy;
    AD_LN_SB;
    const double e = t2 - t4;
    AD_LN_SB;
    double t1n = 0.0, t2n = 0.0, t3n = 0.0;
    if (i + 1 < kLnB) {
      t1n = q[1] * vn;
      t2n = q[2] * vn;
      t3n = q[3] * vn;
    }
    AD_LN_SB;
    const double n0 = e + d1;  // d0 = b1 x - a1 y + d1
    AD_LN_SB;
    const double n1 = t3 - t5;  // d1 = b2 x - a2 y
    AD_LN_SB;
    y = yy;
    yl[i * 64 + lane] = yy;
    if (MASK) {  // lane k at step s0 + i filters sample s0 + i - k (tk = s0 - k)
      const int64_t t = tk + i;
      const bool ok = t >= 0 && t < n;
      d0 = ok ? n0 : d0;
      d1 = ok ? n1 : d1;
    } else {
      d0 = n0;
      d1 = n1;
    }
    t1 = t1n;
    t2 = t2n;
    t3 = t3n;
    AD_LN_SB;
  }
}
#undef AD_LN_SB

template <bool G1>
__global__ __launch_bounds__(64) void k_fx_eq_lanes(FxEqLaneArgs a) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) double xl[kLnSlots][kLnB * kLnRows];  // [slot][dma][row][8]
  __shared__ double yl[kLnB * 64];
  const int lane = threadIdx.x, r = lane >> 4, k = lane & 15;
  const int c = blockIdx.x * kLnRows + r;
  const bool live = c < a.channels;
  const int cc = live ? c : a.channels - 1;
  const int ns = a.eq.nsec;
  const bool sec = k < ns;
  const int64_t n = a.n;
  const double* secp = a.eq.sec + (int64_t)cc * a.eq.sec_ch_stride;
  double q[kSecStride];
#pragma unroll
  for (int e = 0; e < kSecStride; ++e) q[e] = sec ? secp[k * kSecStride + e] : 0.0;
  const double g0 = G1 ? secp[0] : 1.0;
  double* st = a.eq.state + ((int64_t)cc * ns + (sec ? k : 0)) * 2;
  double d0 = sec ? st[0] : 0.0, d1 = sec ? st[1] : 0.0;
  __builtin_amdgcn_s_waitcnt(0);  // coefficients and state before the counted operations
  double y = 0.0;
  double* row = a.buf + (int64_t)cc * a.stride;
  double* dump = a.dump + lane * kLnSt;
  const int64_t S = n + ns - 1, nb = (S + kLnB - 1) / kLnB;
  const unsigned xl0 = lds_addr(&xl[0][0]);
  // block m's input into slot m % kLnSlots: DMA h carries samples 8h .. 8h+7,
  // lane (r, k) dword k & 1 of sample 8h + k / 2
  auto dma_block = [&](int64_t m) {
    const unsigned base = xl0 + (unsigned)(m % kLnSlots) * kLnSlotB;
#pragma unroll
    for (int h = 0; h < kLnDma; ++h) {
      const int64_t t = min(m * kLnB + 8 * h + (k >> 1), n - 1);
      dma4(reinterpret_cast<const char*>(row + t) + 4 * (k & 1), base + h * (kLnRows * 64));
    }
  };
#pragma unroll
  for (int m = 0; m <= kLnD; ++m) dma_block(m);
  const int tail = ns - 1;  // the last section's lane lags the input by tail samples
  for (int64_t b = 0; b < nb; ++b) {
    // DMA(b) was issued at block b - 1 - D, or in the prologue; the operations
    // issued after it (kLnDma DMAs and kLnSt stores per block):
    // prologue blocks b <= D: kLnDma (D - b) + b (kLnDma + kLnSt); later: kLnSt + D (kLnDma + kLnSt)
    static_assert(kLnD == 2, "the wait counts below cover prologue blocks b = 0 .. 2");
    static_assert(kLnSt + kLnD * (kLnDma + kLnSt) <= 63, "vmcnt holds 6 bits");
    if (b > kLnD)
      wait_vm<kLnSt + kLnD * (kLnDma + kLnSt)>();
    else if (b == 0)
      wait_vm<kLnDma * kLnD>();
    else if (b == 1)
      wait_vm<kLnDma * (kLnD - 1) + (kLnDma + kLnSt)>();
    else
      wait_vm<2 * (kLnDma + kLnSt)>();
    dma_block(b + 1 + kLnD);
    const int64_t s0 = b * kLnB;
    const double* xb = &xl[b % kLnSlots][r * 8];
    const bool full = s0 >= tail && s0 + kLnB - 1 <= n - 1;
    if (full)
      lane_steps<false, G1>(q, g0, d0, d1, y, xb, yl, lane, s0 - k, n);
    else
      lane_steps<true, G1>(q, g0, d0, d1, y, xb, yl, lane, s0 - k, n);
    // the last section's outputs of this block: samples s0 - tail + i
#pragma unroll
    for (int h = 0; h < kLnSt; ++h) {
      const int i = 16 * h + k;
      const double v = yl[i * 64 + 16 * r + tail];
      const int64_t t = s0 - tail + i;
      gstore((live && t >= 0 && t < n) ? row + t : dump + h, v);
    }
  }
  wait_vm<0>();
  if (live && sec) {
    st[0] = d0;
    st[1] = d1;
  }
}

}  // namespace

void launch_fx_eq_lanes(const FxEqLaneArgs& a, bool g1, hipStream_t s) {
  if (a.n <= 0 || a.channels <= 0 || a.eq.nsec <= 0) return;
  const dim3 grid((unsigned)((a.channels + kLnRows - 1) / kLnRows));
  if (g1)
    hipLaunchKernelGGL(k_fx_eq_lanes<true>, grid, dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_fx_eq_lanes<false>, grid, dim3(64), 0, s, a);
}

}  // namespace adsp
