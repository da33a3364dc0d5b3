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
//   - the block's outputs stay in registers (kLnB per lane) and are handed
//     to an I/O wave through LDS once per block.
// So the step has no barrier and no hand-over beyond one DPP pair, and the
// loop-carried path is the section's own four-operation chain.  A wave holds
// four channels; lanes are cheap here (the EQ of 256 channels is 64 waves on
// a 1024-SIMD chip), latency is not.
//
// Memory (the I/O wave, see k_fx_eq_lanes): each block's input samples
// (kLnB per channel) are moved into an LDS slot by LDS-DMA
// (global_load_lds_dword: kLnDma 64-B runs per channel), two blocks ahead;
// the outputs are stored with inline-asm stores.  Neither has a VGPR
// destination, and the wave drains its vector-memory counter once per block
// (hipcc would drain it to 0 before the first LDS read behind a DMA anyway).
// Samples past the signal re-read its last one; outputs outside [0, n) and
// the rows of a partial last wave go to a per-lane dump slot.  In place: a
// sample's DMA is issued blocks before its output is stored.
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

#ifndef AD_LN_EXP  // tools/ probe builds only: 1 no output stores, 2 no DMAs (wrong results);
#define AD_LN_EXP 0  // 16384 output writes by every lane (no exec mask), 4096 no output writes,
                     // 8192 16-B output writes
#endif
constexpr int kLnPre = 16;             // input read-ahead of the compute wave (steps)
// yo row stride: rows r and r + 1 (one half-wave of a 64-bit read) on disjoint banks
constexpr int kLnYoS = kLnB + 16;
constexpr int kLnYoN = 2;  // output buffers (block parity)
constexpr int kLnIBar = kLnB - kLnPre;  // the step at which the compute wave meets the barrier

// One block of kLnB steps of the cascade (the operations of eq_section_step
// in its order; the compiler's schedule interleaves consecutive steps).
// side(i) runs at the start of step i (the input read-ahead, the barrier).
template <bool MASK, bool G1, class Side>
__device__ __forceinline__ void lane_steps(const double (&q)[kSecStride], double g0, double& d0, double& d1, double& y,
                                           double (&xv)[kLnB], double (&yb)[kLnB], int64_t tk, int64_t n,
                                           const Side& side) {
#pragma clang fp contract(off)
#pragma unroll
  for (int i = 0; i < kLnB; ++i) {
    side(i);
    // lane 0 takes x * pre_gain (section 0; G1), lanes k > 0 the output of lane k - 1 one step ago
    double v = row_shr1(y, G1 ? xv[i] * g0 : xv[i]);
    if (!G1) v = v * q[0];  // G1: x * 1.0 == x on the other sections
    const double yy = q[1] * v + d0;
    const double n0 = q[2] * v - q[4] * yy + d1;
    const double n1 = q[3] * v - q[5] * yy;
    if (MASK) {  // lane k at step s0 + i filters sample s0 + i - k (tk = s0 - k)
      const int64_t t = tk + i;
      const bool ok = t >= 0 && t < n;
      d0 = ok ? n0 : d0;
      d1 = ok ? n1 : d1;
    } else {
      d0 = n0;
      d1 = n1;
    }
    y = yy;
    yb[i] = yy;  // the block's outputs stay in registers (the last section's lane hands them over)
  }
}

__device__ __forceinline__ void lds_fence_barrier() {
  // the LDS writes before it are visible to the other wave after it (LDS
  // operations of a wave complete in order: a count <= 15 covers every write
  // issued 16 or more LDS operations earlier; callers pass 0 where fewer)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Two waves per workgroup (four channels):
//   wave 0 (compute) runs the cascade: its only memory operations are LDS
//     reads of the inputs (kLnPre steps ahead, from the slot the I/O wave
//     filled) and, once per block, the block's outputs written to LDS (the
//     last section's lane into yo); one barrier per block, at step kLnIBar,
//     before the first read of the next block's slot;
//   wave 1 (I/O) moves the samples: between barrier(b) and barrier(b+1) it
//     waits for its previous phase's operations (DMA(b+2) among them), stores
//     block b-1's outputs from yo and issues the DMAs of block b+D+1.
// Measured (tools/eq_lanes_ab.sh, tools/lane_probe.hip, 256 ch x 2^20): the
// compute wave's own global stores cost ~100 clocks each (a one-wave form:
// 184 clocks per step with them, 62 without), its DMAs ~10 clocks per step,
// and the output writes per block ~11 (74 clocks per step against 63 with
// no hand-over; 16-B writes 76; writes by every lane without an exec mask: 79; four bursts of
// 8 inside the block: 80).  A wave
// alone on its SIMD hides nothing behind a stall.
template <bool G1>
__global__ __launch_bounds__(128) void k_fx_eq_lanes(FxEqLaneArgs a) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) double xl[kLnSlots][kLnB * kLnRows];  // [slot][dma][row][8]
  __shared__ __attribute__((aligned(16))) double yo[kLnYoN][kLnRows][kLnYoS];    // [block % kLnYoN][row][step]
  __shared__ __attribute__((aligned(16))) double junk[2 * 64 + kLnB];            // the other lanes' output writes
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, r = lane >> 4, k = lane & 15;
  const int c = blockIdx.x * kLnRows + r;
  const bool live = c < a.channels;
  const int cc = live ? c : a.channels - 1;
  const int ns = a.eq.nsec;
  const int64_t n = a.n;
  const int64_t S = n + ns - 1, nb = (S + kLnB - 1) / kLnB;
  const int tail = ns - 1;  // the last section's lane lags the input by tail samples
  double* row = a.buf + (int64_t)cc * a.stride;
  static_assert(kLnD == 2, "the wait counts below assume two blocks of DMAs ahead");
  if (wave == 1) {
    // ---- I/O wave
    double* dump = a.dump + lane * kLnSt;
    const unsigned xl0 = lds_addr(&xl[0][0]);
    // block m's input into slot m % kLnSlots: DMA h carries samples 8h .. 8h+7,
    // lane (r, k) dword k & 1 of sample 8h + k / 2
    auto dma_block = [&](int64_t m) {
      if (AD_LN_EXP & 2) return;
      const unsigned base = xl0 + (unsigned)(m % kLnSlots) * kLnSlotB;
#pragma unroll
      for (int h = 0; h < kLnDma; ++h) {
        const int64_t t = min(m * kLnB + 8 * h + (k >> 1), n - 1);
        dma4(reinterpret_cast<const char*>(row + t) + 4 * (k & 1), base + h * (kLnRows * 64));
      }
    };
    // block m's outputs (samples m kLnB - tail + 16 h + k of row r)
    auto store_outputs = [&](int64_t m) {
      if (AD_LN_EXP & 1) return;
      double v[kLnSt];
#pragma unroll
      for (int h = 0; h < kLnSt; ++h) v[h] = yo[m % kLnYoN][r][16 * h + k];
#pragma unroll
      for (int h = 0; h < kLnSt; ++h) {
        const int64_t t = m * kLnB - tail + 16 * h + k;
        gstore((m >= 0 && live && t >= 0 && t < n) ? row + t : dump + h, v[h]);
      }
    };
#pragma unroll
    for (int m = 0; m <= kLnD; ++m) dma_block(m);
    wait_vm<0>();         // DMA(0 .. D)
    lds_fence_barrier();  // the compute wave reads slot 0
    lds_fence_barrier();  // barrier(0): slot 1
    for (int64_t b = 0; b < nb; ++b) {
      wait_vm<0>();  // the previous phase's stores and DMA(b + 2), read after barrier(b + 1)
      store_outputs(b - 1);
      dma_block(b + kLnD + 1);
      lds_fence_barrier();  // barrier(b + 1)
    }
    wait_vm<0>();
    store_outputs(nb - 1);
    wait_vm<0>();
    return;
  }
  // ---- compute wave
  const bool sec = k < ns;
  const double* secp = a.eq.sec + (int64_t)cc * a.eq.sec_ch_stride;
  double q[kSecStride];
#pragma unroll
  for (int e = 0; e < kSecStride; ++e) q[e] = sec ? secp[k * kSecStride + e] : 0.0;
  const double g0 = G1 ? secp[0] : 1.0;
  double* st = a.eq.state + ((int64_t)cc * ns + (sec ? k : 0)) * 2;
  double d0 = sec ? st[0] : 0.0, d1 = sec ? st[1] : 0.0;
  double y = 0.0;
  auto slot_x = [&](int64_t m, int i) {  // the row's input of step i of block m (broadcast read)
    return xl[m % kLnSlots][(i >> 3) * (kLnRows * 8) + r * 8 + (i & 7)];
  };
  lds_fence_barrier();  // slot 0 has landed
  double xv[kLnB], yb[kLnB];
#pragma unroll
  for (int i = 0; i < kLnPre; ++i) xv[i] = slot_x(0, i);
  for (int64_t b = 0; b < nb; ++b) {
    const auto side = [&](int i) {
      if (i == kLnIBar) {
        // barrier(b): block b + 1's slot has landed; the outputs of block b - 1
        // (written a block ago, followed by more than 15 LDS reads) reach the I/O wave
        asm volatile("s_waitcnt lgkmcnt(15)\n\ts_barrier" ::: "memory");
      }
      // every 8 steps, the inputs of the 8 steps kLnPre ahead (one 64-B run per
      // row) in one group the scheduler may not move: it otherwise sinks the
      // reads next to their use, where the LDS latency shows
      if (i % 8 == 0) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int j = i + kLnPre + e;  // the ring slot of step j (this block) or j - kLnB (the next)
          if (j < kLnB)
            xv[j] = slot_x(b, j);
          else
            xv[j - kLnB] = slot_x(b + 1, j - kLnB);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    const int64_t s0 = b * kLnB;
    const bool full = s0 >= tail && s0 + kLnB - 1 <= n - 1;
    if (full)
      lane_steps<false, G1>(q, g0, d0, d1, y, xv, yb, s0 - k, n, side);
    else
      lane_steps<true, G1>(q, g0, d0, d1, y, xv, yb, s0 - k, n, side);
    if (AD_LN_EXP & 16384) {
      // probe: every lane writes its outputs (no exec mask), the last section's
      // lane into yo, the others each into a junk run of their own (distinct
      // addresses within every instruction): 79 against 76 clocks per step
      double2* wp = k == tail ? reinterpret_cast<double2*>(&yo[b % kLnYoN][r][0])
                              : reinterpret_cast<double2*>(&junk[2 * lane]);
#pragma unroll
      for (int i = 0; i < kLnB; i += 2) wp[i / 2] = make_double2(yb[i], yb[i + 1]);
    } else if (k == tail && (AD_LN_EXP & 8192)) {  // probe: the first build's 16-B writes (ds_write_b128)
#pragma unroll
      for (int i = 0; i < kLnB; i += 2)
        *reinterpret_cast<double2*>(&yo[b % kLnYoN][r][i]) = make_double2(yb[i], yb[i + 1]);
    } else if (k == tail && !(AD_LN_EXP & 4096)) {
      // the last section's outputs of block b, one 8-B write each: the sched
      // barriers keep them apart (merged into 16-B writes they measured 75.8
      // against 74.1 clocks per step; an exec-masked ds_write_b128 occupies the
      // LDS issue ~5x as long as a read, SQ_ACTIVE_INST_LDS)
      double* yw = &yo[b % kLnYoN][r][0];
#pragma unroll
      for (int i = 0; i < kLnB; ++i) {
        yw[i] = yb[i];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  lds_fence_barrier();  // barrier(nb): the last block's outputs
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
    hipLaunchKernelGGL(k_fx_eq_lanes<true>, grid, dim3(128), 0, s, a);
  else
    hipLaunchKernelGGL(k_fx_eq_lanes<false>, grid, dim3(128), 0, s, a);
}

}  // namespace adsp
