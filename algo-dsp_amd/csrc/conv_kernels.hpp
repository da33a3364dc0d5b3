// Argument blocks and launchers of the conv kernels (conv_kernels.hip).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace adsp {

// Position of bin q (0..M) in a Z row (k_fdl_mac output, K3 input), M >= 64.
// Wave-lane order, parity split: the bins of K2's pair wave bx, 32bx + l, sit
// at 64bx + 16(l & 1) + (l >> 1), and their mirrors M - (32bx + l) at 32 more,
// so every K2 row store is one aligned 1-KiB line run per wave (a partial
// 128-B line shared by two waves would reach HBM as a read-modify-write).
// K3's split transform reads the even bins (A) and the odd bins (B) as two
// separate streams: with even and odd bins in separate 256-B runs, each of
// its load instructions covers whole lines, so all of A can be requested
// before B and A's transform starts while B is in flight.  Bin M/2 sits at M,
// and bin M (only a separation partner) at 32, which K3 never reads.
__host__ __device__ inline int zrow_pos(int q, int M) {
  if (q == M / 2) return M;
  const bool mir = q > M / 2;
  const int d = mir ? M - q : q;
  return ((d >> 5) << 6) + (mir ? 32 : 0) + ((d & 1) << 4) + ((d & 31) >> 1);
}

// Position of raw bin q (0..M-1) in a block-spectrum row (K1 output: the X
// ring and the partition spectra H; K2 and K3's middle bin read it).  A K2
// pair wave bx reads bins 32bx + l (l < 32) and their mirrors M - (32bx + l),
// i.e. the runs [32bx, 32bx + 31] and [M - 32bx - 31, M - 32bx]: in natural
// order the mirror run starts 16 B past a 128-B line and touches five lines
// for four lines of data.  Bins above M/2 therefore sit one slot lower
// (q - 1), which puts every mirror run on line boundaries, and bin M/2 moves
// to the padding column M.  K1's row stores stay contiguous.
__host__ __device__ inline int xrow_pos(int q, int M) {
  return q < M / 2 ? q : (q == M / 2 ? M : q - 1);
}

// Kernel timing of the engine launchers: when start/stop are set (Upols
// profiling), the launch carries them in its dispatch packet
// (hipExtLaunchKernelGGL), so the recorded interval is the kernel's own
// execution, with no marker packets between the kernels of a call.  start is
// consumed by the first launch; every launch re-records stop, so a kernel
// issued as several launches (K2 partition chunks) spans all of them.
struct LaunchTiming {
  hipEvent_t start = nullptr, stop = nullptr;
};
LaunchTiming& launch_timing();  // per host thread
template <class F, class... Args>
inline void timed_launch(F kernel, dim3 grid, dim3 block, hipStream_t s, Args... args) {
  LaunchTiming& t = launch_timing();
  if (t.stop) {
    hipExtLaunchKernelGGL(kernel, grid, block, 0, s, t.start, t.stop, 0, args...);
    t.start = nullptr;
  } else {
    hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
  }
}

// Pre-enqueued streaming block (the host-buffer streaming call, one block of
// hop >= 2048 per call; capi_conv.cpp stream_convolve).  The K1 -> K2 -> K3
// chain of the NEXT block is enqueued while the current one runs; its K1
// waits in the GPU for the host to publish the block's samples (`go` ==
// seq in mapped host memory) instead of the host launching after them, so the
// launches leave the per-block critical path.  K1 gives up after `timeout`
// ticks of the 100 MHz real-time counter, or at once when go == kGateAbort
// (Reset / destroy / a late block), and reports its decision in `k1_state`
// (seq, or seq | kGateSkipped) and in the device word `gate`; K2 and K3 of
// the chain run only when gate == seq.  K3 publishes the block's completion
// by writing seq to `done` (mapped host memory) after its output stores, so
// the host waits on that word, not on a stream.  All pointers null: an
// ordinary launch.
constexpr uint64_t kGateAbort = ~0ull;
constexpr uint64_t kGateSkipped = 1ull << 63;
struct StreamGate {
  const uint64_t* go;     // K1: host-written (mapped)
  uint64_t* k1_state;     // K1: device-written (mapped)
  uint64_t* gate;         // K1 writes, K2 / K3 read (device memory)
  uint64_t* done;         // K3: device-written (mapped)
  uint64_t seq;
  uint64_t timeout;       // K1's wait, 100 MHz ticks
};

struct RfftArgs {
  const double* x;      // input samples, channel c at x + c*x_stride (call-relative index)
  int64_t x_stride;
  int64_t n;            // valid input samples per channel (beyond: zeros)
  int64_t s0;           // first sample of chunk block 0 (call-relative)
  int jc;               // blocks per channel in this launch
  int channels;
  int aligned;          // x and x_stride allow 16-byte pair loads
  double2* X;           // block-spectra ring [C][Q][MS]
  int64_t x_ch_stride;  // Q*MS
  int Q;
  int slot0;            // ring slot of block 0
  int MS;
  const double2* twM;   // W_M^e, e < M
  const double2* twN;   // W_{2M}^k, k < M
  int per_wg;           // blocks per workgroup (set by the launcher, <= the plan's F)
  // Item order (split kernels; ord_R = 0: XCD-contiguous order).  K2 run ry
  // reads block row ry*R - ord_pc + t at its step t, so K1 writes the rows
  // in decreasing t: the rows K2 needs first are the newest in the Infinity
  // Cache.  Grid: channels * (ord_ny + 1) * ord_R (rows outside [0, jc) idle).
  int ord_R, ord_ny, ord_pc;
  StreamGate sg;        // split kernels, one item: wait for the block (see StreamGate)
};

struct MacArgs {
  const double2* X;
  int64_t x_ch_stride;
  int Q;
  int64_t g0;           // logical spectrum index of chunk block 0 (< 0: zeros)
  int64_t gend;         // last logical block holding input samples (later blocks: zeros)
  int nx, ny;           // bin-pair waves, output runs (set by the launcher)
  int p0;               // first partition of this launch's chunk (set by the launcher)
  int MS;
  const double2* H;     // [n_ir][P][MS]
  int64_t h_ir_stride;  // P*MS
  const int* ir_index;  // [C] device (nullable -> c % n_ir)
  int n_ir;
  double2* Y;           // Z output [C][jc_max + 16][MS] (half-length spectra for the inverse rFFT;
                        // rows >= jc_max absorb the last run's overshoot)
  int64_t y_ch_stride;
  const double2* twN;   // W_{2M}^k, k < M
  int jc;
  int R;                // output blocks per wave run (0: auto, one resident round of waves)
  int P;                // partitions
  int M;                // bins 0..M
  int mid_in_k3;        // 1: no middle-bin wave (K3 computes Z[M/2], MidBin)
  StreamGate sg;        // row form: run only if the chain's K1 ran (see StreamGate)
};

// The middle bin M/2 of an output block's Z row, computed by K3 itself
// (launch_fdl_mac then runs no middle-bin wave: at C channels the K2 grid is
// 128·C·runs pair waves, which fills the resident slots exactly, where one
// extra wave per (channel, run) pushed a second round).  Same quantities as
// K2's middle wave: Y = sum_p X'[g-p] H'[p] over the block-spectrum ring,
// then the Z fold.  on = 0: Z[M/2] comes from the row (K2 wrote it).
struct MidBin {
  int on;
  const double2* X;     // block-spectrum ring [C][Q+1][MS] (row Q: zeros)
  int64_t x_ch_stride;
  int Q;
  int64_t g0;           // logical block of chunk block 0
  int64_t gend;         // last logical block holding input
  const double2* H;     // [n_ir][P][MS] raw partition spectra
  int64_t h_ir_stride;
  const int* ir_index;  // [C] (nullable -> c % n_ir)
  int n_ir;
  int P;
};

struct IrfftArgs {
  const double2* Y;
  int64_t y_ch_stride;
  int MS;
  double* out;
  int64_t out_stride;
  int64_t out_len;      // valid output samples per channel (call-relative)
  int64_t o0;           // output sample of chunk block 0
  int jc;
  int channels;
  int aligned;
  int accumulate;       // 1: add into out (partitioned stages sharing one accumulator)
  const double2* twM;
  const double2* twN;
  MidBin mid;
  // Item order (split kernel; ord_R = 0: XCD-contiguous order): K2 run ry
  // writes output row ry*R + t at its step t, so K3 reads the rows in
  // decreasing t, newest first.  Grid: channels * ord_ny * ord_R.
  int ord_R, ord_ny;
  StreamGate sg;        // split kernel, one item: run only if K1 ran; publish completion
  int mix_parity;       // launch_irfft_mix: global index parity of local channel 0 (out: [2][out_stride] mix)
};

bool launch_window_rfft(int M, const RfftArgs& a, hipStream_t s);
bool launch_irfft_store(int M, const IrfftArgs& a, hipStream_t s);
// K3 with the stereo mixdown fused (M >= 2048; false otherwise): a.out is
// the [2][out_stride] mix (L: even global channels, R: odd), the per-channel
// outputs are not written.
bool launch_irfft_mix(int M, const IrfftArgs& a, hipStream_t s);
bool launch_fdl_mac(int PC, int NH, const MacArgs& a, int channels, hipStream_t s);
// K2's run geometry for a launch (run length R: R_req, or auto when <= 0;
// runs ny), shared with the K1/K3 launches that order their items by it.
void mac_run_geometry(int PC, int NH, int M, int mid_in_k3, int channels, int jc, int R_req, int* R, int* ny);
void launch_copy_f64(const double* src, double* dst, int64_t n, hipStream_t s);
void launch_direct(const double* a, int64_t n, const double* b, int64_t m, double* dst, hipStream_t s);
void launch_direct_circular(const double* a, const double* b, int64_t n, double* dst, hipStream_t s);
void launch_stream_direct(const double* h, int64_t K, const double* buf, int64_t B, double* y, hipStream_t s);
void launch_mixdown(const double* ch, int channels, int64_t stride, int64_t len, double* mix, int64_t mix_stride,
                    int first_parity, hipStream_t s);
// One small partitioned stage (two partitions of p <= 1024 taps) for nb
// consecutive blocks of every channel, fused and stateless: a workgroup per
// (block, channel) transforms both input windows x[d-2p, d) and x[d-p, d+p)
// (N = 2p points), multiplies by the two partition spectra, inverse
// transforms and adds the block's p outputs into the accumulator.
struct PcSmallArgs {
  const double* xin;     // [C][xstride] input FIFO, column 0 = absolute time xbase
  int64_t xstride, xbase;
  int64_t d0;            // absolute time of the first block
  int nb;                // blocks per channel
  const double2* H;      // [2][N] full complex spectra of the two partitions (zero padded to N)
  double* acc;           // [C][acc_stride]; block b adds at acc + (d0 + b*p) - acc_origin
  int64_t acc_stride;
  int64_t acc_off;       // accumulator column of absolute time d0 (includes the stage's tap offset)
  const double2* tw;     // W_2048^m, m < 2048
};
bool launch_pc_small(int N, const PcSmallArgs& a, int channels, hipStream_t s);
// k_pc_emit for one channel and n <= 256 samples, pre-enqueued: waits for the
// host's go word (g.go == g.seq; g.k1_state reports run / skipped), then
// emits + appends and publishes g.seq in g.done (see NupolsDev::process_host).
void launch_pc_emit_gated(const double* in, double* out, const double* acc, int64_t off, int64_t first, int64_t n,
                          int mix, double wet, double dry, double* append_to, const StreamGate& g, hipStream_t s);
// Several fused stages in ONE launch (their accumulator ranges must be
// disjoint): stage k takes grid columns [first[k], first[k+1]).
constexpr int kPcMaxFused = 8;
struct PcSmallMulti {
  PcSmallArgs st[kPcMaxFused];
  int N[kPcMaxFused];
  int first[kPcMaxFused + 1];
  int nst;
};
void launch_pc_small_multi(const PcSmallMulti& m, int channels, hipStream_t s);

// dst[c][j] = j < ncopy ? src[c][j] : 0 for j < ncols (channel strides differ)
void launch_shift_cols(const double* src, int64_t src_stride, double* dst, int64_t dst_stride, int channels,
                       int64_t ncopy, int64_t ncols, hipStream_t s);
// Partitioned-convolution emit: out[c][i] = (i < first ? 0 : acc[c][off + i]) or, with mix,
// dry * in[c][i] + wet * that (ConvolutionReverb.ProcessInPlace, no contraction).
void launch_pc_emit(const double* in, int64_t in_stride, double* out, int64_t out_stride, const double* acc,
                    int64_t acc_stride, int64_t off, int64_t first, int64_t n, int channels, int mix, double wet,
                    double dry, hipStream_t s, double* append_to = nullptr, int64_t append_stride = 0,
                    bool emit = true, int64_t row2 = 0);

}  // namespace adsp
