/*
 * algodsp.h — C ABI of the MI355X-native block-DSP engine (libalgodsp_hip.so).
 *
 * This is the drop-in boundary for the sample-buffer hot path of
 * github.com/cwbudde/algo-dsp (pure Go, reference snapshot 2026-03-06).  Every
 * entry point names the reference API it replaces as `file:line` relative to
 * the reference repository root.  A cgo binding for each is shown in
 * INTEGRATION.md.
 *
 * Conventions
 *  - plain pointers + int64 sizes only; no C++/torch types cross the boundary;
 *  - every fallible call returns an int status (AD_OK = 0); the sentinel codes
 *    mirror the reference's `errors.Is` targets so the Go side can map them
 *    back (conv.go:41-46, partitioned.go:11-15);
 *  - host-pointer calls copy in and out inside the call (cgo forbids C from
 *    retaining Go pointers); `*_device` calls take device pointers and a HIP
 *    stream (`void*`, NULL = the HIP default stream, as in the HIP API) and are
 *    asynchronous with respect to the host;
 *  - a handle is single-caller, like the reference types (no internal locks);
 *  - ad_last_error() returns a thread-local description of the last failure.
 *  - there is no CPU fallback: with no usable GPU the create calls fail with
 *    AD_ERR_NO_DEVICE.
 */
#ifndef ALGODSP_H_
#define ALGODSP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define AD_OK 0
#define AD_ERR_EMPTY_INPUT 1              /* conv.ErrEmptyInput        conv.go:42 */
#define AD_ERR_EMPTY_KERNEL 2             /* conv.ErrEmptyKernel       conv.go:43 */
#define AD_ERR_LENGTH_MISMATCH 3          /* conv.ErrLengthMismatch    conv.go:44 */
#define AD_ERR_INVALID_BLOCK_SIZE 4       /* conv.ErrInvalidBlockSize  conv.go:45 */
#define AD_ERR_INVALID_BLOCK_ORDER 5      /* conv.ErrInvalidBlockOrder partitioned.go:12 */
#define AD_ERR_EMPTY_IMPULSE_RESPONSE 6   /* conv.ErrEmptyImpulseResponse partitioned.go:13 */
#define AD_ERR_STAGE_INDEX_OUT_OF_RANGE 7 /* conv.ErrStageIndexOutOfRange partitioned.go:14 */
#define AD_ERR_INVALID_ARGUMENT 8         /* non-sentinel fmt.Errorf validation errors,
                                             e.g. streaming_overlap_save.go:50-52 */
#define AD_ERR_DIVISION_BY_ZERO 9         /* conv.ErrDivisionByZero    deconvolve.go:14 */
#define AD_ERR_UNKNOWN_EFFECT 10          /* effectchain.ErrUnknownEffect chain.go:11 (here: a node
                                             type the GPU graph runtime does not run) */
#define AD_ERR_DEVICE 100                 /* HIP runtime failure */
#define AD_ERR_NO_DEVICE 101              /* no usable gfx950 device */
#define AD_ERR_INTERNAL 102

/* conv.Mode (conv.go:57-69) */
#define AD_MODE_FULL 0
#define AD_MODE_SAME 1
#define AD_MODE_VALID 2

const char* ad_last_error(void);
int ad_version(void);
/* Number of visible HIP devices (0 when none). */
int ad_device_count(int* count);

/* ======================================================================== */
/* dsp/conv                                                                 */
/* ======================================================================== */

typedef struct ad_conv ad_conv;

/* ---- conv.StreamingConvolverT (streaming.go:27-49) ----------------------
 * NewStreamingOverlapSave(kernel, blockSize)   streaming_overlap_save.go:88
 * NewStreamingOverlapAdd(kernel, blockSize)    streaming_overlap_add.go:87
 * Both are zero-latency: out = linear convolution of the stream, block by
 * block.  FFTSize() reports the reference's nextPow2(blockSize+K-1).      */
int ad_conv_stream_ols_create(const double* kernel, int64_t kernel_len, int64_t block_size, int device,
                              ad_conv** out);
int ad_conv_stream_ola_create(const double* kernel, int64_t kernel_len, int64_t block_size, int device,
                              ad_conv** out);
/* ProcessBlockTo(output, input)  streaming_overlap_save.go:152-164,
 * streaming_overlap_add.go:154-168.  in_len/out_len must equal BlockSize()
 * (AD_ERR_LENGTH_MISMATCH otherwise).  in and out may alias.              */
int ad_conv_process_block(ad_conv* h, const double* in, int64_t in_len, double* out, int64_t out_len);

/* ---- float32 instantiations (F = float32, C = complex64 in the reference) --
 * NewStreamingOverlapSave32 streaming_overlap_save.go:94,
 * NewStreamingOverlapAdd32  streaming_overlap_add.go:93,
 * NewPartitionedConvolution32 partitioned.go:340 (+ ProcessBlock :348-396).
 * Same validation, getters, Reset and destroy as the float64 handles; the
 * *_block32 calls take float32 blocks and refuse float64 handles.  Samples
 * are widened exactly to float64, convolved by the float64 engine and
 * rounded once to float32 (never less accurate than the reference's
 * complex64 path).                                                       */
int ad_conv_stream_ols32_create(const float* kernel, int64_t kernel_len, int64_t block_size, int device,
                                ad_conv** out);
int ad_conv_stream_ola32_create(const float* kernel, int64_t kernel_len, int64_t block_size, int device,
                                ad_conv** out);
int ad_conv_process_block32(ad_conv* h, const float* in, int64_t in_len, float* out, int64_t out_len);
int ad_conv_partitioned32_create(const float* kernel, int64_t kernel_len, int min_block_order, int max_block_order,
                                 int device, ad_conv** out);
int ad_conv_partitioned_process_block32(ad_conv* h, const float* in, int64_t in_len, float* out, int64_t out_len);

/* ---- batch conv.OverlapSave / conv.OverlapAdd ---------------------------
 * NewOverlapSave(kernel, fftSize)  overlap_save.go:53-107 (fftSize<=0: auto,
 *   non-power-of-two: AD_ERR_INVALID_BLOCK_SIZE, < 2K: silently raised)
 * NewOverlapAdd(kernel, blockSize) overlap_add.go:44-89 (blockSize<=0: auto)
 * Process/ProcessTo: out_len must be in_len + K - 1 (overlap_save.go:126-272,
 *   overlap_add.go:108-182); empty input -> AD_ERR_EMPTY_INPUT.           */
int ad_conv_ols_create(const double* kernel, int64_t kernel_len, int64_t fft_size, int device, ad_conv** out);
int ad_conv_ola_create(const double* kernel, int64_t kernel_len, int64_t block_size, int device, ad_conv** out);
int ad_conv_process(ad_conv* h, const double* in, int64_t in_len, double* out, int64_t out_len);

/* ---- conv.PartitionedConvolutionT (partitioned.go:27-436) ---------------
 * Output is the linear convolution delayed by Latency() = 2^minBlockOrder.
 * ProcessBlock(input, output) accepts any length (in_len must equal out_len).
 * Stage layout (StageCount/StageInfo) follows partitionIR (:269-332).     */
int ad_conv_partitioned_create(const double* kernel, int64_t kernel_len, int min_block_order, int max_block_order,
                               int device, ad_conv** out);
int ad_conv_partitioned_process_block(ad_conv* h, const double* in, int64_t in_len, double* out, int64_t out_len);
int ad_conv_stage_count(const ad_conv* h);
int ad_conv_stage_info(const ad_conv* h, int index, int64_t* part_size, int64_t* block_count);

/* ---- reverb.ConvolutionReverb (dsp/effects/reverb/convolution.go:16-95) --
 * NewConvolutionReverb(kernel, minBlockOrder): partitioned engine with
 * maxBlockOrder 13, wet = dry = 1, Latency() = 2^minBlockOrder.
 * ProcessInPlace: block[i] = dry*block[i] + wet*reverb(block)[i] (:60-85).
 * Reset/Latency/destroy: the common handle API below.                    */
int ad_conv_reverb_create(const double* kernel, int64_t kernel_len, int min_block_order, int device, ad_conv** out);
int ad_conv_reverb_set_wet_dry(ad_conv* h, double wet, double dry);
int ad_conv_reverb_process_inplace(ad_conv* h, double* block, int64_t n);

/* ---- host-buffer I/O of the batch / multi-channel calls ------------------
 * ad_conv_process and ad_conv_ols_process_multi move host buffers over PCIe
 * in overlapped chunks (no reference counterpart: OverlapSave.Process /
 * ProcessTo, overlap_save.go:126-272, on host memory).  Mode AUTO page-locks
 * the caller's buffers for the call (hipHostRegister; nothing is retained
 * after it returns) when the call moves >= 64 MiB and stages smaller calls
 * through pinned double buffers with `workers` copy threads (0: 8); STAGE and
 * REGISTER force one form (REGISTER falls back to staging if the runtime
 * refuses to lock the pages).  Results are identical in every mode.
 * host_io_profile: wall-time split (ms) of the handle's last host call:
 * page-locking, transfers + compute, unlocking (0 for the staged form's
 * first and last).                                                          */
#define AD_HOST_IO_AUTO 0
#define AD_HOST_IO_STAGE 1
#define AD_HOST_IO_REGISTER 2
int ad_conv_set_host_io(ad_conv* h, int mode, int workers);
int ad_conv_host_io_profile(const ad_conv* h, double* register_ms, double* transfer_ms, double* unregister_ms);

/* Low-latency host calls (streaming blocks of hop >= 2048, partitioned calls
 * of <= 256 samples): how many calls took a pre-enqueued launch and how many
 * pre-enqueued launches timed out (the call then ran ordinary launches).  A
 * handle pre-enqueues only for back-to-back callers, while no other handle
 * has a launch waiting and while the library owns at most 3 streams (they
 * would otherwise share the device's 4 hardware queues with the caller's);
 * a waiting launch gives up after 4 call intervals (1..20 ms).  No reference
 * counterpart (diagnostics).                                              */
int ad_conv_lowlat_stats(const ad_conv* h, int64_t* pre_enqueued, int64_t* timed_out);

/* ---- common handle API -------------------------------------------------- */
int ad_conv_reset(ad_conv* h);   /* Reset(): clears history/tail/FDL state */
int64_t ad_conv_block_size(const ad_conv* h);
int64_t ad_conv_kernel_len(const ad_conv* h);
int64_t ad_conv_fft_size(const ad_conv* h);
int64_t ad_conv_step_size(const ad_conv* h); /* OverlapSave.StepSize (overlap_save.go:115) */
int64_t ad_conv_latency(const ad_conv* h);   /* PartitionedConvolution.Latency (partitioned.go:410) */
void ad_conv_destroy(ad_conv* h);

/* ---- one-shot functions ------------------------------------------------- */
/* conv.Direct / DirectTo (conv.go:76-154): bit-exact input-stationary
 * scatter-add order.  dst has n+m-1 elements.                             */
int ad_conv_direct(const double* a, int64_t n, const double* b, int64_t m, double* dst, int device);
/* conv.DirectTo (conv.go:97-154) on device buffers: d_dst has n+m-1
 * elements; enqueued on `stream` (NULL: the default stream), not synced.  */
int ad_conv_direct_device(const double* d_a, int64_t n, const double* d_b, int64_t m, double* d_dst, void* stream);
/* conv.DirectCircular (conv.go:158-189): n == m, dst has n elements.      */
int ad_conv_direct_circular(const double* a, int64_t n, const double* b, int64_t m, double* dst, int device);
/* conv.Convolve / ConvolveMode (conv.go:194-247).  dst_cap is the capacity
 * of dst; *dst_len receives the result length.                            */
int ad_conv_convolve(const double* a, int64_t n, const double* b, int64_t m, int mode, double* dst, int64_t dst_cap,
                     int64_t* dst_len, int device);

/* ---- multi-channel device-resident engine (offline / many-channel path) --
 * Uniformly partitioned overlap-save with a frequency-domain delay line.
 * kernels: n_ir impulse responses of kernel_len taps each, row-major.
 * hop: partition/hop length (power of two, 64..8192); 0 = auto (min(8192, nextpow2(max(K, 256))).
 * channels: number of channels processed per call; ir_index[c] selects the
 *   IR of channel c (NULL: c % n_ir).
 * max_chunk_blocks: blocks per channel per internal chunk (0 = auto).     */
int ad_conv_multi_create(const double* kernels, int n_ir, int64_t kernel_len, int64_t hop, int channels,
                         const int32_t* ir_index, int64_t max_chunk_blocks, int device, ad_conv** out);
/* Offline schedule of the device calls below (no reference counterpart: how
 * OverlapSave.Process, overlap_save.go:126-254, is laid out on the GPU).
 * SERIAL: each internal chunk's forward transforms, delay-line MAC and inverse
 * transforms run in turn on the caller's stream.  PIPELINED (hop >= 2048;
 * smaller hops stay serial): chunks of chunk_blocks blocks per channel (0:
 * auto) whose spectra stay in the Infinity Cache, the MAC and the inverse
 * transforms on two internal streams, so consecutive chunks' kernels overlap;
 * the caller's stream still passes the call only when every output is
 * written.  run_blocks: the MAC's run length (0: auto).  Results are
 * bit-identical in both schedules.  Applies from the next signal start (a
 * process_device call, or a segment / mix call with out_begin == 0).       */
#define AD_CONV_SCHED_SERIAL 0
#define AD_CONV_SCHED_PIPELINED 1
#define AD_CONV_SCHED_CHUNKED 2 /* PIPELINED's chunks and rings, every kernel on the caller's stream */
int ad_conv_multi_set_schedule(ad_conv* h, int mode, int64_t chunk_blocks, int64_t run_blocks);
int ad_conv_multi_get_schedule(const ad_conv* h, int* mode, int64_t* chunk_blocks);
/* Full linear convolution of every channel (ModeFull semantics per channel):
 * d_in  [channels][in_stride] (first in_len used),
 * d_out [channels][out_stride] (first out_len written; out_len <= in_len+K-1).
 * Device pointers; asynchronous on `stream` (NULL = default stream).      */
int ad_conv_multi_process_device(ad_conv* h, const double* d_in, int64_t in_stride, int64_t in_len, double* d_out,
                                 int64_t out_stride, int64_t out_len, void* stream);
/* The same full linear convolution computed one output segment at a time:
 * this call writes d_out[c][out_begin .. min(out_end, out_len)) only.
 * out_begin == 0 starts a new signal; a later segment must start where the
 * previous one ended (the frequency-domain delay line carries over), and
 * out_begin / out_end are multiples of the hop (out_end may also be out_len).
 * Segments let a caller overlap per-segment work, such as the multi-GPU
 * mixdown reduce, with the next segment's convolution.  Results are identical
 * to one ad_conv_multi_process_device call.  No reference counterpart: it is
 * the batch OverlapSave.Process (overlap_save.go:126-254) split by output
 * range.  Out-of-order segments return AD_ERR_INVALID_ARGUMENT.            */
int ad_conv_multi_process_device_segment(ad_conv* h, const double* d_in, int64_t in_stride, int64_t in_len,
                                         double* d_out, int64_t out_stride, int64_t out_len, int64_t out_begin,
                                         int64_t out_end, void* stream);
/* The full linear convolution of every channel with the stereo mixdown of
 * the group fused into the inverse transform (config 4's per-GPU work, SURVEY
 * 8(e)): d_mix [2][mix_stride] receives, for out_begin <= t < out_end,
 *   d_mix[t]              (L) = sum of the channels with an even global index,
 *   d_mix[mix_stride + t] (R) = sum of those with an odd global index,
 * where local channel c has global index first_parity + c (mod 2), summed in
 * increasing c.  The per-channel outputs are not written to memory (hop >=
 * 2048; smaller hops convolve into an internal buffer and mix it).  Equal to
 * ad_conv_multi_process_device + ad_conv_mixdown_device to rounding (each
 * channel's block enters the sum as (acc + A) - W B of its split inverse
 * transform's halves, computed at another radix split).  out_begin /
 * out_end follow ad_conv_multi_process_device_segment (out_end <= 0: out_len;
 * 0, 0 = the whole output in one call).  A caller mixing into the RCCL reduce
 * then passes channels = 0 to ad_mixdown_reduce.  Reference: the batch
 * OverlapSave.Process (overlap_save.go:126-254) per channel, then the mix.  */
int ad_conv_multi_process_device_mix(ad_conv* h, const double* d_in, int64_t in_stride, int64_t in_len,
                                     double* d_mix, int64_t mix_stride, int64_t out_len, int first_parity,
                                     int64_t out_begin, int64_t out_end, void* stream);
/* OverlapSave.Process / ProcessTo (overlap_save.go:126-272) of every channel
 * of a multi-channel handle on HOST buffers: in[c] holds n samples, out[c]
 * receives n + kernel_len - 1.  The signal crosses PCIe in chunks through
 * pinned double buffers, overlapping H2D of chunk i+1, the convolution of
 * chunk i and D2H of chunk i-1 (three streams); bit-identical to the device
 * call.  channels must equal the handle's (else AD_ERR_LENGTH_MISMATCH).    */
int ad_conv_ols_process_multi(ad_conv* h, const double* const* in, double* const* out, int channels, int64_t n);

/* ---- multi-channel streaming convolver ----------------------------------
 * `channels` StreamingOverlapSave instances (streaming_overlap_save.go:45-184)
 * sharing n_ir kernels (ir_index[c], NULL: c % n_ir) in one handle: each
 * block call runs every channel with ONE launch per engine kernel, the
 * frequency-domain delay line and input history stay on the device between
 * calls (config 4 real-time form: 64 reverb channels, block by block).
 * Any block_size > 0: with a power-of-two divisor >= 256 (or a power of two
 * >= 64) that divisor is the hop and a call is whole engine blocks; any other
 * size (480, 960, 1000, 4800 ...) runs at hop = nextPow2(block_size) (at least
 * kernel_len/64, within 64..8192) and carries the unfinished block between
 * calls, so a call costs at most ceil((hop - 1 + block_size) / hop) FFT
 * blocks per channel.  Zero latency: out = the newest block_size samples of
 * each channel's linear convolution.
 * Reset / getters: ad_conv_reset, ad_conv_block_size, ad_conv_fft_size.   */
int ad_conv_multi_stream_create(const double* kernels, int n_ir, int64_t kernel_len, int64_t block_size,
                                int channels, const int32_t* ir_index, int device, ad_conv** out);
/* host buffers: in[c], out[c] of n == block_size samples (else AD_ERR_LENGTH_MISMATCH) */
int ad_conv_multi_stream_process_block(ad_conv* h, const double* const* in, double* const* out, int channels,
                                       int64_t n);
/* device buffers [channels][stride]; asynchronous on `stream` */
int ad_conv_multi_stream_process_block_device(ad_conv* h, const double* d_in, int64_t in_stride, double* d_out,
                                              int64_t out_stride, void* stream);
/* ---- many-channel partitioned convolution / convolution reverb ----------
 * `channels` PartitionedConvolution instances (partitioned.go:212-436) that
 * share ONE impulse response, device resident: y[c][t] = (h * x_c)[t - 2^minOrder]
 * for any call length.  Each non-uniform stage is one UPOLS engine over all
 * channels (one launch per engine kernel per stage per call), accumulating
 * into a device buffer; latency 2^minOrder must be 64..8192 here.
 * The reverb form (maxBlockOrder 13, wet = dry = 1 until
 * ad_conv_reverb_set_wet_dry) processes in place as
 * ConvolutionReverb.ProcessInPlace (convolution.go:60-85) -- the
 * effect-chain reverb-conv node.  ad_conv_reset, ad_conv_latency,
 * ad_conv_stage_count / ad_conv_stage_info apply.                          */
int ad_conv_pc_multi_create(const double* kernel, int64_t kernel_len, int min_order, int max_order, int channels,
                            int device, ad_conv** out);
int ad_conv_pc_multi_process_device(ad_conv* h, const double* d_in, int64_t in_stride, double* d_out,
                                    int64_t out_stride, int64_t n, void* stream);
int ad_conv_reverb_multi_create(const double* kernel, int64_t kernel_len, int min_order, int channels, int device,
                                ad_conv** out);
int ad_conv_reverb_multi_process_device(ad_conv* h, double* d_buf, int64_t stride, int64_t n, void* stream);
/* host buffer [channels][n], in place */
int ad_conv_reverb_multi_process(ad_conv* h, double* buf, int64_t n);

/* Live kernel timing (HIP events recorded around every launch on the launch
 * stream) for the FFT engine of a handle.  Kernel index: 0 window rFFT,
 * 1 frequency-domain delay-line MAC, 2 inverse rFFT + overlap-save store.
 * read() synchronises and returns, per kernel, the summed duration (ms),
 * the launch count and the algorithmic bytes those launches moved
 * (DESIGN.md), then clears the counters.  Arrays have 3 entries.          */
int ad_conv_profile_enable(ad_conv* h, int enable);
int ad_conv_profile_read(ad_conv* h, double* total_ms, int64_t* launches, double* alg_bytes);
/* Which kernels enabled timing records: bit k = kernel k (default 7, all).
 * Timing one kernel keeps two events per call inside a timed loop.       */
int ad_conv_profile_kernels(ad_conv* h, int mask);
/* Stereo mixdown of a channel group (build-defined; the
 * reference defines no mixdown):
 *   d_mix[t]              (L) = sum of the group's channels with an even global index,
 *   d_mix[mix_stride + t] (R) = sum of those with an odd global index,
 * t < len; channel c of the group has global index first + c and
 * first_parity = first & 1.  d_chan [channels][stride].  Asynchronous on
 * `stream`.  mix_stride >= len (L and R rows of one [2][mix_stride] buffer,
 * so an output segment can be mixed into its place: pass d_chan + b and
 * d_mix + b).                                                              */
int ad_conv_mixdown_device(const double* d_chan, int channels, int64_t stride, int64_t len, double* d_mix,
                           int64_t mix_stride, int first_parity, void* stream);

/* ---- multi-GPU mixdown over RCCL (SURVEY 8(b) ad_mixdown_reduce, 8(e)) ----
 * One process per GPU; every rank convolves its own channel group and the
 * stereo partial mixes are summed on `root` with ONE RCCL reduce over xGMI.
 * The communicator is created from a unique id that rank 0 makes and the
 * caller distributes (cgo side: any transport -- the reference has no
 * multi-process layer).  librccl.so.1 is loaded on first use (no link-time
 * dependency for single-GPU callers).                                      */
#define AD_COMM_ID_BYTES 128
typedef struct ad_comm ad_comm;
int ad_comm_get_unique_id(uint8_t id[AD_COMM_ID_BYTES]);
/* ncclCommInitRank over `nranks` ranks; `device` is this rank's GPU. */
int ad_comm_create(const uint8_t id[AD_COMM_ID_BYTES], int nranks, int rank, int device, ad_comm** out);
void ad_comm_destroy(ad_comm* comm);
int ad_comm_rank(const ad_comm* comm);
int ad_comm_size(const ad_comm* comm);
/* k_mixdown of this rank's group into d_mix ([2][mix_stride], as
 * ad_conv_mixdown_device), then an in-place sum-reduce of d_mix's 2 x len
 * values to `root` (d_mix on root holds the whole job's stereo mix; on the
 * other ranks it holds the rank's partial mix).  Both are enqueued on
 * `stream` and the call returns without waiting.  channels == 0 skips the
 * mixdown (d_mix already holds the partial mix, e.g. a stereo group).      */
int ad_mixdown_reduce(ad_comm* comm, const double* d_chan, int channels, int64_t stride, int64_t len,
                      int first_parity, double* d_mix, int64_t mix_stride, int root, void* stream);

/* ======================================================================== */
/* dsp/filter, dsp/effects: per-sample processors                           */
/* ======================================================================== */

/* ---- effect chain: biquad EQ -> Compressor -> Freeverb, per channel ------
 * One handle runs `channels` independent instances of the reference
 * processors, each stage optional, fused per sample on the GPU (bit-exact
 * with running the stages block by block, as effectchain.Chain.Process does,
 * chain_process.go:11-33).  Buffers are [channels][n] (host) or
 * [channels][stride] (device), processed in place.
 *
 * EQ stage = biquad.Chain(s) (chain.go:6-138, section.go:26-155): a table of
 * sections {pre_gain, b0, b1, b2, a1, a2}; pre_gain is the Chain gain on a
 * chain's first section (1.0 otherwise).  per_channel = 0: one table [nsec][6]
 * for all channels; 1: [channels][nsec][6].  Replaces Chain.ProcessBlock and,
 * with one section, Section.ProcessBlock (the avx2/generic registry kernels,
 * registry.go:10-100, compute the same DF-II-T recurrence).
 * Compressor stage = dynamics.Compressor ProcessInPlace (compressor.go:362-366)
 * configured by an ad_compressor_config struct, mirroring the setters
 * (compressor.go:130-305).
 * Freeverb stage = reverb.Reverb ProcessInPlace (reverb.go:185-189) with
 * SetWet/SetDry/SetRoomSize/SetDamp/SetGain values (reverb.go:192-220).     */
typedef struct ad_fx_chain ad_fx_chain;
typedef struct ad_compressor_config {
  double sample_rate, threshold_db, ratio, knee_db, attack_ms, release_ms, rms_window_ms, makeup_db;
  double sidechain_low_cut_hz, sidechain_high_cut_hz; /* 0: off; else [1 Hz, Nyquist), low < high */
  int topology;             /* 0 feed-forward, 1 feedback */
  int detector_mode;        /* 0 peak, 1 RMS */
  int feedback_ratio_scale; /* 1: feedback topology scales time constants and ratio */
  int auto_makeup;          /* 1: makeup = -threshold*(1-1/ratio) */
} ad_compressor_config;
/* NewCompressor(sampleRate) defaults (compressor.go:77-127). */
void ad_compressor_default_config(ad_compressor_config* cfg, double sample_rate);
/* The setters' validation of a whole config, host only (no device needed):
 * AD_OK, or AD_ERR_INVALID_ARGUMENT for any value a reference setter rejects:
 * ratio outside [1, 100], knee outside [0, 24] dB, attack outside [0.1, 1000]
 * ms, release outside [1, 5000] ms, RMS window outside [1, 1000] ms
 * (compressor.go:16-23, core.go:10-12, 131-198), a non-finite threshold or
 * makeup, a bad sample rate, topology or detector mode, a side-chain cut
 * that is negative or not in [1 Hz, Nyquist), or low >= high when both are on
 * (core.go:542-564).  ad_fx_chain_set_compressor and the graph's COMPRESSOR
 * node run the same check and change nothing on failure. */
int ad_compressor_validate(const ad_compressor_config* cfg);

int ad_fx_chain_create(int channels, int device, ad_fx_chain** out);
int ad_fx_chain_set_eq(ad_fx_chain* h, const double* sections, int nsec, int per_channel);
/* The EQ round-off noise estimate ad_fx_chain_set_eq computes for the engine
 * choice (eps sqrt(sum NG) of the worst of `sets` tables [nsec][6]; +inf when
 * a section is unstable: |a2| >= 1 or |a1| >= 1 + a2).  Host only, no device
 * needed; no reference counterpart (diagnostics).                         */
int ad_fx_eq_noise(const double* sections, int nsec, int sets, double* noise);
int ad_fx_chain_set_compressor(ad_fx_chain* h, const ad_compressor_config* cfg); /* NULL: stage off */
/* dynamics.Expander / dynamics.Gate (expander.go, gate.go) as the chain's
 * dynamics stage instead of the compressor: cfg gives threshold, ratio, knee,
 * attack, release, detector, topology, RMS window and side-chain filters
 * (makeup fields ignored: these have none); range_db is SetRange, hold_ms is
 * the gate's SetHold (gate != 0).  Out-of-range values -> AD_ERR_INVALID_ARGUMENT
 * (the setters' validation). */
int ad_fx_chain_set_expander(ad_fx_chain* h, const ad_compressor_config* cfg, int gate, double range_db,
                             double hold_ms);
int ad_fx_chain_set_freeverb(ad_fx_chain* h, double wet, double dry, double room_size, double damp, double gain);
int ad_fx_chain_disable_freeverb(ad_fx_chain* h);
int ad_fx_chain_reset(ad_fx_chain* h); /* Chain/Compressor/Reverb Reset() */
int ad_fx_chain_process(ad_fx_chain* h, double* buf, int64_t n);
int ad_fx_chain_process_device(ad_fx_chain* h, double* d_buf, int64_t stride, int64_t n, void* stream);
/* Compressor metrics of one channel (updateMetrics compressor.go:411-423):
 * input peak, output peak, minimum gain (gain reduction, linear). */
int ad_fx_chain_compressor_metrics(ad_fx_chain* h, int channel, double* input_peak, double* output_peak,
                                   double* gain_reduction);
/* EQ section state [channels][nsec][2] {d0, d1} (Chain.State, chain.go:122-130). */
int ad_fx_chain_eq_state(ad_fx_chain* h, double* state, int64_t cap);
/* Chain.SetState (chain.go:130-138) / Section.SetState (section.go:152-155)
 * of every channel, between calls: state [channels][nsec][2] {d0, d1};
 * n < channels*nsec*2 -> AD_ERR_LENGTH_MISMATCH (the reference indexes
 * states[i] for every section).  With ad_fx_chain_eq_state this is the
 * reference's checkpoint / resume surface for the EQ.                       */
int ad_fx_chain_set_eq_state(ad_fx_chain* h, const double* state, int64_t n);
/* Which engine runs the chain:
 *   AUTO            with a compressor, the time-parallel engine (below);
 *                   otherwise the staged engine (stage kernels over time
 *                   chunks on three streams, fx_staged.hip) where it applies
 *                   -- feed-forward dynamics, <= 8 EQ sections, <= 8192
 *                   channels with Freeverb -- with the EQ split over two CUs
 *                   when >= 3 sections are on; else FUSED;
 *   FUSED           the fused per-sample kernels (dsp_kernels.hip k_chain*);
 *   STAGED_NOSPLIT  staged, one EQ pipeline per channel group;
 *   STAGED          staged with the split EQ stage;
 *   TIME_PARALLEL   the time-parallel engine (fx_tp.hip) also for chains
 *                   without a compressor: EQ only, Freeverb only, EQ +
 *                   Freeverb (where the staged engine applies; otherwise as
 *                   AUTO).
 * FUSED, STAGED_NOSPLIT and STAGED perform the reference's operations in its
 * order: their outputs are identical.  The time-parallel engine starts the
 * EQ's time segments from chained states (double-double): its outputs are
 * within 1e-12 relative RMS of those (the serial recurrence's own rounding
 * noise for low-frequency sections), not bit-identical.  That noise grows
 * with the sections' round-off noise gain (poles near z = 1: a low highpass
 * at a high sample rate), so AUTO and TIME_PARALLEL keep the staged engine
 * for an EQ whose noise estimate exceeds 4.5e-13 (ad_fx_chain_last_engine).
 * chunk: samples per staged / time-parallel chunk (0: the engine's default;
 * otherwise >= 256).                                                         */
#define AD_FX_ENGINE_AUTO 0
#define AD_FX_ENGINE_FUSED 1
#define AD_FX_ENGINE_STAGED_NOSPLIT 2
#define AD_FX_ENGINE_STAGED 3
#define AD_FX_ENGINE_TIME_PARALLEL 4
int ad_fx_chain_set_engine(ad_fx_chain* h, int engine, int64_t chunk);
/* The engine that ran the last process call (AD_FX_ENGINE_FUSED, _STAGED,
 * _STAGED_NOSPLIT or _TIME_PARALLEL; -1 before the first call) and the EQ's
 * round-off noise estimate eps sqrt(sum NG) that gates the time-parallel
 * engine (0 without an EQ, inf for an unstable section).  Either pointer may
 * be NULL.  No reference counterpart (engine introspection). */
int ad_fx_chain_last_engine(ad_fx_chain* h, int* engine, double* eq_noise);
/* Per-wave clock counters (s_memtime ticks) of the first chunk of each call,
 * for profiling the serial stages: {compute, barrier wait} pairs per wave. */
int ad_fx_chain_set_profiling(ad_fx_chain* h, int enable);
int ad_fx_chain_read_profile(ad_fx_chain* h, unsigned long long* counters, int cap, int* count);
void ad_fx_chain_destroy(ad_fx_chain* h);

/* ---- batched effectchain graph (dsp/effectchain, 8(f)4) -------------------
 * `channels` copies of one effect-chain graph, each with its own state, run
 * together (one lane per channel).  Replaces effectchain.Chain.Process
 * (chain_process.go:11-33) for graphs made of the node types below; the
 * host-side graph compiler (JSON parse + Kahn order, graph.go:57-165, node
 * Configure param clamps, runtime_*.go) lives in the caller and passes the
 * nodes in topological order, node 0 being `_input`.
 * Per node (processNode, chain_process.go:136-175): the input is the
 * average of the parents' outputs (mixParentEdgesInto :295-318: zeros with
 * no parent, a copy for one, sum in edge order * 1/k for k), then
 *   AD_FXN_SPLIT_FREQ  LR crossover: low = LP chain, high = HP chain, read by
 *                      consumers through parent port 0 / 1 (crossover.go:80-94,
 *                      chain_process.go:177-227; not affected by `bypassed`);
 *   AD_FXN_OUTPUT / AD_FXN_PASS ("split", "sum") / bypassed: mix only;
 *   AD_FXN_BIQUAD      biquad.Chain.ProcessBlock, sections [nsec][6] as in
 *                      ad_fx_chain_set_eq (filter* nodes, runtime_filter_pitch_reverb.go:186-195);
 *   AD_FXN_COMPRESSOR  Compressor.ProcessInPlace with *comp (dyn-compressor,
 *                      and dyn-limiter = NewLimiter's ratio 100 / attack 0.1 ms /
 *                      hard knee / no makeup config, limiter.go:11-44);
 *   AD_FXN_FREEVERB    reverb.Reverb.ProcessInPlace, verb = {wet, dry,
 *                      room_size, damp, gain} (runtime_filter_pitch_reverb.go:330-345);
 *   AD_FXN_CONV_REVERB reverb.ConvolutionReverb.ProcessInPlace (reverb-conv,
 *                      runtime_misc.go:61-67) on the many-channel partitioned engine.
 * The result is the output node's buffer.  Linear runs of in-place nodes fuse
 * into one launch (bit-identical, see capi_fxgraph.cpp).  Other node types
 * return AD_ERR_UNKNOWN_EFFECT; the configs are copied at create.          */
#define AD_FXN_INPUT 0
#define AD_FXN_OUTPUT 1
#define AD_FXN_PASS 2
#define AD_FXN_SPLIT_FREQ 3
#define AD_FXN_BIQUAD 4
#define AD_FXN_COMPRESSOR 5
#define AD_FXN_FREEVERB 6
#define AD_FXN_CONV_REVERB 7 /* reverb-conv (runtime_misc.go:12-67): ConvolutionReverb(ir, conv_min_order)
                                with SetWetDry(conv_wet, conv_dry), in place; the caller
                                mono-averages the provider's IR as Configure does */
#define AD_FX_MAX_PARENTS 8
typedef struct ad_fx_node {
  int type;
  int bypassed;
  int n_parents;
  const int32_t* parents;      /* indices of earlier nodes, in the graph's edge order */
  const int32_t* parent_ports; /* NULL: all 0; 1 = a split-freq node's high band */
  const double* sections;      /* BIQUAD: [nsec][6]; SPLIT_FREQ: low-band (LP) chain */
  int nsec;
  const double* sections2;     /* SPLIT_FREQ: high-band (HP) chain [nsec2][6] */
  int nsec2;
  const ad_compressor_config* comp; /* COMPRESSOR */
  double verb[5];                   /* FREEVERB: wet, dry, room_size, damp, gain */
  int dyn_mode;                     /* COMPRESSOR: 0 compressor / limiter, 1 expander (dyn-expander),
                                       2 gate (dyn-gate); see ad_fx_chain_set_expander */
  double dyn_range_db, dyn_hold_ms; /* expander / gate: SetRange, the gate's SetHold */
  const double* ir;                 /* CONV_REVERB: impulse response [ir_len] */
  int64_t ir_len;
  int conv_min_order;               /* CONV_REVERB: minBlockOrder (reverb-conv uses 7; maxBlockOrder 13) */
  double conv_wet, conv_dry;        /* CONV_REVERB: SetWetDry(wet, dry) (reverb-conv: wet param, dry 1.0) */
} ad_fx_node;
typedef struct ad_fx_graph ad_fx_graph;
int ad_fx_graph_create(const ad_fx_node* nodes, int n_nodes, int channels, int device, ad_fx_graph** out);
/* buf [channels][n] (host) / [channels][stride] (device), processed in place. */
int ad_fx_graph_process(ad_fx_graph* g, double* buf, int64_t n);
int ad_fx_graph_process_device(ad_fx_graph* g, double* d_buf, int64_t stride, int64_t n, void* stream);
int ad_fx_graph_reset(ad_fx_graph* g); /* every node runtime's Reset() */
/* Compiled size: device ops per call, buffers (including the caller's) and
 * streams the independent branches are spread over (the caller's included). */
int ad_fx_graph_op_count(const ad_fx_graph* g, int* launches, int* buffers, int* lanes);
void ad_fx_graph_destroy(ad_fx_graph* g);

/* One-shot biquad.Chain.ProcessBlock over `channels` chains sharing one
 * coefficient set coeffs [sections][5] {b0,b1,b2,a1,a2} and gain (chain.go:59-70);
 * state [channels][sections][2] is read and updated; buf [channels][n]. */
int ad_biquad_chain_process(const double* coeffs, double* state, double gain, double* buf, int channels,
                            int sections, int64_t n, int device);

/* ---- IRLB f16 sample decode (internal/webdemo/irlib.go:68-97, 414-451) ----
 * AUDI chunk payload (little-endian f16, frames interleaved by channel) ->
 * float64 [channels][frames], bit-exact with decodeF16 including its
 * subnormal exponent (every subnormal half decodes to twice its IEEE value). */
int ad_decode_f16(const uint16_t* in, int64_t frames, int channels, double* out, int device);
int ad_decode_f16_device(const uint16_t* d_in, int64_t frames, int channels, double* d_out, void* stream);

/* ---- fir.Filter (dsp/filter/fir/filter.go:11-172) -------------------------
 * New(coeffs) for `channels` independent filters sharing the taps.
 * taps < 32: y[n] = sum_k h[k] x[n-k] (ProcessSample order, :46-69);
 * taps >= 32: the block path's reversed pairing y[n] = sum_j h[j] x[n-N+1+j]
 * (linear-buffer dot product, :74-159).  n == 0 taps: output untouched.     */
typedef struct ad_fir ad_fir;
int ad_fir_create(const double* coeffs, int64_t n_taps, int channels, int device, ad_fir** out);
int ad_fir_process_block(ad_fir* f, double* buf, int64_t n);                        /* :74-114 */
int ad_fir_process_block_to(ad_fir* f, double* dst, const double* src, int64_t n);  /* :119-159 */
int ad_fir_process_device(ad_fir* f, const double* d_src, int64_t src_stride, double* d_dst, int64_t dst_stride,
                          int64_t n, void* stream);
int ad_fir_reset(ad_fir* f); /* :162-172 */
void ad_fir_destroy(ad_fir* f);

/* ---- spectral correlation / deconvolution (dsp/conv/correlate.go,
 * dsp/conv/deconvolve.go) --------------------------------------
 * One power-of-two FFT over the whole zero-padded signal, as the reference's
 * algofft.NewPlan64(n) calls.  Inputs are host arrays copied in inside the
 * call (the _device form takes device pointers on a caller stream).        */

/* CorrelateFFT (correlate.go:111-172): out[n+m-1], index k = lag k-(m-1);
 * FFT size nextPow2(n+m-1); empty a or b -> AD_ERR_EMPTY_INPUT.            */
int ad_correlate_fft(const double* a, int64_t n, const double* b, int64_t m, double* out, int device);
int ad_correlate_fft_device(const double* d_a, int64_t n, const double* d_b, int64_t m, double* d_out, int device,
                            void* stream);

/* DeconvMethod / DeconvOptions (deconvolve.go:20-63) */
#define AD_DECONV_NAIVE 0
#define AD_DECONV_REGULARIZED 1
#define AD_DECONV_WIENER 2
typedef struct {
  int method;
  double epsilon;         /* Regularized: <= 0 -> 1e-6 */
  double noise_variance;  /* Wiener: <= 0 -> 1% of the signal variance */
  double signal_variance; /* Wiener: <= 0 -> variance(signal) */
} ad_deconv_options;
ad_deconv_options ad_deconv_default_options(void); /* :57-63 {Regularized, 1e-6} */

/* Deconvolve (deconvolve.go:72-101 and the three methods :104-323): circular
 * spectral division at FFT size nextPow2(n) (the signal length);
 * *out_len = n-m+1, or n when that is <= 0.  Empty signal ->
 * AD_ERR_EMPTY_INPUT, empty kernel -> AD_ERR_EMPTY_KERNEL, naive method with
 * |H[k]| < 1e-15 -> AD_ERR_DIVISION_BY_ZERO (first bin in ad_last_error);
 * m > nextPow2(n) (the reference indexes out of range) -> AD_ERR_INVALID_ARGUMENT. */
int ad_deconvolve(const double* signal, int64_t n, const double* kernel, int64_t m, const ad_deconv_options* opts,
                  double* out, int64_t out_cap, int64_t* out_len, int device);

/* InverseFilter (deconvolve.go:354-394): out[length] = real(IFFT(conj H /
 * (|H|^2 + eps))), FFT size nextPow2(length), kernel truncated to it;
 * eps <= 0 -> 1e-6; empty kernel -> AD_ERR_EMPTY_KERNEL.                   */
int ad_inverse_filter(const double* kernel, int64_t m, int64_t length, double epsilon, double* out, int device);

#ifdef __cplusplus
}
#endif

#endif /* ALGODSP_H_ */
