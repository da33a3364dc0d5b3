"""dsp/conv mirror over the HIP C ABI.

Names, argument meaning and error behaviour follow the reference package
github.com/cwbudde/algo-dsp/dsp/conv (file:line cited per entry point), so
tests read like the reference's own.  Every call runs on the GPU through
libalgodsp_hip.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import dataclasses
import math

from ._lib import (ADError, DeconvOptionsC, ErrDivisionByZero, ErrEmptyImpulseResponse, ErrEmptyInput,
                   ErrEmptyKernel, ErrInvalidArgument, ErrInvalidBlockOrder, ErrInvalidBlockSize, ErrLengthMismatch,
                   ErrStageIndexOutOfRange, check, f64, lib, ptr)

__all__ = [
    "ADError", "ErrEmptyInput", "ErrEmptyKernel", "ErrLengthMismatch", "ErrInvalidBlockSize",
    "ErrInvalidBlockOrder", "ErrEmptyImpulseResponse", "ErrStageIndexOutOfRange", "ErrInvalidArgument",
    "ModeFull", "ModeSame", "ModeValid",
    "Direct", "DirectCircular", "Convolve", "ConvolveMode",
    "NewStreamingOverlapSave", "NewStreamingOverlapAdd", "NewOverlapSave", "NewOverlapAdd",
    "NewStreamingOverlapSave32", "NewStreamingOverlapAdd32", "NewPartitionedConvolution32",
    "NewPartitionedConvolution", "OverlapAddConvolve", "OverlapSaveConvolve", "MultiChannelConvolver",
    "MultiChannelStreamingConvolver", "PartitionedConvolutionMulti", "NewConvolutionReverbMulti",
    "ErrDivisionByZero", "Correlate", "CorrelateDirect", "CorrelateMode", "AutoCorrelate", "AutoCorrelateNormalized",
    "CorrelateNormalized", "CorrelateFFT", "FindPeak", "LagFromIndex", "IndexFromLag",
    "DeconvNaive", "DeconvRegularized", "DeconvWiener", "DeconvOptions", "DefaultDeconvOptions", "Deconvolve",
    "InverseFilter", "SNR",
]

ModeFull, ModeSame, ModeValid = 0, 1, 2  # conv.go:57-69

DEVICE = 0


class _Handle:
    def __init__(self, h: C.c_void_p):
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().ad_conv_destroy(h)
            except Exception:
                pass
            self._h = None

    def Reset(self) -> None:
        check(lib().ad_conv_reset(self._h))

    def KernelLen(self) -> int:
        return int(lib().ad_conv_kernel_len(self._h))

    def FFTSize(self) -> int:
        return int(lib().ad_conv_fft_size(self._h))

    def LowLatencyStats(self):
        """(calls that took a pre-enqueued launch, pre-enqueued launches that
        timed out) of a streaming or partitioned handle (ad_conv_lowlat_stats)."""
        a, b = C.c_int64(), C.c_int64()
        check(lib().ad_conv_lowlat_stats(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    # host-buffer I/O of batch / multi-channel calls (include/algodsp.h ad_conv_set_host_io)
    HOST_IO_AUTO, HOST_IO_STAGE, HOST_IO_REGISTER = 0, 1, 2

    def set_host_io(self, mode: int, workers: int = 0) -> None:
        check(lib().ad_conv_set_host_io(self._h, int(mode), int(workers)))

    def host_io_profile(self):
        """(register_ms, transfer_ms, unregister_ms) of the last host-buffer call."""
        r, t, u = C.c_double(), C.c_double(), C.c_double()
        check(lib().ad_conv_host_io_profile(self._h, C.byref(r), C.byref(t), C.byref(u)))
        return r.value, t.value, u.value


class StreamingConvolver(_Handle):
    """conv.StreamingConvolverT (streaming.go:27-49)."""

    def BlockSize(self) -> int:
        return int(lib().ad_conv_block_size(self._h))

    def ProcessBlockTo(self, output: np.ndarray, input) -> None:
        x = f64(input)
        if not (isinstance(output, np.ndarray) and output.dtype == np.float64 and output.flags.c_contiguous):
            raise TypeError("output must be a contiguous float64 ndarray")
        check(lib().ad_conv_process_block(self._h, ptr(x), x.size, ptr(output), output.size))

    def ProcessBlock(self, input) -> np.ndarray:
        x = f64(input)
        out = np.empty(self.BlockSize(), dtype=np.float64)
        check(lib().ad_conv_process_block(self._h, ptr(x), x.size, ptr(out), out.size))
        return out


def _create(fn, *args) -> C.c_void_p:
    h = C.c_void_p()
    check(fn(*args, C.byref(h)))
    return h


def NewStreamingOverlapSave(kernel, blockSize: int) -> StreamingConvolver:
    """streaming_overlap_save.go:88"""
    k = f64(kernel)
    return StreamingConvolver(_create(lib().ad_conv_stream_ols_create, ptr(k), k.size, int(blockSize), DEVICE))


def NewStreamingOverlapAdd(kernel, blockSize: int) -> StreamingConvolver:
    """streaming_overlap_add.go:87"""
    k = f64(kernel)
    return StreamingConvolver(_create(lib().ad_conv_stream_ola_create, ptr(k), k.size, int(blockSize), DEVICE))


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _fptr(a: np.ndarray):
    if a.size == 0:
        return C.cast(C.c_void_p(0), C.POINTER(C.c_float))
    return a.ctypes.data_as(C.POINTER(C.c_float))


class StreamingConvolver32(StreamingConvolver):
    """StreamingConvolverT[float32, complex64] (streaming.go:27-49)."""

    def ProcessBlockTo(self, output: np.ndarray, input) -> None:
        x = _f32(input)
        if not (isinstance(output, np.ndarray) and output.dtype == np.float32 and output.flags.c_contiguous):
            raise TypeError("output must be a contiguous float32 ndarray")
        check(lib().ad_conv_process_block32(self._h, _fptr(x), x.size, _fptr(output), output.size))

    def ProcessBlock(self, input) -> np.ndarray:
        out = np.empty(self.BlockSize(), dtype=np.float32)
        self.ProcessBlockTo(out, input)
        return out


def NewStreamingOverlapSave32(kernel, blockSize: int) -> StreamingConvolver32:
    """streaming_overlap_save.go:94"""
    k = _f32(kernel)
    return StreamingConvolver32(_create(lib().ad_conv_stream_ols32_create, _fptr(k), k.size, int(blockSize), DEVICE))


def NewStreamingOverlapAdd32(kernel, blockSize: int) -> StreamingConvolver32:
    """streaming_overlap_add.go:93"""
    k = _f32(kernel)
    return StreamingConvolver32(_create(lib().ad_conv_stream_ola32_create, _fptr(k), k.size, int(blockSize), DEVICE))


class BatchConvolver(_Handle):
    """conv.OverlapSave / conv.OverlapAdd batch convolvers."""

    def BlockSize(self) -> int:
        return int(lib().ad_conv_block_size(self._h))

    def StepSize(self) -> int:
        return int(lib().ad_conv_step_size(self._h))

    def Process(self, input) -> np.ndarray:
        x = f64(input)
        out = np.empty(max(x.size + self.KernelLen() - 1, 0), dtype=np.float64)
        check(lib().ad_conv_process(self._h, ptr(x), x.size, ptr(out), out.size))
        return out

    def ProcessTo(self, output: np.ndarray, input) -> None:
        x = f64(input)
        check(lib().ad_conv_process(self._h, ptr(x), x.size, ptr(output), output.size))


def NewOverlapSave(kernel, fftSize: int = 0) -> BatchConvolver:
    """overlap_save.go:53-107"""
    k = f64(kernel)
    return BatchConvolver(_create(lib().ad_conv_ols_create, ptr(k), k.size, int(fftSize), DEVICE))


def NewOverlapAdd(kernel, blockSize: int = 0) -> BatchConvolver:
    """overlap_add.go:44-89"""
    k = f64(kernel)
    return BatchConvolver(_create(lib().ad_conv_ola_create, ptr(k), k.size, int(blockSize), DEVICE))


def OverlapAddConvolve(signal, kernel) -> np.ndarray:
    """overlap_add.go:221-253"""
    return NewOverlapAdd(kernel, 0).Process(signal)


def OverlapSaveConvolve(signal, kernel) -> np.ndarray:
    """overlap_save.go:313-342"""
    return NewOverlapSave(kernel, 0).Process(signal)


class PartitionedConvolution(_Handle):
    """conv.PartitionedConvolutionT (partitioned.go:27-436)."""

    def ProcessBlock(self, input, output: np.ndarray) -> None:
        x = f64(input)
        check(lib().ad_conv_partitioned_process_block(self._h, ptr(x), x.size, ptr(output), output.size))

    def Latency(self) -> int:
        return int(lib().ad_conv_latency(self._h))

    def StageCount(self) -> int:
        return int(lib().ad_conv_stage_count(self._h))

    def StageInfo(self, index: int):
        p = C.c_int64()
        b = C.c_int64()
        check(lib().ad_conv_stage_info(self._h, int(index), C.byref(p), C.byref(b)))
        return p.value, b.value


def NewPartitionedConvolution(kernel, minBlockOrder: int, maxBlockOrder: int) -> PartitionedConvolution:
    """partitioned.go:335-337"""
    k = f64(kernel)
    return PartitionedConvolution(
        _create(lib().ad_conv_partitioned_create, ptr(k), k.size, int(minBlockOrder), int(maxBlockOrder), DEVICE))


class PartitionedConvolution32(PartitionedConvolution):
    """PartitionedConvolutionT[float32, complex64] (partitioned.go:340)."""

    def ProcessBlock(self, input, output: np.ndarray) -> None:
        x = _f32(input)
        if not (isinstance(output, np.ndarray) and output.dtype == np.float32 and output.flags.c_contiguous):
            raise TypeError("output must be a contiguous float32 ndarray")
        check(lib().ad_conv_partitioned_process_block32(self._h, _fptr(x), x.size, _fptr(output), output.size))


def NewPartitionedConvolution32(kernel, minBlockOrder: int, maxBlockOrder: int) -> PartitionedConvolution32:
    """partitioned.go:340"""
    k = _f32(kernel)
    return PartitionedConvolution32(
        _create(lib().ad_conv_partitioned32_create, _fptr(k), k.size, int(minBlockOrder), int(maxBlockOrder), DEVICE))


class ConvolutionReverb(_Handle):
    """reverb.ConvolutionReverb (dsp/effects/reverb/convolution.go:16-95):
    block = dry*block + wet*PartitionedConvolution(block), latency 2^minBlockOrder."""

    def SetWetDry(self, wet: float, dry: float) -> None:
        check(lib().ad_conv_reverb_set_wet_dry(self._h, float(wet), float(dry)))

    def ProcessInPlace(self, block: np.ndarray) -> None:
        if not (isinstance(block, np.ndarray) and block.dtype == np.float64 and block.flags.c_contiguous):
            raise TypeError("block must be a C-contiguous float64 array")
        check(lib().ad_conv_reverb_process_inplace(self._h, ptr(block), block.size))

    def Latency(self) -> int:
        return int(lib().ad_conv_latency(self._h))


def NewConvolutionReverb(kernel, minBlockOrder: int) -> ConvolutionReverb:
    """convolution.go:28-44 (maxBlockOrder fixed at 13, wet = dry = 1)"""
    k = f64(kernel)
    return ConvolutionReverb(_create(lib().ad_conv_reverb_create, ptr(k), k.size, int(minBlockOrder), DEVICE))


class PartitionedConvolutionMulti(_Handle):
    """`channels` PartitionedConvolution instances sharing one IR, device
    resident (ad_conv_pc_multi_*): one launch per engine kernel per stage
    per call for all channels."""

    def __init__(self, kernel, minBlockOrder: int, maxBlockOrder: int, channels: int, device: int = DEVICE,
                 reverb: bool = False):
        k = f64(kernel)
        h = C.c_void_p()
        if reverb:
            check(lib().ad_conv_reverb_multi_create(ptr(k), k.size, int(minBlockOrder), int(channels), int(device),
                                                    C.byref(h)))
        else:
            check(lib().ad_conv_pc_multi_create(ptr(k), k.size, int(minBlockOrder), int(maxBlockOrder), int(channels),
                                                int(device), C.byref(h)))
        super().__init__(h)
        self.channels = channels

    def Latency(self) -> int:
        return int(lib().ad_conv_latency(self._h))

    def StageCount(self) -> int:
        return int(lib().ad_conv_stage_count(self._h))

    def process_device(self, d_in: int, in_stride: int, d_out: int, out_stride: int, n: int, stream: int = 0):
        check(lib().ad_conv_pc_multi_process_device(self._h, C.c_void_p(d_in), int(in_stride), C.c_void_p(d_out),
                                                    int(out_stride), int(n), C.c_void_p(stream)))

    # ConvolutionReverb form
    def SetWetDry(self, wet: float, dry: float) -> None:
        check(lib().ad_conv_reverb_set_wet_dry(self._h, float(wet), float(dry)))

    def ProcessInPlace(self, block: np.ndarray) -> None:
        """block [channels][n] float64 (host), dry*block + wet*reverb in place."""
        if not (isinstance(block, np.ndarray) and block.dtype == np.float64 and block.flags.c_contiguous):
            raise TypeError("block must be a C-contiguous float64 array")
        check(lib().ad_conv_reverb_multi_process(self._h, ptr(block), block.shape[-1]))

    def process_inplace_device(self, d_buf: int, stride: int, n: int, stream: int = 0) -> None:
        check(lib().ad_conv_reverb_multi_process_device(self._h, C.c_void_p(d_buf), int(stride), int(n),
                                                        C.c_void_p(stream)))


def NewConvolutionReverbMulti(kernel, minBlockOrder: int, channels: int) -> PartitionedConvolutionMulti:
    """NewConvolutionReverb (convolution.go:28-44) x channels, one handle."""
    return PartitionedConvolutionMulti(kernel, minBlockOrder, 13, channels, reverb=True)


def Direct(a, b) -> np.ndarray:
    """conv.go:76-93"""
    x, y = f64(a), f64(b)
    out = np.empty(max(x.size + y.size - 1, 0), dtype=np.float64)
    check(lib().ad_conv_direct(ptr(x), x.size, ptr(y), y.size, ptr(out), DEVICE))
    return out


def direct_device(d_a: int, n: int, d_b: int, m: int, d_dst: int, stream: int = 0) -> None:
    """conv.DirectTo (conv.go:97-154) on device buffers (d_dst: n+m-1 f64),
    enqueued on `stream`."""
    check(lib().ad_conv_direct_device(C.c_void_p(d_a), int(n), C.c_void_p(d_b), int(m), C.c_void_p(d_dst),
                                      C.c_void_p(stream or 0)))


def DirectCircular(a, b) -> np.ndarray:
    """conv.go:158-173"""
    x, y = f64(a), f64(b)
    out = np.empty(x.size, dtype=np.float64)
    check(lib().ad_conv_direct_circular(ptr(x), x.size, ptr(y), y.size, ptr(out), DEVICE))
    return out


def ConvolveMode(a, b, mode: int) -> np.ndarray:
    """conv.go:219-226"""
    x, y = f64(a), f64(b)
    cap = max(x.size + y.size - 1, 1)
    out = np.empty(cap, dtype=np.float64)
    n = C.c_int64()
    check(lib().ad_conv_convolve(ptr(x), x.size, ptr(y), y.size, int(mode), ptr(out), cap, C.byref(n), DEVICE))
    return out[: n.value].copy()


def Convolve(a, b) -> np.ndarray:
    """conv.go:194-216"""
    return ConvolveMode(a, b, ModeFull)


class MultiChannelConvolver(_Handle):
    """Device-resident many-channel UPOLS engine (offline path; include/algodsp.h)."""

    def __init__(self, kernels, hop: int = 0, channels: int = 1, ir_index=None, chunk_blocks: int = 0,
                 device: int = DEVICE):
        k = f64(kernels)
        if k.ndim == 1:
            k = k.reshape(1, -1)
        n_ir, K = k.shape
        irx = None
        if ir_index is not None:
            arr = (C.c_int32 * channels)(*[int(v) for v in ir_index])
            irx = C.cast(arr, C.POINTER(C.c_int32))
        h = C.c_void_p()
        check(lib().ad_conv_multi_create(ptr(k), int(n_ir), int(K), int(hop), int(channels), irx,
                                         int(chunk_blocks), int(device), C.byref(h)))
        super().__init__(h)
        self.channels = channels
        self.kernel_len = K

    KERNELS = ("k_window_rfft", "k_fdl_mac", "k_irfft_store")
    SCHED_SERIAL = 0     # include/algodsp.h AD_CONV_SCHED_*
    SCHED_PIPELINED = 1

    def set_schedule(self, mode: int, chunk_blocks: int = 0, run_blocks: int = 0) -> None:
        """Offline schedule of the device calls (ad_conv_multi_set_schedule):
        SCHED_SERIAL or SCHED_PIPELINED (chunks kept in the Infinity Cache,
        K2 / K3 on internal streams); bit-identical results."""
        check(lib().ad_conv_multi_set_schedule(self._h, int(mode), int(chunk_blocks), int(run_blocks)))

    def schedule(self):
        """(mode, chunk_blocks) the next signal runs with (chunk 0: serial)."""
        m = C.c_int()
        c = C.c_int64()
        check(lib().ad_conv_multi_get_schedule(self._h, C.byref(m), C.byref(c)))
        return m.value, c.value

    def profile_enable(self, on: bool = True, kernels: int = 7) -> None:
        """Event timing of the engine's launches; kernels: bit k = KERNELS[k]."""
        check(lib().ad_conv_profile_kernels(self._h, kernels))
        check(lib().ad_conv_profile_enable(self._h, 1 if on else 0))

    def profile_read(self):
        """{kernel: (total_ms, launches, algorithmic_bytes)}; synchronises and clears."""
        ms = (C.c_double * 3)()
        n = (C.c_int64 * 3)()
        b = (C.c_double * 3)()
        check(lib().ad_conv_profile_read(self._h, ms, n, b))
        return {k: (ms[i], n[i], b[i]) for i, k in enumerate(self.KERNELS)}

    def process_device(self, d_in: int, in_stride: int, in_len: int, d_out: int, out_stride: int, out_len: int,
                       stream: int = 0) -> None:
        check(lib().ad_conv_multi_process_device(self._h, C.c_void_p(d_in), in_stride, in_len, C.c_void_p(d_out),
                                                 out_stride, out_len, C.c_void_p(stream)))

    def process_device_segment(self, d_in: int, in_stride: int, in_len: int, d_out: int, out_stride: int,
                               out_len: int, out_begin: int, out_end: int, stream: int = 0) -> None:
        """process_device restricted to outputs [out_begin, out_end): segments of one
        signal run in order and together equal one process_device call."""
        check(lib().ad_conv_multi_process_device_segment(self._h, C.c_void_p(d_in), in_stride, in_len,
                                                         C.c_void_p(d_out), out_stride, out_len, out_begin,
                                                         out_end, C.c_void_p(stream)))

    def process_device_mix(self, d_in: int, in_stride: int, in_len: int, d_mix: int, mix_stride: int,
                           out_len: int, first_parity: int = 0, out_begin: int = 0, out_end: int = 0,
                           stream: int = 0) -> None:
        """Every channel's full linear convolution with the stereo mixdown fused
        (ad_conv_multi_process_device_mix): d_mix [2][mix_stride] gets L (even
        global channels) and R (odd) over [out_begin, out_end); the per-channel
        outputs are not stored."""
        check(lib().ad_conv_multi_process_device_mix(self._h, C.c_void_p(d_in), in_stride, in_len,
                                                     C.c_void_p(d_mix), mix_stride, out_len, int(first_parity),
                                                     out_begin, out_end, C.c_void_p(stream)))


def _row_ptrs(a: np.ndarray):
    """(c_double_p * rows) of a C-contiguous 2-D float64 array."""
    rows = a.shape[0]
    arr = (C.POINTER(C.c_double) * rows)()
    base = a.ctypes.data
    for r in range(rows):
        arr[r] = C.cast(C.c_void_p(base + r * a.strides[0]), C.POINTER(C.c_double))
    return arr


def _process_host_multi(self, x, out: np.ndarray | None = None) -> np.ndarray:
    """OverlapSave.Process of every channel on host buffers
    (ad_conv_ols_process_multi: chunked, PCIe overlapped with the compute);
    `out` ([C][n+K-1] float64, C-contiguous) is reused when given (ProcessTo)."""
    xs = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    if xs.ndim == 1:
        xs = xs.reshape(1, -1)
    shape = (xs.shape[0], xs.shape[1] + self.kernel_len - 1)
    if out is None:
        out = np.empty(shape, dtype=np.float64)
    elif out.shape != shape or out.dtype != np.float64 or not out.flags.c_contiguous:
        raise ErrLengthMismatch(3, f"conv: output must be a C-contiguous float64 array of shape {shape}")
    check(lib().ad_conv_ols_process_multi(self._h, _row_ptrs(xs), _row_ptrs(out), int(xs.shape[0]),
                                          int(xs.shape[1])))
    return out


MultiChannelConvolver.process_host = _process_host_multi


class MultiChannelStreamingConvolver(_Handle):
    """`channels` StreamingOverlapSave instances in one handle (one launch per
    engine kernel per block for all channels; the frequency-domain delay line
    stays on the device): ad_conv_multi_stream_*."""

    def __init__(self, kernels, block_size: int, channels: int, ir_index=None, device: int = DEVICE):
        k = f64(kernels)
        if k.ndim == 1:
            k = k.reshape(1, -1)
        n_ir, K = k.shape
        irx = None
        if ir_index is not None:
            arr = (C.c_int32 * channels)(*[int(v) for v in ir_index])
            irx = C.cast(arr, C.POINTER(C.c_int32))
        h = C.c_void_p()
        check(lib().ad_conv_multi_stream_create(ptr(k), int(n_ir), int(K), int(block_size), int(channels), irx,
                                                int(device), C.byref(h)))
        super().__init__(h)
        self.channels = channels

    def BlockSize(self) -> int:
        return int(lib().ad_conv_block_size(self._h))

    def ProcessBlock(self, x) -> np.ndarray:
        """x: [channels][block] -> [channels][block] (host buffers)."""
        xs = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
        out = np.empty_like(xs)
        check(lib().ad_conv_multi_stream_process_block(self._h, _row_ptrs(xs), _row_ptrs(out), int(xs.shape[0]),
                                                       int(xs.shape[1])))
        return out

    def process_block_device(self, d_in: int, in_stride: int, d_out: int, out_stride: int, stream: int = 0) -> None:
        check(lib().ad_conv_multi_stream_process_block_device(self._h, C.c_void_p(d_in), int(in_stride),
                                                              C.c_void_p(d_out), int(out_stride), C.c_void_p(stream)))


def mixdown_device(d_chan: int, channels: int, stride: int, length: int, d_mix: int, stream: int = 0,
                   mix_stride: int | None = None, first_parity: int = 0) -> None:
    """Stereo partial mix of a channel group (k_mixdown): L row at d_mix, R row
    at d_mix + mix_stride (default: length) doubles."""
    check(lib().ad_conv_mixdown_device(C.c_void_p(d_chan), channels, stride, length, C.c_void_p(d_mix),
                                       int(length if mix_stride is None else mix_stride), int(first_parity),
                                       C.c_void_p(stream)))


# ---------------------------------------------------------------------------
# dsp/conv/correlate.go
# ---------------------------------------------------------------------------
def _trim_to_mode(full: np.ndarray, lenA: int, lenB: int, mode: int) -> np.ndarray:
    """conv.go:229-247 trimToMode (slicing only)."""
    if mode == ModeSame:
        start = (lenB - 1) // 2
        return full[start:start + lenA].copy()
    if mode == ModeValid:
        return (full[lenB - 1:lenA] if lenA >= lenB else full[lenA - 1:lenB]).copy()
    return full


def Correlate(a, b) -> np.ndarray:
    """correlate.go:16-29: Convolve(a, reverse(b)) on the GPU."""
    x, y = f64(a), f64(b)
    if x.size == 0 or y.size == 0:
        raise ErrEmptyInput(1, "conv: empty input")
    return Convolve(x, y[::-1].copy())


def CorrelateDirect(a, b) -> np.ndarray:
    """correlate.go:32-43: Direct(a, reverse(b)) (bit-exact GPU direct form)."""
    x, y = f64(a), f64(b)
    if x.size == 0 or y.size == 0:
        raise ErrEmptyInput(1, "conv: empty input")
    return Direct(x, y[::-1].copy())


def CorrelateMode(a, b, mode: int) -> np.ndarray:
    """correlate.go:46-53"""
    x, y = f64(a), f64(b)
    return _trim_to_mode(Correlate(x, y), x.size, y.size, mode)


def AutoCorrelate(a) -> np.ndarray:
    """correlate.go:58-60"""
    return Correlate(a, a)


def AutoCorrelateNormalized(a) -> np.ndarray:
    """correlate.go:64-82: zero-lag value scaled to 1 (host rescale of the GPU result)."""
    x = f64(a)
    r = AutoCorrelate(x)
    z = r[x.size - 1]
    return r if z == 0 else r / z


def _l2_norm(x: np.ndarray) -> float:
    """correlate.go:175-183 (sequential sum of squares)."""
    s = 0.0
    for v in x.tolist():
        s += v * v
    return math.sqrt(s)


def CorrelateNormalized(a, b) -> np.ndarray:
    """correlate.go:87-108: divided by |a|*|b|."""
    x, y = f64(a), f64(b)
    r = Correlate(x, y)
    p = _l2_norm(x) * _l2_norm(y)
    return r if p == 0 else r / p


def CorrelateFFT(a, b) -> np.ndarray:
    """correlate.go:111-172: one nextPow2(n+m-1) FFT correlation on the GPU."""
    x, y = f64(a), f64(b)
    out = np.empty(max(x.size + y.size - 1, 0), dtype=np.float64)
    check(lib().ad_correlate_fft(ptr(x), x.size, ptr(y), y.size, ptr(out), DEVICE))
    return out


def _fft_pass_count(N: int) -> int:
    """Passes of the device FFT plan for size N (bigfft.hip BigFft::BigFft)."""
    k = max(0, N.bit_length() - 1)
    if k <= 3:
        return 1
    if k <= 12:
        return 1
    return (k + 8) // 9


def FindPeak(corr):
    """correlate.go:187-205: (index, value) of the first maximum; (-1, 0) when empty."""
    c = f64(corr)
    if c.size == 0:
        return -1, 0.0
    i = int(np.argmax(c))
    return i, float(c[i])


def LagFromIndex(index: int, lenB: int) -> int:
    """correlate.go:210-212"""
    return index - (lenB - 1)


def IndexFromLag(lag: int, lenB: int) -> int:
    """correlate.go:216-218"""
    return lag + (lenB - 1)


# ---------------------------------------------------------------------------
# dsp/conv/deconvolve.go
# ---------------------------------------------------------------------------
DeconvNaive, DeconvRegularized, DeconvWiener = 0, 1, 2  # deconvolve.go:20-35


@dataclasses.dataclass
class DeconvOptions:
    """deconvolve.go:37-54"""

    Method: int = DeconvNaive
    Epsilon: float = 0.0
    NoiseVariance: float = 0.0
    SignalVariance: float = 0.0


def DefaultDeconvOptions() -> DeconvOptions:
    """deconvolve.go:57-63"""
    d = lib().ad_deconv_default_options()
    return DeconvOptions(d.method, d.epsilon, d.noise_variance, d.signal_variance)


def Deconvolve(signal, kernel, opts: DeconvOptions) -> np.ndarray:
    """deconvolve.go:72-101 (naive / regularized / Wiener spectral division on the GPU)."""
    x, h = f64(signal), f64(kernel)
    o = DeconvOptionsC(int(opts.Method), float(opts.Epsilon), float(opts.NoiseVariance), float(opts.SignalVariance))
    cap = max(x.size, 1)
    out = np.empty(cap, dtype=np.float64)
    n = C.c_int64()
    check(lib().ad_deconvolve(ptr(x), x.size, ptr(h), h.size, C.byref(o), ptr(out), cap, C.byref(n), DEVICE))
    return out[: n.value].copy()


def InverseFilter(kernel, length: int, epsilon: float) -> np.ndarray:
    """deconvolve.go:354-394"""
    h = f64(kernel)
    out = np.empty(max(int(length), 0), dtype=np.float64)
    check(lib().ad_inverse_filter(ptr(h), h.size, int(length), float(epsilon), ptr(out), DEVICE))
    return out


def SNR(original, recovered) -> float:
    """deconvolve.go:399-421 (host metric)."""
    a, b = f64(original), f64(recovered)
    if a.size != b.size or a.size == 0:
        return -math.inf
    sp = npow = 0.0
    for x, y in zip(a.tolist(), b.tolist()):
        sp += x * x
        d = x - y
        npow += d * d
    if npow == 0:
        return math.inf
    return 10 * math.log10(sp / npow)
