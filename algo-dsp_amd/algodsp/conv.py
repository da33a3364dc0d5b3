"""dsp/conv mirror over the HIP C ABI.

Names, argument meaning and error behaviour follow the reference package
github.com/cwbudde/algo-dsp/dsp/conv (file:line cited per entry point), so
tests read like the reference's own.  Every call runs on the GPU through
libalgodsp_hip.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import (ADError, ErrEmptyImpulseResponse, ErrEmptyInput, ErrEmptyKernel, ErrInvalidArgument,
                   ErrInvalidBlockOrder, ErrInvalidBlockSize, ErrLengthMismatch, ErrStageIndexOutOfRange, check,
                   f64, lib, ptr)

__all__ = [
    "ADError", "ErrEmptyInput", "ErrEmptyKernel", "ErrLengthMismatch", "ErrInvalidBlockSize",
    "ErrInvalidBlockOrder", "ErrEmptyImpulseResponse", "ErrStageIndexOutOfRange", "ErrInvalidArgument",
    "ModeFull", "ModeSame", "ModeValid",
    "Direct", "DirectCircular", "Convolve", "ConvolveMode",
    "NewStreamingOverlapSave", "NewStreamingOverlapAdd", "NewOverlapSave", "NewOverlapAdd",
    "NewPartitionedConvolution", "OverlapAddConvolve", "OverlapSaveConvolve", "MultiChannelConvolver",
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


def Direct(a, b) -> np.ndarray:
    """conv.go:76-93"""
    x, y = f64(a), f64(b)
    out = np.empty(max(x.size + y.size - 1, 0), dtype=np.float64)
    check(lib().ad_conv_direct(ptr(x), x.size, ptr(y), y.size, ptr(out), DEVICE))
    return out


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

    def profile_enable(self, on: bool = True) -> None:
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


def mixdown_device(d_chan: int, channels: int, stride: int, length: int, d_mix: int, stream: int = 0) -> None:
    check(lib().ad_conv_mixdown_device(C.c_void_p(d_chan), channels, stride, length, C.c_void_p(d_mix),
                                       C.c_void_p(stream)))
