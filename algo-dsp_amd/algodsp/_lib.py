"""ctypes loader for libalgodsp_hip.so (the C ABI declared in include/algodsp.h).

The product path is the HIP library only: if it cannot be loaded, or no
gfx950 device is visible, every create call raises -- there is no CPU
fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = _HERE.parent / "libalgodsp_hip.so"
HEADER_PATH = _HERE.parent.parent / "include" / "algodsp.h"

# status codes (include/algodsp.h)
AD_OK = 0
AD_ERR_EMPTY_INPUT = 1
AD_ERR_EMPTY_KERNEL = 2
AD_ERR_LENGTH_MISMATCH = 3
AD_ERR_INVALID_BLOCK_SIZE = 4
AD_ERR_INVALID_BLOCK_ORDER = 5
AD_ERR_EMPTY_IMPULSE_RESPONSE = 6
AD_ERR_STAGE_INDEX_OUT_OF_RANGE = 7
AD_ERR_INVALID_ARGUMENT = 8
AD_ERR_DIVISION_BY_ZERO = 9
AD_ERR_DEVICE = 100
AD_ERR_NO_DEVICE = 101
AD_ERR_INTERNAL = 102


class ADError(Exception):
    """Error returned through the C ABI; `code` is the AD_* status."""

    code = None

    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class ErrEmptyInput(ADError):
    pass


class ErrEmptyKernel(ADError):
    pass


class ErrLengthMismatch(ADError):
    pass


class ErrInvalidBlockSize(ADError):
    pass


class ErrInvalidBlockOrder(ADError):
    pass


class ErrEmptyImpulseResponse(ADError):
    pass


class ErrStageIndexOutOfRange(ADError):
    pass


class ErrInvalidArgument(ADError):
    pass


class ErrDivisionByZero(ADError):
    pass


class ErrDevice(ADError):
    pass


_BY_CODE = {
    AD_ERR_EMPTY_INPUT: ErrEmptyInput,
    AD_ERR_EMPTY_KERNEL: ErrEmptyKernel,
    AD_ERR_LENGTH_MISMATCH: ErrLengthMismatch,
    AD_ERR_INVALID_BLOCK_SIZE: ErrInvalidBlockSize,
    AD_ERR_INVALID_BLOCK_ORDER: ErrInvalidBlockOrder,
    AD_ERR_EMPTY_IMPULSE_RESPONSE: ErrEmptyImpulseResponse,
    AD_ERR_STAGE_INDEX_OUT_OF_RANGE: ErrStageIndexOutOfRange,
    AD_ERR_INVALID_ARGUMENT: ErrInvalidArgument,
    AD_ERR_DIVISION_BY_ZERO: ErrDivisionByZero,
}

class CompressorConfig(C.Structure):
    """ad_compressor_config (include/algodsp.h)."""

    _fields_ = [(n, C.c_double) for n in ("sample_rate", "threshold_db", "ratio", "knee_db", "attack_ms",
                                          "release_ms", "rms_window_ms", "makeup_db", "sidechain_low_cut_hz",
                                          "sidechain_high_cut_hz")] + \
               [(n, C.c_int) for n in ("topology", "detector_mode", "feedback_ratio_scale", "auto_makeup")]


class DeconvOptionsC(C.Structure):
    """ad_deconv_options (include/algodsp.h)."""

    _fields_ = [("method", C.c_int), ("epsilon", C.c_double), ("noise_variance", C.c_double),
                ("signal_variance", C.c_double)]


_lib = None

c_double_p = C.POINTER(C.c_double)
c_float_p = C.POINTER(C.c_float)
c_int64_p = C.POINTER(C.c_int64)


def lib() -> C.CDLL:
    """Loads (once) and returns the HIP library; raises if it is missing."""
    global _lib
    if _lib is None:
        # PyTorch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7) and
        # refers to it by the unversioned name, so if our library pulled in
        # /opt/rocm's copy first the process would end up with two HIP/HSA
        # runtimes and torch would see no GPU.  Importing torch first makes the
        # dynamic linker bind our NEEDED libamdhip64.so.7 to torch's runtime:
        # one runtime, shared device pointers and streams.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        path = os.environ.get("ALGODSP_LIB", str(LIB_PATH))
        if not pathlib.Path(path).exists():
            raise ImportError(f"libalgodsp_hip.so not built at {path}; run `make -C algo-dsp_amd`")
        _lib = C.CDLL(path)
        _declare(_lib)
    return _lib


def _declare(L: C.CDLL) -> None:
    vp = C.c_void_p
    i64 = C.c_int64
    sig = {
        "ad_last_error": (C.c_char_p, []),
        "ad_version": (C.c_int, []),
        "ad_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "ad_conv_stream_ols_create": (C.c_int, [c_double_p, i64, i64, C.c_int, C.POINTER(vp)]),
        "ad_conv_stream_ola_create": (C.c_int, [c_double_p, i64, i64, C.c_int, C.POINTER(vp)]),
        "ad_conv_process_block": (C.c_int, [vp, c_double_p, i64, c_double_p, i64]),
        "ad_conv_stream_ols32_create": (C.c_int, [c_float_p, i64, i64, C.c_int, C.POINTER(vp)]),
        "ad_conv_stream_ola32_create": (C.c_int, [c_float_p, i64, i64, C.c_int, C.POINTER(vp)]),
        "ad_conv_process_block32": (C.c_int, [vp, c_float_p, i64, c_float_p, i64]),
        "ad_conv_partitioned32_create": (C.c_int, [c_float_p, i64, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
        "ad_conv_partitioned_process_block32": (C.c_int, [vp, c_float_p, i64, c_float_p, i64]),
        "ad_conv_ols_create": (C.c_int, [c_double_p, i64, i64, C.c_int, C.POINTER(vp)]),
        "ad_conv_ola_create": (C.c_int, [c_double_p, i64, i64, C.c_int, C.POINTER(vp)]),
        "ad_conv_process": (C.c_int, [vp, c_double_p, i64, c_double_p, i64]),
        "ad_conv_partitioned_create": (C.c_int, [c_double_p, i64, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
        "ad_conv_partitioned_process_block": (C.c_int, [vp, c_double_p, i64, c_double_p, i64]),
        "ad_conv_stage_count": (C.c_int, [vp]),
        "ad_conv_stage_info": (C.c_int, [vp, C.c_int, c_int64_p, c_int64_p]),
        "ad_conv_reset": (C.c_int, [vp]),
        "ad_conv_block_size": (i64, [vp]),
        "ad_conv_kernel_len": (i64, [vp]),
        "ad_conv_fft_size": (i64, [vp]),
        "ad_conv_step_size": (i64, [vp]),
        "ad_conv_latency": (i64, [vp]),
        "ad_conv_set_host_io": (C.c_int, [vp, C.c_int, C.c_int]),
        "ad_conv_host_io_profile": (C.c_int, [vp, c_double_p, c_double_p, c_double_p]),
        "ad_conv_destroy": (None, [vp]),
        "ad_conv_direct": (C.c_int, [c_double_p, i64, c_double_p, i64, c_double_p, C.c_int]),
        "ad_conv_direct_circular": (C.c_int, [c_double_p, i64, c_double_p, i64, c_double_p, C.c_int]),
        "ad_conv_direct_device": (C.c_int, [C.c_void_p, i64, C.c_void_p, i64, C.c_void_p, C.c_void_p]),
        "ad_conv_convolve": (C.c_int, [c_double_p, i64, c_double_p, i64, C.c_int, c_double_p, i64, c_int64_p,
                                       C.c_int]),
        "ad_conv_multi_create": (C.c_int, [c_double_p, C.c_int, i64, i64, C.c_int, C.POINTER(C.c_int32), i64,
                                           C.c_int, C.POINTER(vp)]),
        "ad_conv_multi_set_schedule": (C.c_int, [vp, C.c_int, i64, i64]),
        "ad_conv_lowlat_stats": (C.c_int, [vp, c_int64_p, c_int64_p]),
        "ad_conv_multi_get_schedule": (C.c_int, [vp, C.POINTER(C.c_int), c_int64_p]),
        "ad_conv_multi_process_device": (C.c_int, [vp, vp, i64, i64, vp, i64, i64, vp]),
        "ad_conv_multi_process_device_segment": (C.c_int, [vp, vp, i64, i64, vp, i64, i64, i64, i64, vp]),
        "ad_conv_multi_process_device_mix": (C.c_int, [vp, vp, i64, i64, vp, i64, i64, C.c_int, i64, i64, vp]),
        "ad_conv_mixdown_device": (C.c_int, [vp, C.c_int, i64, i64, vp, i64, C.c_int, vp]),
        "ad_comm_get_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
        "ad_comm_create": (C.c_int, [C.POINTER(C.c_uint8), C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
        "ad_comm_destroy": (None, [vp]),
        "ad_comm_rank": (C.c_int, [vp]),
        "ad_comm_size": (C.c_int, [vp]),
        "ad_mixdown_reduce": (C.c_int, [vp, vp, C.c_int, i64, i64, C.c_int, vp, i64, C.c_int, vp]),
        "ad_conv_ols_process_multi": (C.c_int, [vp, C.POINTER(c_double_p), C.POINTER(c_double_p), C.c_int, i64]),
        "ad_conv_multi_stream_create": (C.c_int, [c_double_p, C.c_int, i64, i64, C.c_int, C.POINTER(C.c_int32),
                                                  C.c_int, C.POINTER(vp)]),
        "ad_conv_multi_stream_process_block": (C.c_int, [vp, C.POINTER(c_double_p), C.POINTER(c_double_p), C.c_int,
                                                         i64]),
        "ad_conv_multi_stream_process_block_device": (C.c_int, [vp, vp, i64, vp, i64, vp]),
        "ad_conv_pc_multi_create": (C.c_int, [c_double_p, i64, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
        "ad_conv_pc_multi_process_device": (C.c_int, [vp, vp, i64, vp, i64, i64, vp]),
        "ad_conv_reverb_multi_create": (C.c_int, [c_double_p, i64, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
        "ad_conv_reverb_multi_process_device": (C.c_int, [vp, vp, i64, i64, vp]),
        "ad_conv_reverb_multi_process": (C.c_int, [vp, c_double_p, i64]),
        "ad_conv_profile_enable": (C.c_int, [vp, C.c_int]),
        "ad_conv_profile_kernels": (C.c_int, [vp, C.c_int]),
        "ad_conv_profile_read": (C.c_int, [vp, c_double_p, c_int64_p, c_double_p]),
        "ad_compressor_default_config": (None, [C.POINTER(CompressorConfig), C.c_double]),
        "ad_compressor_validate": (C.c_int, [C.POINTER(CompressorConfig)]),
        "ad_fx_chain_create": (C.c_int, [C.c_int, C.c_int, C.POINTER(vp)]),
        "ad_fx_chain_set_eq": (C.c_int, [vp, c_double_p, C.c_int, C.c_int]),
        "ad_fx_eq_noise": (C.c_int, [c_double_p, C.c_int, C.c_int, c_double_p]),
        "ad_fx_chain_set_compressor": (C.c_int, [vp, C.POINTER(CompressorConfig)]),
        "ad_fx_chain_set_expander": (C.c_int, [vp, C.POINTER(CompressorConfig), C.c_int, C.c_double, C.c_double]),
        "ad_fx_chain_set_freeverb": (C.c_int, [vp, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double]),
        "ad_fx_chain_disable_freeverb": (C.c_int, [vp]),
        "ad_fx_chain_reset": (C.c_int, [vp]),
        "ad_fx_chain_process": (C.c_int, [vp, c_double_p, i64]),
        "ad_fx_chain_process_device": (C.c_int, [vp, vp, i64, i64, vp]),
        "ad_fx_chain_compressor_metrics": (C.c_int, [vp, C.c_int, c_double_p, c_double_p, c_double_p]),
        "ad_fx_chain_eq_state": (C.c_int, [vp, c_double_p, i64]),
        "ad_fx_chain_set_eq_state": (C.c_int, [vp, c_double_p, i64]),
        "ad_fx_chain_set_engine": (C.c_int, [vp, C.c_int, i64]),
        "ad_fx_chain_last_engine": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_double)]),
        "ad_fx_chain_set_profiling": (C.c_int, [vp, C.c_int]),
        "ad_fx_chain_read_profile": (C.c_int, [vp, C.POINTER(C.c_ulonglong), C.c_int, C.POINTER(C.c_int)]),
        "ad_fx_chain_destroy": (None, [vp]),
        "ad_fx_graph_create": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]),
        "ad_fx_graph_process": (C.c_int, [vp, c_double_p, i64]),
        "ad_fx_graph_process_device": (C.c_int, [vp, vp, i64, i64, vp]),
        "ad_fx_graph_reset": (C.c_int, [vp]),
        "ad_fx_graph_op_count": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "ad_fx_graph_destroy": (None, [vp]),
        "ad_biquad_chain_process": (C.c_int, [c_double_p, c_double_p, C.c_double, c_double_p, C.c_int, C.c_int, i64,
                                              C.c_int]),
        "ad_conv_reverb_create": (C.c_int, [c_double_p, i64, C.c_int, C.c_int, C.POINTER(vp)]),
        "ad_conv_reverb_set_wet_dry": (C.c_int, [vp, C.c_double, C.c_double]),
        "ad_conv_reverb_process_inplace": (C.c_int, [vp, c_double_p, i64]),
        "ad_decode_f16": (C.c_int, [C.POINTER(C.c_uint16), i64, C.c_int, c_double_p, C.c_int]),
        "ad_decode_f16_device": (C.c_int, [vp, i64, C.c_int, vp, vp]),
        "ad_fir_create": (C.c_int, [c_double_p, i64, C.c_int, C.c_int, C.POINTER(vp)]),
        "ad_fir_process_block": (C.c_int, [vp, c_double_p, i64]),
        "ad_fir_process_block_to": (C.c_int, [vp, c_double_p, c_double_p, i64]),
        "ad_fir_process_device": (C.c_int, [vp, vp, i64, vp, i64, i64, vp]),
        "ad_fir_reset": (C.c_int, [vp]),
        "ad_fir_destroy": (None, [vp]),
        "ad_correlate_fft": (C.c_int, [c_double_p, i64, c_double_p, i64, c_double_p, C.c_int]),
        "ad_correlate_fft_device": (C.c_int, [vp, i64, vp, i64, vp, C.c_int, vp]),
        "ad_deconv_default_options": (DeconvOptionsC, []),
        "ad_deconvolve": (C.c_int, [c_double_p, i64, c_double_p, i64, C.POINTER(DeconvOptionsC), c_double_p, i64,
                                    c_int64_p, C.c_int]),
        "ad_inverse_filter": (C.c_int, [c_double_p, i64, i64, C.c_double, c_double_p, C.c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args


def check(rc: int) -> None:
    if rc == AD_OK:
        return
    msg = lib().ad_last_error().decode("utf-8", "replace")
    raise _BY_CODE.get(rc, ErrDevice if rc >= 100 else ADError)(rc, msg)


def f64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def ptr(a: np.ndarray):
    if a.size == 0:
        return C.cast(C.c_void_p(0), c_double_p)
    return a.ctypes.data_as(c_double_p)


def device_count() -> int:
    n = C.c_int(0)
    lib().ad_device_count(C.byref(n))
    return n.value


def exported_symbols() -> list[str]:
    """Every ad_* symbol declared in include/algodsp.h."""
    import re

    text = HEADER_PATH.read_text()
    return sorted(set(re.findall(r"\b(ad_[a-z0-9_]+)\s*\(", text)))
