"""algodsp — Python harness over the MI355X-native block-DSP engine.

The product is the HIP library libalgodsp_hip.so (C ABI: include/algodsp.h).
These modules mirror the reference Go packages (dsp/conv, dsp/filter/...,
dsp/effects/...) for tests and benchmarks.  There is no CPU fallback.
"""
from . import conv  # noqa: F401
from ._lib import ADError, device_count, exported_symbols, lib  # noqa: F401
