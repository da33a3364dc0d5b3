"""Host-side biquad coefficient designers (RBJ cookbook), restating
dsp/filter/design/design.go:37-223 and design/pass/butterworth.go:56-125.

Coefficients are computed once on the host (Python float64 = IEEE double;
trig/pow from libm, which may differ from Go's math package by 1 ulp) and
handed to both the GPU and the oracle, so parity tests never depend on the
designers.  Each returns (b0, b1, b2, a1, a2) normalised by a0; an invalid
frequency returns the zero section like the reference.
"""
from __future__ import annotations

import math

_DEFAULT_Q = 1 / math.sqrt(2)
_ZERO = (0.0, 0.0, 0.0, 0.0, 0.0)


def _w0(freq, fs):  # normalizedW0 design.go:192-204
    if fs <= 0 or math.isnan(fs) or math.isinf(fs):
        return None
    if freq <= 0 or freq >= fs / 2 or math.isnan(freq) or math.isinf(freq):
        return None
    return 2 * math.pi * freq / fs


def _q(q):  # normalizedQ design.go:206-212
    return _DEFAULT_Q if (q <= 0 or math.isnan(q) or math.isinf(q)) else q


def _norm(b0, b1, b2, a0, a1, a2):  # normalizeBiquad design.go:214-223
    if a0 == 0 or math.isnan(a0) or math.isinf(a0):
        return _ZERO
    return (b0 / a0, b1 / a0, b2 / a0, a1 / a0, a2 / a0)


def lowpass(freq, q, fs):  # pass.LowpassRBJ butterworth.go:56-88
    if fs <= 0 or freq <= 0 or freq >= fs / 2:
        return _ZERO
    if q <= 0:
        q = 1 / math.sqrt(2)
    w0 = 2 * math.pi * freq / fs
    cw, sw = math.cos(w0), math.sin(w0)
    alpha = sw / (2 * q)
    return _norm((1 - cw) / 2, 1 - cw, (1 - cw) / 2, 1 + alpha, -2 * cw, 1 - alpha)


def highpass(freq, q, fs):  # pass.HighpassRBJ butterworth.go:91-123
    if fs <= 0 or freq <= 0 or freq >= fs / 2:
        return _ZERO
    if q <= 0:
        q = 1 / math.sqrt(2)
    w0 = 2 * math.pi * freq / fs
    cw, sw = math.cos(w0), math.sin(w0)
    alpha = sw / (2 * q)
    return _norm((1 + cw) / 2, -(1 + cw), (1 + cw) / 2, 1 + alpha, -2 * cw, 1 - alpha)


def peak(freq, gain_db, q, fs):  # peakRBJ design.go:114-137
    w0 = _w0(freq, fs)
    if w0 is None:
        return _ZERO
    q = _q(q)
    cw, sw = math.cos(w0), math.sin(w0)
    alpha = sw / (2 * q)
    a = math.pow(10, gain_db / 40)
    return _norm(1 + alpha * a, -2 * cw, 1 - alpha * a, 1 + alpha / a, -2 * cw, 1 - alpha / a)


def low_shelf(freq, gain_db, q, fs):  # design.go:139-161
    w0 = _w0(freq, fs)
    if w0 is None:
        return _ZERO
    q = _q(q)
    cw, sw = math.cos(w0), math.sin(w0)
    alpha = sw / (2 * q)
    a = math.pow(10, gain_db / 40)
    beta = 2 * math.sqrt(a) * alpha
    return _norm(a * ((a + 1) - (a - 1) * cw + beta), 2 * a * ((a - 1) - (a + 1) * cw),
                 a * ((a + 1) - (a - 1) * cw - beta), (a + 1) + (a - 1) * cw + beta,
                 -2 * ((a - 1) + (a + 1) * cw), (a + 1) + (a - 1) * cw - beta)


def high_shelf(freq, gain_db, q, fs):  # design.go:163-185
    w0 = _w0(freq, fs)
    if w0 is None:
        return _ZERO
    q = _q(q)
    cw, sw = math.cos(w0), math.sin(w0)
    alpha = sw / (2 * q)
    a = math.pow(10, gain_db / 40)
    beta = 2 * math.sqrt(a) * alpha
    return _norm(a * ((a + 1) + (a - 1) * cw + beta), -2 * a * ((a - 1) + (a + 1) * cw),
                 a * ((a + 1) + (a - 1) * cw - beta), (a + 1) - (a - 1) * cw + beta,
                 2 * ((a - 1) - (a + 1) * cw), (a + 1) - (a - 1) * cw - beta)


def config5_eq(fs: float = 48000.0):
    """The BASELINE config-5 EQ: HP 40 Hz Q .707, LowShelf 100 Hz
    +3 dB, Peak 1 kHz -2 dB Q 1, HighShelf 8 kHz +2 dB, LP 18 kHz Q .707; one
    filter node (a one-section biquad.Chain, gain 1) each."""
    return [
        ([highpass(40.0, 0.707, fs)], 1.0),
        ([low_shelf(100.0, 3.0, 0.707, fs)], 1.0),
        ([peak(1000.0, -2.0, 1.0, fs)], 1.0),
        ([high_shelf(8000.0, 2.0, 0.707, fs)], 1.0),
        ([lowpass(18000.0, 0.707, fs)], 1.0),
    ]
