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


def bilinear_transform(s_coeffs, fs):  # BilinearTransform design.go:17-35
    """c0 s^2 + c1 s + c2 -> (1, d1/d0, d2/d0); (1, 0, 0) for fs <= 0 or a
    degenerate d0."""
    if fs <= 0:
        return (1.0, 0.0, 0.0)
    k = 2 * fs
    c0, c1, c2 = s_coeffs
    d0 = c0 * k * k + c1 * k + c2
    d1 = -2 * c0 * k * k + 2 * c2
    d2 = c0 * k * k - c1 * k + c2
    if d0 == 0 or math.isnan(d0) or math.isinf(d0):
        return (1.0, 0.0, 0.0)
    return (1.0, d1 / d0, d2 / d0)


def bandpass(freq, q, fs):  # Bandpass design.go:47-69 (constant skirt gain)
    w0 = _w0(freq, fs)
    if w0 is None:
        return _ZERO
    q = _q(q)
    cw, sw = math.cos(w0), math.sin(w0)
    alpha = sw / (2 * q)
    return _norm(sw / 2, 0.0, -sw / 2, 1 + alpha, -2 * cw, 1 - alpha)


def notch(freq, q, fs):  # Notch design.go:71-92
    w0 = _w0(freq, fs)
    if w0 is None:
        return _ZERO
    q = _q(q)
    cw, sw = math.cos(w0), math.sin(w0)
    alpha = sw / (2 * q)
    return _norm(1.0, -2 * cw, 1.0, 1 + alpha, -2 * cw, 1 - alpha)


def allpass(freq, q, fs):  # Allpass design.go:94-115
    w0 = _w0(freq, fs)
    if w0 is None:
        return _ZERO
    q = _q(q)
    cw, sw = math.cos(w0), math.sin(w0)
    alpha = sw / (2 * q)
    return _norm(1 - alpha, -2 * cw, 1 + alpha, 1 + alpha, -2 * cw, 1 - alpha)


def response(sec, freq, fs):  # Coefficients.Response biquad/response.go:10-19
    """H(e^{jw}) of one section (b0, b1, b2, a1, a2)."""
    import cmath

    b0, b1, b2, a1, a2 = sec
    w = 2 * math.pi * freq / fs
    ejw, ej2w = cmath.exp(complex(0, -w)), cmath.exp(complex(0, -2 * w))
    return (b0 + b1 * ejw + b2 * ej2w) / (1 + a1 * ejw + a2 * ej2w)


def chain_response(secs, freq, fs, gain=1.0):  # Chain.Response biquad/response.go:52-59
    h = complex(gain, 0)
    for sec in secs:
        h *= response(sec, freq, fs)
    return h


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


# ---- Butterworth / Linkwitz-Riley cascades (crossover nodes) --------------
def butterworth_q(order, index):  # butterworthQ pass/common.go:20-30
    theta = math.pi * float(2 * index + 1) / (2 * float(order))
    s = math.sin(theta)
    if s == 0:
        return 1 / math.sqrt(2)
    return 1 / (2 * s)


def _bw_first_order(freq, fs, high):  # butterworthFirstOrderLP/HP pass/common.go:34-70
    if fs <= 0 or freq <= 0 or freq >= fs / 2:
        return _ZERO
    k = math.tan(math.pi * freq / fs)
    norm = 1 / (1 + k)
    return (norm, -norm, 0.0, (k - 1) * norm, 0.0) if high else (k * norm, k * norm, 0.0, (k - 1) * norm, 0.0)


def butterworth_lp(freq, order, fs):  # ButterworthLP pass/butterworth.go:12-30
    if order <= 0:
        return None
    secs = [lowpass(freq, butterworth_q(order, i), fs) for i in range(order // 2 - 1, -1, -1)]
    if order % 2:
        secs.append(_bw_first_order(freq, fs, False))
    return secs


def butterworth_hp(freq, order, fs):  # ButterworthHP pass/butterworth.go:35-53
    if order <= 0:
        return None
    secs = [highpass(freq, butterworth_q(order, i), fs) for i in range(order // 2 - 1, -1, -1)]
    if order % 2:
        secs.append(_bw_first_order(freq, fs, True))
    return secs


def _lr_orders(order):  # linkwitzRileyPrototypeOrders pass/linkwitz_riley.go:116-122
    return (order // 2, (order + 1) // 2) if order >= 2 else None


def linkwitz_riley_lp(freq, order, fs):  # LinkwitzRileyLP pass/linkwitz_riley.go:23-45
    o = _lr_orders(order)
    if o is None or fs <= 0 or freq <= 0 or freq >= fs / 2:
        return None
    return butterworth_lp(freq, o[0], fs) + butterworth_lp(freq, o[1], fs)


def linkwitz_riley_hp(freq, order, fs, inverted=False):  # pass/linkwitz_riley.go:61-105
    o = _lr_orders(order)
    if o is None or fs <= 0 or freq <= 0 or freq >= fs / 2:
        return None
    secs = butterworth_hp(freq, o[0], fs) + butterworth_hp(freq, o[1], fs)
    if inverted:  # negate the first section's B coefficients
        b0, b1, b2, a1, a2 = secs[0]
        secs[0] = (-b0, -b1, -b2, a1, a2)
    return secs


def crossover(freq, order, fs):
    """crossover.New (filter/crossover/crossover.go:31-65): (LP sections, HP
    sections) of a two-way Linkwitz-Riley network, HP polarity-inverted for
    orders = 2 mod 4; None where New returns an error."""
    if order <= 0 or order % 2 or fs <= 0 or freq <= 0 or freq >= fs / 2:
        return None
    lp = linkwitz_riley_lp(freq, order, fs)
    hp = linkwitz_riley_hp(freq, order, fs, inverted=(order % 4 == 2))
    if lp is None or hp is None:
        return None
    return lp, hp


class RBJDesigner:
    """A FilterDesigner (effectchain/runtime_filter_pitch_reverb.go:18-24) for
    the batched graph runtime: family "rbj" (one cookbook section) and
    "butterworth" (lowpass/highpass cascades of the given order).  The
    reference injects the webdemo's designer here; any designer works, since
    the coefficients it returns are inputs to both the GPU and the oracle."""

    KINDS = ("lowpass", "highpass", "peak", "lowshelf", "highshelf")

    def NormalizeFamily(self, family):
        return family if family in ("rbj", "butterworth") else "rbj"

    def NormalizeFamilyForType(self, kind, family):
        return family if kind in ("lowpass", "highpass") else "rbj"

    def NormalizeOrder(self, kind, family, order):
        return max(1, min(int(order), 8)) if family == "butterworth" else 2

    def ClampShape(self, kind, family, freq, fs, q):
        return q

    def BuildChain(self, family, kind, order, freq, gain_db, q, fs):
        """-> (sections [(b0, b1, b2, a1, a2)], chain gain)"""
        if family == "butterworth":
            secs = butterworth_lp(freq, order, fs) if kind == "lowpass" else butterworth_hp(freq, order, fs)
            return secs, 1.0
        if kind == "lowpass":
            return [lowpass(freq, q, fs)], 1.0
        if kind == "highpass":
            return [highpass(freq, q, fs)], 1.0
        if kind == "peak":
            return [peak(freq, gain_db, q, fs)], 1.0
        if kind == "lowshelf":
            return [low_shelf(freq, gain_db, q, fs)], 1.0
        if kind == "highshelf":
            return [high_shelf(freq, gain_db, q, fs)], 1.0
        raise NotImplementedError(f"RBJDesigner: filter kind {kind!r}")
