"""CPU tests of the host-side coefficient designers (SURVEY 8(a) a19,
algodsp/design.py) against the properties the reference's own tests assert
(dsp/filter/design/design_test.go:18-325), plus the config-5 EQ pinned bit for
bit by tests/golden/config5_eq_coeffs.json (tests/golden/make_config5_eq.py).

The designers' outputs are inputs to both the GPU and the oracle, so no
parity test depends on them; these tests pin the designers themselves.  The
reference's exact bits are unpinned (Go's math package is not run here), so
beyond the fixture the checks are design_test.go's tolerance properties and
the RBJ cookbook's magnitudes at the design frequency.
"""
import cmath
import json
import math
import pathlib

import numpy as np
import pytest

from algodsp import design

GOLDEN = pathlib.Path(__file__).parent / "golden" / "config5_eq_coeffs.json"
TOL = 1e-9  # design_test.go:12


def mag(sec, f, fs):  # design_test.go:288-291
    return abs(design.response(sec, f, fs))


def mag_chain(secs, f, fs):  # design_test.go:293-296
    return abs(design.chain_response(secs, f, fs))


def finite(sec):  # assertFiniteCoefficients design_test.go:298-307
    return all(math.isfinite(v) for v in sec)


def stable(sec):  # assertStableSection / sectionRoots design_test.go:309-325
    _, _, _, a1, a2 = sec
    d = cmath.sqrt(complex(a1 * a1 - 4 * a2, 0))
    r1, r2 = (-a1 + d) / 2, (-a1 - d) / 2
    return abs(r1) < 1 + TOL and abs(r2) < 1 + TOL


def test_bilinear_normalizes_a0():  # design_test.go:18-29
    got = design.bilinear_transform((1, 1, 1), 48000)
    assert abs(got[0] - 1) <= 1e-12
    assert all(math.isfinite(v) for v in got)


def test_basic_response_shape():  # design_test.go:31-62
    sr, f, q = 48000.0, 1000.0, 1 / math.sqrt(2)
    lp, hp = design.lowpass(f, q, sr), design.highpass(f, q, sr)
    assert mag(lp, 100, sr) > mag(lp, 10000, sr)
    assert mag(hp, 10000, sr) > mag(hp, 100, sr)
    bp = design.bandpass(f, q, sr)
    assert mag(bp, f, sr) > mag(bp, 100, sr) and mag(bp, f, sr) > mag(bp, 10000, sr)
    n = design.notch(f, q, sr)
    assert mag(n, f, sr) < mag(n, 100, sr) and mag(n, f, sr) < mag(n, 10000, sr)
    ap = design.allpass(f, q, sr)
    for hz in (100, 500, 1000, 5000, 10000):
        assert abs(mag(ap, hz, sr) - 1) <= 1e-6


def test_eq_basic_behavior():  # design_test.go:64-87
    sr, f, q = 48000.0, 1000.0, 1.0
    assert mag(design.peak(f, 6, q, sr), f, sr) > 1 and mag(design.peak(f, -6, q, sr), f, sr) < 1
    ls = design.low_shelf(500, 6, q, sr)
    assert mag(ls, 100, sr) > mag(ls, 10000, sr)
    hs = design.high_shelf(4000, 6, q, sr)
    assert mag(hs, 10000, sr) > mag(hs, 100, sr)


@pytest.mark.parametrize("sr", [44100.0, 48000.0, 96000.0, 192000.0])
def test_validate_across_sample_rates(sr):  # design_test.go:89-106
    for c in (design.lowpass(1000, 0.707, sr), design.highpass(1000, 0.707, sr), design.bandpass(1000, 1.2, sr),
              design.notch(1000, 1.2, sr), design.allpass(1000, 1.2, sr), design.peak(1000, 3, 1.0, sr),
              design.low_shelf(300, 6, 1.0, sr), design.high_shelf(3000, -6, 1.0, sr)):
        assert finite(c) and stable(c), c


@pytest.mark.parametrize("kind", ["lp", "hp"])
def test_butterworth_order_and_shape(kind):  # design_test.go:108-146
    sr = 48000.0
    secs = design.butterworth_lp(1000, 5, sr) if kind == "lp" else design.butterworth_hp(1000, 5, sr)
    assert len(secs) == 3
    assert secs[-1][4] == 0 and secs[-1][2] == 0  # final first-order section (A2 = B2 = 0)
    assert all(stable(c) for c in secs)
    lo, hi = mag_chain(secs, 100, sr), mag_chain(secs, 10000, sr)
    assert (lo > hi) if kind == "lp" else (hi > lo)


def test_invalid_inputs():  # design_test.go:231-268
    zero = (0.0, 0.0, 0.0, 0.0, 0.0)
    assert design.lowpass(1000, 0.707, 0) == zero
    assert design.highpass(0, 0.707, 48000) == zero
    for c in (design.bandpass(1000, 0, 48000), design.notch(1000, -1, 48000), design.allpass(1000, 0, 48000),
              design.peak(1000, 3, 0, 48000), design.low_shelf(1000, 3, 0, 48000),
              design.high_shelf(1000, 3, 0, 48000)):
        assert finite(c) and stable(c)  # q <= 0 takes defaultQ
    assert design.bilinear_transform((1, 1, 1), 0) == (1.0, 0.0, 0.0)
    assert design.bilinear_transform((0, 0, 0), 48000) == (1.0, 0.0, 0.0)
    assert design.butterworth_lp(1000, 0, 48000) is None
    assert design.butterworth_hp(1000, 0, 48000) is None


def test_mag_helper_non_default_sample_rate():  # design_test.go:270-277
    assert math.isfinite(mag(design.lowpass(1000, 0.707, 44100), 1000, 44100))


# ---------------------------------------------------------------- config 5
@pytest.mark.parametrize("fs", ["44100", "48000", "96000", "192000"])
def test_config5_eq_matches_fixture(fs):
    """The config-5 EQ coefficients, bit for bit, at four sample rates."""
    want = json.loads(GOLDEN.read_text())[fs]
    got = [list(co[0]) for co, g in design.config5_eq(float(fs))]
    assert [[float.fromhex(v) for v in sec] for sec in want] == got
    assert all(g == 1.0 for _, g in design.config5_eq(float(fs)))


@pytest.mark.parametrize("fs", [44100.0, 48000.0, 96000.0, 192000.0])
def test_config5_eq_design_frequency_magnitudes(fs):
    """RBJ cookbook magnitudes at each section's design frequency: |H| = Q for
    the 2nd-order highpass / lowpass, 10^(G/40) (half the dB gain) for the
    shelves, 10^(G/20) for the peak; plus a0 = 1 (the normalised form has no
    a0: the section's DC / Nyquist gains agree with their closed forms), every
    section finite and stable."""
    (hp,), (ls,), (pk,), (hs,), (lp,) = [co for co, _ in design.config5_eq(fs)]
    close = lambda a, b: abs(a - b) <= 1e-9 * max(1.0, abs(b))  # noqa: E731
    assert close(mag(hp, 40.0, fs), 0.707)
    assert close(mag(ls, 100.0, fs), 10 ** (3.0 / 40))
    assert close(mag(pk, 1000.0, fs), 10 ** (-2.0 / 20))
    assert close(mag(hs, 8000.0, fs), 10 ** (2.0 / 40))
    assert close(mag(lp, 18000.0, fs), 0.707)
    # DC and Nyquist from the coefficient sums (shelves: 10^(G/20) at their end)
    dc = lambda s: (s[0] + s[1] + s[2]) / (1 + s[3] + s[4])  # noqa: E731
    ny = lambda s: (s[0] - s[1] + s[2]) / (1 - s[3] + s[4])  # noqa: E731
    assert abs(dc(hp)) <= 1e-12 and close(ny(lp) + 1.0, 1.0)
    assert close(dc(ls), 10 ** (3.0 / 20)) and close(ny(hs), 10 ** (2.0 / 20))
    for s in (hp, ls, pk, hs, lp):
        assert finite(s) and stable(s)
    assert np.isfinite([mag_chain([hp, ls, pk, hs, lp], f, fs) for f in (10, 100, 1000, 10000, 20000)]).all()
