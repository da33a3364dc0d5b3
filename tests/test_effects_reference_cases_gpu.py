"""The reference's Compressor, Gate and Freeverb unit tests, restated against
the HIP engine.

Each test names the test it follows (dsp/effects/dynamics/compressor_test.go,
gate_test.go, dsp/effects/reverb/reverb_test.go under github.com/cwbudde/algo-dsp) and keeps
its settings and inputs.  The reference's `calculateGain` and `peakLevel` are
internals with no ABI entry, so the gain tests observe them through the
output (auto makeup off and 0 dB makeup: output = gain x input) and through
the metrics.  A reference `ProcessSample` call is a one-sample
`ProcessInPlace` on the GPU.  Bars: Freeverb bit-exact; the compressor
within 1e-12 of the oracle (GPU log/exp2 against libm), and the engine equal
to itself bit for bit across call sizes.
"""
import math

import numpy as np
import pytest

import oracle_lib as O
from algodsp import processors as P

pytestmark = pytest.mark.gpu
FS = 48000.0


def one_sample_calls(proc, xs):
    out = []
    for x in xs:
        b = np.array([x], dtype=np.float64)
        proc.ProcessInPlace(b)
        out.append(b[0])
    return np.array(out)


def settled_gain(level, n=4000, **cfg):
    """Output / input of a constant `level` after the envelope settles, auto
    makeup off, 0 dB makeup (so the ratio is the gain computer's value)."""
    c = P.Compressor(FS, auto_makeup=0, makeup_db=0.0, **cfg)
    x = np.full(n, level)
    c.ProcessInPlace(x)
    return x[-1] / level, x


# ---------------------------------------------------------------- Compressor
def test_gain_below_threshold(gpu):
    """TestGainCalculationBelowThreshold (compressor_test.go:356-372): levels
    0.001, 0.01, 0.05 under a -20 dB threshold keep unit gain: every output
    sample equals its input."""
    for level in (0.001, 0.01, 0.05):
        g, y = settled_gain(level, n=2000, threshold_db=-20.0, knee_db=0.0)
        assert g == 1.0
        assert np.all(y == level)


def test_gain_above_threshold(gpu):
    """TestGainCalculationAboveThreshold (compressor_test.go:375-404): 0.2
    over -20 dB at 4:1, hard knee: 0 < gain < 1, and the settled gain is the
    hard-knee value 2^(-(log2 0.2 - log2 0.1) (1 - 1/4)) to 1e-9 relative
    (Python's log2 / pow against the device's)."""
    g, _ = settled_gain(0.2, threshold_db=-20.0, ratio=4.0, knee_db=0.0, attack_ms=1.0)
    assert 0.0 < g < 1.0
    # the envelope settles to the level; overshoot in log2 units (core.go:293-308)
    thr = -20.0 * math.log2(10.0) / 20.0
    want = 2.0 ** (-(math.log2(0.2) - thr) * (1.0 - 1.0 / 4.0))
    assert abs(g - want) <= 1e-9 * want


def test_gain_ratios(gpu):
    """TestGainCalculationRatios (compressor_test.go:407-453): ratios 1, 2, 4,
    10 at levels 0.2 and 0.3: ratio 1 is unit gain, higher ratios never give
    more gain."""
    for level in (0.2, 0.3):
        prev = None
        for ratio in (1.0, 2.0, 4.0, 10.0):
            g, _ = settled_gain(level, threshold_db=-20.0, ratio=ratio, knee_db=0.0, attack_ms=1.0)
            if ratio == 1.0:
                assert g == 1.0
            else:
                assert g < 1.0
            if prev is not None:
                assert g <= prev
            prev = g


def test_process_sample_zero(gpu):
    """TestProcessSampleZero (compressor_test.go:456-467)."""
    c = P.Compressor(FS)
    c.Reset()
    assert np.all(one_sample_calls(c, np.zeros(100)) == 0.0)
    z = np.zeros(1000)
    c.ProcessInPlace(z)
    assert np.all(z == 0.0)


def test_process_in_place_matches_sample(gpu):
    """TestProcessInPlaceMatchesSample (compressor_test.go:470-505): 256
    samples of 0.1 sin(2 pi 440 i / 48000); one-sample calls against one
    block call (bit for bit here), both within 1e-12 of the oracle."""
    x = 0.1 * np.sin(2 * np.pi * 440 * np.arange(256) / FS)
    want = one_sample_calls(P.Compressor(FS), x)
    got = x.copy()
    P.Compressor(FS).ProcessInPlace(got)
    assert np.array_equal(got, want)
    ref = O.Compressor(FS).process_in_place(x)
    assert float(np.max(np.abs(got - ref))) <= 1e-12


def test_reset(gpu):
    """TestReset (compressor_test.go:507-532): after 100 x 0.5 the metrics
    are non-zero; Reset clears them, and the next output is a fresh
    compressor's."""
    c = P.Compressor(FS)
    one_sample_calls(c, np.full(100, 0.5))
    ip, op, _ = c.Metrics()
    assert ip == 0.5 and op > 0
    c.Reset()
    ip, op, gr = c.Metrics()
    assert ip == 0.0 and op == 0.0 and gr == 1.0
    x = 0.3 * np.sin(np.arange(500) * 0.05)
    a = x.copy()
    c.ProcessInPlace(a)
    b = x.copy()
    P.Compressor(FS).ProcessInPlace(b)
    assert np.array_equal(a, b)


def test_metrics_tracking(gpu):
    """TestMetricsTracking (compressor_test.go:535-570): threshold -20 dB,
    1 ms attack, 500 x 0.8: InputPeak == 0.8, OutputPeak > 0,
    GainReduction < 1, and all three match the oracle's."""
    c = P.Compressor(FS, threshold_db=-20.0, attack_ms=1.0)
    one_sample_calls(c, np.full(500, 0.8))
    ip, op, gr = c.Metrics()
    assert ip == 0.8
    assert op > 0.0
    assert gr < 1.0
    o = O.Compressor(FS, threshold_db=-20.0, attack_ms=1.0)
    o.process_in_place(np.full(500, 0.8))
    np.testing.assert_allclose([ip, op, gr], o.metrics(), rtol=1e-12, atol=0)


def test_envelope_attack_and_release(gpu):
    """TestEnvelopeFollowerAttack / Release (compressor_test.go:573-660),
    observed through the gain: with a 1 ms attack a 0.5 step is compressed
    more and more (gain never rises while the envelope climbs), and after
    the step the gain recovers to 1 within the 50 ms release's decay."""
    c = P.Compressor(FS, attack_ms=1.0, release_ms=50.0, threshold_db=-20.0, knee_db=0.0, auto_makeup=0,
                     makeup_db=0.0)
    x = np.concatenate([np.full(2000, 0.5), np.full(12000, 0.01)])
    y = x.copy()
    c.ProcessInPlace(y)
    g = y / x
    assert np.all(np.diff(g[:2000]) <= 1e-15)           # attack: gain falls monotonically
    assert g[1999] < 0.6                                 # and reaches deep compression
    assert np.all(np.diff(g[2000:]) >= -1e-15)          # release: gain rises monotonically
    assert g[-1] == 1.0                                  # back under threshold


# ------------------------------------------------------------------ Freeverb
def test_reverb_process_in_place_matches_sample(gpu):
    """TestReverbProcessInPlaceMatchesSample (reverb_test.go:8-33): 128
    samples of sin(2 pi i / 23), one-sample calls against one block call and
    the oracle, bit for bit."""
    x = np.sin(2 * np.pi * np.arange(128) / 23)
    want = one_sample_calls(P.Reverb(), x)
    got = x.copy()
    P.Reverb().ProcessInPlace(got)
    assert np.array_equal(got, want)
    assert np.array_equal(got, O.Freeverb().process_in_place(x))


def test_reverb_reset_restores_state(gpu):
    """TestReverbResetRestoresState (reverb_test.go:35-58)."""
    r = P.Reverb()
    x = np.zeros(128)
    x[0] = 1.0
    out1 = one_sample_calls(r, x)
    r.Reset()
    out2 = one_sample_calls(r, x)
    assert np.array_equal(out1, out2)


def test_reverb_impulse_tail_exists(gpu):
    """TestReverbImpulseTailExists (reverb_test.go:60-84): dry 0, an impulse,
    some |y[i]| > 1e-10 for i > 0 within 4096 samples; the tail equals the
    oracle's bit for bit."""
    r = P.Reverb()
    r.SetDry(0.0)
    x = np.zeros(4096)
    x[0] = 1.0
    y = x.copy()
    r.ProcessInPlace(y)
    assert np.any(np.abs(y[1:]) > 1e-10)
    o = O.Freeverb()
    o.set(0.22, 0.0, 0.72, 0.45, 0.015)
    assert np.array_equal(y, o.process_in_place(x))


# ---------------------------------------------------------------------- Gate
def test_gate_process_sample_zero(gpu):
    """TestGateProcessSampleZero (gate_test.go:534-545)."""
    g = P.Gate(FS)
    g.Reset()
    assert np.all(one_sample_calls(g, np.zeros(100)) == 0.0)


def test_gate_process_in_place_matches_sample(gpu):
    """TestGateProcessInPlaceMatchesSample (gate_test.go:548-589): 0.5 / 0.001
    / 0.5 sections of a 440 Hz sine; one-sample calls against one block (bit
    for bit here), within 1e-12 of the oracle."""
    i = np.arange(256)
    amp = np.where((i >= 100) & (i < 200), 0.001, 0.5)
    x = amp * np.sin(2 * np.pi * 440 * i / FS)
    want = one_sample_calls(P.Gate(FS), x)
    got = x.copy()
    P.Gate(FS).ProcessInPlace(got)
    assert np.array_equal(got, want)
    ref = O.Expander(FS, gate=True).process_in_place(x)
    assert float(np.max(np.abs(got - ref))) <= 1e-12


def test_gate_reset_and_metrics(gpu):
    """TestGateReset (gate_test.go:591-620) and TestGateMetricsTracking
    (:623-654): Reset clears the metrics; with threshold -10 dB and no hold,
    500 x 0.01 report InputPeak 0.01 and GainReduction < 1."""
    g = P.Gate(FS)
    one_sample_calls(g, np.full(100, 0.5))
    assert g.Metrics()[0] == 0.5
    g.Reset()
    ip, op, _ = g.Metrics()
    assert ip == 0.0 and op == 0.0
    g = P.Gate(FS, threshold_db=-10.0, hold_ms=0.0)
    one_sample_calls(g, np.full(500, 0.01))
    ip, _, gr = g.Metrics()
    assert abs(ip - 0.01) <= 1e-10
    assert gr < 1.0


def test_gate_range_clamp(gpu):
    """TestGateRangeClamp (gate_test.go:460-490): threshold -10 dB, 100:1,
    range -40 dB, hard knee: a 0.0001 level is attenuated by no more than
    the range, and once settled by exactly the oracle's gain."""
    cfg = dict(threshold_db=-10.0, ratio=100.0, range_db=-40.0, knee_db=0.0)
    x = np.full(4000, 1e-4)
    y = x.copy()
    P.Gate(FS, **cfg).ProcessInPlace(y)
    assert np.all(y / x >= 10 ** (-40 / 20) - 1e-10)
    ref = O.Expander(FS, gate=True, **cfg).process_in_place(x)
    assert float(np.max(np.abs(y - ref))) <= 1e-12 * 1e-4


def test_gate_ratio_one_passthrough(gpu):
    """TestGateRatioOnePassthrough (gate_test.go:912-933): ratio 1, hard knee:
    unit gain at levels 0.001 ... 0.5 (every output sample equals its input)."""
    for level in (0.001, 0.01, 0.05, 0.1, 0.5):
        x = np.full(1000, level)
        y = x.copy()
        P.Gate(FS, ratio=1.0, knee_db=0.0).ProcessInPlace(y)
        assert np.array_equal(y, x)


def test_gate_negative_input(gpu):
    """TestGateNegativeInput (gate_test.go:936-945)."""
    g = P.Gate(FS)
    g.Reset()
    assert one_sample_calls(g, [-0.5])[0] <= 0.0


# ------------------------------------------------------------------ Expander
def test_expander_parameter_validation(gpu):
    """TestExpanderParameterValidation (expander_test.go:65-92): ratio 0.5,
    knee 25, attack 0.05 ms, release 0.5 ms and range -121 dB are rejected."""
    for field, value in (("ratio", 0.5), ("knee_db", 25.0), ("attack_ms", 0.05), ("release_ms", 0.5)):
        e = P.Expander(FS)
        with pytest.raises(Exception):
            e._set(**{field: value})
    e = P.Expander(FS)
    with pytest.raises(Exception):
        e.SetRange(-121.0)
    assert e.range_db == -60.0  # the rejected value left the stage as it was


def test_expander_gain_behavior(gpu):
    """TestExpanderGainBehavior (expander_test.go:94-121): threshold -20 dB,
    6:1, hard knee, range -80 dB: 1024 x 0.5 settle at >= 0.49; after Reset,
    1024 x 0.02 are attenuated below 0.02.  Both against the oracle, 1e-12."""
    cfg = dict(threshold_db=-20.0, ratio=6.0, knee_db=0.0, range_db=-80.0)
    e = P.Expander(FS, **cfg)
    hi = np.full(1024, 0.5)
    e.ProcessInPlace(hi)
    assert hi[-1] >= 0.49
    e.Reset()
    lo = np.full(1024, 0.02)
    e.ProcessInPlace(lo)
    assert lo[-1] < 0.02
    o = O.Expander(FS, **cfg)
    assert float(np.max(np.abs(hi - o.process_in_place(np.full(1024, 0.5))))) <= 1e-12
    o.reset()
    assert float(np.max(np.abs(lo - o.process_in_place(np.full(1024, 0.02))))) <= 1e-12


def test_expander_topology_changes_output(gpu):
    """TestExpanderTopologyDetectorAndSidechain (expander_test.go:123-150):
    RMS detector, 20 ms window, threshold -25 dB, 4:1; 512 x 0.05 give a
    different last output in feedback and feed-forward topology."""
    base = dict(threshold_db=-25.0, ratio=4.0, detector_mode=1, rms_window_ms=20.0)
    fb = np.full(512, 0.05)
    P.Expander(FS, topology=1, **base).ProcessInPlace(fb)
    ff = np.full(512, 0.05)
    P.Expander(FS, topology=0, **base).ProcessInPlace(ff)
    assert fb[-1] != ff[-1]
