"""The reference's biquad Chain unit tests, restated against the HIP engine.

Each test names the test it follows (dsp/filter/biquad/chain_test.go under
github.com/cwbudde/algo-dsp) and keeps its coefficients and inputs.  The
reference checks its chain against standalone Sections with `almostEqual`;
here the standalone sections are the oracle's DF-II-T restatement
(oracle/or_filters.c, section.go:47-53) and the bar is bit equality, the
engine's parity gate for biquads.  A reference `ProcessSample` call is a
one-sample `ProcessBlock` on the GPU (the state carries between calls).
"""
import numpy as np
import pytest

import oracle_lib as O
from algodsp import processors as P

pytestmark = pytest.mark.gpu

TWO = [[0.25, 0.5, 0.25, -0.2, 0.04], [0.1, 0.2, 0.1, -0.5, 0.1]]  # twoSectionCoeffs, chain_test.go:10-15
NEW = [[0.3, 0.4, 0.3, -0.3, 0.05], [0.2, 0.1, 0.2, -0.4, 0.08]]  # chain_test.go:273-276


def sample_by_sample(chain, xs):
    out = []
    for x in xs:
        b = np.array([x], dtype=np.float64)
        chain.ProcessBlock(b)
        out.append(b[0])
    return np.array(out)


def cascade(coeffs, xs, gain=1.0):
    """Standalone oracle sections in cascade, sample by sample (the
    reference's `section2.ProcessSample(section1.ProcessSample(x * gain))`)."""
    states = [np.zeros(2) for _ in coeffs]
    out = []
    for x in xs:
        v = x * gain
        for k, c in enumerate(coeffs):
            v, states[k] = O.biquad_sample(c, states[k], v)
        out.append(v)
    return np.array(out)


def test_new_chain(gpu):
    """TestNewChain / TestNewChain_WithGain (chain_test.go:17-41)."""
    c = P.Chain(TWO)
    assert c.NumSections() == 2 and 2 * c.NumSections() == 4  # Order()
    assert c.Gain() == 1.0
    assert P.Chain(TWO, gain=0.5).Gain() == 0.5


@pytest.mark.parametrize("gain, xs", [
    (1.0, [1, 0.5, -0.3, 0.7, 0, -1, 0.2, 0.8]),  # TestChain_ProcessSample_MatchesManualCascade :43-61
    (2.0, [1, 0.5, -0.3, 0.7]),                    # TestChain_ProcessSample_WithGain :63-82
])
def test_chain_sample_matches_manual_cascade(gpu, gain, xs):
    got = sample_by_sample(P.Chain(TWO, gain=gain), xs)
    assert np.array_equal(got, cascade(TWO, xs, gain))


@pytest.mark.parametrize("gain, xs", [
    (1.0, [1, 0.5, -0.3, 0.7, 0, -1, 0.2, 0.8]),  # TestChain_ProcessBlock_MatchesSample :84-107
    (0.5, [1, 0.5, -0.3, 0.7]),                    # TestChain_ProcessBlock_WithGain :109-131
])
def test_chain_block_matches_sample(gpu, gain, xs):
    ref = sample_by_sample(P.Chain(TWO, gain=gain), xs)
    blk = np.array(xs, dtype=np.float64)
    P.Chain(TWO, gain=gain).ProcessBlock(blk)
    assert np.array_equal(blk, ref)


def test_chain_single_section(gpu):
    """TestChain_SingleSection (chain_test.go:133-148)."""
    c = [0.25, 0.5, 0.25, -0.2, 0.04]
    xs = [1, 0.5, -0.3, 0.7, 0]
    assert np.array_equal(sample_by_sample(P.Chain([c]), xs), cascade([c], xs))


def test_chain_three_sections(gpu):
    """TestChain_ThreeSections (chain_test.go:150-175): 6th order, impulse."""
    co = TWO + [[0.3, 0.3, 0.3, -0.1, 0.02]]
    xs = [1, 0, 0, 0, 0, 0, 0, 0]
    ch = P.Chain(co)
    assert 2 * ch.NumSections() == 6
    assert np.array_equal(sample_by_sample(ch, xs), cascade(co, xs))


def test_chain_reset(gpu):
    """TestChain_Reset (chain_test.go:177-190)."""
    ch = P.Chain(TWO)
    sample_by_sample(ch, [1, 0.5])
    assert np.any(ch.State() != 0)
    ch.Reset()
    assert np.array_equal(ch.State(), np.zeros((1, 2, 2)))


def test_chain_state_save_restore(gpu):
    """TestChain_State_SaveRestore (chain_test.go:192-212)."""
    ch = P.Chain(TWO)
    sample_by_sample(ch, [1, 0.5])
    saved = ch.State()
    y = sample_by_sample(ch, [-0.3, 0.7])
    ch.SetState(saved)
    assert np.array_equal(sample_by_sample(ch, [-0.3, 0.7]), y)


def test_chain_odd_order_first_order_section(gpu):
    """TestChain_OddOrder_FirstOrderSection (chain_test.go:226-246): a
    first-order section (B2 = A2 = 0) after a second-order one."""
    second = [0.25, 0.5, 0.25, -0.2, 0.04]
    first = [0.3, 0.3, 0.0, -0.4, 0.0]
    xs = [1, 0, 0, 0, 0.5, -0.5, 0, 0]
    assert np.array_equal(sample_by_sample(P.Chain([second, first]), xs), cascade([second, first], xs))


def test_chain_stability_long_run(gpu):
    """TestChain_StabilityLongRun (chain_test.go:248-262): an impulse then
    10000 zeros leave every state below 1e-100 (one block call here, the
    states the same bits as the oracle's)."""
    ch = P.Chain(TWO)
    x = np.zeros(10001)
    x[0] = 1.0
    ref, st = O.biquad_chain_block(np.array(TWO).ravel(), np.zeros(4), 1.0, x)
    ch.ProcessBlock(x)
    assert np.array_equal(x, ref)
    states = ch.State()[0]
    assert np.all(np.abs(states) <= 1e-100)
    assert np.array_equal(states.ravel(), st)


def test_update_coefficients_preserves_state(gpu):
    """TestChain_UpdateCoefficients_PreservesStateWhenSectionCountMatches
    (chain_test.go:264-286)."""
    ch = P.Chain(TWO)
    sample_by_sample(ch, [1, 0.5, -0.3])
    saved = ch.State()
    ch.UpdateCoefficients(NEW, 1.0)
    assert np.array_equal(ch.State(), saved)


def test_update_coefficients_applies_new(gpu):
    """TestChain_UpdateCoefficients_AppliesNewCoefficients (chain_test.go:288-311)."""
    ch = P.Chain(TWO)
    ch.UpdateCoefficients(NEW, 1.0)
    ref = P.Chain(NEW)
    xs = [1, 0.5, -0.3, 0.7, 0, -1, 0.2, 0.8]
    assert np.array_equal(sample_by_sample(ch, xs), sample_by_sample(ref, xs))
    assert np.array_equal(sample_by_sample(P.Chain(NEW), xs), cascade(NEW, xs))


def test_update_coefficients_updates_gain(gpu):
    """TestChain_UpdateCoefficients_UpdatesGain (chain_test.go:313-320), and
    the new gain is the one applied."""
    ch = P.Chain(TWO, gain=1.0)
    ch.UpdateCoefficients(TWO, 0.5)
    assert ch.Gain() == 0.5
    xs = [1, 0.5, -0.3, 0.7]
    assert np.array_equal(sample_by_sample(ch, xs), cascade(TWO, xs, 0.5))


def test_update_coefficients_section_count_change_resets(gpu):
    """TestChain_UpdateCoefficients_DifferentSectionCountResetsState
    (chain_test.go:322-344)."""
    ch = P.Chain(TWO)
    sample_by_sample(ch, [1, 0.5])
    ch.UpdateCoefficients([TWO[0]], 1.0)
    assert ch.NumSections() == 1
    assert np.array_equal(ch.State(), np.zeros((1, 1, 2)))
    xs = [0.25, -1, 0.5]
    assert np.array_equal(sample_by_sample(ch, xs), cascade([TWO[0]], xs))
