"""The reference's fir.Filter unit tests, restated against the HIP engine.

Each test names the test it follows (dsp/filter/fir/filter_test.go under
github.com/cwbudde/algo-dsp) and keeps its taps, inputs and 1e-12 bar; the
block paths are also held to the oracle's bits (the GPU's FIR below 32
taps is bit-exact).  `Response` / `MagnitudeDB` are host-side analysis
outside the hot path and are not restated.
"""
import numpy as np
import pytest

import oracle_lib as O
from algodsp import processors as P

pytestmark = pytest.mark.gpu
EPS = 1e-12  # filter_test.go:9


def test_new_copies_coefficients(gpu):
    """TestNew / TestCoefficients_IsCopy (filter_test.go:15-34, 198-206)."""
    c = np.array([0.25, 0.5, 0.25])
    f = P.Filter(c)
    assert f.coeffs.size - 1 == 2  # Order()
    c[0] = 999.0
    assert f.ProcessSample(1.0) == 0.25


def test_process_sample_impulse(gpu):
    """TestProcessSample_Impulse (filter_test.go:36-59)."""
    co = [0.25, 0.5, 0.25]
    f = P.Filter(co)
    for i, want in enumerate(co):
        assert abs(f.ProcessSample(1.0 if i == 0 else 0.0) - want) <= EPS
    for _ in range(5):
        assert abs(f.ProcessSample(0.0)) <= EPS


@pytest.mark.parametrize("co, xs, want", [
    ([1.0 / 3, 1.0 / 3, 1.0 / 3], [1, 1, 1, 1, 1], [1.0 / 3, 2.0 / 3, 1, 1, 1]),  # MovingAverage :61-74
    ([1.0, -1.0], [0, 1, 3, 6, 10], [0, 1, 2, 3, 4]),                              # Differentiator :76-89
    ([0.5], [1, 2, 3], [0.5, 1.0, 1.5]),                                           # TestSingleTap :208-222
], ids=["moving_average", "differentiator", "single_tap"])
def test_process_sample_closed_forms(gpu, co, xs, want):
    f = P.Filter(co)
    got = [f.ProcessSample(float(x)) for x in xs]
    assert np.max(np.abs(np.array(got) - np.array(want))) <= EPS


def test_process_block_and_block_to_match_sample(gpu):
    """TestProcessBlock_MatchesSample / TestProcessBlockTo_MatchesSample
    (filter_test.go:91-134); bit for bit, and equal to the oracle's block."""
    co = [0.25, 0.5, 0.25]
    xs = np.array([1, 0.5, -0.3, 0.7, 0, -1, 0.2, 0.8])
    f1 = P.Filter(co)
    ref = np.array([f1.ProcessSample(x) for x in xs])
    blk = xs.copy()
    P.Filter(co).ProcessBlock(blk)
    assert np.array_equal(blk, ref)
    dst = np.zeros_like(xs)
    P.Filter(co).ProcessBlockTo(dst, xs)
    assert np.array_equal(dst, ref)
    assert np.array_equal(blk, O.Fir(co).process_block(xs))


def test_reset(gpu):
    """TestReset (filter_test.go:136-154)."""
    co = [0.25, 0.5, 0.25]
    f = P.Filter(co)
    f.ProcessSample(1.0)
    f.ProcessSample(0.5)
    f.Reset()
    for i, want in enumerate(co):
        assert abs(f.ProcessSample(1.0 if i == 0 else 0.0) - want) <= EPS
