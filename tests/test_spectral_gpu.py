"""GPU parity of the spectral row: CorrelateFFT, Deconvolve and
InverseFilter (dsp/conv/correlate.go:111-172, deconvolve.go:72-394) through
the HIP C ABI against the CPU oracle (oracle/or_spectral.c).

The reference pins these only by tolerance (conv_test.go:463-485: 1e-8 vs
Direct); FFT-level bits are unpinned (algo-fft is not in the container), so
the GPU result must match the oracle within FFT rounding:
  max |gpu - oracle| <= TOL * max(1, max |oracle|), TOL = 1e-10
(1e-8 for the regularised inverses, whose 1/(|H|^2 + eps) gain amplifies
rounding by up to 1/(2 sqrt(eps))).  Sizes cover the one-pass (N <= 4096),
two-pass and three-pass (N > 2^18) device FFT plans and the naive DFT (N <= 8).
"""
import numpy as np
import pytest

import oracle_lib as O
from algodsp import conv, signals

pytestmark = pytest.mark.gpu
TOL = 1e-10


def close(got, want, tol=TOL):
    got, want = np.asarray(got), np.asarray(want)
    assert got.shape == want.shape
    if want.size:
        err = float(np.max(np.abs(got - want)))
        assert err <= tol * max(1.0, float(np.max(np.abs(want)))), err


# ------------------------------------------------------------- CorrelateFFT
def test_correlate_fft_kat(gpu):
    # conv_test.go:463-485
    a, b = [1, 2, 3, 4, 5], [1, 2, 3]
    r = conv.CorrelateFFT(a, b)
    d = conv.Correlate(a, b)
    assert r.size == d.size == 7
    assert np.max(np.abs(r - d)) < 1e-8


@pytest.mark.parametrize("n,m", [(1, 1), (2, 1), (3, 3), (5, 3), (9, 8), (20, 12), (17, 16), (33, 31), (1000, 37),
                                 (4096, 1), (3000, 1100), (40000, 25000), (131072, 131072), (600000, 3)])
def test_correlate_fft_matches_oracle(gpu, n, m):
    a, b = signals.white_noise(n, 31 + n), signals.white_noise(m, 57 + m)
    close(conv.CorrelateFFT(a, b), O.correlate_fft(a, b))


@pytest.mark.parametrize("n,m", [(3, 3), (5, 3), (20, 12), (33, 31), (1000, 37), (40000, 25000), (1 << 17, 3)])
def test_correlate_fft_device_matches_host(gpu, n, m):
    """ad_correlate_fft_device (device arrays on the caller's stream; the
    product and the lag order fused into the transforms' passes) against the
    host-buffer entry point, bit for bit, and against the oracle."""
    import ctypes as C

    import torch

    from algodsp._lib import check, lib

    a, b = signals.white_noise(n, 5 + n), signals.white_noise(m, 9 + m)
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    dout = torch.full((n + m - 1,), np.nan, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream()
    check(lib().ad_correlate_fft_device(C.c_void_p(da.data_ptr()), n, C.c_void_p(db.data_ptr()), m,
                                        C.c_void_p(dout.data_ptr()), 0, C.c_void_p(st.cuda_stream)))
    st.synchronize()
    got = dout.cpu().numpy()
    assert np.array_equal(got, conv.CorrelateFFT(a, b))
    close(got, O.correlate_fft(a, b))


def test_correlate_fft_device_two_streams(gpu):
    """device calls alternating between two streams share the
    per-device work buffers and the first pass's max-abs counter; each call
    waits for the previous one when that ran on another stream, so every
    result equals the single-stream result bit for bit (and a later call on
    the first stream is not corrupted either)."""
    import ctypes as C

    import torch

    from algodsp._lib import check, lib

    n = m = 1 << 20  # the split first pass with the max-abs partials (N = 2^21)
    pairs = [(signals.white_noise(n, 300 + i), 10.0 ** (3 * i) * signals.white_noise(m, 400 + i)) for i in range(6)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    devs = [(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()) for a, b in pairs]
    torch.cuda.synchronize()
    for i, (da, db) in enumerate(devs):
        st = streams[i % 2]
        dout = torch.full((n + m - 1,), np.nan, dtype=torch.float64, device="cuda")
        check(lib().ad_correlate_fft_device(C.c_void_p(da.data_ptr()), n, C.c_void_p(db.data_ptr()), m,
                                            C.c_void_p(dout.data_ptr()), 0, C.c_void_p(st.cuda_stream)))
        outs.append(dout)
    torch.cuda.synchronize()
    for (a, b), dout in zip(pairs, outs):
        assert np.array_equal(dout.cpu().numpy(), conv.CorrelateFFT(a, b))


@pytest.mark.parametrize("sa,sb", [(3.0e4, 3.0e-3), (1.0e-4, 2.0e3), (1.0, 1.0e-9), (2.0**600, 2.0**-600),
                                   (2.0**-600, 2.0**560)])
@pytest.mark.parametrize("n,m", [(40000, 25000), (1 << 17, 4096)])
def test_correlate_fft_unequal_scales(gpu, n, m, sa, sb):
    """Signals whose magnitudes differ by 1e6 .. 1e9 (an int16-scale recording
    against a normalised template): the device packs both into one transform of
    a + i b, so without its power-of-two rescaling of b, B's spectrum would
    carry rounding of order eps |A| and the correlation's error would grow by
    |a| / |b|.  The reference transforms a and b separately (correlate.go:122-147);
    the result must stay within the same relative bar as equal-scale inputs.
    Ratios beyond 2^1000 take the scale's clamped two-factor path:
    a single 2^e would overflow there (parity unpinned: no reference fixture
    covers it, the oracle transforms a and b separately)."""
    a, b = sa * signals.white_noise(n, 3 + n), sb * signals.white_noise(m, 4 + m)
    close(conv.CorrelateFFT(a, b), O.correlate_fft(a, b))


def _np_correlate_fft(a, b):  # same lag order as correlate.go:165-171
    n, m = len(a), len(b)
    N = 1 << max(0, (n + m - 2).bit_length())
    r = np.fft.irfft(np.fft.rfft(a, N) * np.conj(np.fft.rfft(b, N)), N)
    return np.concatenate([r[N - m + 1:], r[:n]])


@pytest.mark.parametrize("n,m,sa,sb", [(1 << 23, 1 << 23, 1.0, 1.0), (10_000_000, 3_000_000, 3.0e4, 3.0e-3),
                                       ((1 << 24) - 9, 10, 2.0**600, 2.0**-600)])
def test_correlate_fft_2p24(gpu, n, m, sa, sb):
    """The bench size's plan (n + m - 1 in (2^23, 2^24]: N = 2^24, passes
    256 x 256 x 256): the first pass with the max-abs folded in
    (k_corr_split0), the second forming the packed spectrum at its load
    (k_fft_pass_pf PACKIN), the fused forward-last / inverse-first pass, at
    equal, 1e7-apart and 2^1200-apart scales.  Checked against numpy's fp64
    FFT at the spectral bar: the oracle's C restatement takes ~30 s per call
    at this size, and test_oracle.py::test_correlate_fft_matches_numpy pins it
    to the same numpy expression at smaller sizes."""
    a, b = sa * signals.white_noise(n, 5 + n), sb * signals.white_noise(m, 6 + m)
    close(conv.CorrelateFFT(a, b), _np_correlate_fft(a, b))


def test_correlate_fft_empty(gpu):
    with pytest.raises(conv.ErrEmptyInput):
        conv.CorrelateFFT([], [1.0, 2.0])
    with pytest.raises(conv.ErrEmptyInput):
        conv.CorrelateFFT([1.0], [])


def test_correlate_family(gpu):
    # conv_test.go:244-280, 494-561
    x = np.cos(2 * np.pi * np.arange(256) / 32)
    r = conv.AutoCorrelate(x)
    assert conv.FindPeak(r)[0] == 255 and conv.LagFromIndex(255, 256) == 0
    a, b = [1, 2, 3, 4, 5], [1, 2, 3]
    np.testing.assert_allclose(conv.CorrelateDirect(a, b), conv.Correlate(a, b), atol=1e-10, rtol=0)
    assert abs(conv.AutoCorrelateNormalized(a)[4] - 1.0) < 1e-10
    assert abs(conv.FindPeak(conv.CorrelateNormalized(a, a))[1] - 1.0) < 0.1
    assert conv.CorrelateMode(a, b, conv.ModeFull).size == 7
    assert conv.CorrelateMode(a, b, conv.ModeSame).size == 5
    assert conv.CorrelateMode(a, b, conv.ModeValid).size == 3
    assert conv.FindPeak([]) == (-1, 0.0)
    assert conv.IndexFromLag(0, 3) == 2


# --------------------------------------------------------------- Deconvolve
def _opts(method, eps=0.0, nv=0.0, sv=0.0):
    return conv.DeconvOptions(method, eps, nv, sv)


@pytest.mark.parametrize("n,m", [(3, 1), (8, 3), (102, 3), (5000, 64), (300000, 1500)])
@pytest.mark.parametrize("method,eps", [(conv.DeconvRegularized, 1e-3), (conv.DeconvRegularized, 0.0),
                                        (conv.DeconvWiener, 0.0)])
def test_deconvolve_matches_oracle(gpu, n, m, method, eps):
    x = signals.white_noise(n, 7 + n)
    h = np.hanning(m + 2)[1:-1] if m > 1 else np.array([0.8])
    got = conv.Deconvolve(x, h, _opts(method, eps))
    want = O.deconvolve(x, h, method, eps)
    close(got, want, 1e-8)


def test_deconvolve_naive_and_wiener_given_variances(gpu):
    # conv_test.go:563-617
    orig = np.sin(2 * np.pi * np.arange(50) / 10)
    rec = conv.Deconvolve(conv.Direct(orig, [1.0]), [1.0], _opts(conv.DeconvNaive))
    assert np.max(np.abs(rec - orig)) < 1e-12
    y = conv.Direct(orig, [0.25, 0.5, 0.25])
    got = conv.Deconvolve(y, [0.25, 0.5, 0.25], _opts(conv.DeconvWiener, 0.0, 0.01, 1.0))
    close(got, O.deconvolve(y, [0.25, 0.5, 0.25], 2, 0.0, 0.01, 1.0), 1e-8)
    h = [1.0, 0.3]
    x = signals.white_noise(4000, 3)
    close(conv.Deconvolve(x, h, _opts(conv.DeconvNaive)), O.deconvolve(x, h, 0), 1e-9)


def test_deconvolve_errors(gpu):
    # conv_test.go:619-631 and the naive zero-bin error (deconvolve.go:146-154)
    d = conv.DefaultDeconvOptions()
    assert d.Method == conv.DeconvRegularized and d.Epsilon == 1e-6
    with pytest.raises(conv.ErrEmptyInput):
        conv.Deconvolve([], [1.0, 2.0], d)
    with pytest.raises(conv.ErrEmptyKernel):
        conv.Deconvolve([1.0, 2.0], [], d)
    with pytest.raises(conv.ErrDivisionByZero) as e:
        conv.Deconvolve([1.0, 2.0, 3.0, 4.0], [1.0, 1.0], _opts(conv.DeconvNaive))
    with pytest.raises(O.OracleError) as eo:
        O.deconvolve([1.0, 2.0, 3.0, 4.0], [1.0, 1.0], 0)
    assert f"bin {eo.value.bad_bin}" in str(e.value)


def test_deconvolve_round_trip(gpu):
    # property at a size past the oracle's comfort: deconvolve(conv(x, h), h) ~ x
    # (circular deconvolution at nextPow2(n) = n: exact up to rounding for a
    # kernel without spectral zeros)
    x = signals.white_noise(1 << 20, 99)
    h = np.array([1.0, -0.5, 0.25])
    y = conv.Direct(x, h)[: x.size]  # circular-compatible: drop the tail
    y[: h.size - 1] += conv.Direct(x, h)[x.size:]  # wrap the tail (circular convolution)
    rec = conv.Deconvolve(y, h, _opts(conv.DeconvNaive))
    # olen = n - m + 1
    assert np.max(np.abs(rec - x[: rec.size])) < 1e-9


# ------------------------------------------------------------ InverseFilter
@pytest.mark.parametrize("m,length,eps", [(3, 64, 1e-3), (3, 1, 1e-3), (5, 7, 0.0), (1000, 4096, 1e-4),
                                          (100000, 65536, 1e-2), (7, 1 << 21, 1e-3)])
def test_inverse_filter_matches_oracle(gpu, m, length, eps):
    h = signals.white_noise(m, 5 + m)
    close(conv.InverseFilter(h, length, eps), O.inverse_filter(h, length, eps), 1e-8)


def test_inverse_filter_kat_and_errors(gpu):
    # conv_test.go:312-340
    inv = conv.InverseFilter([0.5, 1.0, 0.5], 64, 1e-3)
    assert conv.FindPeak(conv.Direct([0.5, 1.0, 0.5], inv))[1] > 0.1
    assert conv.InverseFilter([1.0], 0, 1e-3).size == 0
    with pytest.raises(conv.ErrEmptyKernel):
        conv.InverseFilter([], 8, 1e-3)
