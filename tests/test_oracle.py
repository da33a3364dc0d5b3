"""Pins the CPU oracle (oracle/liboracle.so) against the reference's own
known-answer vectors and equivalence tests, plus independent
cross-checks (numpy FFT convolution, long-double direct sums).  CPU only.
"""
import json
import math
import pathlib

import numpy as np
import pytest

import oracle_lib as O
from algodsp import signals

KATS = json.loads((pathlib.Path(__file__).parent / "golden" / "reference_kats.json").read_text())


# ---------------------------------------------------------------- conv.Direct
@pytest.mark.parametrize("case", KATS["direct"], ids=lambda c: c["source"])
def test_direct_kat(case):
    got = O.direct(case["a"], case["b"])
    np.testing.assert_allclose(got, case["expected"], atol=case["tol"], rtol=0)


def test_direct_circular_kat():
    c = KATS["direct_circular"][0]
    np.testing.assert_allclose(O.direct_circular(c["a"], c["b"]), c["expected"], atol=c["tol"], rtol=0)


def test_direct_errors():
    # conv_test.go:71-81
    with pytest.raises(O.OracleError) as e:
        O.direct([], [1, 2])
    assert e.value.code == 1
    with pytest.raises(O.OracleError) as e:
        O.direct([1, 2], [])
    assert e.value.code == 2


def test_direct_matches_long_double():
    a = signals.white_noise(4000, 11)
    b = signals.make_test_kernel(256)
    got = O.direct(a, b)
    ref = O.direct_ld(a, b)
    assert np.max(np.abs(got - ref)) < 1e-12


def test_fft_matches_numpy():
    for n in (1, 2, 8, 1024, 32768):
        x = signals.white_noise(2 * n, n).view(np.complex128)
        np.testing.assert_allclose(O.fft(x), np.fft.fft(x), atol=1e-9 * math.log2(max(n, 2)))
        np.testing.assert_allclose(O.fft(x, inverse=True), np.fft.ifft(x), atol=1e-12)


# ------------------------------------------------------- batch OLA / OLS
@pytest.mark.parametrize("K,n", [(3, 10), (64, 1000), (256, 4096), (1000, 3000), (5000, 20000)])
def test_batch_ola_ols_match_direct(K, n):
    # conv_test.go:100-169: OLA vs Direct 1e-10, OLS vs Direct 1e-8
    x = signals.white_noise(n, K)
    h = signals.make_test_kernel(K)
    ref = O.direct_ld(x, h)
    np.testing.assert_allclose(O.OverlapAdd(h).process(x), ref, atol=1e-10 * max(1, K / 64), rtol=0)
    np.testing.assert_allclose(O.OverlapSave(h).process(x), ref, atol=1e-8, rtol=0)


def test_ols_fft_size_rules():
    # overlap_save.go:61-76
    h = np.ones(100)
    assert O.OverlapSave(h, 0).fft_size() == 256
    assert O.OverlapSave(h, 64).fft_size() == 256  # silently raised to nextPow2(2K)
    assert O.OverlapSave(h, 1024).step_size() == 1024 - 100 + 1
    with pytest.raises(O.OracleError) as e:
        O.OverlapSave(h, 300)
    assert e.value.code == 4


def test_convolve_modes():
    # conv_test.go:171-243
    a = signals.make_test_signal(200)
    for m in (5, 64, 65, 300):
        b = signals.make_test_kernel(m)
        full = O.direct_ld(a, b)
        np.testing.assert_allclose(O.convolve_mode(a, b, 0), full, atol=1e-8)
        same = O.convolve_mode(a, b, 1)
        assert same.size == a.size
        np.testing.assert_allclose(same, full[(m - 1) // 2:(m - 1) // 2 + a.size], atol=1e-8)
        valid = O.convolve_mode(a, b, 2)
        assert valid.size == max(a.size, m) - min(a.size, m) + 1


# ------------------------------------------------------------- streaming
def test_streaming_ols_impulse_kat():
    c = KATS["streaming_ols_impulse"]
    s = O.Streaming(c["kernel"], c["block_size"])
    out1 = s.process_block(c["blocks"][0])
    np.testing.assert_allclose(out1, c["expected_first"], atol=c["tol"])


@pytest.mark.parametrize("ola", [False, True])
def test_streaming_vs_batch(ola):
    c = KATS["streaming_ols_vs_batch"]
    h, B, nb = c["kernel"], c["block_size"], c["num_blocks"]
    sig = np.sin(np.arange(B * nb) * 0.1)
    s = O.Streaming(h, B, ola=ola)
    got = np.concatenate([s.process_block(sig[i * B:(i + 1) * B]) for i in range(nb)])
    want = O.OverlapSave(h).process(sig)[: B * nb]
    np.testing.assert_allclose(got, want, atol=c["tol"])


@pytest.mark.parametrize("K,B", [(16384, 4096), (100, 64), (5, 3), (1000, 4096)])
def test_streaming_long_kernel_continuity(K, B):
    h = signals.make_test_kernel(K)
    nb = 3
    x = np.sin(np.arange(B * nb) * 0.2)
    s_ols = O.Streaming(h, B)
    s_ola = O.Streaming(h, B, ola=True)
    a = np.concatenate([s_ols.process_block(x[i * B:(i + 1) * B]) for i in range(nb)])
    b = np.concatenate([s_ola.process_block(x[i * B:(i + 1) * B]) for i in range(nb)])
    ref = O.direct_ld(x, h)[: B * nb]
    np.testing.assert_allclose(a, ref, atol=1e-9)
    np.testing.assert_allclose(b, ref, atol=1e-9)
    assert s_ols.fft_size() == 1 << math.ceil(math.log2(B + K - 1))


# ------------------------------------------------------------ partitioned
@pytest.mark.parametrize("K,n,lo,hi", KATS["partitioned_vs_soa"]["cases"])
def test_partitioned_matches_soa(K, n, lo, hi):
    # partitioned_test.go:121-165 (PCG input replaced by SplitMix64 noise)
    h = signals.make_impulse_kernel(K)
    x = signals.white_noise(n, 42)
    lat = 1 << lo
    pc = O.Partitioned(h, lo, hi)
    xin = np.concatenate([x, np.zeros(lat)])
    out = pc.process_block(xin)[lat:]
    soa = O.Streaming(h, lat, ola=True)
    ref = np.concatenate([soa.process_block(xin[i:i + lat]) for i in range(0, n, lat)])
    assert np.max(np.abs(out[:n] - ref[:n])) < 1e-7


def test_partitioned_dirac_and_latency():
    c = KATS["partitioned_dirac"]
    x = signals.white_noise(c["signal_len"], 3)
    pc = O.Partitioned(c["kernel"], c["min_order"], c["max_order"])
    lat = 1 << c["min_order"]
    out = pc.process_block(np.concatenate([x, np.zeros(lat)]))
    np.testing.assert_allclose(out[lat:], x, atol=c["tol"])
    for order in KATS["partitioned_latency"]["orders"]:
        assert O.Partitioned(signals.make_impulse_kernel(64), order, order + 4).latency() == 1 << order


@pytest.mark.parametrize("K,lo,hi", [(131072, 7, 13), (95432, 7, 13), (1000, 7, 13), (5000, 4, 8), (3, 2, 5),
                                     (777, 5, 5)])
def test_partitioned_is_delayed_linear_conv(K, lo, hi):
    """The reference's stage layout covers the kernel: output == conv delayed by latency."""
    h = signals.white_noise(K, K) * np.exp(-np.arange(K) / max(K / 4, 1))
    lat = 1 << lo
    n = min(3 * K, 40000) + lat
    x = signals.white_noise(n, 5)
    pc = O.Partitioned(h, lo, hi)
    # arbitrary call sizes (ProcessBlock accepts any length)
    outs, pos, step = [], 0, 0
    sizes = [lat * 3 + 5, 1, lat - 1, 2 * lat]
    while pos < n:
        m = min(sizes[step % len(sizes)], n - pos)
        outs.append(pc.process_block(x[pos:pos + m]))
        pos += m
        step += 1
    out = np.concatenate(outs)
    nf = 2 * n + K
    ref = np.fft.irfft(np.fft.rfft(x, nf) * np.fft.rfft(h, nf), nf)[: n - lat]
    assert np.sqrt(np.mean((out[lat:] - ref) ** 2)) < 1e-9


def test_partitioned_stage_layout_131072():
    # (7,13) on 131072 taps -> (128x2), 256, 512, 1024, 2048, 4096, (8192x15)
    pc = O.Partitioned(np.ones(131072), 7, 13)
    layout = [pc.stage_info(i) for i in range(pc.stage_count())]
    assert layout == [(128, 2), (256, 1), (512, 1), (1024, 1), (2048, 1), (4096, 1), (8192, 15)]
    pc = O.Partitioned(np.ones(95432), 7, 13)
    layout = [pc.stage_info(i) for i in range(pc.stage_count())]
    assert layout == [(128, 2), (256, 2), (512, 1), (1024, 2), (2048, 1), (4096, 2), (8192, 10)]


# --------------------------------------------------------------- filters
def test_biquad_kat_and_kernels():
    c = KATS["biquad_dfiit_impulse"]
    st = np.zeros(2)
    ys = []
    for x in c["input"]:
        y, st = O.biquad_sample(c["coeffs"], st, x)
        ys.append(y)
    np.testing.assert_allclose(ys, c["expected"], atol=c["tol"])
    v = KATS["biquad_avx2_vector"]
    ref = []
    st = np.zeros(2)
    for x in v["input"]:
        y, st = O.biquad_sample(v["coeffs"], st, x)
        ref.append(y)
    for kern in ("avx2", "generic"):
        got, st2 = O.biquad_block(v["coeffs"], [0, 0], v["input"], kernel=kern)
        assert np.array_equal(got, ref)  # same operation order -> bit-exact
        assert np.array_equal(st2, st)


def test_fir_block_vs_sample():
    c = KATS["fir_block_vs_sample"]
    f1, f2 = O.Fir(c["coeffs"]), O.Fir(c["coeffs"])
    ref = [f1.process_sample(x) for x in c["input"]]
    np.testing.assert_allclose(f2.process_block(c["input"]), ref, atol=c["tol"])


def test_fir_long_block_is_reversed_convolution():
    # for >= 32 taps ProcessBlock computes sum h[N-1-j] x[n-j]
    h = signals.white_noise(64, 9)
    x = signals.white_noise(500, 10)
    got = O.Fir(h).process_block(x)
    ref = O.direct_ld(x, h[::-1].copy())[: x.size]
    assert np.max(np.abs(got - ref)) < 1e-12
    sample = O.Fir(h)
    ref2 = [sample.process_sample(v) for v in x]
    np.testing.assert_allclose(ref2, O.direct_ld(x, h)[: x.size], atol=1e-12)


# --------------------------------------------------------------- effects
def test_compressor_coefficients():
    c = KATS["compressor_coefficients"]
    comp = O.Compressor(c["sample_rate"])
    thr, knee, att, rel, mk = comp.params()
    assert abs(thr - c["expected_threshold_log2"]) < c["tol"]
    assert abs(knee - c["expected_knee_width_log2"]) < c["tol"]
    assert 0 < att < 1 and 0 < rel < 1
    assert abs(mk - 10 ** (c["expected_auto_makeup_db"] / 20)) < 1e-12


def _legacy_signal():
    i = np.arange(4096, dtype=np.float64)
    out = np.empty(4096)
    for k in range(4096):
        if k < 1024:
            out[k] = 0.08 * math.sin(2 * math.pi * 440 * k / 48000)
        elif k < 2048:
            out[k] = 0.7 * math.sin(2 * math.pi * 440 * k / 48000)
        elif k < 3072:
            out[k] = 0.2 * math.sin(2 * math.pi * 440 * k / 48000)
        else:
            out[k] = 0.9 * math.sin(2 * math.pi * 880 * k / 48000)
    return out


def _legacy_sim(x, sr, thr_db, ratio, att_ms, rel_ms, topology, detector, rms_ms=0.0):
    """Closed-form legacy compressor of legacy_parity_test.go:156-259, restated."""
    threshold = 10 ** (thr_db / 20.0)
    lr = 1.0 / ratio
    scale = ratio if topology == 1 else 1.0
    attack = 1.0 - math.exp(-math.log(2) / (att_ms * 0.001 * sr * scale))
    release = math.exp(-math.log(2) / (rel_ms * 0.001 * sr * scale))
    out = np.empty_like(x)
    peak = 0.0
    if topology == 1:
        makeup1 = threshold ** ((1.0 - lr) * ratio)
        prev = 0.0
        for i, s in enumerate(x):
            if prev > peak:
                peak += (prev - peak) * attack
            else:
                peak = prev + (peak - prev) * release
            g = makeup1 * peak ** (1.0 - ratio) if peak >= threshold else 1.0
            y = s * g
            out[i] = y
            prev = abs(y)
        return out
    makeup1 = threshold ** (1.0 - lr)
    size = max(int(round(sr * 0.001 * rms_ms)), 1) if detector == 1 else 0
    buf = np.zeros(max(size, 1))
    pos, ssum = 0, 0.0
    for i, s in enumerate(x):
        if detector == 1:
            sq = s * s
            ssum += sq - buf[pos]
            buf[pos] = sq
            pos = (pos + 1) % size
            a = math.sqrt(ssum / size)
        else:
            a = abs(s)
        if a > peak:
            peak += (a - peak) * attack
        else:
            peak = a + (peak - a) * release
        g = makeup1 * peak ** (lr - 1.0) if peak >= threshold else 1.0
        out[i] = s * g
    return out


@pytest.mark.parametrize("case", KATS["compressor_legacy_parity"]["cases"], ids=lambda c: c["name"])
def test_compressor_legacy_parity(case):
    x = _legacy_signal()
    kw = dict(auto_makeup=0, makeup_db=0.0, knee_db=0.0, threshold_db=float(case["threshold_db"]),
              ratio=float(case["ratio"]), attack_ms=float(case["attack_ms"]), release_ms=float(case["release_ms"]),
              topology=case["topology"], detector_mode=case["detector"], feedback_ratio_scale=1)
    if "rms_ms" in case:
        kw["rms_window_ms"] = float(case["rms_ms"])
    got = O.Compressor(48000.0, **kw).process_in_place(x)
    want = _legacy_sim(x, 48000.0, case["threshold_db"], case["ratio"], case["attack_ms"], case["release_ms"],
                       case["topology"], case["detector"], case.get("rms_ms", 0.0))
    assert np.max(np.abs(got - want)) < KATS["compressor_legacy_parity"]["tol"]


def test_freeverb_block_vs_sample():
    x = np.sin(2 * math.pi * np.arange(128) / 23)
    r1, r2 = O.Freeverb(), O.Freeverb()
    want = [r1.process_sample(v) for v in x]
    got = r2.process_in_place(x)
    assert np.max(np.abs(got - np.array(want))) <= 1e-12
    r2.reset()
    imp = np.zeros(4000)
    imp[0] = 1
    tail = r2.process_in_place(imp)
    assert np.any(np.abs(tail[1200:]) > 0)  # reverb_test.go:62+: impulse tail exists


# ------------------------------------------------------------------- IRLB
def test_irlib_layout():
    data = (pathlib.Path(__file__).parent.parent / "data" / "irs.irlib").read_bytes()
    irs = O.irlib_read(data)
    exp = KATS["irlib"]
    assert [(n, s.shape[1]) for n, fs, s in irs] == [tuple(e) for e in exp["irs"]]
    assert all(fs == exp["sample_rate"] and s.shape[0] == exp["channels"] for n, fs, s in irs)


def test_decode_f16_subnormal_quirk():
    # irlib.go:87 doubles every subnormal half
    assert O.decode_f16(0x0001) == 2.0 * 2.0 ** -24
    assert O.decode_f16(0x3C00) == 1.0
    assert O.decode_f16(0xC000) == -2.0
    assert O.decode_f16(0x03FF) == 2.0 * (1023 / 1024) * 2.0 ** -14


# ------------------------------------------------ correlate.go / deconvolve.go
def _np_correlate_fft(a, b):
    n, m = len(a), len(b)
    N = 1 << max(0, (n + m - 2).bit_length())
    r = np.fft.ifft(np.fft.fft(a, N) * np.conj(np.fft.fft(b, N))).real
    return np.concatenate([r[N - m + 1:], r[:n]])


def test_correlate_fft_kat():
    # conv_test.go:463-485: CorrelateFFT([1..5], [1,2,3]) == Correlate within 1e-8
    a, b = [1, 2, 3, 4, 5], [1, 2, 3]
    r = O.correlate_fft(a, b)
    ref = O.direct(a, b[::-1])  # Correlate = Convolve(a, reverse b); m <= 64 -> Direct
    assert r.size == 7
    assert np.max(np.abs(r - ref)) < 1e-8
    assert np.allclose(ref, [3, 8, 14, 20, 26, 14, 5])


@pytest.mark.parametrize("n,m", [(1, 1), (7, 3), (1000, 37), (4096, 4097), (30000, 2500)])
def test_correlate_fft_matches_numpy(n, m):
    a, b = signals.white_noise(n, 11), signals.white_noise(m, 12)
    r = O.correlate_fft(a, b)
    assert np.max(np.abs(r - _np_correlate_fft(a, b))) < 1e-10 * max(1.0, np.max(np.abs(r)))


def test_correlate_autocorr_peak_kat():
    # conv_test.go:244-265: cos(2 pi i / 32) auto-correlation peaks at zero lag (index n-1)
    x = np.cos(2 * np.pi * np.arange(256) / 32)
    r = O.correlate_fft(x, x)
    assert int(np.argmax(r)) == 255


def test_correlate_fft_empty():
    with pytest.raises(O.OracleError) as e:
        O.correlate_fft([], [1, 2])
    assert e.value.code == 1


def _np_deconv(s, h, eps=None):
    n, m = len(s), len(h)
    N = 1 << max(0, (n - 1).bit_length())
    S, H = np.fft.fft(s, N), np.fft.fft(h, N)
    R = S / H if eps is None else S * np.conj(H) / (np.abs(H) ** 2 + eps)
    olen = n - m + 1 if n - m + 1 > 0 else n
    return np.fft.ifft(R).real[:olen]


@pytest.mark.parametrize("method,eps", [(0, None), (1, 1e-3), (1, 1e-6), (2, None)])
def test_deconvolve_matches_numpy(method, eps):
    orig = np.sin(2 * np.pi * np.arange(100) / 20)
    h = np.array([0.25, 0.5, 0.25])
    y = O.direct(orig, h)
    if method == 0:
        h = np.array([1.0, 0.3])  # no spectral zero (|H| >= 0.7)
        y = O.direct(orig, h)
    if method == 2:  # Wiener, auto variances: nsr = 0.01
        got = O.deconvolve(y, h, 2)
        ref = _np_deconv(y, h, 0.01)
    else:
        got = O.deconvolve(y, h, method, eps or 0.0)
        ref = _np_deconv(y, h, eps)
    assert got.size == y.size - h.size + 1
    assert np.max(np.abs(got - ref)) < 1e-9 * max(1.0, np.max(np.abs(ref)))


def test_deconvolve_reference_kats():
    # conv_test.go:282-310 (regularized eps 1e-3: SNR logged only) and :563-583 (naive, identity kernel)
    orig = np.sin(2 * np.pi * np.arange(100) / 20)
    rec = O.deconvolve(O.direct(orig, [0.25, 0.5, 0.25]), [0.25, 0.5, 0.25], 1, 1e-3)
    assert rec.size == 100 and np.all(np.isfinite(rec))
    o2 = np.sin(2 * np.pi * np.arange(50) / 10)
    rec2 = O.deconvolve(o2, [1.0], 0)
    assert np.max(np.abs(rec2 - o2)) < 1e-12


def test_deconvolve_errors_and_zero_bin():
    # conv_test.go:619-631; deconvolve.go:146-154 (first bin with |H| < 1e-15)
    with pytest.raises(O.OracleError) as e:
        O.deconvolve([], [1, 2])
    assert e.value.code == 1
    with pytest.raises(O.OracleError) as e:
        O.deconvolve([1, 2], [])
    assert e.value.code == 2
    with pytest.raises(O.OracleError) as e:
        O.deconvolve([1.0, 2.0, 3.0, 4.0], [1.0, 1.0], 0)  # H = 1 + W^k: zero at k = N/2 = 2
    assert e.value.code == 9 and e.value.bad_bin == 2


def test_inverse_filter_kat():
    # conv_test.go:312-340: InverseFilter([.5, 1, .5], 64, 1e-3) -> conv with kernel has a dominant peak
    inv = O.inverse_filter([0.5, 1.0, 0.5], 64, 1e-3)
    r = O.direct([0.5, 1.0, 0.5], inv)
    assert np.max(r) > 0.1
    H = np.fft.fft([0.5, 1.0, 0.5], 64)
    ref = np.fft.ifft(np.conj(H) / (np.abs(H) ** 2 + 1e-3)).real
    assert np.max(np.abs(inv - ref)) < 1e-9 * np.max(np.abs(ref))


# ------------------------------------------------------------------ Gate / Expander (dynamics/gate.go, expander.go)
def test_gate_gain_kats():
    """gate_test.go:352-458: unity above threshold, attenuation below it,
    more attenuation for larger ratios (ratio 1 is unity), rangeLin at silence."""
    g = O.Expander(48000.0, gate=True, threshold_db=-40.0)
    assert all(g.gain(l) == 1.0 for l in (0.1, 0.5, 1.0))
    assert g.gain(0.0) == 10 ** (-80 / 20)
    g = O.Expander(48000.0, gate=True, threshold_db=-20.0, ratio=10.0, knee_db=0.0)
    assert 0.0 < g.gain(0.05) < 1.0
    prev = None
    for ratio in (1.0, 2.0, 4.0, 10.0):
        gr = O.Expander(48000.0, gate=True, threshold_db=-20.0, ratio=ratio, knee_db=0.0, range_db=-120.0).gain(0.01)
        if ratio == 1.0:
            assert gr == 1.0
        else:
            assert gr < prev
        prev = gr
    # the floor: gain never drops below rangeLin (gate_test.go:460-491)
    g = O.Expander(48000.0, gate=True, threshold_db=-20.0, ratio=100.0, knee_db=0.0, range_db=-20.0)
    assert g.gain(1e-6) == 10 ** (-20 / 20)


def test_gate_hold_behaviour():
    """gate_test.go:657-712 and 714-759: the hold counter is full after a loud
    passage, reaches 0 after decay + hold, and refills on a loud return."""
    g = O.Expander(48000.0, gate=True, threshold_db=-20.0, attack_ms=0.1, release_ms=1.0, hold_ms=10.0, knee_db=0.0)
    for _ in range(2000):
        g.process_sample(0.5)
    assert g.hold_counter() == 480
    for _ in range(1000 + 480):
        g.process_sample(0.0)
    assert g.hold_counter() == 0
    g = O.Expander(48000.0, gate=True, threshold_db=-20.0, hold_ms=100.0, attack_ms=0.1)
    for _ in range(2000):
        g.process_sample(0.5)
    full = g.hold_counter()
    for _ in range(10):
        g.process_sample(0.0)
    for _ in range(2000):
        g.process_sample(0.5)
    assert g.hold_counter() == full == 4800


def test_expander_gain_behaviour():
    """expander_test.go:94-158: above-threshold pass-through, attenuation below,
    and feedback vs feed-forward topologies differ."""
    e = O.Expander(48000.0, threshold_db=-20.0, ratio=6.0, knee_db=0.0, range_db=-80.0)
    assert e.process_in_place(np.full(1024, 0.5))[-1] >= 0.49
    e = O.Expander(48000.0, threshold_db=-20.0, ratio=6.0, knee_db=0.0, range_db=-80.0)
    assert e.process_in_place(np.full(1024, 0.02))[-1] < 0.02
    kw = dict(threshold_db=-25.0, ratio=4.0, detector_mode=1, rms_window_ms=20.0)
    fb = O.Expander(48000.0, topology=1, **kw).process_in_place(np.full(512, 0.05))[-1]
    ff = O.Expander(48000.0, topology=0, **kw).process_in_place(np.full(512, 0.05))[-1]
    assert fb != ff


# ---------------------------------------------------------- float32 variants
def test_oracle_streaming32_kats():
    """The float32 restatement (or_conv32.c) against the reference's own float32
    tests: impulse response (streaming_test.go:236-266) and OLA == OLS within
    1e-4 (:175-234); plus partitioned32 vs the float64 oracle."""
    c = KATS["streaming32_impulse"]
    for ola in (False, True):
        s = O.Streaming32(c["kernel"], c["block_size"], ola=ola)
        np.testing.assert_allclose(s.process_block(c["input"]), c["expected"], atol=c["tol"], rtol=0)
    e = KATS["streaming32_equivalence"]
    B, nb = e["block_size"], e["num_blocks"]
    i = np.arange(B * nb)
    sig = (np.sin(i * 0.1) + 0.5 * np.cos(i * 0.05)).astype(np.float32)
    a = O.Streaming32(e["kernel"], B, ola=True)
    b = O.Streaming32(e["kernel"], B, ola=False)
    ya = np.concatenate([a.process_block(sig[k * B:(k + 1) * B]) for k in range(nb)])
    yb = np.concatenate([b.process_block(sig[k * B:(k + 1) * B]) for k in range(nb)])
    assert np.max(np.abs(ya.astype(np.float64) - yb)) <= e["tol"]
    h = signals.make_impulse_kernel(1000)
    x = signals.white_noise(3000, 5)
    p32 = O.Partitioned32(h, 6, 9).process_block(x)
    p64 = O.Partitioned(h, 6, 9).process_block(x)
    assert np.max(np.abs(p32 - p64)) < 1e-4
