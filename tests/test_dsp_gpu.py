"""GPU parity of the per-sample processors and the FIR filter through the HIP
C ABI against the CPU oracle.

Tolerances (BASELINE.json north_star / SURVEY 8(d) parity gates):
  * biquad chains, Freeverb, FIR with < 32 taps: bit-exact (same operation
    order, no FMA contraction on either side);
  * FIR with >= 32 taps: <= 1e-12 RMS (the reference's vecmath.DotProduct
    summation order is unpinned; both sides sum sequentially, so in practice
    this is exact too);
  * Compressor and the fused effect chain: <= 1e-12 RMS (log2/pow come from
    the GPU's math library vs the host libm, and the envelope follower computes
    the reference's map as two FMAs: last-ulp differences, never more).
"""
import json
import pathlib

import numpy as np
import pytest

import oracle_lib as O
from algodsp import design, processors as P, signals

pytestmark = pytest.mark.gpu

KATS = json.loads((pathlib.Path(__file__).parent / "golden" / "reference_kats.json").read_text())
RMS_TOL = 1e-12
# compressor metrics (peaks, minimum gain): relative, the processors' 1e-12 bar
# (the envelope is the reference's map with its own rounding, dsp_device.hpp
# env_step; the feedback topology feeds that rounding back through the gain)
METRIC_RTOL = 1e-12


def rms(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    return float(np.sqrt(np.mean((a - b) ** 2))) if a.size else 0.0


def stable_sections(k, seed):
    """k stable biquads (poles inside the unit circle) from a seeded RNG."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        r, th = rng.uniform(0.2, 0.97), rng.uniform(0.05, 3.0)
        a1, a2 = -2 * r * np.cos(th), r * r
        b = rng.uniform(-1, 1, 3)
        out.append([b[0], b[1], b[2], a1, a2])
    return np.array(out)


def legacy_signal(n=4096, fs=48000.0):
    """makeLegacyParitySignal (dsp/effects/dynamics/legacy_parity_test.go:8-40):
    440 Hz at 0.08 / 0.7 / 0.2, then 880 Hz at 0.9, in four equal segments."""
    k = np.arange(n, dtype=np.float64)
    q = n // 4
    amp = np.where(k < q, 0.08, np.where(k < 2 * q, 0.7, np.where(k < 3 * q, 0.2, 0.9)))
    f = np.where(k < 3 * q, 440.0, 880.0)
    return amp * np.sin(2 * np.pi * f * k / fs)


# ------------------------------------------------------------------ biquad
def test_biquad_section_kat(gpu):
    case = KATS["biquad_dfiit_impulse"]
    x = np.array(case["input"], dtype=np.float64)
    s = P.Section(*case["coeffs"])
    s.ProcessBlock(x)
    np.testing.assert_allclose(x, case["expected"], atol=case["tol"], rtol=0)


def test_biquad_avx2_vector_bit_exact(gpu):
    case = KATS["biquad_avx2_vector"]
    x = np.array(case["input"], dtype=np.float64)
    want, _ = O.biquad_block(case["coeffs"], [0.0, 0.0], x)
    per_sample = []
    st = np.zeros(2)
    for v in x:  # register_test.go: block kernel == ProcessSample loop
        y, st = O.biquad_sample(case["coeffs"], st, v)
        per_sample.append(y)
    s = P.Section(*case["coeffs"])
    s.ProcessBlock(x)
    assert np.array_equal(x, want)
    np.testing.assert_allclose(x, per_sample, atol=case["tol"], rtol=0)


@pytest.mark.parametrize("sections,gain", [(1, 1.0), (5, 1.0), (3, 0.5), (8, 1.0), (11, 1.7)])
def test_chain_bit_exact_multichannel(gpu, sections, gain):
    coeffs = stable_sections(sections, 10 + sections)
    C, n = 70, 5003  # two workgroups, ragged last one
    x = np.stack([signals.white_noise(n, 300 + c) for c in range(C)])
    gpu_ch = P.Chain(coeffs, gain, channels=C)
    y = x.copy()
    gpu_ch.ProcessBlock(np.zeros((C, 0)))  # empty block: no-op
    a, b = y[:, :2000].copy(), y[:, 2000:].copy()  # state carried across blocks
    gpu_ch.ProcessBlock(a)
    gpu_ch.ProcessBlock(b)
    got = np.concatenate([a, b], axis=1)
    for c in (0, 33, 69):
        want, st = O.biquad_chain_block(coeffs.ravel(), np.zeros(2 * sections), gain, x[c])
        assert np.array_equal(got[c], want), (c, float(np.max(np.abs(got[c] - want))))
        np.testing.assert_array_equal(gpu_ch.State()[c].ravel(), st)


def test_chain_one_shot_state_io(gpu):
    coeffs = stable_sections(4, 3)
    x = np.stack([signals.white_noise(777, 9), signals.white_noise(777, 10)])
    state = np.zeros((2, 4, 2))
    y1, y2 = x[:, :300].copy(), x[:, 300:].copy()
    P.chain_process(coeffs, state, 0.8, y1)
    P.chain_process(coeffs, state, 0.8, y2)
    got = np.concatenate([y1, y2], axis=1)
    for c in range(2):
        want, st = O.biquad_chain_block(coeffs.ravel(), np.zeros(8), 0.8, x[c])
        assert np.array_equal(got[c], want)
        np.testing.assert_array_equal(state[c].ravel(), st)


@pytest.mark.parametrize("sections", [3, 11])
def test_chain_set_state_round_trip(gpu, sections):
    """Chain.State / Chain.SetState (chain.go:122-138) as a checkpoint at a call
    boundary: run A, save the state, run B; a second chain restored from the
    saved state produces B's block bit for bit, and both equal the oracle run
    over A + B in one pass.  Covers > 8 sections (several EQ passes)."""
    coeffs = stable_sections(sections, 40 + sections)
    C, n1, n2 = 5, 1500, 2200
    x = np.stack([signals.white_noise(n1 + n2, 600 + c) for c in range(C)])
    ch = P.Chain(coeffs, 0.9, channels=C)
    a, b = x[:, :n1].copy(), x[:, n1:].copy()
    ch.ProcessBlock(a)
    saved = ch.State().copy()
    ch.ProcessBlock(b)
    ch2 = P.Chain(coeffs, 0.9, channels=C)
    ch2.SetState(saved)
    np.testing.assert_array_equal(ch2.State(), saved)
    b2 = x[:, n1:].copy()
    ch2.ProcessBlock(b2)
    assert np.array_equal(b2, b)
    for c in (0, C - 1):
        want, st = O.biquad_chain_block(coeffs.ravel(), np.zeros(2 * sections), 0.9, x[c])
        assert np.array_equal(np.concatenate([a[c], b[c]]), want)
        np.testing.assert_array_equal(ch.State()[c].ravel(), st)
    with pytest.raises(Exception):
        ch2.SetState(saved[:, :1])  # too short: the reference indexes every section


def test_chain_reset(gpu):
    coeffs = stable_sections(2, 5)
    ch = P.Chain(coeffs)
    x = signals.white_noise(100, 1)
    a = x.copy()
    ch.ProcessBlock(a)
    ch.Reset()
    b = x.copy()
    ch.ProcessBlock(b)
    assert np.array_equal(a, b)


# ------------------------------------------------------------------ compressor
@pytest.mark.parametrize("cfg", [
    {},
    {"knee_db": 0.0},
    {"detector_mode": 1, "rms_window_ms": 5.0},
    {"topology": 1},
    {"topology": 1, "feedback_ratio_scale": 0},
    {"sidechain_low_cut_hz": 80.0, "sidechain_high_cut_hz": 6000.0},
    {"auto_makeup": 0, "makeup_db": 6.0, "ratio": 10.0, "threshold_db": -30.0},
], ids=lambda c: ",".join(f"{k}={v}" for k, v in c.items()) or "defaults")
def test_compressor_vs_oracle(gpu, cfg):
    C = 3
    n = 4096
    sig = [legacy_signal(n), 0.5 * signals.white_noise(n, 77), legacy_signal(n) * 0.3]
    x = np.stack(sig)
    comp = P.Compressor(48000.0, channels=C, **cfg)
    y = x.copy()
    a, b = y[:, :1500].copy(), y[:, 1500:].copy()
    comp.ProcessInPlace(a)
    comp.ProcessInPlace(b)
    got = np.concatenate([a, b], axis=1)
    for c in range(C):
        oc = O.Compressor(48000.0, **cfg)
        want = oc.process_in_place(x[c])
        assert rms(got[c], want) <= RMS_TOL, rms(got[c], want)
        assert float(np.max(np.abs(got[c] - want))) < 1e-12
        gm, om = np.array(comp.Metrics(c)), np.array(oc.metrics())
        np.testing.assert_allclose(gm, om, rtol=METRIC_RTOL, atol=0)


def test_compressor_setters_reject_out_of_range(gpu):
    """Every value a reference setter rejects (compressor.go:16-23, core.go:131-198,
    542-564) makes ad_fx_chain_set_compressor return AD_ERR_INVALID_ARGUMENT,
    and the stage keeps its previous config: the output afterwards equals an
    untouched compressor's bit for bit."""
    from algodsp import _lib
    from test_abi import BAD_COMPRESSOR_VALUES

    n = 4096
    x = np.stack([legacy_signal(n), 0.5 * signals.white_noise(n, 77)])
    comp = P.Compressor(48000.0, channels=2)
    setters = {"ratio": comp.SetRatio, "knee_db": comp.SetKnee, "attack_ms": comp.SetAttack,
               "release_ms": comp.SetRelease, "rms_window_ms": comp.SetRMSWindow,
               "threshold_db": comp.SetThreshold, "makeup_db": comp.SetMakeupGain,
               "sidechain_low_cut_hz": comp.SetSidechainLowCut, "sidechain_high_cut_hz": comp.SetSidechainHighCut}
    for field, value in BAD_COMPRESSOR_VALUES:
        with pytest.raises(_lib.ADError) as e:
            if field in setters:
                setters[field](value)
            else:
                comp._set(**{field: value})
        assert e.value.code == _lib.AD_ERR_INVALID_ARGUMENT, (field, value)
    comp.SetSidechainHighCut(6000.0)
    with pytest.raises(_lib.ADError) as e:
        comp.SetSidechainLowCut(6000.0)  # low >= high
    assert e.value.code == _lib.AD_ERR_INVALID_ARGUMENT
    comp.SetSidechainHighCut(0.0)
    a = x.copy()
    comp.ProcessInPlace(a)
    b = x.copy()
    P.Compressor(48000.0, channels=2).ProcessInPlace(b)
    assert np.array_equal(a, b)


# ------------------------------------------------------------------ Expander / Gate
@pytest.mark.parametrize("kind,cfg", [
    ("expander", {}),
    ("expander", {"knee_db": 0.0, "ratio": 6.0, "threshold_db": -20.0, "range_db": -80.0}),
    ("expander", {"topology": 1, "detector_mode": 1, "rms_window_ms": 20.0, "threshold_db": -25.0}),
    ("expander", {"sidechain_low_cut_hz": 300.0, "sidechain_high_cut_hz": 5000.0}),
    ("gate", {}),
    ("gate", {"threshold_db": -20.0, "attack_ms": 0.1, "release_ms": 1.0, "hold_ms": 10.0, "knee_db": 0.0}),
    ("gate", {"hold_ms": 0.0, "range_db": -120.0, "ratio": 100.0}),
], ids=lambda v: v if isinstance(v, str) else (",".join(f"{k}={x}" for k, x in v.items()) or "defaults"))
def test_expander_gate_vs_oracle(gpu, kind, cfg):
    """dynamics.Expander / dynamics.Gate (expander.go:358-440, gate.go:360-450)
    on a bursty signal that opens and closes them, over a call boundary: the
    output within 1e-12 RMS of the oracle and the metrics to 1e-12."""
    C, n = 3, 6000
    env = np.where((np.arange(n) // 900) % 2 == 0, 0.5, 0.003)
    x = np.stack([env * signals.white_noise(n, 60 + c) for c in range(C)])
    for engine in (P.EffectChain.ENGINE_AUTO, P.EffectChain.ENGINE_FUSED):
        ex = (P.Gate if kind == "gate" else P.Expander)(48000.0, channels=C, **cfg)
        ex.SetEngine(engine)
        a, b = x[:, :2500].copy(), x[:, 2500:].copy()
        ex.ProcessInPlace(a)
        ex.ProcessInPlace(b)
        got = np.concatenate([a, b], axis=1)
        for c in range(C):
            oc = O.Expander(48000.0, gate=kind == "gate", **cfg)
            want = oc.process_in_place(x[c])
            assert rms(got[c], want) <= RMS_TOL, rms(got[c], want)
            assert float(np.max(np.abs(got[c] - want))) < 1e-12
            np.testing.assert_allclose(np.array(ex.Metrics(c)), np.array(oc.metrics()), rtol=METRIC_RTOL, atol=0)


def test_gate_setters(gpu):
    """SetRange / SetHold re-derive the parameters without touching the state."""
    g = P.Gate(48000.0, channels=1, threshold_db=-20.0)
    o = O.Expander(48000.0, gate=True, threshold_db=-20.0)
    x = np.where(np.arange(4000) < 1500, 0.4, 0.001) * signals.white_noise(4000, 5)
    a, b = x[None, :2000].copy(), x[None, 2000:].copy()
    g.ProcessInPlace(a)
    g.SetHold(0.0)
    g.SetRange(-30.0)
    g.ProcessInPlace(b)
    want_a = o.process_in_place(x[:2000])
    assert rms(a[0], want_a) <= RMS_TOL
    assert np.all(np.abs(b[0]) <= np.abs(x[2000:]) + 1e-15)
    assert np.min(np.abs(b[0][-500:]) / np.maximum(np.abs(x[2000:][-500:]), 1e-300)) >= 10 ** (-30 / 20) - 1e-12
    with pytest.raises(Exception):
        g.SetRange(10.0)


# ------------------------------------------------------------------ Freeverb
def test_freeverb_bit_exact(gpu):
    C, n = 65, 6000
    x = np.stack([np.sin(2 * np.pi * np.arange(n) / 23) * (1 + 0.01 * c) for c in range(C)])
    x[5] = signals.white_noise(n, 5)
    rv = P.Reverb(channels=C)
    y = x.copy()
    a, b = y[:, :2345].copy(), y[:, 2345:].copy()
    rv.ProcessInPlace(a)
    rv.ProcessInPlace(b)
    got = np.concatenate([a, b], axis=1)
    for c in (0, 5, 64):
        want = O.Freeverb().process_in_place(x[c])
        assert np.array_equal(got[c], want), (c, float(np.max(np.abs(got[c] - want))))


def test_freeverb_params(gpu):
    rv = P.Reverb()
    rv.SetWet(0.5)
    rv.SetRoomSize(0.9)
    rv.SetDamp(0.2)
    rv.SetDry(0.3)
    rv.SetGain(0.02)
    x = signals.white_noise(3000, 8)
    y = x.copy()
    rv.ProcessInPlace(y)
    o = O.Freeverb()
    o.set(0.5, 0.3, 0.9, 0.2, 0.02)
    assert np.array_equal(y, o.process_in_place(x))


# ------------------------------------------------------------------ effect chain (config 5)
def test_effect_chain_config5(gpu):
    fs = 48000.0
    eq = design.config5_eq(fs)
    comp_cfg = {"auto_makeup": 0, "makeup_db": 0.0}
    verb = (0.22, 1.0, 0.72, 0.45, 0.015)
    C, n = 9, 8192
    x = np.stack([0.5 * signals.white_noise(n, 0x5EED + c) for c in range(C)])
    fx = P.EffectChain(C, eq, comp_cfg, verb, fs)
    y = x.copy()
    fx.Process(y)
    for c in (0, 4, 8):
        v = x[c].copy()
        for co, g in eq:
            v, _ = O.biquad_chain_block(np.ravel(co), np.zeros(2 * len(co)), g, v)
        v = O.Compressor(fs, **comp_cfg).process_in_place(v)
        o = O.Freeverb()
        o.set(*verb)
        v = o.process_in_place(v)
        assert rms(y[c], v) <= RMS_TOL, rms(y[c], v)


# the 256-channel bench-shape test lives in test_configs_gpu.py (test_config5_chain)


# ------------------------------------------------------------------ staged engine == fused kernels
STAGED_CASES = {
    "eq": dict(eq=True),
    "comp": dict(comp={}),
    "comp-rms-sidechain": dict(comp={"detector_mode": 1, "rms_window_ms": 3.0, "sidechain_low_cut_hz": 80.0,
                                     "sidechain_high_cut_hz": 6000.0}),
    "verb": dict(verb=True),
    "eq-verb": dict(eq=True, verb=True),
    "eq-comp": dict(eq=True, comp={"knee_db": 0.0, "auto_makeup": 1}),
    "config5": dict(eq=True, comp={"auto_makeup": 0, "makeup_db": 0.0}, verb=True),
}


@pytest.mark.parametrize("case", list(STAGED_CASES), ids=list(STAGED_CASES))
def test_staged_engine_matches_fused(gpu, case):
    """The staged engine (stage kernels over time chunks on three streams)
    computes every value with the fused kernels' operations: outputs, EQ
    state and compressor metrics are identical, over chunk boundaries
    (ad_fx_chain_set_engine chunk 256), calls that end mid-chunk, and a
    partial channel group.  The time-parallel engine (the default, fx_tp.hip)
    starts EQ segments from chained states, so it matches the fused kernels
    to the rounding noise of the EQ's low-frequency sections (the serial
    recurrence's own, ~1e-13): <= 1e-12 relative RMS on the outputs (the
    chain's parity bar), metrics to 1e-11."""
    fs = 48000.0
    cfg = STAGED_CASES[case]
    eq = design.config5_eq(fs) if cfg.get("eq") else ()
    comp = cfg.get("comp")
    verb = (0.3, 0.8, 0.8, 0.3, 0.02) if cfg.get("verb") else None
    C, n = 70, 3000
    x = np.stack([0.5 * signals.white_noise(n, 900 + c) * (1 + 0.02 * c) for c in range(C)])
    outs = {}
    # "tp": time-parallel (the default), "2": staged with the split
    # EQ/detector stage, "1": staged, one EQ pipeline per channel group, "0": fused
    engines = {"tp": P.EffectChain.ENGINE_AUTO, "2": P.EffectChain.ENGINE_STAGED,
               "1": P.EffectChain.ENGINE_STAGED_NOSPLIT, "0": P.EffectChain.ENGINE_FUSED}
    for staged in ("tp", "2", "1", "0"):
        fx = P.EffectChain(C, eq, comp, verb, fs)
        fx.SetEngine(engines[staged], 256)
        y = x.copy()
        parts = []
        for lo, hi in [(0, 700), (700, 701), (701, 3000)]:
            b = y[:, lo:hi].copy()
            fx.Process(b)
            parts.append(b)
        outs[staged] = (np.concatenate(parts, axis=1), fx)
    b = outs["0"][0]
    for k in ("2", "1"):
        a = outs[k][0]
        assert np.array_equal(a, b), (k, float(np.max(np.abs(a - b))))
    a = outs["tp"][0]
    assert rms(a, b) <= 1e-12 * max(1.0, float(np.sqrt(np.mean(b ** 2)))), rms(a, b)
    if comp is not None:
        from algodsp._lib import lib
        import ctypes as Cc

        for c in (0, 33, 69):
            m = []
            for k in ("2", "1", "0", "tp"):
                v = [Cc.c_double() for _ in range(3)]
                lib().ad_fx_chain_compressor_metrics(outs[k][1]._h, c, *[Cc.byref(t) for t in v])
                m.append([t.value for t in v])
            assert m[0] == m[1] == m[2], (c, m)
            assert np.allclose(m[3], m[2], rtol=1e-11, atol=0), (c, m)


@pytest.mark.parametrize("chunk,nsec", [(0, 5), (4096, 5), (0, 8), (4096, 8), (0, 1)])
def test_time_parallel_per_channel_eq(gpu, chunk, nsec):
    """The time-parallel engine with a coefficient table per channel
    (ad_fx_chain_set_eq per_channel = 1: one set of segment maps per channel
    in K_carry) against the fused kernels: <= 1e-12 relative RMS, over a full
    49152-sample chunk (256 segments, every scan step) and a partial one
    (chunk 0 = the engine's default), or 4096-sample chunks; 1, 5 (config 5)
    and 8 (the most a pass takes) sections with a chain gain != 1, every
    table's noise estimate under the engine's gate (<= 4.4e-13 at the highest
    channel rate; a 20 Hz highpass among them would send the chain to the
    staged engine, test_time_parallel_noise_guard); then a coefficient update
    with the same section count keeps the state (the maps are rebuilt)."""
    import ctypes as Cc

    from algodsp._lib import lib
    from algodsp.processors import section_table

    fs = 48000.0
    C, n = 70, 70000
    comp = {"auto_makeup": 0, "makeup_db": 0.0}
    verb = (0.3, 0.8, 0.8, 0.3, 0.02)
    x = np.stack([0.5 * signals.white_noise(n, 4100 + c) for c in range(C)])

    def table(scale):
        tabs = []
        for c in range(C):
            f = fs * (1.0 + scale * 0.01 * (c % 7))
            secs = [co[0] for co, _ in design.config5_eq(f)]
            secs += [design.peak(300.0, 4.0, 2.0, f), design.highpass(120.0, 0.707, f),
                     design.low_shelf(250.0, 6.0, 0.707, f)]
            if nsec == 1:
                secs = [design.highpass(40.0, 0.707, f)]
            tabs.append(section_table(np.array(secs[:nsec]), 0.8))
        return np.ascontiguousarray(np.stack(tabs))

    outs = {}
    for eng in ("tp", "0"):
        fx = P.EffectChain(C, (), comp, verb, fs)
        t = table(1.0)
        assert lib().ad_fx_chain_set_eq(fx._h, t.ctypes.data_as(Cc.POINTER(Cc.c_double)), t.shape[1], 1) == 0
        fx.SetEngine(P.EffectChain.ENGINE_AUTO if eng == "tp" else P.EffectChain.ENGINE_FUSED, chunk)
        y = x.copy()
        a, b = y[:, :66000].copy(), y[:, 66000:].copy()
        fx.Process(a)
        t = table(2.0)
        assert lib().ad_fx_chain_set_eq(fx._h, t.ctypes.data_as(Cc.POINTER(Cc.c_double)), t.shape[1], 1) == 0
        fx.Process(b)
        outs[eng] = np.concatenate([a, b], axis=1)
        assert fx.LastEngine()[0] == (P.EffectChain.ENGINE_TIME_PARALLEL if eng == "tp" else
                                      P.EffectChain.ENGINE_FUSED)
    a, b = outs["tp"], outs["0"]
    assert rms(a, b) <= 1e-12 * max(1.0, float(np.sqrt(np.mean(b ** 2)))), rms(a, b)


@pytest.mark.parametrize("fs", [96000.0, 192000.0])
@pytest.mark.parametrize("what", ["config5", "eq-only"])
def test_time_parallel_noise_guard(gpu, fs, what):
    """the time-parallel engine's distance from the serial
    recurrence grows with the EQ's round-off noise gain (tools/tp_cond.py: a
    10 Hz highpass at 192 kHz puts it near 4e-11).  A 10 Hz highpass at 96 and
    192 kHz ahead of config 5's other sections (designed at that rate): the
    noise estimate is past the gate, so AUTO (with the compressor) and an
    explicit TIME_PARALLEL request (EQ only) run the staged engine, and the
    output is within 1e-12 RMS of the oracle chain (EQ only: bit-exact)."""
    eq = [([design.highpass(10.0, 0.707, fs)], 1.0)] + design.config5_eq(fs)[1:]
    comp = {"auto_makeup": 0, "makeup_db": 0.0} if what == "config5" else None
    verb = (0.22, 1.0, 0.72, 0.45, 0.015) if what == "config5" else None
    C, n = 8, 70000
    x = np.stack([0.5 * signals.white_noise(n, 8100 + c) for c in range(C)])
    fx = P.EffectChain(C, eq, comp, verb, fs)
    fx.SetEngine(P.EffectChain.ENGINE_AUTO if what == "config5" else P.EffectChain.ENGINE_TIME_PARALLEL)
    a, b = x[:, :40000].copy(), x[:, 40000:].copy()
    fx.Process(a)
    fx.Process(b)
    y = np.concatenate([a, b], axis=1)
    engine, noise = fx.LastEngine()
    assert noise > 4.5e-13, noise
    assert engine in (P.EffectChain.ENGINE_STAGED, P.EffectChain.ENGINE_STAGED_NOSPLIT), engine
    for c in (0, 7):
        v = x[c].copy()
        for co, g in eq:
            v, _ = O.biquad_chain_block(np.ravel(co), np.zeros(2 * len(co)), g, v)
        if what == "config5":
            v = O.Compressor(fs, **comp).process_in_place(v)
            o = O.Freeverb()
            o.set(*verb)
            v = o.process_in_place(v)
            assert rms(y[c], v) <= RMS_TOL, (c, rms(y[c], v))
        else:
            assert np.array_equal(y[c], v), (c, float(np.max(np.abs(y[c] - v))))


@pytest.mark.parametrize("what", ["eq", "eq+comp", "verb", "eq+verb"])
def test_time_parallel_engine_on_request(gpu, what):
    """AD_FX_ENGINE_TIME_PARALLEL runs chains without a compressor on the
    time-parallel engine too (EQ-only, Freeverb-only -- the per-channel
    K_verb in place on the caller's buffer -- and EQ + Freeverb): outputs
    within 1e-12 relative RMS of the fused kernels and EQ end states within
    the serial recurrence's noise, over a full 49152-sample chunk and a
    partial one; then the fused engine continues from the state the
    time-parallel one left (the delay lines move back to its layout)."""
    fs = 48000.0
    eq = design.config5_eq(fs) if "eq" in what else ()
    comp = {"auto_makeup": 0, "makeup_db": 0.0} if "comp" in what else None
    verb = (0.3, 0.8, 0.8, 0.3, 0.02) if "verb" in what else None
    C, n = 70, 70000
    x = np.stack([0.5 * signals.white_noise(n, 5100 + c) for c in range(C)])
    outs, states = {}, {}
    for eng in (P.EffectChain.ENGINE_TIME_PARALLEL, P.EffectChain.ENGINE_FUSED):
        fx = P.EffectChain(C, eq, comp, verb, fs)
        fx.SetEngine(eng)
        y = x.copy()
        a, b = y[:, :66000].copy(), y[:, 66000:].copy()
        fx.Process(a)
        fx.Process(b)
        c = y[:, :3000].copy()
        fx.SetEngine(P.EffectChain.ENGINE_FUSED)
        fx.Process(c)
        outs[eng] = np.concatenate([a, b, c], axis=1)
        if eq:
            from algodsp._lib import lib
            import ctypes as Cc

            st = np.zeros(C * len(eq) * 2)
            assert lib().ad_fx_chain_eq_state(fx._h, st.ctypes.data_as(Cc.POINTER(Cc.c_double)), st.size) == 0
            states[eng] = st
    a, b = outs[P.EffectChain.ENGINE_TIME_PARALLEL], outs[P.EffectChain.ENGINE_FUSED]
    assert rms(a, b) <= 1e-12 * max(1.0, float(np.sqrt(np.mean(b ** 2)))), rms(a, b)
    if eq:
        sa, sb = states[P.EffectChain.ENGINE_TIME_PARALLEL], states[P.EffectChain.ENGINE_FUSED]
        assert np.max(np.abs(sa - sb)) <= 1e-11 * max(1.0, float(np.max(np.abs(sb)))), np.max(np.abs(sa - sb))


def test_engine_switch_growing_calls(gpu):
    """the staged and time-parallel engines share the chunk
    row stride tmax; alternating them with growing call lengths (each call
    larger than the other engine's buffers) must resize every buffer a kernel
    indexes at that stride.  Config-5 chain, engines switched between calls,
    against the fused kernels run over the same calls (the staged calls are
    bit-identical to fused, the time-parallel ones within 1e-12 relative)."""
    fs = 48000.0
    eq = design.config5_eq(fs)
    comp = {"auto_makeup": 0, "makeup_db": 0.0}
    verb = (0.3, 0.8, 0.8, 0.3, 0.02)
    C = 70
    E = P.EffectChain
    calls = [(E.ENGINE_TIME_PARALLEL, 1000), (E.ENGINE_STAGED, 16384), (E.ENGINE_TIME_PARALLEL, 20000),
             (E.ENGINE_STAGED, 30000), (E.ENGINE_STAGED_NOSPLIT, 40000), (E.ENGINE_TIME_PARALLEL, 70000),
             (E.ENGINE_STAGED, 1000)]
    n = sum(k for _, k in calls)
    x = np.stack([0.5 * signals.white_noise(n, 7100 + c) for c in range(C)])
    outs = {}
    for mode in ("switch", "fused"):
        fx = P.EffectChain(C, eq, comp, verb, fs)
        parts, t = [], 0
        for eng, k in calls:
            fx.SetEngine(eng if mode == "switch" else E.ENGINE_FUSED)
            b = x[:, t:t + k].copy()
            fx.Process(b)
            parts.append(b)
            t += k
        outs[mode] = np.concatenate(parts, axis=1)
    a, b = outs["switch"], outs["fused"]
    assert np.all(np.isfinite(a))
    assert rms(a, b) <= 1e-12 * max(1.0, float(np.sqrt(np.mean(b ** 2)))), rms(a, b)


@pytest.mark.parametrize("C,n", [(1, 5000), (3, 257), (65, 64), (2, 1)])
def test_time_parallel_small_shapes(gpu, C, n):
    """The time-parallel engine at edge shapes -- one channel, a ragged
    channel group, one segment (len <= 64), a one-sample call -- against the
    fused kernels (config-5 chain, then two more calls continuing the state)."""
    fs = 48000.0
    eq = design.config5_eq(fs)
    comp = {"auto_makeup": 0, "makeup_db": 0.0}
    verb = (0.3, 0.8, 0.8, 0.3, 0.02)
    x = np.stack([0.5 * signals.white_noise(3 * n, 6100 + c) for c in range(C)])
    outs = {}
    for eng in (P.EffectChain.ENGINE_AUTO, P.EffectChain.ENGINE_FUSED):
        fx = P.EffectChain(C, eq, comp, verb, fs)
        fx.SetEngine(eng)
        parts = []
        for k in range(3):
            b = x[:, k * n:(k + 1) * n].copy()
            fx.Process(b)
            parts.append(b)
        outs[eng] = np.concatenate(parts, axis=1)
    a, b = outs[P.EffectChain.ENGINE_AUTO], outs[P.EffectChain.ENGINE_FUSED]
    assert rms(a, b) <= 1e-12 * max(1.0, float(np.sqrt(np.mean(b ** 2)))), rms(a, b)


# ------------------------------------------------------------------ FIR
@pytest.mark.parametrize("taps", [1, 5, 31, 32, 64, 257])
def test_fir_vs_oracle(gpu, taps):
    h = signals.make_test_kernel(taps)
    C = 3
    n = 2500
    x = np.stack([signals.white_noise(n, 40 + c) for c in range(C)])
    f = P.Filter(h, channels=C)
    parts = []
    for lo, hi in [(0, 7), (7, 1200), (1200, 2500)]:  # blocks shorter and longer than the taps
        blk = x[:, lo:hi].copy()
        f.ProcessBlock(blk)
        parts.append(blk)
    got = np.concatenate(parts, axis=1)
    for c in range(C):
        of = O.Fir(h)
        want = np.concatenate([of.process_block(x[c, lo:hi]) for lo, hi in [(0, 7), (7, 1200), (1200, 2500)]])
        if taps < 32:
            assert np.array_equal(got[c], want)
        else:
            assert rms(got[c], want) <= RMS_TOL


@pytest.mark.parametrize("taps", [7, 300, 1500])
def test_fir_device_paths(gpu, taps):
    """ad_fir_process_device: out-of-place and in-place calls on device
    buffers, blocks shorter and longer than the taps (delay-line ping-pong),
    more taps than one LDS chunk (1024), and Reset ordered after the last
    call's stream."""
    import torch

    h = signals.make_test_kernel(taps)
    C, n = 4, 5000
    x = np.stack([signals.white_noise(n, 60 + c) for c in range(C)])
    cuts = [(0, 3), (3, 1700), (1700, 1710), (1710, 5000)]
    f = P.Filter(h, channels=C)
    s = torch.cuda.current_stream()
    dx = torch.from_numpy(x).cuda()
    dy = torch.zeros_like(dx)
    for k, (lo, hi) in enumerate(cuts):
        if k % 2:  # in place: dst is the source itself
            tmp = dx.clone()
            f.process_device(tmp.data_ptr() + 8 * lo, n, tmp.data_ptr() + 8 * lo, n, hi - lo, s.cuda_stream)
            dy[:, lo:hi] = tmp[:, lo:hi]
        else:
            f.process_device(dx.data_ptr() + 8 * lo, n, dy.data_ptr() + 8 * lo, n, hi - lo, s.cuda_stream)
    s.synchronize()
    got = dy.cpu().numpy()
    for c in range(C):
        of = O.Fir(h)
        want = np.concatenate([of.process_block(x[c, lo:hi]) for lo, hi in cuts])
        if taps < 32:
            assert np.array_equal(got[c], want)
        else:
            assert rms(got[c], want) <= RMS_TOL
    f.Reset()
    f.process_device(dx.data_ptr(), n, dy.data_ptr(), n, n, s.cuda_stream)
    s.synchronize()
    assert rms(dy.cpu().numpy()[1], O.Fir(h).process_block(x[1])) <= RMS_TOL


def test_fir_mixed_streams(gpu):
    """Calls on the NULL stream, a side stream and the host-buffer path, then
    Reset, then more calls: the shared delay line is ordered across streams
    (each call waits for the previous call's last operation), so the result
    equals one sequential filter."""
    import torch

    h = signals.make_test_kernel(300)
    C, n = 2, 4000
    x = np.stack([signals.white_noise(n, 90 + c) for c in range(C)])
    dx = torch.from_numpy(x).cuda()
    dy = torch.zeros_like(dx)
    side = torch.cuda.Stream()
    f = P.Filter(h, channels=C)
    for rep in range(2):
        f.process_device(dx.data_ptr(), n, dy.data_ptr(), n, 1000, 0)
        f.process_device(dx.data_ptr() + 8 * 1000, n, dy.data_ptr() + 8 * 1000, n, 1000, side.cuda_stream)
        blk = x[:, 2000:2500].copy()
        f.ProcessBlock(blk)
        f.process_device(dx.data_ptr() + 8 * 2500, n, dy.data_ptr() + 8 * 2500, n, 1500, 0)
        torch.cuda.synchronize()
        got = dy.cpu().numpy()
        got[:, 2000:2500] = blk
        for c in range(C):
            assert rms(got[c], O.Fir(h).process_block(x[c])) <= RMS_TOL
        f.process_device(dx.data_ptr(), n, dy.data_ptr(), n, 700, side.cuda_stream)
        f.Reset()


def test_fir_block_to_and_reset(gpu):
    h = signals.make_test_kernel(40)
    x = signals.white_noise(500, 3)
    f = P.Filter(h)
    dst = np.zeros_like(x)
    f.ProcessBlockTo(dst, x)
    f.Reset()
    y = x.copy()
    f.ProcessBlock(y)
    assert np.array_equal(dst, y)
    case = KATS["fir_block_vs_sample"]  # filter_test.go:91-134: block == per-sample
    g = P.Filter(case["coeffs"])
    vals = [g.ProcessSample(v) for v in case["input"]]
    of = O.Fir(case["coeffs"])
    want = [of.process_sample(v) for v in case["input"]]
    blk = np.array(case["input"], dtype=np.float64)
    P.Filter(case["coeffs"]).ProcessBlock(blk)
    np.testing.assert_allclose(vals, want, atol=case["tol"], rtol=0)
    np.testing.assert_allclose(blk, want, atol=case["tol"], rtol=0)


# ------------------------------------------------------------------ IRLB f16 decode (8(f)2)
def test_decode_f16_all_codes(gpu):
    from algodsp import irlib

    codes = np.arange(65536, dtype=np.uint16)
    got = irlib.decode_f16_gpu(codes, 1)[0]
    want = np.array([O.decode_f16(int(h)) for h in codes], dtype=np.float64)
    same = (got == want) | (np.isnan(got) & np.isnan(want))
    assert same.all(), np.flatnonzero(~same)[:10]
    # subnormal quirk (irlib.go:87): 0x0001 decodes to 2^-23, twice IEEE's 2^-24
    assert got[1] == 2.0 ** -23


@pytest.mark.parametrize("channels,frames", [(1, 65536), (2, 32768), (2, 1030), (2, 1031), (1, 7), (3, 5000)])
def test_decode_f16_layouts(gpu, channels, frames):
    """Interleaved AUDI codes -> channel-major f64: the mono/stereo vector
    kernel (4 frames per lane, scalar tail) and the generic one."""
    from algodsp import irlib

    codes = (np.arange(frames * channels, dtype=np.int64) * 7919 % 65536).astype(np.uint16)
    got = irlib.decode_f16_gpu(codes, channels)
    want = np.array([O.decode_f16(int(h)) for h in codes], dtype=np.float64).reshape(frames, channels).T
    assert np.array_equal(got, want, equal_nan=True)


def test_irlib_gpu_decode_matches_oracle(gpu):
    from algodsp import irlib

    data = irlib.DEFAULT_IRLIB.read_bytes()
    ref = O.irlib_read(data)
    got = irlib.read_irlib(gpu=True)
    assert len(got) == len(ref)
    for g, (name, fs, samples) in zip(got, ref):
        assert g["name"] == name and g["sample_rate"] == fs
        assert np.array_equal(g["samples"], samples)


# ------------------------------------------------------------------ ConvolutionReverb (a10)
@pytest.mark.parametrize("min_order", [6, 7])
def test_convolution_reverb(gpu, min_order):
    from algodsp import conv

    ir = signals.make_impulse_kernel(3000)
    rv = conv.NewConvolutionReverb(ir, min_order)
    assert rv.Latency() == 1 << min_order
    rv.SetWetDry(0.4, 0.9)
    x = signals.white_noise(5000, 21)
    blocks = [(0, 100), (100, 1337), (1337, 5000)]  # variable block lengths (convolution.go:60)
    parts = []
    for a, b in blocks:
        seg = x[a:b].copy()
        rv.ProcessInPlace(seg)
        parts.append(seg)
    got = np.concatenate(parts)
    pc = O.Partitioned(ir, min_order, 13)
    wet = np.concatenate([pc.process_block(x[a:b]) for a, b in blocks])
    want = 0.9 * x + 0.4 * wet
    assert rms(got, want) <= 1e-7


def test_eq_only_per_section_pipeline_bit_exact(gpu):
    """EQ-only chains (a12-a14) run one K_sec workgroup per section, each on
    its own chunk (fx_run_staged): bit-exact against the oracle's
    biquad.Chain.ProcessBlock (chain.go:59-70, section.go:47-53) over several
    16384-sample chunks, calls that end mid-step and mid-chunk, a partial
    channel group (130 channels), and the EQ state afterwards."""
    fs = 48000.0
    eq = design.config5_eq(fs)
    C, n = 130, 40000
    x = np.stack([0.5 * signals.white_noise(n, 1300 + c) for c in range(C)])
    fx = P.EffectChain(C, eq, None, None, fs)
    y = x.copy()
    parts = []
    for lo, hi in [(0, 17001), (17001, 17040), (17040, n)]:
        b = y[:, lo:hi].copy()
        fx.Process(b)
        parts.append(b)
    y = np.concatenate(parts, axis=1)
    engine, _ = fx.LastEngine()
    assert engine == P.EffectChain.ENGINE_STAGED, engine
    for c in (0, 63, 64, 129):
        v = x[c].copy()
        for co, g in eq:
            v, _ = O.biquad_chain_block(np.ravel(co), np.zeros(2 * len(co)), g, v)
        assert np.array_equal(y[c], v), (c, float(np.max(np.abs(y[c] - v))))


def test_eq_only_many_channels_whole_chain_bit_exact(gpu):
    """Many channels: an EQ-only chain at 4160 channels (a partial last group
    of every engine's channel grouping) runs K_lanes, bit-exact against the
    oracle's biquad.Chain.ProcessBlock (chain.go:59-70) on device buffers, on
    the first and last channels of the groups at both ends; the
    one-workgroup-per-channel-group staged kernel (ENGINE_STAGED_NOSPLIT)
    gives the same bits."""
    import torch

    fs = 48000.0
    eq = design.config5_eq(fs)
    C, n = 4160, 20000
    base = np.stack([0.5 * signals.white_noise(n, 4160 + c) for c in range(4)])
    x = np.concatenate([base] * (C // 4))
    fx = P.EffectChain(C, eq, None, None, fs)
    dx = torch.from_numpy(x).cuda()
    s = torch.cuda.current_stream()
    fx.process_device(dx.data_ptr(), n, n, s.cuda_stream)
    s.synchronize()
    y = dx.cpu().numpy()
    engine, _ = fx.LastEngine()
    assert engine == P.EffectChain.ENGINE_STAGED, engine
    for c in (0, 63, 4097, 4159):
        v = x[c].copy()
        for co, g in eq:
            v, _ = O.biquad_chain_block(np.ravel(co), np.zeros(2 * len(co)), g, v)
        assert np.array_equal(y[c], v), (c, float(np.max(np.abs(y[c] - v))))
    fx.close()
    fx = P.EffectChain(C, eq, None, None, fs)
    fx.SetEngine(P.EffectChain.ENGINE_STAGED_NOSPLIT)
    dx = torch.from_numpy(x).cuda()
    fx.process_device(dx.data_ptr(), n, n, s.cuda_stream)
    s.synchronize()
    assert np.array_equal(dx.cpu().numpy(), y)
    fx.close()


def _lane_oracle(tab, x):
    """The fx chain's section table [nsec][6] {pre_gain, b0, b1, b2, a1, a2}
    through the oracle: each section a one-section biquad.Chain with gain
    pre_gain (chain.go:59-70), states from zero."""
    v = x.copy()
    for row in np.asarray(tab):
        v, _ = O.biquad_chain_block(np.ravel(row[1:]), np.zeros(2), row[0], v)
    return v


@pytest.mark.parametrize("nsec,gains,per_channel", [(1, "one", False), (2, "first", False), (5, "first", False),
                                                   (8, "first", True), (3, "every", False), (7, "every", True)])
def test_eq_lanes_bit_exact(gpu, nsec, gains, per_channel):
    """K_lanes (fx_eq_lanes.hip): an EQ-only chain with its sections across the
    lanes of a DPP row, one launch over the call, in place on the caller's
    buffer.  Bit-exact against the oracle's biquad chain (section.go:47-53,
    chain.go:59-70) for 1 to 8 sections, a pre-gain on the first section only
    (the kernel's pre-gained input) or on every section (its per-lane
    multiply), one table or one per channel, 1 to 9 channels (partial rows of
    a wave), calls of 1, 31, 32, 33 and 5000 samples (shorter than the
    section skew, block edges, several blocks) that carry the state, and
    the EQ state read back afterwards (Chain.State, chain.go:119-128)."""
    import ctypes as Cc

    from algodsp._lib import lib
    from algodsp.processors import section_table

    rng = np.random.default_rng(77 + nsec)
    for C in (1, 4, 9):
        tabs = []
        for c in range(C if per_channel else 1):
            secs = stable_sections(nsec, 1000 * nsec + c)
            t = section_table(secs, 0.75 if gains != "one" else 1.0)
            if gains == "every":
                t[1:, 0] = rng.uniform(0.5, 1.5, nsec - 1)
            tabs.append(t)
        tab = np.ascontiguousarray(np.stack(tabs) if per_channel else tabs[0])
        fx = P.EffectChain(C, (), None, None, 48000.0)
        assert lib().ad_fx_chain_set_eq(fx._h, tab.ctypes.data_as(Cc.POINTER(Cc.c_double)), nsec,
                                        1 if per_channel else 0) == 0
        lens = [1, 31, 32, 33, 5000]
        x = np.stack([0.5 * signals.white_noise(sum(lens), 5100 + c) for c in range(C)])
        parts, lo = [], 0
        for L in lens:
            b = x[:, lo:lo + L].copy()
            fx.Process(b)
            parts.append(b)
            lo += L
        y = np.concatenate(parts, axis=1)
        assert fx.LastEngine()[0] == P.EffectChain.ENGINE_STAGED
        for c in range(C):
            want = _lane_oracle(tab[c] if per_channel else tab, x[c])
            assert np.array_equal(y[c], want), (C, c, float(np.max(np.abs(y[c] - want))))
        fx.close()


def test_eq_lanes_edge_values_bitwise(gpu):
    """K_lanes on inputs with signed zeros, subnormals, silence runs and large
    values: every output's bit pattern (including the sign of a zero result)
    equals the oracle's biquad chain (section.go:47-53), the staged one-workgroup
    kernel's and the fused kernel's; 5 sections, 6 channels, two calls."""
    fs = 48000.0
    eq = design.config5_eq(fs)
    C, n = 6, 3000
    rng = np.random.default_rng(11)
    x = 0.5 * rng.standard_normal((C, n))
    x[0, :] = -0.0                                  # negative-zero silence
    x[1, 100:900] = 0.0                             # a silence run inside noise
    x[2, ::7] = -0.0
    x[3, :] = rng.standard_normal(n) * 1e-310       # subnormal input
    x[4, :] *= 1e150                                # large values
    x[5, 1500:] = 5e-324                            # the smallest subnormal
    outs = {}
    for name, eng in [("lanes", P.EffectChain.ENGINE_AUTO), ("nosplit", P.EffectChain.ENGINE_STAGED_NOSPLIT),
                      ("fused", P.EffectChain.ENGINE_FUSED)]:
        fx = P.EffectChain(C, eq, None, None, fs)
        fx.SetEngine(eng)
        a, b = x[:, :1234].copy(), x[:, 1234:].copy()
        fx.Process(a)
        fx.Process(b)
        outs[name] = np.concatenate([a, b], axis=1)
        fx.close()
    for c in range(C):
        v = x[c].copy()
        for co, g in eq:
            v, _ = O.biquad_chain_block(np.ravel(co), np.zeros(2 * len(co)), g, v)
        for name, y in outs.items():
            assert np.array_equal(y[c].view(np.uint64), v.view(np.uint64)), (name, c)


def test_eq_lanes_device_stride_matches_staged(gpu):
    """K_lanes on a device buffer whose row stride exceeds the call (the
    samples past n stay untouched), at 256 channels x 70000 samples over two
    calls, gives the staged one-workgroup kernel's bits (ENGINE_STAGED_NOSPLIT)
    and its EQ state."""
    import ctypes as Cc

    import torch

    from algodsp._lib import lib

    fs = 48000.0
    eq = design.config5_eq(fs)
    C, n, stride = 256, 70000, 70013
    x = np.zeros((C, stride))
    x[:, :n] = np.stack([0.5 * signals.white_noise(n, 7000 + c) for c in range(C)])
    x[:, n:] = 9.0
    outs, states = [], []
    for eng in (P.EffectChain.ENGINE_AUTO, P.EffectChain.ENGINE_STAGED_NOSPLIT):
        fx = P.EffectChain(C, eq, None, None, fs)
        fx.SetEngine(eng)
        dx = torch.from_numpy(x.copy()).cuda()
        s = torch.cuda.current_stream()
        fx.process_device(dx.data_ptr(), stride, 40000, s.cuda_stream)
        fx.process_device(dx.data_ptr() + 40000 * 8, stride, n - 40000, s.cuda_stream)
        s.synchronize()
        outs.append(dx.cpu().numpy())
        st = np.zeros((C, len(eq), 2))
        assert lib().ad_fx_chain_eq_state(fx._h, st.ctypes.data_as(Cc.POINTER(Cc.c_double)), st.size) == 0
        states.append(st)
        fx.close()
    assert np.array_equal(outs[0], outs[1])
    assert np.all(outs[0][:, n:] == 9.0)
    assert np.array_equal(np.asarray(states[0]), np.asarray(states[1]))
