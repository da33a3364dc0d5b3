"""Batched effectchain graph runtime: `channels` copies of one
dsp/effectchain graph on the GPU vs the oracle's restatement of
Chain.Process (chain_process.go:11-319) channel by channel.

Tolerance: <= 1e-12 RMS (the compressor's log2/exp2 come from the GPU math
library vs the host libm, see test_dsp_gpu.py); the biquad, Freeverb, mix
and crossover paths are bit-exact.  The CPU tests cover the host-side graph
compiler (graph.go parse/order rules) and the crossover designer against the
reference's own crossover test properties (crossover_test.go:73-161).
"""
import json

import numpy as np
import pytest

import oracle_lib as O
from algodsp import design, effectchain as E, signals

RMS_TOL = 1e-12
FS = 48000.0


def rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a) - np.asarray(b)) ** 2)))


def graph(nodes, edges):
    return json.dumps({
        "nodes": [{"id": "_input", "type": "_input"}, {"id": "_output", "type": "_output"}] + nodes,
        "connections": [dict(zip(("from", "to", "fromPortIndex"), e)) for e in edges],
    })


CONFIG5 = graph(
    [{"id": "hp", "type": "filter-highpass", "params": {"freq": 40, "q": 0.707}},
     {"id": "ls", "type": "filter-lowshelf", "params": {"freq": 100, "gain": 3, "q": 0.707}},
     {"id": "pk", "type": "filter-peak", "params": {"freq": 1000, "gain": -2, "q": 1}},
     {"id": "hs", "type": "filter-highshelf", "params": {"freq": 8000, "gain": 2, "q": 0.707}},
     {"id": "lp", "type": "filter-lowpass", "params": {"freq": 18000, "q": 0.707}},
     {"id": "comp", "type": "dyn-compressor", "params": {"thresholdDB": -20, "ratio": 4}},
     {"id": "verb", "type": "reverb-freeverb", "params": {}}],
    [("_input", "hp"), ("hp", "ls"), ("ls", "pk"), ("pk", "hs"), ("hs", "lp"), ("lp", "comp"),
     ("comp", "verb"), ("verb", "_output")])

# split-freq crossover, a limiter on the low band, Freeverb on the high band,
# a dry path straight from the input, a bypassed node and a fan-in of three
BRANCHED = graph(
    [{"id": "xo", "type": "split-freq", "params": {"freqHz": 800}},
     {"id": "lim", "type": "dyn-limiter", "params": {"thresholdDB": -6, "releaseMs": 50}},
     {"id": "eq", "type": "filter-peak", "params": {"freq": 3000, "gain": 4, "q": 2}},
     {"id": "verb", "type": "reverb-freeverb", "params": {"wet": 0.5, "roomSize": 0.9}},
     {"id": "byp", "type": "dyn-compressor", "bypassed": True, "params": {"ratio": 10}},
     {"id": "comp", "type": "dyn-compressor", "params": {"thresholdDB": -30, "ratio": 3, "kneeDB": 0}}],
    [("_input", "xo"), ("xo", "lim", 0), ("xo", "eq", 1), ("eq", "verb"), ("_input", "byp"),
     ("lim", "comp"), ("comp", "_output"), ("verb", "_output"), ("byp", "_output")])


# ------------------------------------------------------------------ CPU tests
def test_parse_graph_rules():
    g = E.parse_graph(graph([{"id": "a", "type": "split"}, {"id": "", "type": "x"}, {"id": "b", "type": "sum"}],
                            [("_input", "a"), ("a", "b"), ("b", "_output"), ("a", "a"), ("a", "ghost")]))
    assert set(g.Order) == {"_input", "_output", "a", "b"}
    assert g.Order.index("_input") < g.Order.index("a") < g.Order.index("b") < g.Order.index("_output")
    assert len(g.Incoming["a"]) == 1  # self-loop and unknown target dropped
    with pytest.raises(E.GraphError):
        E.parse_graph(graph([{"id": "a", "type": "split"}, {"id": "b", "type": "split"}],
                            [("a", "b"), ("b", "a")]))
    assert E.parse_graph(json.dumps({"nodes": [{"id": "_input", "type": "_input"}]})).Order == []
    assert E.parse_graph("").Order == []
    with pytest.raises(E.GraphError):
        E.parse_graph("{not json")


def test_param_clamps():
    p = E.Params("c", "dyn-compressor", num={"thresholdDB": -90, "ratio": 500, "attackMs": 0.0})
    c = E.compressor_config(p, FS)
    assert (c.threshold_db, c.ratio, c.attack_ms, c.auto_makeup) == (-60, 100, 0.1, 0)
    lim = E.limiter_config(E.Params("l", "dyn-limiter", num={"thresholdDB": float("nan")}), FS)
    assert (lim.threshold_db, lim.ratio, lim.attack_ms, lim.knee_db) == (-0.1, 100.0, 0.1, 0.0)
    assert E.freeverb_params(E.Params("v", "reverb-freeverb", num={"roomSize": 2})) == (0.22, 1, 0.98, 0.45, 0.015)
    lp, hp = E.split_freq_sections(E.Params("x", "split-freq", num={"freqHz": 1e6}), FS)
    assert lp == design.crossover(FS * 0.5 * 0.95, 4, FS)[0]


def _chain_response(secs, f, fs):
    z = np.exp(-2j * np.pi * f / fs)
    h = 1.0
    for b0, b1, b2, a1, a2 in secs:
        h *= (b0 + b1 * z + b2 * z * z) / (1 + a1 * z + a2 * z * z)
    return h


@pytest.mark.parametrize("order", [2, 4, 8, 12])
def test_crossover_allpass_sum(order):
    """crossover_test.go:73-103: |LP + HP| = 0 dB within 0.1 dB at 20 Hz .. 20 kHz."""
    lp, hp = design.crossover(1000, order, FS)
    for f in (20, 50, 100, 200, 500, 1000, 2000, 5000, 10000, 20000):
        mag = 20 * np.log10(abs(_chain_response(lp, f, FS) + _chain_response(hp, f, FS)))
        assert abs(mag) < 0.1
    assert design.crossover(1000, 3, FS) is None and design.crossover(30000, 4, FS) is None


def test_dynamics_gate_expander_clamps():
    """gateRuntime / expanderRuntime Configure (runtime_dynamics.go:130-235)."""
    c, rng, hold = E.gate_config(E.Params("g", "dyn-gate", num={"thresholdDB": -99, "holdMs": 9000,
                                                              "rangeDB": -200}), FS)
    assert (c.threshold_db, c.ratio, c.attack_ms, rng, hold) == (-80, 10, 0.1, -120, 5000)
    assert (c.auto_makeup, c.makeup_db, c.topology, c.detector_mode) == (0, 0.0, 0, 0)
    c, rng, hold = E.expander_config(E.Params("e", "dyn-expander", num={"ratio": 0.5, "rmsWindowMs": 5000},
                                              str_={"topology": "feedback", "detector": "rms"}), FS)
    assert (c.threshold_db, c.ratio, c.attack_ms, c.rms_window_ms, rng, hold) == (-35, 1, 1, 1000, -60, 0.0)
    assert (c.topology, c.detector_mode, c.feedback_ratio_scale) == (1, 1, 0)


def test_unknown_effects_rejected():
    for t in ("chorus", "filter-moog", "dyn-lookahead", "vocoder"):
        ch = E.Chain(FS, 2, designer=design.RBJDesigner())
        with pytest.raises(E.UnknownEffect):
            ch.LoadGraph(graph([{"id": "n", "type": t}], [("_input", "n"), ("n", "_output")]))


class _Prov:
    def __init__(self, irs):
        self.irs = irs

    def GetIR(self, i):
        if 0 <= i < len(self.irs):
            return self.irs[i], 48000.0, True
        return None, 0.0, False


def test_conv_reverb_configure_semantics():
    """convReverbRuntime.Configure (runtime_misc.go:18-58): irIndex default 0,
    stereo -> (ch0 + ch1) * 0.5 over the shorter length with ch0's tail kept,
    wet default 0.35, no provider / missing IR -> no engine (pass-through)."""
    a = np.array([1.0, 2.0, 3.0, 4.0])
    b = np.array([3.0, 0.5])
    prov = _Prov([[a, b], [b]])
    k, wet = E.conv_reverb_kernel(E.Params("r", "reverb-conv"), prov)
    np.testing.assert_array_equal(k, [2.0, 1.25, 3.0, 4.0])
    assert wet == 0.35
    k, wet = E.conv_reverb_kernel(E.Params("r", "reverb-conv", num={"irIndex": 1.9, "wet": 0.8}), prov)
    np.testing.assert_array_equal(k, b)
    assert wet == 0.8
    assert E.conv_reverb_kernel(E.Params("r", "reverb-conv", num={"irIndex": 5}), prov) is None
    assert E.conv_reverb_kernel(E.Params("r", "reverb-conv"), None) is None
    with pytest.raises(ValueError):
        E.conv_reverb_kernel(E.Params("r", "reverb-conv"), _Prov([[np.zeros(0)]]))


# ------------------------------------------------------------------ GPU tests
def _run_both(g, C, n, calls=1, designer=None, scale=0.5):
    ch = E.Chain(FS, C, designer=designer or design.RBJDesigner())
    ch.LoadGraph(g)
    oracles = [O.FxGraph(ch.spec, FS) for _ in range(C)]
    worst = 0.0
    for k in range(calls):
        x = np.stack([scale * signals.white_noise(n, 1000 * k + c) for c in range(C)])
        y = x.copy()
        assert ch.Process(y)
        for c in range(C):
            want = oracles[c].process(x[c])
            worst = max(worst, rms(y[c], want))
            assert np.max(np.abs(y[c] - want)) < 1e-10
    return ch, worst


@pytest.mark.gpu
def test_config5_graph_fuses_and_matches(gpu):
    ch, err = _run_both(CONFIG5, 5, 3000, calls=2)
    assert err < RMS_TOL
    launches, buffers, lanes = ch.op_count()
    assert (launches, buffers, lanes) == (1, 1, 1)  # filter x5 -> compressor -> Freeverb in one in-place launch


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 777, 4096])
def test_branched_graph(gpu, n):
    ch, err = _run_both(BRANCHED, 3, n, calls=3)
    assert err < RMS_TOL
    assert ch.op_count()[2] >= 2  # the crossover's two bands run on their own streams


# a gate on the low band and an RMS feedback expander on the high band of a
# crossover, on a bursty signal so both open and close
DYNAMICS = graph(
    [{"id": "xo", "type": "split-freq", "params": {"freqHz": 1200}},
     {"id": "gate", "type": "dyn-gate", "params": {"thresholdDB": -30, "holdMs": 5, "releaseMs": 20}},
     {"id": "exp", "type": "dyn-expander", "params": {"thresholdDB": -28, "ratio": 4, "rangeDB": -40,
                                                      "topology": "feedback", "detector": "rms"}},
     {"id": "comp", "type": "dyn-compressor", "params": {"thresholdDB": -12}}],
    [("_input", "xo"), ("xo", "gate", 0), ("xo", "exp", 1), ("gate", "comp"), ("comp", "_output"),
     ("exp", "_output")])


@pytest.mark.gpu
def test_dynamics_gate_expander_graph(gpu):
    C, n = 4, 6000
    ch = E.Chain(FS, C, designer=design.RBJDesigner())
    ch.LoadGraph(DYNAMICS)
    oracles = [O.FxGraph(ch.spec, FS) for _ in range(C)]
    env = np.where((np.arange(n) // 700) % 2 == 0, 0.6, 0.004)
    x = np.stack([env * signals.white_noise(n, 50 + c) for c in range(C)])
    y = x.copy()
    for lo, hi in [(0, 1000), (1000, 1001), (1001, n)]:
        b = y[:, lo:hi].copy()
        assert ch.Process(b)
        y[:, lo:hi] = b
    for c in range(C):
        want = oracles[c].process(x[c])
        assert rms(y[c], want) < RMS_TOL
        assert np.max(np.abs(y[c] - want)) < 1e-10


@pytest.mark.gpu
def test_crossover_impulse_energy(gpu):
    """crossover_test.go:138-161: LP + HP of an impulse is allpass (energy 1 +- 0.001);
    the output node averages the two bands, so the sum is 2 * out."""
    g = graph([{"id": "xo", "type": "split-freq", "params": {"freqHz": 1000}}],
              [("_input", "xo"), ("xo", "_output", 0), ("xo", "_output", 1)])
    ch = E.Chain(FS, 2)
    ch.LoadGraph(g)
    x = np.zeros((2, 4096))
    x[:, 0] = 1.0
    ch.Process(x)
    e = np.sum((2 * x) ** 2, axis=1)
    assert np.all(np.abs(e - 1.0) < 0.001)


@pytest.mark.gpu
def test_unconnected_and_passthrough_nodes(gpu):
    """A node without parents processes zeros; without a designer, filter nodes
    keep the passthrough chain {B0: 1} (registry_defaults.go:152-158)."""
    g = graph([{"id": "v", "type": "reverb-freeverb"}, {"id": "f", "type": "filter-lowpass"},
               {"id": "s", "type": "sum"}],
              [("_input", "f"), ("f", "s"), ("s", "_output"), ("v", "_output")])
    ch = E.Chain(FS, 2, designer=None)
    ch.LoadGraph(g)
    x = np.stack([signals.white_noise(500, c) for c in range(2)])
    y = x.copy()
    ch.Process(y)
    oracle = O.FxGraph(ch.spec, FS)
    np.testing.assert_array_equal(y[1], oracle.process(x[1]))
    np.testing.assert_array_equal(y, x * 0.5)


@pytest.mark.gpu
def test_reset_and_device_path(gpu):
    import torch

    ch = E.Chain(FS, 4, designer=design.RBJDesigner())
    ch.LoadGraph(BRANCHED)
    x = np.stack([0.5 * signals.white_noise(2048, c) for c in range(4)])
    first = x.copy()
    ch.Process(first)
    ch.Process(x.copy())
    ch.Reset()
    again = x.copy()
    ch.Process(again)
    np.testing.assert_array_equal(again, first)
    ch.Reset()
    d = torch.zeros((4, 3000), dtype=torch.float64, device="cuda")
    d[:, :2048] = torch.from_numpy(x).cuda()
    ch.process_device(d.data_ptr(), 3000, 2048)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d[:, :2048].cpu().numpy(), first)
    assert not d[:, 2048:].any()


def _conv_graph(wet=0.4, with_dry=False, index=0):
    nodes = [{"id": "cv", "type": "reverb-conv", "params": {"irIndex": index, "wet": wet}}]
    edges = [("_input", "cv"), ("cv", "_output")]
    if with_dry:
        nodes.insert(0, {"id": "comp", "type": "dyn-compressor", "params": {"thresholdDB": -12, "ratio": 3}})
        edges = [("_input", "comp"), ("comp", "cv"), ("cv", "_output"), ("_input", "_output")]
    return graph(nodes, edges)


@pytest.mark.gpu
@pytest.mark.parametrize("with_dry", [False, True])
def test_reverb_conv_node_vs_oracle(gpu, with_dry):
    """reverb-conv nodes (runtime_misc.go:12-67) on the many-channel
    partitioned engine: Large Church (stereo, averaged to mono) at latency 128,
    calls of varying length, against the oracle's Chain.Process restatement
    (Partitioned(kernel, 7, 13) + dry/wet mix).  FFT tolerance 1e-7 RMS."""
    from algodsp import irlib

    prov = irlib.LibraryProvider()
    idx = prov.IRNames().index("Large Church")
    C = 4
    ch = E.Chain(FS, C, designer=design.RBJDesigner(), ir_provider=prov)
    ch.LoadGraph(_conv_graph(0.4, with_dry, idx))
    kinds = [d["type"] for d in ch.spec]
    assert "conv" in kinds
    oracles = [O.FxGraph(ch.spec, FS) for _ in range(C)]
    for k, n in enumerate([128, 4096, 1000, 20011, 128, 7]):
        x = np.stack([0.5 * signals.white_noise(n, 500 * k + c) for c in range(C)])
        y = x.copy()
        assert ch.Process(y)
        for c in range(C):
            want = oracles[c].process(x[c])
            assert rms(y[c], want) < 1e-7
            assert np.max(np.abs(y[c] - want)) < 1e-9
    # without a provider the node passes the block through (no engine)
    ch2 = E.Chain(FS, 2)
    ch2.LoadGraph(_conv_graph())
    x = signals.white_noise(300, 1).reshape(1, -1).repeat(2, 0).copy()
    y = x.copy()
    assert ch2.Process(y)
    np.testing.assert_array_equal(y, x)


@pytest.mark.gpu
@pytest.mark.parametrize("field,value", [("ratio", 100.5), ("attack_ms", 0.05), ("release_ms", 5001.0),
                                         ("rms_window_ms", 0.5), ("makeup_db", float("nan")),
                                         ("sidechain_low_cut_hz", 30000.0)])
def test_graph_compressor_node_rejects_setter_ranges(gpu, field, value):
    """A COMPRESSOR node whose config a reference setter would reject
    (compressor.go:16-23, core.go:131-198, 542-564) fails ad_fx_graph_create
    with AD_ERR_INVALID_ARGUMENT, as the node's Configure would fail; the same
    graph with an in-range config builds."""
    import ctypes as C

    from algodsp import _lib

    def build(cfg):
        nodes = (E._Node * 3)()
        par = [(C.c_int32 * 1)(0), (C.c_int32 * 1)(1)]
        ports = [(C.c_int32 * 1)(0), (C.c_int32 * 1)(0)]
        nodes[0].type = 0  # AD_FXN_INPUT
        nodes[1].type = 5  # AD_FXN_COMPRESSOR
        nodes[1].n_parents, nodes[1].parents, nodes[1].parent_ports = 1, par[0], ports[0]
        nodes[1].comp = C.pointer(cfg)
        nodes[2].type = 1  # AD_FXN_OUTPUT
        nodes[2].n_parents, nodes[2].parents, nodes[2].parent_ports = 1, par[1], ports[1]
        h = C.c_void_p()
        rc = _lib.lib().ad_fx_graph_create(C.cast(nodes, C.c_void_p), 3, 4, 0, C.byref(h))
        if rc == _lib.AD_OK:
            _lib.lib().ad_fx_graph_destroy(h)
        return rc

    good = _lib.CompressorConfig()
    _lib.lib().ad_compressor_default_config(C.byref(good), FS)
    assert build(good) == _lib.AD_OK
    bad = _lib.CompressorConfig()
    _lib.lib().ad_compressor_default_config(C.byref(bad), FS)
    setattr(bad, field, value)
    assert build(bad) == _lib.AD_ERR_INVALID_ARGUMENT


# the reference's own integration graphs (integration_test.go), at its 44.1 kHz;
# its "threshold" key is not one the dynamics runtime reads (runtime_dynamics.go:21
# reads thresholdDB), so the default applies on both sides
def _ref_graph_run(g, x, fs=44100.0, calls=(0, None)):
    ch = E.Chain(fs, x.shape[0], designer=design.RBJDesigner())
    ch.LoadGraph(g)
    oracles = [O.FxGraph(ch.spec, fs) for _ in range(x.shape[0])]
    y = x.copy()
    assert ch.Process(y)
    for c in range(x.shape[0]):
        want = oracles[c].process(x[c])
        assert np.all(np.isfinite(y[c]))
        assert rms(y[c], want) < RMS_TOL
        assert np.max(np.abs(y[c] - want)) < 1e-10
    return y


@pytest.mark.gpu
def test_reference_integration_linear(gpu):
    """TestChainIntegrationLinear (integration_test.go:153-193): _input ->
    dyn-compressor (ratio 4, attack 10 ms, release 100 ms) -> _output on 512
    samples of 0.8 sin(2 pi 1000 i / 44100): finite, and the oracle's."""
    g = graph([{"id": "comp", "type": "dyn-compressor",
                "params": {"threshold": -20.0, "ratio": 4.0, "attackMs": 10.0, "releaseMs": 100.0}}],
              [("_input", "comp"), ("comp", "_output")])
    i = np.arange(512)
    _ref_graph_run(g, np.stack([0.8 * np.sin(2 * np.pi * 1000 * i / 44100.0)] * 2))


@pytest.mark.gpu
def test_reference_integration_split_freq(gpu):
    """TestChainIntegrationSplitFreq (integration_test.go:196-248): a 1 kHz
    split-freq, a compressor per band, summed: finite, and the oracle's."""
    p = {"threshold": -10.0, "ratio": 2.0, "attackMs": 5.0, "releaseMs": 50.0}
    g = graph([{"id": "xo", "type": "split-freq", "params": {"freqHz": 1000.0}},
               {"id": "low_comp", "type": "dyn-compressor", "params": p},
               {"id": "hi_comp", "type": "dyn-compressor", "params": p},
               {"id": "sum", "type": "sum"}],
              [("_input", "xo"), ("xo", "low_comp", 0), ("xo", "hi_comp", 1), ("low_comp", "sum"),
               ("hi_comp", "sum"), ("sum", "_output")])
    i = np.arange(512)
    x = 0.5 * np.sin(2 * np.pi * 200 * i / 44100.0) + 0.3 * np.sin(2 * np.pi * 5000 * i / 44100.0)
    _ref_graph_run(g, np.stack([x, x]))
