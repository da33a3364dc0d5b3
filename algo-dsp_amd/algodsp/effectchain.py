"""Batched effectchain runtime: `channels` copies of one
dsp/effectchain graph processed together on the GPU.

Mirrors the reference's Chain API (dsp/effectchain/chain.go, chain_process.go):

    ch = Chain(48000.0, channels=256)            # effectchain.New(ctx, DefaultRegistry(...))
    ch.LoadGraph(json_graph)                      # chain.go LoadGraph: parse + Kahn order + Configure
    ch.Process(block)                             # chain_process.go:11-33, block [channels][n] in place

The host side here is the graph compiler: JSON parsing and the topological
order restate graph.go:57-165; each node's parameters are clamped exactly as
its runtime's Configure does (runtime_dynamics.go, runtime_filter_pitch_reverb.go,
chain_process.go:177-227 for split-freq).  The compiled node list goes to
ad_fx_graph_create (include/algodsp.h), which runs every node on the GPU;
there is no CPU path.  Node types outside {filter*, dyn-compressor,
dyn-limiter, dyn-gate, dyn-expander, reverb-freeverb, split-freq, split, sum,
_input, _output} raise
UnknownEffect (the GPU runtime's ErrUnknownEffect).
"""
from __future__ import annotations

import ctypes as C
import json
import math

import numpy as np

from . import design
from ._lib import CompressorConfig, check, lib, ptr
from .processors import section_table

INPUT_NODE_ID = "_input"  # graph.go:10-13
OUTPUT_NODE_ID = "_output"
NODE_TYPE_SPLIT_FREQ = "split-freq"

FXN_INPUT, FXN_OUTPUT, FXN_PASS, FXN_SPLIT_FREQ, FXN_BIQUAD, FXN_COMPRESSOR, FXN_FREEVERB, FXN_CONV_REVERB = range(8)
MAX_PARENTS = 8

FILTER_TYPES = ("filter", "filter-lowpass", "filter-highpass", "filter-bandpass", "filter-notch",
                "filter-allpass", "filter-peak", "filter-lowshelf", "filter-highshelf")  # registry_defaults.go:141-151


class UnknownEffect(ValueError):
    """effectchain.ErrUnknownEffect (chain.go:11) for node types the GPU runtime lacks."""


class GraphError(ValueError):
    """parseGraph errors (graph.go:63-66, 157-159)."""


class _Node(C.Structure):
    _fields_ = [("type", C.c_int), ("bypassed", C.c_int), ("n_parents", C.c_int),
                ("parents", C.POINTER(C.c_int32)), ("parent_ports", C.POINTER(C.c_int32)),
                ("sections", C.POINTER(C.c_double)), ("nsec", C.c_int),
                ("sections2", C.POINTER(C.c_double)), ("nsec2", C.c_int),
                ("comp", C.POINTER(CompressorConfig)), ("verb", C.c_double * 5),
                ("dyn_mode", C.c_int), ("dyn_range_db", C.c_double), ("dyn_hold_ms", C.c_double),
                ("ir", C.POINTER(C.c_double)), ("ir_len", C.c_int64), ("conv_min_order", C.c_int),
                ("conv_wet", C.c_double), ("conv_dry", C.c_double)]


def clamp(v, lo, hi):  # core.Clamp
    return lo if v < lo else (hi if v > hi else v)


class Params:
    """effectchain.Params (params.go): ID, Type, Bypassed, Num, Str."""

    def __init__(self, id_, type_, bypassed=False, num=None, str_=None):
        self.ID, self.Type, self.Bypassed = id_, type_, bool(bypassed)
        self.Num, self.Str = num or {}, str_ or {}

    def GetNum(self, key, default):  # params.go:15-27
        v = self.Num.get(key)
        if v is None or math.isnan(v) or math.isinf(v):
            return default
        return v


def _parse_params(raw):  # parseNodeParams graph.go:169-199
    num, st = {}, {}
    if isinstance(raw, dict):
        for k, v in raw.items():
            if isinstance(v, bool):
                num[k] = 1.0 if v else 0.0
            elif isinstance(v, (int, float)):
                num[k] = float(v)
            elif isinstance(v, str):
                st[k] = v
    return num, st


class CompiledGraph:
    def __init__(self, nodes, incoming, outgoing, order):
        self.Nodes, self.Incoming, self.Outgoing, self.Order = nodes, incoming, outgoing, order


def parse_graph(raw: str) -> CompiledGraph:
    """parseGraph (graph.go:57-165): nodes without id/type are dropped, a graph
    without _input/_output is empty, edges to unknown nodes and self-loops are
    dropped, Kahn's algorithm orders the nodes (any topological order gives
    the same result), a cycle is an error."""
    if raw == "":
        return CompiledGraph({}, {}, {}, [])
    try:
        state = json.loads(raw)
    except json.JSONDecodeError as e:
        raise GraphError(f"invalid chain graph json: {e}") from e
    nodes = {}
    for n in state.get("nodes") or []:
        if not n.get("id") or not n.get("type"):
            continue
        num, st = _parse_params(n.get("params"))
        nodes[n["id"]] = Params(n["id"], n["type"], n.get("bypassed", False), num, st)
    if INPUT_NODE_ID not in nodes or OUTPUT_NODE_ID not in nodes:
        return CompiledGraph({}, {}, {}, [])
    incoming = {k: [] for k in nodes}
    outgoing = {k: [] for k in nodes}
    indeg = {k: 0 for k in nodes}
    for c in state.get("connections") or []:
        f, t = c.get("from", ""), c.get("to", "")
        if not f or not t or f == t or f not in nodes or t not in nodes:
            continue
        e = (f, t, max(0, int(c.get("fromPortIndex", 0) or 0)), max(0, int(c.get("toPortIndex", 0) or 0)))
        outgoing[f].append(e)
        incoming[t].append(e)
        indeg[t] += 1
    queue = [k for k in nodes if indeg[k] == 0]
    order = []
    while queue:
        k = queue.pop(0)
        order.append(k)
        for e in outgoing[k]:
            indeg[e[1]] -= 1
            if indeg[e[1]] == 0:
                queue.append(e[1])
    if len(order) != len(nodes):
        raise GraphError("invalid chain graph: contains cycle")
    return CompiledGraph(nodes, incoming, outgoing, order)


# ---- node configuration (each runtime's Configure) -------------------------
def compressor_config(p: Params, fs: float) -> CompressorConfig:
    """compressorRuntime.Configure (runtime_dynamics.go:15-57) on NewCompressor defaults."""
    c = CompressorConfig()
    lib().ad_compressor_default_config(C.byref(c), float(fs))
    c.threshold_db = clamp(p.GetNum("thresholdDB", -20), -60, 0)
    c.ratio = clamp(p.GetNum("ratio", 4), 1, 100)
    c.knee_db = clamp(p.GetNum("kneeDB", 6), 0, 24)
    c.attack_ms = clamp(p.GetNum("attackMs", 10), 0.1, 1000)
    c.release_ms = clamp(p.GetNum("releaseMs", 100), 1, 5000)
    c.auto_makeup = 0
    c.makeup_db = clamp(p.GetNum("makeupGainDB", 0), 0, 24)
    return c


def limiter_config(p: Params, fs: float) -> CompressorConfig:
    """NewLimiter (dynamics/limiter.go:11-44: ratio 100, attack 0.1 ms, hard
    knee, no makeup) + limiterRuntime.Configure (runtime_dynamics.go:67-85)."""
    c = CompressorConfig()
    lib().ad_compressor_default_config(C.byref(c), float(fs))
    c.ratio, c.attack_ms, c.knee_db, c.auto_makeup, c.makeup_db = 100.0, 0.1, 0.0, 0, 0.0
    c.threshold_db = clamp(p.GetNum("thresholdDB", -0.1), -24, 0)
    c.release_ms = clamp(p.GetNum("releaseMs", 100), 1, 5000)
    return c


def gate_config(p: Params, fs: float):
    """gateRuntime.Configure (runtime_dynamics.go:130-170) on NewGate defaults:
    (config, range dB, hold ms).  Topology and detector stay NewGate's
    (feed-forward, peak)."""
    c = CompressorConfig()
    lib().ad_compressor_default_config(C.byref(c), float(fs))
    c.threshold_db = clamp(p.GetNum("thresholdDB", -40), -80, 0)
    c.ratio = clamp(p.GetNum("ratio", 10), 1, 100)
    c.knee_db = clamp(p.GetNum("kneeDB", 6), 0, 24)
    c.attack_ms = clamp(p.GetNum("attackMs", 0.1), 0.1, 1000)
    c.release_ms = clamp(p.GetNum("releaseMs", 100), 1, 5000)
    c.auto_makeup, c.makeup_db, c.feedback_ratio_scale = 0, 0.0, 0
    return c, clamp(p.GetNum("rangeDB", -80), -120, 0), clamp(p.GetNum("holdMs", 50), 0, 5000)


def expander_config(p: Params, fs: float):
    """expanderRuntime.Configure (runtime_dynamics.go:180-235) on NewExpander
    defaults: (config, range dB, hold ms = 0)."""
    c = CompressorConfig()
    lib().ad_compressor_default_config(C.byref(c), float(fs))
    c.threshold_db = clamp(p.GetNum("thresholdDB", -35), -80, 0)
    c.ratio = clamp(p.GetNum("ratio", 2), 1, 100)
    c.knee_db = clamp(p.GetNum("kneeDB", 6), 0, 24)
    c.attack_ms = clamp(p.GetNum("attackMs", 1), 0.1, 1000)
    c.release_ms = clamp(p.GetNum("releaseMs", 100), 1, 5000)
    c.topology = 1 if p.Str.get("topology", "") == "feedback" else 0  # normalize.go:185-194
    c.detector_mode = 1 if p.Str.get("detector", "") == "rms" else 0  # normalize.go:196-205
    c.rms_window_ms = clamp(p.GetNum("rmsWindowMs", 30), 1, 1000)
    c.auto_makeup, c.makeup_db, c.feedback_ratio_scale = 0, 0.0, 0
    return c, clamp(p.GetNum("rangeDB", -60), -120, 0), 0.0


def freeverb_params(p: Params):
    """freeverbRuntime.Configure (runtime_filter_pitch_reverb.go:330-341)."""
    return (clamp(p.GetNum("wet", 0.22), 0, 1.5), clamp(p.GetNum("dry", 1), 0, 1.5),
            clamp(p.GetNum("roomSize", 0.72), 0, 0.98), clamp(p.GetNum("damp", 0.45), 0, 0.99),
            clamp(p.GetNum("gain", 0.015), 0, 0.1))


def _filter_kind(node_type, raw):  # normalizeFilterKind normalize.go:42-86
    k = raw.strip().lower()
    if k in ("bandeq", "band-eq", "bandeqpeak", "bell", "bandbell"):
        k = "peak"
    if raw.strip():
        return k if k in ("highpass", "lowpass", "bandpass", "notch", "allpass", "peak", "highshelf",
                          "lowshelf") else "peak"
    return {"filter-highpass": "highpass", "filter-bandpass": "bandpass", "filter-notch": "notch",
            "filter-allpass": "allpass", "filter-peak": "peak", "filter-lowshelf": "lowshelf",
            "filter-highshelf": "highshelf"}.get(node_type, "lowpass")


def filter_chain(p: Params, fs: float, designer):
    """filterRuntime.Configure (runtime_filter_pitch_reverb.go:40-176) -> (sections, gain).
    Without a designer the runtime keeps its passthrough chain {B0: 1}."""
    fam = (p.Str.get("family", "") or "").strip().lower() or "rbj"
    if p.Type == "filter-moog" or fam == "moog":  # normalizeFilterFamily: the moog ladder, designer or not
        raise UnknownEffect("filter-moog is not run by the GPU graph runtime")
    if designer is None:
        return [(1.0, 0.0, 0.0, 0.0, 0.0)], 1.0
    kind = _filter_kind(p.Type, p.Str.get("kind", ""))
    freq = clamp(p.GetNum("freq", 1200), 20, fs * 0.49)
    gain_db = clamp(p.GetNum("gain", 0), -24, 24)
    shape = clamp(p.GetNum("q", 0.707), 0.2, 8)
    fam = designer.NormalizeFamilyForType(kind, designer.NormalizeFamily(fam))
    order = designer.NormalizeOrder(kind, fam, int(round(p.GetNum("order", 2))))
    shape = designer.ClampShape(kind, fam, freq, fs, shape)
    try:
        return designer.BuildChain(fam, kind, order, freq, gain_db, shape, fs)
    except NotImplementedError as e:
        raise UnknownEffect(str(e)) from e


def split_freq_sections(p: Params, fs: float):
    """processSplitFreqNode (chain_process.go:177-227): LR4 at clamp(freqHz).
    crossover.New failing leaves both bands a copy (identity sections)."""
    freq = p.GetNum("freqHz", 1200)
    freq = max(freq, 20.0)
    max_freq = max(20.0, fs * 0.5 * 0.95)
    freq = min(freq, max_freq)
    xo = design.crossover(freq, 4, fs)
    if xo is None:
        ident = [(1.0, 0.0, 0.0, 0.0, 0.0)]
        return ident, ident
    return xo


def conv_reverb_kernel(p: Params, provider):
    """convReverbRuntime.Configure (runtime_misc.go:18-58): the IR at irIndex
    (default 0), stereo averaged to mono ((ch0 + ch1) * 0.5 over the shorter
    length, ch0's tail kept), and the wet level (default 0.35; dry 1.0).
    None when there is no provider or no such IR: the runtime then has no
    engine and Process leaves the block untouched (a pass-through node)."""
    ir_index = int(p.GetNum("irIndex", 0))
    wet = p.GetNum("wet", 0.35)
    if provider is None:
        return None
    samples, _fs, ok = provider.GetIR(ir_index)
    if not ok or samples is None or len(samples) == 0:
        return None
    ch0 = np.asarray(samples[0], dtype=np.float64)
    kernel = ch0.copy()
    if len(samples) > 1:
        ch1 = np.asarray(samples[1], dtype=np.float64)
        n = min(ch0.size, ch1.size)
        kernel[:n] = (ch0[:n] + ch1[:n]) * 0.5
    if kernel.size == 0:  # NewConvolutionReverb: "reverb: empty impulse response kernel"
        raise ValueError("effectchain: create convolution reverb: reverb: empty impulse response kernel")
    return kernel, wet


class Chain:
    """effectchain.Chain for `channels` independent channels of one graph.
    `ir_provider` is effectchain.WithIRProvider's IRProvider (GetIR(index) ->
    (samples [ch][n], sample_rate, ok)) for reverb-conv nodes."""

    def __init__(self, sample_rate: float = 48000.0, channels: int = 1, designer=None, device: int = 0,
                 ir_provider=None):
        self.sample_rate = float(sample_rate)
        self.channels = int(channels)
        self.designer = designer
        self.ir_provider = ir_provider
        self.device = int(device)
        self.graph = CompiledGraph({}, {}, {}, [])
        self._h = None
        self._keep = []
        # the compiled nodes in execution order, as plain data (node id, kind,
        # bypassed, parents [(index, port)] and the designed parameters):
        # what the GPU runs, and what the parity tests hand to the oracle
        self.spec = []

    def HasGraph(self) -> bool:
        return bool(self.graph.Order)

    def _free(self):
        if self._h:
            lib().ad_fx_graph_destroy(self._h)
            self._h = None

    def LoadGraph(self, json_graph: str) -> None:
        g = parse_graph(json_graph)
        self._free()
        self.graph = g
        if not g.Order:
            return
        order = [INPUT_NODE_ID] + [k for k in g.Order if k != INPUT_NODE_ID]
        idx = {k: i for i, k in enumerate(order)}
        fs = self.sample_rate
        nodes = (_Node * len(order))()
        keep = []
        spec = []
        for i, k in enumerate(order):
            p = g.Nodes[k]
            d = nodes[i]
            # mainParents (splitMainAndSideParents, chain_process.go:120-134): the
            # GPU runtime has no sidechain node types, so every edge is a main edge
            par = [(idx[e[0]], e[2]) for e in g.Incoming[k]]
            if len(par) > MAX_PARENTS:
                raise UnknownEffect(f"node {k}: more than {MAX_PARENTS} parents")
            if par:
                pa = (C.c_int32 * len(par))(*[q[0] for q in par])
                po = (C.c_int32 * len(par))(*[q[1] if g.Nodes[order[q[0]]].Type == NODE_TYPE_SPLIT_FREQ and q[1] == 1
                                              else 0 for q in par])
                keep += [pa, po]
                d.parents, d.parent_ports = C.cast(pa, C.POINTER(C.c_int32)), C.cast(po, C.POINTER(C.c_int32))
            d.n_parents = len(par)
            d.bypassed = 1 if p.Bypassed else 0
            t = p.Type
            sd = {"id": k, "bypassed": bool(p.Bypassed),
                  "parents": [(q[0], 1 if g.Nodes[order[q[0]]].Type == NODE_TYPE_SPLIT_FREQ and q[1] == 1 else 0)
                              for q in par]}
            if k == INPUT_NODE_ID:
                d.type = FXN_INPUT
                sd["type"] = "input"
            elif k == OUTPUT_NODE_ID:
                d.type = FXN_OUTPUT
                sd["type"] = "output"
            elif t == NODE_TYPE_SPLIT_FREQ:
                d.type = FXN_SPLIT_FREQ
                lp, hp = split_freq_sections(p, fs)
                sd.update(type="split", sections=lp, sections2=hp)
                a, b = section_table(np.asarray(lp)), section_table(np.asarray(hp))
                keep += [a, b]
                d.sections, d.nsec = ptr(a), a.shape[0]
                d.sections2, d.nsec2 = ptr(b), b.shape[0]
            elif t in ("split", "sum", INPUT_NODE_ID, OUTPUT_NODE_ID):
                d.type = FXN_PASS
                sd["type"] = "pass"
            elif t in FILTER_TYPES or t == "filter-moog":
                d.type = FXN_BIQUAD
                sd.update(type="biquad", sections=([], 1.0))
                if not p.Bypassed:
                    secs, gain = filter_chain(p, fs, self.designer)
                    sd["sections"] = (list(secs), gain)
                    a = section_table(np.asarray(secs, dtype=np.float64), gain)
                    keep.append(a)
                    d.sections, d.nsec = ptr(a), a.shape[0]
            elif t in ("dyn-compressor", "dyn-limiter"):
                d.type = FXN_COMPRESSOR
                cfg = compressor_config(p, fs) if t == "dyn-compressor" else limiter_config(p, fs)
                keep.append(cfg)
                d.comp = C.pointer(cfg)
                sd.update(type="comp", comp={f: getattr(cfg, f) for f, _ in cfg._fields_})
            elif t in ("dyn-gate", "dyn-expander"):
                d.type = FXN_COMPRESSOR
                gate = t == "dyn-gate"
                cfg, rng, hold = gate_config(p, fs) if gate else expander_config(p, fs)
                keep.append(cfg)
                d.comp = C.pointer(cfg)
                d.dyn_mode, d.dyn_range_db, d.dyn_hold_ms = (2 if gate else 1), rng, hold
                sd.update(type="comp", comp={f: getattr(cfg, f) for f, _ in cfg._fields_},
                          expander=dict(gate=gate, range_db=rng, hold_ms=hold))
            elif t == "reverb-freeverb":
                d.type = FXN_FREEVERB
                for j, v in enumerate(freeverb_params(p)):
                    d.verb[j] = v
                sd.update(type="verb", verb=freeverb_params(p))
            elif t == "reverb-conv":
                kw = None if p.Bypassed else conv_reverb_kernel(p, self.ir_provider)
                if kw is None:
                    d.type = FXN_PASS  # no engine: Process is a no-op (runtime_misc.go:61-64)
                    sd["type"] = "pass"
                else:
                    kern, wet = kw
                    kern = np.ascontiguousarray(kern)
                    keep.append(kern)
                    d.type = FXN_CONV_REVERB
                    d.ir, d.ir_len = ptr(kern), kern.size
                    d.conv_min_order, d.conv_wet, d.conv_dry = 7, wet, 1.0  # NewConvolutionReverb(kernel, 7)
                    sd.update(type="conv", kernel=kern, min_order=7, wet=wet, dry=1.0)
            else:
                raise UnknownEffect(f"effect type {t!r} is not run by the GPU graph runtime")
            spec.append(sd)
        h = C.c_void_p()
        check(lib().ad_fx_graph_create(C.cast(nodes, C.c_void_p), len(order), self.channels, self.device, C.byref(h)))
        self._h = h
        self._keep = keep
        self.spec = spec

    def op_count(self):
        """(device ops per call, buffers, streams) of the compiled graph."""
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        check(lib().ad_fx_graph_op_count(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def Process(self, block) -> bool:
        """chain_process.go:11-33; block [channels][n] float64, in place.
        False (block untouched) without a valid graph."""
        if not isinstance(block, np.ndarray) or block.dtype != np.float64 or not block.flags.c_contiguous:
            raise TypeError("block must be a C-contiguous float64 numpy array")
        b = block.reshape(1, -1) if block.ndim == 1 else block
        if b.shape[0] != self.channels:
            raise ValueError(f"block has {b.shape[0]} channels, chain has {self.channels}")
        if b.shape[1] == 0:
            return True
        if not self._h:
            return False
        check(lib().ad_fx_graph_process(self._h, ptr(b), b.shape[1]))
        return True

    def process_device(self, d_buf: int, stride: int, n: int, stream: int = 0) -> bool:
        if not self._h:
            return False
        check(lib().ad_fx_graph_process_device(self._h, C.c_void_p(d_buf), int(stride), int(n),
                                               C.c_void_p(stream)))
        return True

    def Reset(self) -> None:
        if self._h:
            check(lib().ad_fx_graph_reset(self._h))

    def close(self):
        self._free()

    def __del__(self):
        try:
            self._free()
        except Exception:
            pass


def _graph_json(nodes, edges):
    return json.dumps({
        "nodes": [{"id": INPUT_NODE_ID, "type": INPUT_NODE_ID}, {"id": OUTPUT_NODE_ID, "type": OUTPUT_NODE_ID}] + nodes,
        "connections": [dict(zip(("from", "to", "fromPortIndex"), e)) for e in edges],
    })


# Example graphs (bench.py --workload fx --graph ...).  config5: BASELINE
# config 5 as an effectchain graph (fuses into one launch); branched: an LR4
# split-freq crossover, a limiter -> compressor low band, an EQ -> Freeverb
# high band and a dry path, averaged at the output.
EXAMPLE_GRAPHS = {
    "config5": _graph_json(
        [{"id": "hp", "type": "filter-highpass", "params": {"freq": 40, "q": 0.707}},
         {"id": "ls", "type": "filter-lowshelf", "params": {"freq": 100, "gain": 3, "q": 0.707}},
         {"id": "pk", "type": "filter-peak", "params": {"freq": 1000, "gain": -2, "q": 1}},
         {"id": "hs", "type": "filter-highshelf", "params": {"freq": 8000, "gain": 2, "q": 0.707}},
         {"id": "lp", "type": "filter-lowpass", "params": {"freq": 18000, "q": 0.707}},
         {"id": "comp", "type": "dyn-compressor", "params": {"thresholdDB": -20, "ratio": 4}},
         {"id": "verb", "type": "reverb-freeverb", "params": {}}],
        [(INPUT_NODE_ID, "hp"), ("hp", "ls"), ("ls", "pk"), ("pk", "hs"), ("hs", "lp"), ("lp", "comp"),
         ("comp", "verb"), ("verb", OUTPUT_NODE_ID)]),
    "branched": _graph_json(
        [{"id": "xo", "type": "split-freq", "params": {"freqHz": 800}},
         {"id": "lim", "type": "dyn-limiter", "params": {"thresholdDB": -6, "releaseMs": 50}},
         {"id": "eq", "type": "filter-peak", "params": {"freq": 3000, "gain": 4, "q": 2}},
         {"id": "verb", "type": "reverb-freeverb", "params": {"wet": 0.5, "roomSize": 0.9}},
         {"id": "comp", "type": "dyn-compressor", "params": {"thresholdDB": -30, "ratio": 3, "kneeDB": 0}}],
        [(INPUT_NODE_ID, "xo"), ("xo", "lim", 0), ("xo", "eq", 1), ("eq", "verb"), (INPUT_NODE_ID, OUTPUT_NODE_ID),
         ("lim", "comp"), ("comp", OUTPUT_NODE_ID), ("verb", OUTPUT_NODE_ID)]),
}
