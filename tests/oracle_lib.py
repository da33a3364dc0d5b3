"""ctypes wrapper of oracle/liboracle.so — the CPU parity checker.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product path.
"""
from __future__ import annotations

import ctypes as C
import pathlib
import subprocess

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "liboracle.so"

dp = C.POINTER(C.c_double)
fp = C.POINTER(C.c_float)
i64 = C.c_int64
vp = C.c_void_p

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not ORACLE_LIB.exists():
            build()
        L = C.CDLL(str(ORACLE_LIB))
        sig = {
            "or_fft": (C.c_int, [vp, vp, i64, C.c_int]),
            "or_direct": (C.c_int, [dp, i64, dp, i64, dp]),
            "or_direct_circular": (C.c_int, [dp, i64, dp, i64, dp]),
            "or_direct_ld": (None, [dp, i64, dp, i64, dp]),
            "or_convolve": (C.c_int, [dp, i64, dp, i64, C.c_int, dp, i64, C.POINTER(i64)]),
            "or_ola_new": (C.c_int, [dp, i64, i64, C.POINTER(vp)]),
            "or_ola_process": (C.c_int, [vp, dp, i64, dp]),
            "or_ola_block_size": (i64, [vp]),
            "or_ola_fft_size": (i64, [vp]),
            "or_ola_free": (None, [vp]),
            "or_ola_convolve": (C.c_int, [dp, i64, dp, i64, dp]),
            "or_ols_new": (C.c_int, [dp, i64, i64, C.POINTER(vp)]),
            "or_ols_process": (C.c_int, [vp, dp, i64, dp]),
            "or_ols_fft_size": (i64, [vp]),
            "or_ols_step_size": (i64, [vp]),
            "or_ols_free": (None, [vp]),
            "or_sols_new": (C.c_int, [dp, i64, i64, C.POINTER(vp)]),
            "or_sola_new": (C.c_int, [dp, i64, i64, C.POINTER(vp)]),
            "or_stream_process_block": (C.c_int, [vp, dp, i64, dp, i64]),
            "or_stream_reset": (None, [vp]),
            "or_stream_fft_size": (i64, [vp]),
            "or_stream_free": (None, [vp]),
            "or_stream32_new": (C.c_int, [C.c_int, fp, i64, i64, C.POINTER(vp)]),
            "or_stream32_process_block": (C.c_int, [vp, fp, fp, i64]),
            "or_stream32_fft_size": (i64, [vp]),
            "or_stream32_free": (None, [vp]),
            "or_pc32_new": (C.c_int, [fp, i64, C.c_int, C.c_int, C.POINTER(vp)]),
            "or_pc32_process_block": (C.c_int, [vp, fp, fp, i64]),
            "or_pc32_free": (None, [vp]),
            "or_pc_new": (C.c_int, [dp, i64, C.c_int, C.c_int, C.POINTER(vp)]),
            "or_pc_process_block": (C.c_int, [vp, dp, dp, i64]),
            "or_pc_reset": (None, [vp]),
            "or_correlate_fft": (C.c_int, [dp, i64, dp, i64, dp]),
            "or_deconvolve": (C.c_int, [dp, i64, dp, i64, C.c_int, C.c_double, C.c_double, C.c_double, dp, i64,
                                        C.POINTER(i64), C.POINTER(i64)]),
            "or_inverse_filter": (C.c_int, [dp, i64, i64, C.c_double, dp]),
            "or_pc_latency": (i64, [vp]),
            "or_pc_stage_count": (C.c_int, [vp]),
            "or_pc_stage_info": (C.c_int, [vp, C.c_int, C.POINTER(i64), C.POINTER(i64)]),
            "or_pc_free": (None, [vp]),
            "or_fir_new": (vp, [dp, i64]),
            "or_fir_process_sample": (C.c_double, [vp, C.c_double]),
            "or_fir_process_block": (None, [vp, dp, i64]),
            "or_fir_process_block_to": (None, [vp, dp, dp, i64]),
            "or_fir_reset": (None, [vp]),
            "or_fir_free": (None, [vp]),
            "or_biquad_process_sample": (C.c_double, [dp, dp, C.c_double]),
            "or_biquad_process_block": (None, [dp, dp, dp, i64]),
            "or_biquad_process_block_generic": (None, [dp, dp, dp, i64]),
            "or_biquad_process_block_to": (None, [dp, dp, dp, dp, i64]),
            "or_biquad_chain_process_block": (None, [dp, dp, C.c_int, C.c_double, dp, i64]),
            "or_biquad_chain_process_sample": (C.c_double, [dp, dp, C.c_int, C.c_double, C.c_double]),
            "or_comp_default_cfg": (None, [vp, C.c_double]),
            "or_comp_new": (vp, [vp]),
            "or_comp_process_sample": (C.c_double, [vp, C.c_double]),
            "or_comp_process_in_place": (None, [vp, dp, i64]),
            "or_comp_reset": (None, [vp]),
            "or_comp_metrics": (None, [vp, dp, dp, dp]),
            "or_comp_params": (None, [vp, dp, dp, dp, dp, dp]),
            "or_comp_free": (None, [vp]),
            "or_comp_set_expander": (None, [vp, C.c_int, C.c_double, C.c_double]),
            "or_comp_hold_counter": (C.c_int, [vp]),
            "or_comp_gain_for_level": (C.c_double, [vp, C.c_double]),
            "or_verb_new": (vp, []),
            "or_verb_set": (None, [vp, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double]),
            "or_verb_process_sample": (C.c_double, [vp, C.c_double]),
            "or_verb_process_in_place": (None, [vp, dp, i64]),
            "or_verb_reset": (None, [vp]),
            "or_verb_free": (None, [vp]),
            "or_decode_f16": (C.c_float, [C.c_uint16]),
            "or_irlib_count": (C.c_int, [C.c_char_p, i64]),
            "or_irlib_get": (C.c_int, [C.c_char_p, i64, C.c_int, C.c_char_p, C.c_int, dp, C.POINTER(C.c_int),
                                       C.POINTER(i64), dp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def f64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def P(a: np.ndarray):
    return a.ctypes.data_as(dp)


class OracleError(Exception):
    def __init__(self, code):
        super().__init__(f"oracle status {code}")
        self.code = code


def _ck(rc):
    if rc != 0:
        raise OracleError(rc)


# ---- conv ----
def direct(a, b):
    a, b = f64(a), f64(b)
    out = np.empty(max(a.size + b.size - 1, 1))
    _ck(lib().or_direct(P(a), a.size, P(b), b.size, P(out)))
    return out[: a.size + b.size - 1]


def direct_circular(a, b):
    a, b = f64(a), f64(b)
    out = np.empty(max(a.size, 1))
    _ck(lib().or_direct_circular(P(a), a.size, P(b), b.size, P(out)))
    return out[: a.size]


def direct_ld(a, b):
    a, b = f64(a), f64(b)
    out = np.empty(a.size + b.size - 1)
    lib().or_direct_ld(P(a), a.size, P(b), b.size, P(out))
    return out


def convolve_mode(a, b, mode=0):
    a, b = f64(a), f64(b)
    cap = max(a.size + b.size - 1, 1)
    out = np.empty(cap)
    n = i64()
    _ck(lib().or_convolve(P(a), a.size, P(b), b.size, mode, P(out), cap, C.byref(n)))
    return out[: n.value].copy()


# ---- correlate.go / deconvolve.go ----
def correlate_fft(a, b):
    a, b = f64(a), f64(b)
    out = np.empty(max(a.size + b.size - 1, 1))
    _ck(lib().or_correlate_fft(P(a), a.size, P(b), b.size, P(out)))
    return out[: a.size + b.size - 1]


def deconvolve(signal, kernel, method=1, epsilon=0.0, noise_var=0.0, signal_var=0.0):
    """Returns (output, bad_bin); raises OracleError on a non-zero status (bad_bin in .bad_bin)."""
    x, h = f64(signal), f64(kernel)
    cap = max(x.size, 1)
    out = np.empty(cap)
    n, bad = i64(), i64(-1)
    rc = lib().or_deconvolve(P(x), x.size, P(h), h.size, method, epsilon, noise_var, signal_var, P(out), cap,
                             C.byref(n), C.byref(bad))
    if rc != 0:
        e = OracleError(rc)
        e.bad_bin = bad.value
        raise e
    return out[: n.value].copy()


def inverse_filter(kernel, length, epsilon):
    h = f64(kernel)
    out = np.empty(max(length, 1))
    _ck(lib().or_inverse_filter(P(h), h.size, length, epsilon, P(out)))
    return out[:length]


def fft(x, inverse=False):
    x = np.ascontiguousarray(np.asarray(x, dtype=np.complex128))
    out = np.empty_like(x)
    _ck(lib().or_fft(x.ctypes.data, out.ctypes.data, x.size, 1 if inverse else 0))
    return out


class OverlapAdd:
    def __init__(self, kernel, block_size=0):
        k = f64(kernel)
        self.K = k.size
        self.h = vp()
        _ck(lib().or_ola_new(P(k) if k.size else None, k.size, block_size, C.byref(self.h)))

    def process(self, x):
        x = f64(x)
        out = np.empty(max(x.size + self.K - 1, 1))
        _ck(lib().or_ola_process(self.h, P(x), x.size, P(out)))
        return out[: x.size + self.K - 1]

    def block_size(self):
        return lib().or_ola_block_size(self.h)

    def fft_size(self):
        return lib().or_ola_fft_size(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_ola_free(self.h)


class OverlapSave:
    def __init__(self, kernel, fft_size=0):
        k = f64(kernel)
        self.K = k.size
        self.h = vp()
        _ck(lib().or_ols_new(P(k) if k.size else None, k.size, fft_size, C.byref(self.h)))

    def process(self, x):
        x = f64(x)
        out = np.empty(max(x.size + self.K - 1, 1))
        _ck(lib().or_ols_process(self.h, P(x), x.size, P(out)))
        return out[: x.size + self.K - 1]

    def fft_size(self):
        return lib().or_ols_fft_size(self.h)

    def step_size(self):
        return lib().or_ols_step_size(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_ols_free(self.h)


class Streaming:
    def __init__(self, kernel, block, ola=False):
        k = f64(kernel)
        self.B = block
        self.h = vp()
        fn = lib().or_sola_new if ola else lib().or_sols_new
        _ck(fn(P(k) if k.size else None, k.size, block, C.byref(self.h)))

    def process_block(self, x):
        x = f64(x)
        out = np.empty(self.B)
        _ck(lib().or_stream_process_block(self.h, P(x), x.size, P(out), out.size))
        return out

    def reset(self):
        lib().or_stream_reset(self.h)

    def fft_size(self):
        return lib().or_stream_fft_size(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_stream_free(self.h)


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


class Streaming32:
    """NewStreamingOverlapSave32 / NewStreamingOverlapAdd32 (float32, complex64)."""

    def __init__(self, kernel, block, ola=False):
        k = _f32(kernel)
        self._h = C.c_void_p()
        _ck(lib().or_stream32_new(1 if ola else 0, k.ctypes.data_as(fp), k.size, int(block), C.byref(self._h)))
        self.block = int(block)

    def process_block(self, x):
        xi = _f32(x)
        out = np.empty(self.block, dtype=np.float32)
        _ck(lib().or_stream32_process_block(self._h, xi.ctypes.data_as(fp), out.ctypes.data_as(fp), xi.size))
        return out

    def fft_size(self):
        return int(lib().or_stream32_fft_size(self._h))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_stream32_free(self._h)


class Partitioned32:
    """NewPartitionedConvolution32 (float32, complex64)."""

    def __init__(self, kernel, min_order, max_order):
        k = _f32(kernel)
        self._h = C.c_void_p()
        _ck(lib().or_pc32_new(k.ctypes.data_as(fp), k.size, int(min_order), int(max_order), C.byref(self._h)))

    def process_block(self, x):
        xi = _f32(x)
        out = np.empty(xi.size, dtype=np.float32)
        _ck(lib().or_pc32_process_block(self._h, xi.ctypes.data_as(fp), out.ctypes.data_as(fp), xi.size))
        return out

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_pc32_free(self._h)


class Partitioned:
    def __init__(self, kernel, min_order, max_order):
        k = f64(kernel)
        self.h = vp()
        _ck(lib().or_pc_new(P(k) if k.size else None, k.size, min_order, max_order, C.byref(self.h)))

    def process_block(self, x):
        x = f64(x)
        out = np.empty(x.size)
        _ck(lib().or_pc_process_block(self.h, P(x), P(out), x.size))
        return out

    def latency(self):
        return lib().or_pc_latency(self.h)

    def stage_count(self):
        return lib().or_pc_stage_count(self.h)

    def stage_info(self, i):
        p, b = i64(), i64()
        _ck(lib().or_pc_stage_info(self.h, i, C.byref(p), C.byref(b)))
        return p.value, b.value

    def reset(self):
        lib().or_pc_reset(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_pc_free(self.h)


# ---- filters ----
class Fir:
    def __init__(self, coeffs):
        c = f64(coeffs)
        self.h = lib().or_fir_new(P(c), c.size)

    def process_sample(self, x):
        return lib().or_fir_process_sample(self.h, float(x))

    def process_block(self, buf):
        b = f64(buf).copy()
        lib().or_fir_process_block(self.h, P(b), b.size)
        return b

    def reset(self):
        lib().or_fir_reset(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_fir_free(self.h)


def biquad_block(coeffs, state, buf, kernel="avx2"):
    c, s, b = f64(coeffs), f64(state).copy(), f64(buf).copy()
    fn = lib().or_biquad_process_block if kernel == "avx2" else lib().or_biquad_process_block_generic
    fn(P(c), P(s), P(b), b.size)
    return b, s


def biquad_sample(coeffs, state, x):
    c = f64(coeffs)
    s = f64(state).copy()
    y = lib().or_biquad_process_sample(P(c), P(s), float(x))
    return y, s


def biquad_chain_block(coeffs, state, gain, buf):
    c, s, b = f64(coeffs), f64(state).copy(), f64(buf).copy()
    sections = c.size // 5
    lib().or_biquad_chain_process_block(P(c), P(s), sections, float(gain), P(b), b.size)
    return b, s


# ---- effects ----
class CompCfg(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("sample_rate", "threshold_db", "ratio", "knee_db", "attack_ms",
                                           "release_ms", "rms_window_ms", "makeup_db", "sidechain_low_cut_hz",
                                           "sidechain_high_cut_hz")] + \
               [(n, C.c_int) for n in ("topology", "detector_mode", "feedback_ratio_scale", "auto_makeup")]


class Compressor:
    def __init__(self, sample_rate=48000.0, **kw):
        cfg = CompCfg()
        lib().or_comp_default_cfg(C.byref(cfg), float(sample_rate))
        for k, v in kw.items():
            setattr(cfg, k, v)
        self.cfg = cfg
        self.h = lib().or_comp_new(C.byref(cfg))

    def process_in_place(self, buf):
        b = f64(buf).copy()
        lib().or_comp_process_in_place(self.h, P(b), b.size)
        return b

    def process_sample(self, x):
        return lib().or_comp_process_sample(self.h, float(x))

    def metrics(self):
        a, b, c = C.c_double(), C.c_double(), C.c_double()
        lib().or_comp_metrics(self.h, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value

    def params(self):
        v = [C.c_double() for _ in range(5)]
        lib().or_comp_params(self.h, *[C.byref(x) for x in v])
        return [x.value for x in v]

    def reset(self):
        lib().or_comp_reset(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_comp_free(self.h)


class Expander(Compressor):
    """dynamics.Expander (mode 1) / dynamics.Gate (mode 2) over the oracle's
    shared detector core; defaults of NewExpander / NewGate."""

    def __init__(self, sample_rate=48000.0, gate=False, range_db=None, hold_ms=None, **kw):
        base = dict(threshold_db=-40.0, ratio=10.0, knee_db=6.0, attack_ms=0.1, release_ms=100.0) if gate else \
            dict(threshold_db=-35.0, ratio=2.0, knee_db=6.0, attack_ms=1.0, release_ms=100.0)
        base.update(kw)
        super().__init__(sample_rate, **base)
        lib().or_comp_set_expander(self.h, 2 if gate else 1,
                                   float((-80.0 if gate else -60.0) if range_db is None else range_db),
                                   float((50.0 if gate else 0.0) if hold_ms is None else hold_ms))

    def hold_counter(self):
        return lib().or_comp_hold_counter(self.h)

    def gain(self, level):
        return lib().or_comp_gain_for_level(self.h, float(level))


class Freeverb:
    def __init__(self):
        self.h = lib().or_verb_new()

    def set(self, wet, dry, room, damp, gain=0.015):
        lib().or_verb_set(self.h, wet, dry, room, damp, gain)

    def process_in_place(self, buf):
        b = f64(buf).copy()
        lib().or_verb_process_in_place(self.h, P(b), b.size)
        return b

    def process_sample(self, x):
        return lib().or_verb_process_sample(self.h, float(x))

    def reset(self):
        lib().or_verb_reset(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_verb_free(self.h)


def decode_f16(h):
    return lib().or_decode_f16(int(h))


def irlib_read(data: bytes):
    """Returns [(name, sample_rate, samples[ch][n])] for every IR in an IRLB image."""
    n = lib().or_irlib_count(data, len(data))
    if n < 0:
        raise OracleError(-1)
    res = []
    for i in range(n):
        name = C.create_string_buffer(256)
        fs = C.c_double()
        ch = C.c_int()
        ln = i64()
        _ck(lib().or_irlib_get(data, len(data), i, name, 256, C.byref(fs), C.byref(ch), C.byref(ln), None))
        buf = np.empty(ch.value * ln.value)
        _ck(lib().or_irlib_get(data, len(data), i, name, 256, C.byref(fs), C.byref(ch), C.byref(ln), P(buf)))
        res.append((name.value.decode(), fs.value, buf.reshape(ch.value, ln.value)))
    return res


# ---- effectchain graph (chain_process.go:11-319), one channel -------------
class FxGraph:
    """Restatement of effectchain.Chain.Process over the oracle's node
    runtimes for ONE channel: nodes in topological order, input of a node =
    mixParentEdgesInto (zeros / copy / sum in edge order * 1/k), split-freq ->
    crossover LP/HP chains read by port, _output/bypassed mix only, others in
    place; the result is the _output buffer.  `nodes` is the compiled list of
    algodsp.effectchain: dicts {type, bypassed, parents [(idx, port)],
    sections, sections2 ([n][5] + gain), comp (field dict), verb}."""

    def __init__(self, nodes, fs):
        self.nodes = nodes
        self.rt = []
        for d in nodes:
            t = d["type"]
            if t == "biquad":
                secs, gain = d["sections"]
                self.rt.append(["biquad", np.asarray(secs, dtype=np.float64).ravel(), np.zeros(2 * len(secs)), gain])
            elif t == "split":
                lp, hp = d["sections"], d["sections2"]
                self.rt.append(["split", np.asarray(lp, dtype=np.float64).ravel(), np.zeros(2 * len(lp)),
                                np.asarray(hp, dtype=np.float64).ravel(), np.zeros(2 * len(hp))])
            elif t == "comp":
                cfg = {k: v for k, v in d["comp"].items() if k != "sample_rate"}
                if "expander" in d:
                    self.rt.append(["comp", Expander(d["comp"]["sample_rate"], **d["expander"], **cfg)])
                else:
                    self.rt.append(["comp", Compressor(d["comp"]["sample_rate"], **cfg)])
            elif t == "verb":
                v = Freeverb()
                v.set(*d["verb"])
                self.rt.append(["verb", v])
            elif t == "conv":  # ConvolutionReverb(kernel, minOrder) + SetWetDry (convolution.go:28-85)
                self.rt.append(["conv", Partitioned(d["kernel"], d["min_order"], 13), d["wet"], d["dry"]])
            else:
                self.rt.append([t])

    def process(self, block):
        n = len(block)
        buf, low, high = {}, {}, {}
        for i, d in enumerate(self.nodes):
            if i == 0:
                buf[0] = np.array(block, dtype=np.float64)
                continue
            par = d["parents"]

            def src(e):
                j, port = e
                if self.nodes[j]["type"] == "split":
                    return high[j] if port == 1 else low[j]
                return buf[j]

            if not par:
                dst = np.zeros(n)
            elif len(par) == 1:
                dst = src(par[0]).copy()
            else:
                mix = np.zeros(n)
                for e in par:
                    mix = mix + src(e)
                dst = mix * (1.0 / len(par))
            buf[i] = dst
            r = self.rt[i]
            if r[0] == "split":
                low[i], r[2] = biquad_chain_block(r[1], r[2], 1.0, dst)
                high[i], r[4] = biquad_chain_block(r[3], r[4], 1.0, dst)
                continue
            if d["type"] in ("output", "pass") or d["bypassed"]:
                continue
            if r[0] == "biquad":
                buf[i], r[2] = biquad_chain_block(r[1], r[2], r[3], dst)
            elif r[0] == "comp":
                buf[i] = r[1].process_in_place(dst)
            elif r[0] == "verb":
                buf[i] = r[1].process_in_place(dst)
            elif r[0] == "conv":
                rev = r[1].process_block(dst)
                buf[i] = r[3] * dst + r[2] * rev  # block[i] = dry*block[i] + wet*reverbOut[i]
        return buf[[i for i, d in enumerate(self.nodes) if d["type"] == "output"][0]]
