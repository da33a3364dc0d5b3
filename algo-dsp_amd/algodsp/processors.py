"""Host-side mirror of the reference's per-sample processors on the HIP engine.

Names and argument meaning follow the Go packages so the parity tests read
like the reference's own tests:

  biquad.Chain / biquad.Section  dsp/filter/biquad/chain.go, section.go
  dynamics.Compressor            dsp/effects/dynamics/compressor.go
  reverb.Reverb (Freeverb)       dsp/effects/reverb/reverb.go
  fir.Filter                     dsp/filter/fir/filter.go
  effectchain filter -> dyn-compressor -> reverb-freeverb (EffectChain)

Every instance can carry `channels` independent reference instances (one
lane each on the GPU); buffers are [channels][n] float64 (a 1-D buffer is
one channel).  All work runs in libalgodsp_hip.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import CompressorConfig, check, f64, lib, ptr

DEVICE = 0
SEC_STRIDE = 6  # {pre_gain, b0, b1, b2, a1, a2}


def _as2d(buf, channels: int):
    if not isinstance(buf, np.ndarray) or buf.dtype != np.float64 or not buf.flags.c_contiguous:
        raise TypeError("buffer must be a C-contiguous float64 numpy array")
    b2 = buf.reshape(1, -1) if buf.ndim == 1 else buf
    if b2.shape[0] != channels:
        raise ValueError(f"buffer has {b2.shape[0]} channels, processor has {channels}")
    return b2


def section_table(coeffs, gain: float = 1.0) -> np.ndarray:
    """[sections][5] {b0,b1,b2,a1,a2} (+ chain gain) -> [sections][6] device table."""
    c = f64(coeffs).reshape(-1, 5)
    t = np.ones((c.shape[0], SEC_STRIDE))
    t[:, 1:] = c
    if c.shape[0]:
        t[0, 0] = gain
    return t


class _FxChain:
    def __init__(self, channels: int, device: int):
        self.channels = int(channels)
        self._h = C.c_void_p()
        check(lib().ad_fx_chain_create(self.channels, int(device), C.byref(self._h)))

    def _process(self, buf):
        b = _as2d(buf, self.channels)
        check(lib().ad_fx_chain_process(self._h, ptr(b), b.shape[1]))

    def process_device(self, d_buf: int, stride: int, n: int, stream: int | None = None):
        check(lib().ad_fx_chain_process_device(self._h, C.c_void_p(d_buf), int(stride), int(n),
                                               C.c_void_p(stream or 0)))

    def Reset(self):
        check(lib().ad_fx_chain_reset(self._h))

    # engine selection (include/algodsp.h ad_fx_chain_set_engine); the fused
    # and staged engines give identical results, the time-parallel one within
    # 1e-12 relative RMS of them
    ENGINE_AUTO, ENGINE_FUSED, ENGINE_STAGED_NOSPLIT, ENGINE_STAGED, ENGINE_TIME_PARALLEL = 0, 1, 2, 3, 4

    def SetEngine(self, engine: int, chunk: int = 0):
        check(lib().ad_fx_chain_set_engine(self._h, int(engine), int(chunk)))

    def LastEngine(self) -> tuple[int, float]:
        """(engine that ran the last call, the EQ's round-off noise estimate)
        (ad_fx_chain_last_engine)."""
        e, ng = C.c_int(), C.c_double()
        check(lib().ad_fx_chain_last_engine(self._h, C.byref(e), C.byref(ng)))
        return e.value, ng.value

    def close(self):
        if self._h:
            lib().ad_fx_chain_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Chain(_FxChain):
    """biquad.Chain (chain.go:6-138): optional gain, then sections in order."""

    def __init__(self, coeffs, gain: float = 1.0, channels: int = 1, device: int = DEVICE):
        super().__init__(channels, device)
        self._coeffs = f64(coeffs).reshape(-1, 5)
        self._gain = float(gain)
        self._load()

    def _load(self):
        t = section_table(self._coeffs, self._gain)
        check(lib().ad_fx_chain_set_eq(self._h, ptr(t), t.shape[0], 0))

    def NumSections(self) -> int:
        return self._coeffs.shape[0]

    def Gain(self) -> float:
        return self._gain

    def SetGain(self, g: float):  # chain.go:89-97
        self._gain = float(g)
        self._load()

    def UpdateCoefficients(self, coeffs, gain: float | None = None):  # chain.go:99-115
        self._coeffs = f64(coeffs).reshape(-1, 5)
        if gain is not None:
            self._gain = float(gain)
        self._load()

    def ProcessBlock(self, buf):  # chain.go:59-70
        self._process(buf)

    def State(self) -> np.ndarray:  # chain.go:122-130 -> [channels][sections][2]
        out = np.zeros((self.channels, self.NumSections(), 2))
        check(lib().ad_fx_chain_eq_state(self._h, ptr(out), out.size))
        return out

    def SetState(self, states):  # chain.go:130-138: [channels][sections][2] (a [sections][2] list for 1 channel)
        st = np.ascontiguousarray(np.asarray(states, dtype=np.float64))
        check(lib().ad_fx_chain_set_eq_state(self._h, ptr(st), st.size))


def Section(b0, b1, b2, a1, a2, channels: int = 1, device: int = DEVICE) -> Chain:
    """biquad.Section (section.go:26-155) = a one-section chain with unit gain."""
    return Chain([[b0, b1, b2, a1, a2]], 1.0, channels, device)


class Compressor(_FxChain):
    """dynamics.Compressor (compressor.go:39-431) on `channels` lanes."""

    def __init__(self, sample_rate: float = 48000.0, channels: int = 1, device: int = DEVICE, **cfg):
        super().__init__(channels, device)
        self.cfg = CompressorConfig()
        lib().ad_compressor_default_config(C.byref(self.cfg), float(sample_rate))
        for k, v in cfg.items():
            setattr(self.cfg, k, v)
        self._apply()

    def _apply(self):
        check(lib().ad_fx_chain_set_compressor(self._h, C.byref(self.cfg)))

    def _set(self, **kv):
        # a setter the reference rejects returns its error and leaves the
        # config as it was (core.go:131-198): restore the fields, then raise
        old = {k: getattr(self.cfg, k) for k in kv}
        for k, v in kv.items():
            setattr(self.cfg, k, v)
        try:
            self._apply()
        except Exception:
            for k, v in old.items():
                setattr(self.cfg, k, v)
            raise

    # setters (compressor.go:130-305, core.go:131-250)
    def SetThreshold(self, db):
        self._set(threshold_db=db)

    def SetRatio(self, r):
        self._set(ratio=r)

    def SetKnee(self, db):
        self._set(knee_db=db)

    def SetAttack(self, ms):
        self._set(attack_ms=ms)

    def SetRelease(self, ms):
        self._set(release_ms=ms)

    def SetRMSWindow(self, ms):
        self._set(rms_window_ms=ms)

    def SetSidechainLowCut(self, hz):
        self._set(sidechain_low_cut_hz=hz)

    def SetSidechainHighCut(self, hz):
        self._set(sidechain_high_cut_hz=hz)

    def SetAutoMakeup(self, on: bool):
        self._set(auto_makeup=int(bool(on)))

    def SetMakeupGain(self, db):
        self._set(makeup_db=db)

    def ProcessInPlace(self, buf):  # compressor.go:362-366
        self._process(buf)

    def Metrics(self, channel: int = 0):
        ip, op, gr = C.c_double(), C.c_double(), C.c_double()
        check(lib().ad_fx_chain_compressor_metrics(self._h, int(channel), C.byref(ip), C.byref(op), C.byref(gr)))
        return ip.value, op.value, gr.value


class Expander(Compressor):
    """dynamics.Expander (expander.go) on `channels` lanes: the compressor's
    detector core with the downward-expansion gain and a range floor.
    Defaults of NewExpander (expander.go:9-15)."""

    GATE = False

    def __init__(self, sample_rate: float = 48000.0, channels: int = 1, device: int = DEVICE, **cfg):
        _FxChain.__init__(self, channels, device)
        self.cfg = CompressorConfig()
        lib().ad_compressor_default_config(C.byref(self.cfg), float(sample_rate))
        defaults = dict(threshold_db=-40.0, ratio=10.0, knee_db=6.0, attack_ms=0.1, release_ms=100.0) \
            if self.GATE else dict(threshold_db=-35.0, ratio=2.0, knee_db=6.0, attack_ms=1.0, release_ms=100.0)
        self.range_db = cfg.pop("range_db", -80.0 if self.GATE else -60.0)
        self.hold_ms = cfg.pop("hold_ms", 50.0 if self.GATE else 0.0)
        for k, v in {**defaults, **cfg}.items():
            setattr(self.cfg, k, v)
        self._apply()

    def _apply(self):
        check(lib().ad_fx_chain_set_expander(self._h, C.byref(self.cfg), int(self.GATE), float(self.range_db),
                                             float(self.hold_ms)))

    def _set_attr(self, name, value):
        # a rejected value raises and leaves the stage as it was (like _set)
        old = getattr(self, name)
        setattr(self, name, value)
        try:
            self._apply()
        except Exception:
            setattr(self, name, old)
            raise

    def SetRange(self, db):  # expander.go / gate.go SetRange
        self._set_attr("range_db", db)


class Gate(Expander):
    """dynamics.Gate (gate.go): Expander gain plus a hold counter; defaults of
    NewGate (gate.go:9-17)."""

    GATE = True

    def SetHold(self, ms):  # gate.go:196-223
        self._set_attr("hold_ms", ms)


class Reverb(_FxChain):
    """reverb.Reverb (Freeverb, reverb.go:33-235) with NewReverb defaults."""

    def __init__(self, channels: int = 1, device: int = DEVICE):
        super().__init__(channels, device)
        self.wet, self.dry, self.room, self.damp, self.gain = 0.22, 1.0, 0.72, 0.45, 0.015
        self._apply()

    def _apply(self):
        check(lib().ad_fx_chain_set_freeverb(self._h, self.wet, self.dry, self.room, self.damp, self.gain))

    def SetWet(self, v):
        self.wet = float(v)
        self._apply()

    def SetDry(self, v):
        self.dry = float(v)
        self._apply()

    def SetRoomSize(self, v):
        self.room = float(v)
        self._apply()

    def SetDamp(self, v):
        self.damp = float(v)
        self._apply()

    def SetGain(self, v):
        self.gain = float(v)
        self._apply()

    def ProcessInPlace(self, buf):  # reverb.go:185-189
        self._process(buf)


class EffectChain(_FxChain):
    """effectchain `_input -> filter-* -> dyn-compressor -> reverb-freeverb ->
    _output` for `channels` chains, fused per sample (chain_process.go:11-33).

    eq: list of (coeffs [sections][5], gain) biquad chains (filter nodes, in
    order); compressor: dict of ad_compressor_config fields or None;
    freeverb: (wet, dry, room, damp, gain) or None."""

    def __init__(self, channels: int, eq=(), compressor=None, freeverb=None, sample_rate: float = 48000.0,
                 device: int = DEVICE):
        super().__init__(channels, device)
        tabs = [section_table(c, g) for c, g in eq]
        t = np.concatenate(tabs) if tabs else np.zeros((0, SEC_STRIDE))
        check(lib().ad_fx_chain_set_eq(self._h, ptr(f64(t)), t.shape[0], 0))
        if compressor is not None:
            cfg = CompressorConfig()
            lib().ad_compressor_default_config(C.byref(cfg), float(sample_rate))
            for k, v in compressor.items():
                setattr(cfg, k, v)
            self.cfg = cfg
            check(lib().ad_fx_chain_set_compressor(self._h, C.byref(cfg)))
        if freeverb is not None:
            check(lib().ad_fx_chain_set_freeverb(self._h, *map(float, freeverb)))

    def Process(self, buf):
        self._process(buf)


class Filter:
    """fir.Filter (filter.go:11-172) for `channels` lanes sharing the taps."""

    def __init__(self, coeffs, channels: int = 1, device: int = DEVICE):
        self.coeffs = f64(coeffs).ravel()
        self.channels = int(channels)
        self._h = C.c_void_p()
        check(lib().ad_fir_create(ptr(self.coeffs), self.coeffs.size, self.channels, int(device),
                                  C.byref(self._h)))

    def ProcessBlock(self, buf):  # :74-114
        b = _as2d(buf, self.channels)
        check(lib().ad_fir_process_block(self._h, ptr(b), b.shape[1]))

    def ProcessBlockTo(self, dst, src):  # :119-159
        d, s = _as2d(dst, self.channels), _as2d(f64(src), self.channels)
        if d.shape != s.shape:
            raise ValueError("dst/src length mismatch")
        check(lib().ad_fir_process_block_to(self._h, ptr(d), ptr(s), s.shape[1]))

    def ProcessSample(self, x: float) -> float:  # :46-69 (one channel)
        b = np.array([[x]] * self.channels, dtype=np.float64)
        self.ProcessBlock(b)
        return float(b[0, 0])

    def process_device(self, d_src: int, src_stride: int, d_dst: int, dst_stride: int, n: int,
                       stream: int | None = None):
        check(lib().ad_fir_process_device(self._h, C.c_void_p(d_src), int(src_stride), C.c_void_p(d_dst),
                                          int(dst_stride), int(n), C.c_void_p(stream or 0)))

    def Reset(self):
        check(lib().ad_fir_reset(self._h))

    def close(self):
        if self._h:
            lib().ad_fir_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def chain_process(coeffs, state, gain, buf):
    """ad_biquad_chain_process: one-shot Chain.ProcessBlock, state in/out."""
    c = f64(coeffs).reshape(-1, 5)
    b = _as2d(buf, buf.shape[0] if buf.ndim == 2 else 1)
    st = state
    if not (isinstance(st, np.ndarray) and st.dtype == np.float64 and st.flags.c_contiguous
            and st.size == b.shape[0] * c.shape[0] * 2):
        raise TypeError("state must be a C-contiguous float64 array [channels][sections][2]")
    check(lib().ad_biquad_chain_process(ptr(c), ptr(st), float(gain), ptr(b), b.shape[0], c.shape[0], b.shape[1],
                                        DEVICE))
