"""IRLB impulse-response library reader (internal/webdemo/irlib.go:17-451).

Host-side data-format parsing for the IRs the benchmark configs use
(Large Church from web/irs.irlib).  The f16 decoder keeps the
reference's subnormal exponent (irlib.go:87: 127-14-e+1, i.e. every
subnormal half decodes to twice its IEEE value) so inputs match the
reference's IRs exactly.
"""
from __future__ import annotations

import pathlib
import struct

import numpy as np

DATA_DIR = pathlib.Path(__file__).resolve().parent.parent.parent / "data"
DEFAULT_IRLIB = DATA_DIR / "irs.irlib"


def decode_f16(h: np.ndarray) -> np.ndarray:
    """decodeF16 irlib.go:68-97, vectorised; returns float32."""
    h = np.asarray(h, dtype=np.uint16).astype(np.uint32)
    sign = (h >> 15) << 31
    exp = (h >> 10) & 0x1F
    frac = h & 0x3FF
    bits = sign | ((exp + 112) << 23) | (frac << 13)  # normal numbers
    bits = np.where(exp == 31, sign | 0x7F800000 | (frac << 13), bits)
    zero = (exp == 0) & (frac == 0)
    bits = np.where(zero, sign, bits)
    sub = (exp == 0) & (frac != 0)
    if np.any(sub):
        f = np.where(sub, frac, 1)
        # shifts e until bit 10 is set: e = 10 - floor(log2(frac))
        e = 10 - np.floor(np.log2(f.astype(np.float64))).astype(np.int64)
        m = (f.astype(np.int64) << e) & 0x3FF
        sb = sign.astype(np.int64) | ((127 - 14 - e + 1) << 23) | (m << 13)
        bits = np.where(sub, sb.astype(np.uint32), bits)
    return bits.astype(np.uint32).view(np.float32)


def _read_string(buf: bytes, pos: int):
    (n,) = struct.unpack_from("<H", buf, pos)
    pos += 2
    return buf[pos:pos + n].decode("utf-8", "replace"), pos + n


def decode_f16_gpu(raw: np.ndarray, channels: int, device: int = 0) -> np.ndarray:
    """AUDI payload (interleaved f16) -> float64 [channels][frames] on the GPU
    (ad_decode_f16, bit-exact with decodeF16 incl. its subnormal quirk)."""
    import ctypes as C

    from ._lib import check, lib

    raw = np.ascontiguousarray(raw, dtype=np.uint16)
    frames = raw.size // channels
    out = np.empty((channels, frames), dtype=np.float64)
    check(lib().ad_decode_f16(raw.ctypes.data_as(C.POINTER(C.c_uint16)), frames, channels,
                              out.ctypes.data_as(C.POINTER(C.c_double)), device))
    return out


def read_irlib(path=DEFAULT_IRLIB, gpu: bool = False):
    """Returns a list of dicts {name, category, sample_rate, samples[ch][n] (float64)}.
    gpu=True decodes the AUDI payloads with the HIP kernel (ad_decode_f16)."""
    buf = pathlib.Path(path).read_bytes()
    if buf[:4] != b"IRLB":
        raise ValueError("irlib: invalid magic")
    version, count, index_offset = struct.unpack_from("<HIQ", buf, 4)
    if version != 1:
        raise ValueError(f"irlib: unsupported version {version}")
    pos = index_offset
    if buf[pos:pos + 4] != b"INDX":
        raise ValueError("irlib: expected INDX chunk")
    (indx_size,) = struct.unpack_from("<Q", buf, pos + 4)
    pos += 12
    end = pos + indx_size
    entries = []
    while pos < end:
        off, sr, ch, ln = struct.unpack_from("<QdII", buf, pos)
        pos += 24
        name, pos = _read_string(buf, pos)
        cat, pos = _read_string(buf, pos)
        entries.append((off, sr, ch, ln, name, cat))
    out = []
    for off, sr, ch, ln, name, cat in entries:
        try:
            out.append(_read_chunk(buf, off, ch, gpu))
        except (ValueError, struct.error):
            continue  # bad chunks are skipped (irlib.go:255-263)
    return out


def _read_chunk(buf: bytes, off: int, idx_channels: int, gpu: bool = False):
    if buf[off:off + 4] != b"IR--":
        raise ValueError("irlib: expected IR--")
    (chunk_size,) = struct.unpack_from("<Q", buf, off + 4)
    pos = off + 12
    read = 0
    meta = None
    samples = None
    while read < chunk_size:
        if pos + 8 > len(buf):
            break
        magic = buf[pos:pos + 4]
        (sub,) = struct.unpack_from("<I", buf, pos + 4)
        pos += 8
        read += 8
        body = pos
        if magic == b"META":
            sr, ch, ln = struct.unpack_from("<dII", buf, body)
            p = body + 16
            name, p = _read_string(buf, p)
            _desc, p = _read_string(buf, p)
            cat, p = _read_string(buf, p)
            (ntags,) = struct.unpack_from("<H", buf, p)
            p += 2
            for _ in range(ntags):
                _t, p = _read_string(buf, p)
            meta = dict(name=name, category=cat, sample_rate=sr, channels=ch, length=ln)
            pos = p
        elif magic == b"AUDI":
            raw = np.frombuffer(buf, dtype="<u2", count=sub // 2, offset=body)
            ch = meta["channels"] if meta else idx_channels
            frames = raw.size // ch
            if frames:
                if gpu:
                    samples = decode_f16_gpu(raw[: frames * ch], ch)
                else:
                    vals = decode_f16(raw[: frames * ch]).astype(np.float64)
                    samples = vals.reshape(frames, ch).T.copy()
            pos = body + sub
        else:
            pos = body + sub
        read += sub
    if meta is None or samples is None:
        raise ValueError("irlib: incomplete IR chunk")
    meta["samples"] = samples
    return meta


def large_church(path=DEFAULT_IRLIB, pad_to: int | None = 131072) -> np.ndarray:
    """Stereo Large Church IR [2][n], zero padded to `pad_to` taps."""
    for ir in read_irlib(path):
        if ir["name"] == "Large Church":
            s = ir["samples"]
            if pad_to and s.shape[1] < pad_to:
                s = np.pad(s, ((0, 0), (0, pad_to - s.shape[1])))
            return s
    raise KeyError("Large Church not found in IR library")


class LibraryProvider:
    """effectchain.IRProvider over an IR library (internal/webdemo
    effects_chain_adapter.go:12-23 + irlib.go:59-65): GetIR(index) returns
    (samples [ch][n], sample_rate, ok); ok is False out of range."""

    def __init__(self, path=DEFAULT_IRLIB, gpu: bool = False):
        self.irs = read_irlib(path, gpu=gpu)

    def GetIR(self, index: int):
        if index < 0 or index >= len(self.irs):
            return None, 0.0, False
        ir = self.irs[index]
        if ir["samples"] is None or len(ir["samples"]) == 0:
            return None, 0.0, False
        return ir["samples"], ir["sample_rate"], True

    def IRNames(self):
        return [ir["name"] for ir in self.irs]
