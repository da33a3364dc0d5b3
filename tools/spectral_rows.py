"""8(f)3 host-buffer rows (Deconvolve, InverseFilter) for tools/rows_bench.py,
measured in a process of their own without torch (the Go caller's situation).
Prints one JSON row per line."""
from __future__ import annotations

import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tools"))

import oracle_lib as O  # noqa: E402
from algodsp import conv, signals  # noqa: E402
from rows_bench import cpu_time, row  # noqa: E402


def main():
    q = "--quick" in sys.argv
    rows = []
    nd = 1 << (16 if q else 22)
    xd = signals.white_noise(nd, 41)
    hd = np.hanning(1502)[1:-1]
    opts = conv.DeconvOptions(conv.DeconvRegularized, 1e-3, 0.0, 0.0)
    got = conv.Deconvolve(xd, hd, opts)
    ncs = 1 << 16
    want = O.deconvolve(xd[:ncs], hd, 1, 1e-3)
    assert np.max(np.abs(conv.Deconvolve(xd[:ncs], hd, opts) - want)) <= 1e-8 * max(1.0, np.max(np.abs(want)))
    t0 = time.perf_counter()
    for _ in range(5):
        conv.Deconvolve(xd, hd, opts)
    ms = (time.perf_counter() - t0) / 5 * 1e3
    cs = cpu_time(lambda: O.deconvolve(xd[:ncs], hd, 1, 1e-3), budget_s=1.0, max_reps=5)
    rows.append(row("8(f)3", "conv.Deconvolve deconvolve.go:72-330 (DeconvRegularized)",
                    f"{nd} samples / 1500-tap Hann kernel, eps 1e-3, host buffers", nd, "samples", ms, cs, ncs,
                    f"oracle Deconvolve, {ncs} samples", None, 0,
                    "FFT(signal) and FFT(kernel) in one launch per pass, the regularised division fused into the "
                    "inverse's first pass, inverse at half length (Hermitian); PCIe in/out included"))
    ni = 1 << (16 if q else 22)
    hi = signals.white_noise(4096, 43)
    conv.InverseFilter(hi, ni, 1e-3)
    t0 = time.perf_counter()
    for _ in range(5):
        conv.InverseFilter(hi, ni, 1e-3)
    ms = (time.perf_counter() - t0) / 5 * 1e3
    wi = O.inverse_filter(hi, 1 << 16, 1e-3)
    assert np.max(np.abs(conv.InverseFilter(hi, 1 << 16, 1e-3) - wi)) <= 1e-8 * max(1.0, np.max(np.abs(wi)))
    cs = cpu_time(lambda: O.inverse_filter(hi, 1 << 16, 1e-3), budget_s=1.0, max_reps=5)
    rows.append(row("8(f)3", "conv.InverseFilter deconvolve.go:354-394", f"4096-tap kernel, length {ni}, "
                    "eps 1e-3, host buffers", ni, "samples", ms, cs, 1 << 16, "oracle InverseFilter, length 65536",
                    None, 0, "one real transform, conj(H)/(|H|^2 + eps) fused into the half-length inverse"))



if __name__ == "__main__":
    main()
