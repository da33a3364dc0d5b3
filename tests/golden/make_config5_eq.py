"""Writes tests/golden/config5_eq_coeffs.json: the config-5 EQ sections
(BASELINE config 5, SURVEY 8(d): HP 40 Hz Q .707, LowShelf 100 Hz +3 dB,
Peak 1 kHz -2 dB Q 1, HighShelf 8 kHz +2 dB, LP 18 kHz Q .707) as produced by
algodsp/design.py, the restatement of dsp/filter/design/design.go:37-223 and
design/pass/butterworth.go:56-125, in hex floats (exact bits) at 44.1, 48,
96 and 192 kHz.  These are the coefficients every config-5 parity test and
bench.py --workload fx hand to both the GPU and the oracle; the fixture pins
them against silent designer changes.  The reference's own bits are unpinned
(Go's math.Cos / Sin / Pow are not run here; both are correctly rounded or
within 1 ulp), so tests/test_design.py checks the designers against the
properties design_test.go asserts instead.

Usage: python tests/golden/make_config5_eq.py
"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))

from algodsp import design  # noqa: E402


def main():
    out = {"_source": "algodsp.design.config5_eq (design.go:37-223 restated); tests/golden/make_config5_eq.py",
           "_layout": "per sample rate: [[b0, b1, b2, a1, a2] as float.hex()] per section, chain gains 1"}
    for fs in (44100.0, 48000.0, 96000.0, 192000.0):
        out[str(int(fs))] = [[float(v).hex() for v in co[0]] for co, _ in design.config5_eq(fs)]
    path = pathlib.Path(__file__).with_name("config5_eq_coeffs.json")
    path.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
