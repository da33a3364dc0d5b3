"""Calibrates the time-parallel EQ engine's conditioning guard on the CPU.

The time-parallel engine (fx_tp.hip) starts each EQ segment from a chained
start state instead of running the DF-II-T cascade serially.  Its output
differs from the serial recurrence (the reference's, and the bit-exact
engines') by the rounding noise both carry, and that noise grows with the
sections' round-off noise gain: poles near z = 1 (a low highpass at a high
sample rate) amplify every state rounding.

This script simulates the engine's arithmetic in numpy -- zero-state segment
runs in double, the segment-start states chained in long double (the
engine chains in double-double), the rerun in double from the chained states
rounded to double -- and compares it with the serial recurrence (the C oracle)
for highpass cutoffs and sample rates, next to the closed-form noise gain of
each section's all-pole part,

    NG = (1 + a2) / ((1 - a2) ((1 + a2)^2 - a1^2)),

which the library's guard (fx_tp_noise_gain, capi_dsp.cpp) evaluates.
Usage: python tools/tp_cond.py
"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import oracle_lib as O  # noqa: E402
from algodsp import design, signals  # noqa: E402


def noise_gain(sec):
    b0, b1, b2, a1, a2 = (np.longdouble(v) for v in sec)
    d = (1 - a2) * ((1 + a2) ** 2 - a1 ** 2)
    if d <= 0:
        return np.inf
    return float((1 + a2) / d)


def run_cascade(secs, x, st):
    """DF-II-T cascade (section.go:47-53 operation order) over x[..., t],
    states st[..., k, 2] updated in place; returns y."""
    y = np.empty_like(x)
    for t in range(x.shape[-1]):
        v = x[..., t]
        for k, (b0, b1, b2, a1, a2) in enumerate(secs):
            o = b0 * v + st[..., k, 0]
            st[..., k, 0] = (b1 * v - a1 * o) + st[..., k, 1]
            st[..., k, 1] = b2 * v - a2 * o
            v = o
        y[..., t] = v
    return y


def tp_sim(secs, x, seg):
    C, n = x.shape
    ns = len(secs)
    nseg = n // seg
    xs = x[:, :nseg * seg].reshape(C, nseg, seg)
    # zero-state runs (double)
    z = np.zeros((C, nseg, ns, 2))
    run_cascade(secs, xs, z)
    # A: zero-input step of the cascade, long double
    D = 2 * ns
    A = np.zeros((D, D), dtype=np.longdouble)
    for i in range(D):
        st = np.zeros(D, dtype=np.longdouble)
        st[i] = 1
        v = np.longdouble(0)
        for k, (b0, b1, b2, a1, a2) in enumerate(secs):
            y = np.longdouble(b0) * v + st[2 * k]
            A[2 * k, i] = np.longdouble(b1) * v - np.longdouble(a1) * y + st[2 * k + 1]
            A[2 * k + 1, i] = np.longdouble(b2) * v - np.longdouble(a2) * y
            v = y
    B = np.eye(D, dtype=np.longdouble)
    for _ in range(seg):
        B = A @ B
    s = np.zeros((C, D), dtype=np.longdouble)
    starts = np.zeros((C, nseg, D))
    for v in range(nseg):
        starts[:, v] = s.astype(np.float64)
        s = s @ B.T + z[:, v].reshape(C, D).astype(np.longdouble)
    st = starts.reshape(C, nseg, ns, 2).copy()
    y = run_cascade(secs, xs, st)
    return y.reshape(C, nseg * seg)


def main():
    C, n, seg = 16, 65536, 256
    x = np.stack([0.5 * signals.white_noise(n, 4242 + c) for c in range(C)])
    print(f"{'fs':>7} {'hp Hz':>6} {'sqrtNG*eps':>11} {'tp-serial rel rms':>18}")
    for fs in (48000.0, 96000.0, 192000.0):
        for fc in (10.0, 20.0, 40.0, 80.0):
            eq = design.config5_eq(fs)
            secs = [design.highpass(fc, 0.707, fs)] + [co[0] for co, _ in eq[1:]]
            ng = max(noise_gain(s) for s in secs)
            ref = np.stack([O.biquad_chain_block(np.ravel(secs), np.zeros(2 * len(secs)), 1.0, x[c])[0]
                            for c in range(C)])
            got = tp_sim(secs, x, seg)
            r = ref[:, :got.shape[1]]
            rel = float(np.sqrt(np.mean((got - r) ** 2)) / np.sqrt(np.mean(r ** 2)))
            print(f"{fs:7.0f} {fc:6.0f} {np.sqrt(ng) * 2.0 ** -52:11.3e} {rel:18.3e}", flush=True)


if __name__ == "__main__":
    main()
