"""Bit-identity of the fused CorrelateFFT pass (k_corr_fwd_last_inv_first)
with the unfused passes: runs CorrelateFFT of two 2^23-sample signals (and a
few other sizes) through the default library and through a build without the
fusion (tools/build_variant.sh corr_unfused "-DAD_CORR_FUSED=0" bigfft.hip),
each in its own child process (ALGODSP_LIB selects the .so), and compares the
outputs bit for bit.  Usage: python tools/corr_fused_check.py [ab/corr_unfused.so]
"""
import os
import pathlib
import subprocess
import sys
import tempfile

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
SIZES = [(1 << 23, 1 << 23), (3_000_000, 1_000_000), (1 << 16, 1 << 16), (40000, 25000), (70000, 3)]


def child(out_dir):
    sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
    from algodsp import conv, signals

    for i, (n, m) in enumerate(SIZES):
        a, b = signals.white_noise(n, 11 + n), 1e-3 * signals.white_noise(m, 13 + m)
        np.save(os.path.join(out_dir, f"c{i}.npy"), conv.CorrelateFFT(a, b))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    alt = sys.argv[1] if len(sys.argv) > 1 else "ab/corr_unfused.so"
    with tempfile.TemporaryDirectory() as d:
        outs = []
        for lib in (None, str(ROOT / alt)):
            od = os.path.join(d, "alt" if lib else "def")
            os.makedirs(od)
            env = dict(os.environ)
            if lib:
                env["ALGODSP_LIB"] = lib
            subprocess.run([sys.executable, __file__, "--child", od], check=True, env=env, timeout=600)
            outs.append(od)
        ok = True
        for i, (n, m) in enumerate(SIZES):
            x, y = np.load(os.path.join(outs[0], f"c{i}.npy")), np.load(os.path.join(outs[1], f"c{i}.npy"))
            same = x.shape == y.shape and np.array_equal(x, y)
            ok &= same
            print(f"n={n} m={m}: {'bit-identical' if same else 'DIFFERENT, max %.3e' % float(np.max(np.abs(x - y)))}")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
