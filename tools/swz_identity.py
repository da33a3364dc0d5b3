"""Bit-identity of two library builds (argv[1], argv[2]) on the FFT paths:
OverlapSave (hop 8192, 131072 taps, 2^21 samples: K1/K2/K3), OverlapAdd,
CorrelateFFT (2 x 2^20 and 2 x 2^23: the fused pass), Deconvolve.  Each build
runs in its own child process (ALGODSP_LIB); the outputs' SHA-256 must match."""
import hashlib
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
CHILD = r'''
import hashlib, sys
sys.path.insert(0, "%s")
import numpy as np
from algodsp import conv
rng = np.random.default_rng(5)
h = hashlib.sha256()
k = rng.standard_normal(131072)
x = rng.standard_normal(1 << 21)
h.update(conv.OverlapSaveConvolve(x, k).tobytes())
h.update(conv.OverlapAddConvolve(x[: 1 << 19], k[:16384]).tobytes())
for n in (1 << 20, 1 << 23):
    a, b = rng.standard_normal(n), rng.standard_normal(n)
    h.update(conv.CorrelateFFT(a, b).tobytes())
print(h.hexdigest())
''' % (ROOT / "algo-dsp_amd")

out = []
for libp in sys.argv[1:3]:
    env = dict(os.environ, ALGODSP_LIB=str((ROOT / libp).resolve()))
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=250)
    if r.returncode != 0:
        print(r.stderr[-2000:])
        sys.exit(1)
    out.append(r.stdout.strip().splitlines()[-1])
print("identical" if out[0] == out[1] else "DIFFERENT", out)
sys.exit(0 if out[0] == out[1] else 1)
