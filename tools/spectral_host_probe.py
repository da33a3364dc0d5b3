"""Where a host-buffer Deconvolve / InverseFilter call spends its time:
wall time per call for 2^22 samples, with fresh and with reused output
arrays (run under rocprofv3 --kernel-trace --hip-trace --stats)."""
import pathlib
import sys
import time

import numpy as np

if "--torch-first" in sys.argv:  # torch's HIP runtime loaded before the library (rows_bench, bench.py)
    import torch  # noqa: F401

    if "--init" in sys.argv:
        torch.cuda.set_device(0)

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
from algodsp import conv, signals  # noqa: E402

if "--torch" in sys.argv:  # the rows_bench process state: torch's HIP runtime initialised first
    import torch

    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")

n = 1 << 22
hi = signals.white_noise(4096, 43)
conv.InverseFilter(hi, n, 1e-3)
for rep in range(3):
    t0 = time.perf_counter()
    conv.InverseFilter(hi, n, 1e-3)
    print(f"InverseFilter fresh output: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
xd = signals.white_noise(n, 41)
hd = np.hanning(1502)[1:-1]
opts = conv.DeconvOptions(conv.DeconvRegularized, 1e-3, 0.0, 0.0)
conv.Deconvolve(xd, hd, opts)
for rep in range(3):
    t0 = time.perf_counter()
    conv.Deconvolve(xd, hd, opts)
    print(f"Deconvolve: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
