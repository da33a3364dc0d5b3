"""Compressor-only and config-5 chains at 256 and 16384 channels: Msamples/s of
one call, best of 3 (device buffers, AUTO engine)."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "algo-dsp_amd"))
from algodsp import design, processors, signals  # noqa: E402

fs = 48000.0
comp = {"auto_makeup": 0, "makeup_db": 0.0}
verb = (0.22, 1.0, 0.72, 0.45, 0.015)
cases = [("comp", 256, 1 << 20, dict(compressor=comp)), ("comp", 16384, 1 << 15, dict(compressor=comp)),
         ("config5", 256, 1 << 20, dict(eq=design.config5_eq(fs), compressor=comp, freeverb=verb))]
for name, C, n, kw in cases:
    xb = torch.from_numpy(np.stack([0.5 * signals.white_noise(n, 0x5EED + c) for c in range(min(C, 256))]))
    xb = xb.repeat(C // xb.shape[0], 1).contiguous().cuda()
    fx = processors.EffectChain(C, sample_rate=fs, **kw)
    s = torch.cuda.current_stream()
    fx.process_device(xb.data_ptr(), n, n, s.cuda_stream)
    s.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        fx.process_device(xb.data_ptr(), n, n, s.cuda_stream)
        s.synchronize()
        best = min(best, time.perf_counter() - t)
    print(f"{name:8s} {C:6d} ch x {n:8d}: {C * n / best / 1e6:10.1f} Msamples/s", flush=True)
    fx.close()
