"""Freeverb-only chain on the time-parallel engine (K_verb in place on the
caller's buffer), 256 ch x 2^20, and config 5: Msamples/s, best of 3."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "algo-dsp_amd"))
from algodsp import design, processors, signals  # noqa: E402

fs = 48000.0
verb = (0.22, 1.0, 0.72, 0.45, 0.015)
comp = {"auto_makeup": 0, "makeup_db": 0.0}
C, n = 256, 1 << 20
xb = torch.from_numpy(np.stack([0.5 * signals.white_noise(n, 0x5EED + c) for c in range(C)])).cuda()
for name, kw, eng in (("verb-tp", dict(freeverb=verb), processors.EffectChain.ENGINE_TIME_PARALLEL),
                      ("config5", dict(eq=design.config5_eq(fs), compressor=comp, freeverb=verb), None)):
    fx = processors.EffectChain(C, sample_rate=fs, **kw)
    if eng is not None:
        fx.SetEngine(eng)
    s = torch.cuda.current_stream()
    fx.process_device(xb.data_ptr(), n, n, s.cuda_stream)
    s.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        fx.process_device(xb.data_ptr(), n, n, s.cuda_stream)
        s.synchronize()
        best = min(best, time.perf_counter() - t)
    print(f"{name:8s}: {C * n / best / 1e6:10.1f} Msamples/s", flush=True)
    fx.close()
