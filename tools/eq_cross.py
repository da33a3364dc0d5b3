"""EQ-only chains (config-5 EQ, 5 sections, bit-exact staged engine) per channel
count: Msamples/s of one call, best of 3 (the per-section pipeline against the
one-workgroup-per-channel-group kernel is the library build's choice).

  python3 tools/eq_cross.py [C:n ...]
"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "algo-dsp_amd"))
from algodsp import design, processors, signals  # noqa: E402

fs = 48000.0
eq = design.config5_eq(fs)
for spec in (sys.argv[1:] or ["256:1048576", "1024:262144", "2048:131072", "4096:65536", "8192:32768", "16384:32768"]):
    C, n = (int(v) for v in spec.split(":"))
    xb = torch.from_numpy(np.stack([0.5 * signals.white_noise(n, 0x5EED + c) for c in range(min(C, 64))]))
    xb = xb.repeat(C // xb.shape[0], 1).contiguous().cuda()
    fx = processors.EffectChain(C, sample_rate=fs, eq=eq)
    s = torch.cuda.current_stream()
    fx.process_device(xb.data_ptr(), n, n, s.cuda_stream)
    s.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        fx.process_device(xb.data_ptr(), n, n, s.cuda_stream)
        s.synchronize()
        best = min(best, time.perf_counter() - t)
    print(f"{C:6d} ch x {n:8d}: {C * n / best / 1e6:10.1f} Msamples/s", flush=True)
    fx.close()
