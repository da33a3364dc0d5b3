"""PCIe / host-copy probe for the host-buffer pipeline: pinned H2D / D2H
rates through torch, and ad_conv_ols_process_multi at several worker counts."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "algo-dsp_amd"))

n = 1 << 27  # doubles (1 GiB)
h = torch.empty(n, dtype=torch.float64).pin_memory()
d = torch.empty(n, dtype=torch.float64, device="cuda")
for name, f in [("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))]:
    f(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    print(name, round(3 * n * 8 / (time.perf_counter() - t) / 1e9, 1), "GB/s", flush=True)
a = np.ones(n)
b = np.empty(n)
b[:] = 0
t = time.perf_counter(); np.copyto(b, a); print("host memcpy 1 thread", round(n * 8 / (time.perf_counter() - t) / 1e9, 1), "GB/s")
del a, b, h, d
