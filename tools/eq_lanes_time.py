"""K_lanes call time at 256 channels x 2^20 samples (config 5's EQ), device
buffers: ms per call over 3 calls after a warm-up (A/B builds via ALGODSP_LIB).
FRESH=1: every call filters a fresh copy of the same input (event-timed around
the call only), instead of the previous call's output in place."""
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
import torch

from algodsp import design, processors, signals

fs = 48000.0
C_, n = 256, 1 << 20
fx = processors.EffectChain(C_, design.config5_eq(fs), None, None, fs)
x0 = torch.from_numpy(0.5 * signals.white_noise(C_ * n, 3).reshape(C_, n)).cuda()
x = x0.clone()
s = torch.cuda.current_stream()
fresh = os.environ.get("FRESH") == "1"
fx.process_device(x.data_ptr(), n, n, s.cuda_stream)
torch.cuda.synchronize()
if fresh:
    tot = 0.0
    for _ in range(3):
        x.copy_(x0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fx.process_device(x.data_ptr(), n, n, s.cuda_stream)
        e1.record()
        torch.cuda.synchronize()
        tot += e0.elapsed_time(e1) * 1e-3
    dt = tot / 3
else:
    t0 = time.perf_counter()
    for _ in range(3):
        fx.process_device(x.data_ptr(), n, n, s.cuda_stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
print(f"{'fresh ' if fresh else ''}{dt * 1e3:.2f} ms/call = {C_ * n / dt / 1e9:.2f} Gsamples/s = {dt * 2.4e9 / n:.1f} clocks per step at 2.4 GHz")
