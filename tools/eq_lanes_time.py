"""K_lanes call time at 256 channels x 2^20 samples (config 5's EQ), device
buffers: ms per call over 3 calls after a warm-up (A/B builds via ALGODSP_LIB)."""
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
x = torch.from_numpy(0.5 * signals.white_noise(C_ * n, 3).reshape(C_, n)).cuda()
s = torch.cuda.current_stream().cuda_stream
fx.process_device(x.data_ptr(), n, n, s)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    fx.process_device(x.data_ptr(), n, n, s)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 3
print(f"{dt * 1e3:.2f} ms/call = {C_ * n / dt / 1e9:.2f} Gsamples/s = {dt * 2.4e9 / n:.1f} clocks per step at 2.4 GHz")
