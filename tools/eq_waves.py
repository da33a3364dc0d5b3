"""The bit-exact EQ-only chain (a12-a14: config 5's five RBJ sections, no
compressor or reverb, 256 channels, the staged engine AUTO picks): call time
per 2^20 samples and the per-wave clock counters of K_eq's first chunk
(ad_fx_chain_set_profiling: {compute, barrier wait} per section wave)."""
import ctypes as C
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
import numpy as np
import torch

from algodsp import design, processors, signals
from algodsp._lib import check, lib

fs = 48000.0
C_ = 256
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
fx = processors.EffectChain(C_, design.config5_eq(fs), None, None, fs)
x = torch.from_numpy(0.5 * signals.white_noise(C_ * n, 1).reshape(C_, n)).cuda()
s = torch.cuda.current_stream().cuda_stream
fx.process_device(x.data_ptr(), n, n, s)
torch.cuda.synchronize()
reps = 3
t0 = time.perf_counter()
for _ in range(reps):
    fx.process_device(x.data_ptr(), n, n, s)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
print(f"engine {fx.LastEngine()}  {C_} ch x {n}: {dt * 1e3:.2f} ms/call = {C_ * n / dt / 1e6:.1f} Msamples/s "
      f"= {dt * 2.4e9 / n:.1f} clocks per channel-group sample")
check(lib().ad_fx_chain_set_profiling(fx._h, 1))
fx.process_device(x.data_ptr(), n, n, s)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 64)()
cnt = C.c_int()
check(lib().ad_fx_chain_read_profile(fx._h, buf, 64, C.byref(cnt)))
v = list(buf)[: cnt.value]
for w in range(len(v) // 2):
    if v[2 * w] or v[2 * w + 1]:
        print(f"K_eq wave {w}: compute {v[2*w]:>10d}  barrier wait {v[2*w+1]:>10d}  ticks per first chunk")
