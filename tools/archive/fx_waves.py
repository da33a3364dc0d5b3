"""Per-wave clock counters of the config-5 staged engine's first chunk
(ad_fx_chain_set_profiling): {compute, barrier wait} per K_eq wave."""
import ctypes as C
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
import numpy as np
import torch

from algodsp import design, processors, signals
from algodsp._lib import check, lib

fs = 48000.0
C_, n = 256, 1 << 16
fx = processors.EffectChain(C_, design.config5_eq(fs), {"auto_makeup": 0, "makeup_db": 0.0},
                            (0.22, 1.0, 0.72, 0.45, 0.015), fs)
x = torch.from_numpy(0.5 * signals.white_noise(C_ * n, 1).reshape(C_, n)).cuda()
s = torch.cuda.current_stream().cuda_stream
fx.process_device(x.data_ptr(), n, n, s)
check(lib().ad_fx_chain_set_profiling(fx._h, 1))
fx.process_device(x.data_ptr(), n, n, s)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 64)()
cnt = C.c_int()
check(lib().ad_fx_chain_read_profile(fx._h, buf, 64, C.byref(cnt)))
v = list(buf)[: cnt.value]
for w in range(len(v) // 2):
    if v[2 * w] or v[2 * w + 1]:
        print(f"K_eq wave (section/detector) {w}: compute {v[2*w]:>10d}  barrier wait {v[2*w+1]:>10d}  ticks/chunk")
