"""EQ-only chains (a12-a14, bit-exact): K_lanes (the default, AUTO) against the
staged one-workgroup kernel (ENGINE_STAGED_NOSPLIT) and, up to 4096 channels,
the per-section pipeline (an AD_FX_EQ_LANES=0 build, when given as argv[1]):
ms per call and Gsamples/s at config 5's five sections, several channel
counts, device-resident buffers, the same input for every engine (outputs
compared bit for bit)."""
import ctypes as C
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
import numpy as np
import torch

from algodsp import design, processors, signals

fs = 48000.0
eq = design.config5_eq(fs)
P = processors.EffectChain
for C_, n in [(256, 1 << 20), (1024, 1 << 18), (4096, 1 << 16), (8192, 1 << 15), (16384, 1 << 15)]:
    x0 = torch.from_numpy(0.5 * signals.white_noise(C_ * n, 3).reshape(C_, n)).cuda()
    res = {}
    outs = {}
    for name, eng in [("lanes", P.ENGINE_AUTO), ("nosplit", P.ENGINE_STAGED_NOSPLIT)]:
        fx = P(C_, eq, None, None, fs)
        fx.SetEngine(eng)
        x = x0.clone()
        s = torch.cuda.current_stream().cuda_stream
        fx.process_device(x.data_ptr(), n, n, s)  # warm-up (and the compared output)
        torch.cuda.synchronize()
        outs[name] = x.cpu().numpy()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            fx.process_device(x.data_ptr(), n, n, s)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        res[name] = dt
        fx.close()
    same = np.array_equal(outs["lanes"], outs["nosplit"])
    print(f"{C_:6d} ch x {n:8d}: " + "  ".join(f"{k} {v * 1e3:8.2f} ms = {C_ * n / v / 1e9:6.2f} G" for k, v in res.items())
          + f"  lanes clocks/sample@2.4GHz {res['lanes'] * 2.4e9 / n:6.1f}  bit-identical {same}", flush=True)
