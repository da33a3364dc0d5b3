"""Staged engine vs fused kernels over channel counts (config-5 chain and its
single stages); prints Msamples/s per engine.  Used to pick the crossover."""
import os, sys, time, pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
import numpy as np, torch
from algodsp import design, processors, signals

fs = 48000.0
eq = design.config5_eq(fs)
comp = {"auto_makeup": 0, "makeup_db": 0.0}
verb = (0.22, 1.0, 0.72, 0.45, 0.015)
cases = {"config5": dict(eq=eq, compressor=comp, freeverb=verb), "verb": dict(freeverb=verb),
         "eq": dict(eq=eq), "comp": dict(compressor=comp)}
s = torch.cuda.current_stream().cuda_stream
for C in (256, 1024, 4096, 16384):
    n = (1 << 28) // C
    x = torch.from_numpy(0.5 * signals.white_noise(C * n, 1).reshape(C, n)).cuda()
    for name, kw in cases.items():
        res = {}
        for st in ("1", "0"):
            fx = processors.EffectChain(C, sample_rate=fs, **kw)
            fx.SetEngine(fx.ENGINE_AUTO if st == "1" else fx.ENGINE_FUSED)
            fx.process_device(x.data_ptr(), n, n, s)
            torch.cuda.synchronize()
            t = time.perf_counter()
            fx.process_device(x.data_ptr(), n, n, s)
            torch.cuda.synchronize()
            res[st] = C * n / (time.perf_counter() - t) / 1e6
            fx.close()
        print(f"C={C:6d} {name:8s} staged {res['1']:9.1f}  fused {res['0']:9.1f} Msamples/s", flush=True)
