import sys, time, numpy as np, torch
sys.path.insert(0, "algo-dsp_amd")
from algodsp import processors as P, design
fs = 48000.0; C, n = 256, 1 << 20
x = torch.randn(C, n, dtype=torch.float64, device="cuda") * 0.3
for eng in (P.EffectChain.ENGINE_AUTO, P.EffectChain.ENGINE_TIME_PARALLEL):
    fx = P.EffectChain(C, design.config5_eq(fs), None, None, fs)
    fx.SetEngine(eng)
    s = torch.cuda.current_stream()
    fx.process_device(x.data_ptr(), n, n, s.cuda_stream); s.synchronize()
    t = time.perf_counter()
    for _ in range(3): fx.process_device(x.data_ptr(), n, n, s.cuda_stream)
    s.synchronize(); dt = (time.perf_counter() - t) / 3
    print(eng, f"{C * n / dt / 1e9:.2f} Gsamples/s", f"{dt*1e3:.2f} ms")
    fx.close()
