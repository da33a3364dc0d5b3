"""Config 5 (256 ch x 2^20, device buffers) per time-parallel chunk length
(ad_fx_chain_set_engine chunk): Gsamples/s, best of three timed calls."""
import sys
import time

import torch

sys.path.insert(0, "algo-dsp_amd")
from algodsp import design, processors as P  # noqa: E402

fs = 48000.0
C, n = 256, 1 << 20
x = torch.randn(C, n, dtype=torch.float64, device="cuda") * 0.3
for chunk in [int(c) for c in (sys.argv[1:] or (16384, 32768, 49152, 65536, 98304, 131072))]:
    fx = P.EffectChain(C, design.config5_eq(fs), {"auto_makeup": 0, "makeup_db": 0.0},
                       (0.22, 1.0, 0.72, 0.45, 0.015), fs)
    fx.SetEngine(P.EffectChain.ENGINE_AUTO, chunk)
    s = torch.cuda.current_stream()
    fx.process_device(x.data_ptr(), n, n, s.cuda_stream)
    s.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        fx.process_device(x.data_ptr(), n, n, s.cuda_stream)
        s.synchronize()
        best = min(best, time.perf_counter() - t)
    print(chunk, f"{C * n / best / 1e9:.2f} Gsamples/s", flush=True)
    fx.close()
