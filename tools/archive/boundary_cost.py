"""Diagnostic: wall time per engine call vs chunk count (kernel boundaries)."""
import sys, time, pathlib
ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
import numpy as np, torch
from algodsp import conv, irlib, signals
dev = torch.device("cuda", 0)
ir = irlib.large_church()
n = 1 << 24; K = ir.shape[1]; out_len = n + K - 1
x = torch.from_numpy(np.stack([signals.white_noise(n, c) for c in range(2)])).to(dev)
y = torch.empty((2, out_len), dtype=torch.float64, device=dev)
s = torch.cuda.current_stream(dev)
for hop, chunk in ((8192, 4096), (8192, 1032), (8192, 516), (8192, 258), (4096, 4200), (4096, 1032)):
    eng = conv.MultiChannelConvolver(ir, hop=hop, channels=2, chunk_blocks=chunk)
    for _ in range(3): eng.process_device(x.data_ptr(), n, n, y.data_ptr(), out_len, out_len, s.cuda_stream)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10): eng.process_device(x.data_ptr(), n, n, y.data_ptr(), out_len, out_len, s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    wall = e0.elapsed_time(e1) / 10
    eng.profile_enable(True)
    for _ in range(3): eng.process_device(x.data_ptr(), n, n, y.data_ptr(), out_len, out_len, s.cuda_stream)
    eng.profile_enable(False)
    p = eng.profile_read()
    busy = sum(v[0] for v in p.values()) / 3
    nk = sum(v[1] for v in p.values()) / 3
    print(f"hop {hop} chunk {chunk}: gpu-wall {wall:.3f} ms/call, kernel busy {busy:.3f} ms, kernels/call {nk:.0f}, "
          f"gap/kernel {(wall-busy)/nk*1e3:.1f} us", {k: round(v[0]/v[1]*1e3, 1) for k, v in p.items()})
    del eng
