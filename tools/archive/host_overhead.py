"""Measures host-side cost of one engine call vs GPU time (diagnostic)."""
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
for hop in (8192,):
    eng = conv.MultiChannelConvolver(ir, hop=hop, channels=2)
    for sname, sp in (("torch-current", torch.cuda.current_stream(dev).cuda_stream), ("handle", 0),
                      ("side", torch.cuda.Stream(dev).cuda_stream)):
        for _ in range(3): eng.process_device(x.data_ptr(), n, n, y.data_ptr(), out_len, out_len, sp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10): eng.process_device(x.data_ptr(), n, n, y.data_ptr(), out_len, out_len, sp)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"hop {hop} stream {sname}: host issue {(t1-t0)/10*1e3:.3f} ms/call, total {(t2-t0)/10*1e3:.3f} ms/call")
