"""Experiment: stereo config-3 step as one 2-channel engine on one stream vs
two 1-channel engines on two streams (channel pipelines overlap, so one
kernel's compute phase can run beside the other's HBM phase).
Prints ms/step for each arrangement.  Not part of the product path."""
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from algodsp import conv, irlib, signals  # noqa: E402

ir = irlib.large_church()
K = ir.shape[1]
n = 1 << 24
out_len = n + K - 1
x = torch.from_numpy(np.stack([signals.white_noise(n, 0x5EED + c) for c in range(2)])).cuda()
y = torch.empty((2, out_len), dtype=torch.float64, device="cuda")
hop = int(sys.argv[1]) if len(sys.argv) > 1 else 8192


def timeit(fn, steps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


e2 = conv.MultiChannelConvolver(ir, hop=hop, channels=2)
s0 = torch.cuda.current_stream()
one = timeit(lambda: e2.process_device(x.data_ptr(), n, n, y.data_ptr(), out_len, out_len, s0.cuda_stream))
ref = y.clone()
del e2

ea = conv.MultiChannelConvolver(ir[0:1], hop=hop, channels=1)
eb = conv.MultiChannelConvolver(ir[1:2], hop=hop, channels=1)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def two():
    ev = torch.cuda.Event()
    ev.record(s0)
    sa.wait_event(ev)
    sb.wait_event(ev)
    ea.process_device(x[0].data_ptr(), n, n, y[0].data_ptr(), out_len, out_len, sa.cuda_stream)
    eb.process_device(x[1].data_ptr(), n, n, y[1].data_ptr(), out_len, out_len, sb.cuda_stream)
    fa, fb = torch.cuda.Event(), torch.cuda.Event()
    fa.record(sa)
    fb.record(sb)
    s0.wait_event(fa)
    s0.wait_event(fb)


t2 = timeit(two)
same = bool(torch.equal(y, ref))
print(f"hop {hop}: one 2-ch engine {one:.4f} ms/step; two 1-ch engines on two streams {t2:.4f} ms/step; "
      f"identical={same}", flush=True)
