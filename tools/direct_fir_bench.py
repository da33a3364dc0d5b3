#!/usr/bin/env python3
"""A/B timing of the time-domain FIR-shaped kernels (conv.Direct, fir.Filter)
on one MI355X: TFLOP/s (2 flops per product: rounded mul + rounded add) at a
few sizes, with a parity check against the oracle on each.

  python tools/direct_fir_bench.py            # default kernels
  AD_DIRECT_R=0 python tools/direct_fir_bench.py   # input-stationary k_direct_lds
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
from rows_bench import ROOT, dev_time  # noqa: E402  (also sets sys.path)


def main():
    import torch

    import oracle_lib as O
    from algodsp import conv, processors, signals

    cuda = torch.device("cuda", 0)
    out = []
    for n, m in ((48000, 256), (1 << 20, 256), (1 << 22, 256), (1 << 22, 64), (1 << 20, 2048)):
        a = signals.white_noise(n, 0x5EED)
        b = signals.make_test_kernel(m)
        da, db = torch.from_numpy(a).to(cuda), torch.from_numpy(b).to(cuda)
        dd = torch.empty(n + m - 1, dtype=torch.float64, device=cuda)
        ms = dev_time(lambda s: conv.direct_device(da.data_ptr(), n, db.data_ptr(), m, dd.data_ptr(), s),
                      reps=20)
        ok = bool(np.array_equal(dd.cpu().numpy(), O.direct(a, b))) if n <= (1 << 20) else None
        out.append(dict(op="direct", n=n, m=m, us=round(ms * 1e3, 2), tflops=round(2.0 * n * m / ms / 1e9, 2),
                        bit_exact=ok))
    for ch, n, taps in ((64, 1 << 20, 256), (8, 1 << 16, 256), (64, 1 << 18, 33), (16, 1 << 18, 1024)):
        h = signals.make_test_kernel(taps)
        f = processors.Filter(h, channels=ch)
        xs = np.stack([signals.white_noise(n, 0x5EED + c) for c in range(ch)])
        x = torch.from_numpy(xs).to(cuda)
        y = torch.empty_like(x)
        ms = dev_time(lambda s: f.process_device(x.data_ptr(), n, y.data_ptr(), n, n, s), reps=5)
        f.Reset()
        f.process_device(x.data_ptr(), n, y.data_ptr(), n, n, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want = O.Fir(h).process_block(xs[ch - 1, :8192])
        err = float(np.sqrt(np.mean((y[ch - 1, :8192].cpu().numpy() - want) ** 2)))
        out.append(dict(op="fir", channels=ch, n=n, taps=taps, us=round(ms * 1e3, 2),
                        tflops=round(2.0 * ch * n * taps / ms / 1e9, 2), rms_err=err))
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
