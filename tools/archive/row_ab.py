"""Same-box A/B of the latency- and PCIe-bound conv rows (a3, a4, a5, a6 of
tools/rows_bench.py) for several builds of the library: each ALGODSP_LIB in
argv runs in its own child process, in turn, for --rounds rounds.

    python tools/row_ab.py ab/old.so algo-dsp_amd/libalgodsp_hip.so
"""
import argparse
import json
import os
import pathlib
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent


def child():
    sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
    import numpy as np

    from algodsp import conv, irlib, signals

    k16 = irlib.large_church()[0, :16384]
    out = {}
    B, nblk = 4096, 512
    xs = signals.white_noise(nblk * B, 0x5EED)
    ys = np.empty_like(xs)
    for ctor, name in ((conv.NewStreamingOverlapSave, "a5"), (conv.NewStreamingOverlapAdd, "a6")):
        s = ctor(k16, B)
        for i in range(16):
            s.ProcessBlockTo(ys[i * B:(i + 1) * B], xs[i * B:(i + 1) * B])
        t0 = time.perf_counter()
        for i in range(nblk):
            s.ProcessBlockTo(ys[i * B:(i + 1) * B], xs[i * B:(i + 1) * B])
        out[name + " us/block"] = round((time.perf_counter() - t0) / nblk * 1e6, 1)
    xbt = signals.white_noise(1 << 22, 3)
    for ctor, name in ((conv.NewOverlapSave, "a4"), (conv.NewOverlapAdd, "a3")):
        e = ctor(k16)
        e.Process(xbt[:1 << 16])
        e.Process(xbt)
        t0 = time.perf_counter()
        for _ in range(6):
            e.Process(xbt)
        out[name + " Msamples/s"] = round(6 * len(xbt) / (time.perf_counter() - t0) / 1e6, 1)
        yb = np.empty(len(xbt) + len(k16) - 1)
        e.ProcessTo(yb, xbt)
        t0 = time.perf_counter()
        for _ in range(6):
            e.ProcessTo(yb, xbt)
        out[name + " ProcessTo Msamples/s"] = round(6 * len(xbt) / (time.perf_counter() - t0) / 1e6, 1)
    print(json.dumps(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child()
    for r in range(a.rounds):
        for lib in a.libs:
            env = dict(os.environ, ALGODSP_LIB=str(pathlib.Path(lib).resolve()))
            p = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True,
                               timeout=300)
            if p.returncode != 0:
                print(lib, "rc", p.returncode, p.stderr[-800:])
                return p.returncode
            print(r, lib, p.stdout.strip().splitlines()[-1], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
