"""Per-step time of the headline step over a long back-to-back run, and the
same steps with idle gaps between them: does the board slow down under
sustained load (power / thermal management) within the bench's timed region?

  python3 tools/step_curve.py [--steps 60] [--gap-ms 20]
"""
import argparse
import json
import subprocess
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "algo-dsp_amd"))


def smi():
    try:
        r = subprocess.run(["rocm-smi", "--showpower", "--showtemp", "--showclocks", "--json"], capture_output=True,
                           text=True, timeout=20)
        d = json.loads(r.stdout)
        card = d.get("card0", next(iter(d.values())))
        keep = {k: v for k, v in card.items() if any(s in k for s in ("Power", "Temperature", "sclk", "mclk", "fclk"))}
        return keep
    except Exception as e:  # noqa: BLE001 - diagnostics only
        return {"error": str(e)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--gap-ms", type=float, default=20.0)
    a = ap.parse_args()
    import numpy as np
    import torch

    from algodsp import conv, irlib, signals

    n, C, hop = 1 << 24, 2, 8192
    ir = irlib.large_church()
    out_len = n + ir.shape[1] - 1
    x = torch.from_numpy(np.stack([signals.white_noise(n, 0x5EED + c) for c in range(C)])).cuda()
    y = torch.empty((C, out_len), dtype=torch.float64, device="cuda")
    eng = conv.MultiChannelConvolver(ir, hop=hop, channels=C, ir_index=[0, 1], chunk_blocks=0, device=0)
    s = torch.cuda.current_stream()

    def step():
        eng.process_device(x.data_ptr(), n, n, y.data_ptr(), out_len, out_len, s.cuda_stream)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    before = smi()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    ev[0].record(s)
    for i in range(a.steps):
        step()
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    during = smi()
    b2b = [round(ev[i].elapsed_time(ev[i + 1]), 4) for i in range(a.steps)]
    time.sleep(1.0)
    gapped = []
    for i in range(a.steps // 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        step()
        e1.record(s)
        e1.synchronize()
        gapped.append(round(e0.elapsed_time(e1), 4))
        time.sleep(a.gap_ms / 1e3)
    print(json.dumps({"back_to_back_ms": b2b, "gapped_ms": gapped, "gap_ms": a.gap_ms,
                      "smi_before": before, "smi_after_b2b": during}))


if __name__ == "__main__":
    main()
