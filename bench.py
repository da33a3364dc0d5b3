#!/usr/bin/env python3
"""Benchmark: overlap-save partitioned convolution, stereo x 131072-tap IR
(BASELINE.json configs[2] / metric), one step = one pass of the hot path over
2 channels x 2^24 samples of synthetic 48 kHz white noise resident in HBM.

  python bench.py --gpus N --steps K --warmup W

N > 1 (torchrun, one rank per GPU): every rank convolves its own stereo
channel pair (weak scaling; channel group per GPU) and the
per-rank stereo outputs are summed to rank 0 with one RCCL reduce over xGMI
(the north star's stereo mixdown), inside the timed step.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--samples", type=int, default=1 << 24, help="samples per channel per step")
    p.add_argument("--hop", type=int, default=8192)
    p.add_argument("--chunk", type=int, default=0, help="blocks per channel per engine chunk (0 = auto)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=1 << 24, help="samples of one channel for the CPU leg")
    p.add_argument("--mixdown", choices=["auto", "on", "off"], default="auto")
    p.add_argument("--kernel-timing", choices=["on", "off"], default="on",
                   help="HIP events around every engine kernel launch inside the timed region")
    return p.parse_args()


def cpu_baseline(ir, sample_len):
    """Times the oracle (C restatement of the reference's batch OverlapSave.Process,
    dsp/conv/overlap_save.go:126-254, N = 262144, step 131073) on one host core
    over a bounded sample of the same workload (one channel, `sample_len` samples)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np

    import oracle_lib as O
    from algodsp import signals

    x = signals.white_noise(sample_len, 0x5EED)
    ols = O.OverlapSave(ir[0], 0)
    t0 = time.perf_counter()
    ols.process(x)
    dt = time.perf_counter() - t0
    del np
    return {
        "value": sample_len / dt / 1e6,
        "unit": "Msamples/s",
        "cores": 1,
        "kind": "port",
        "sample": f"1 channel x {sample_len} samples (2^{sample_len.bit_length() - 1}) white noise, "
                  f"Large Church L (131072 taps), oracle OverlapSave.Process N=262144; {dt:.1f} s",
    }


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from algodsp import conv, irlib, signals

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    mixdown = world > 1 if args.mixdown == "auto" else args.mixdown == "on"

    ir = irlib.large_church()                       # [2][131072], Large Church zero padded
    K = ir.shape[1]
    n = args.samples
    out_len = n + K - 1                             # full linear convolution (OverlapSave.Process)
    x_host = np.stack([signals.white_noise(n, 0x5EED + 2 * rank + c) for c in range(2)])
    x = torch.from_numpy(x_host).to(dev)
    y = torch.empty((2, out_len), dtype=torch.float64, device=dev)
    del x_host

    eng = conv.MultiChannelConvolver(ir, hop=args.hop, channels=2, chunk_blocks=args.chunk, device=local)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def step():
        eng.process_device(x.data_ptr(), n, n, y.data_ptr(), out_len, out_len, sptr)
        if mixdown:
            dist.reduce(y, dst=0, op=dist.ReduceOp.SUM)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    eng.profile_read()  # clear

    live = args.kernel_timing == "on"
    eng.profile_enable(live)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not live:  # kernel durations from a separate event-timed pass
        eng.profile_enable(True)
        for _ in range(max(2, args.steps // 2)):
            step()
        torch.cuda.synchronize(dev)
    eng.profile_enable(False)
    prof = eng.profile_read()

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_samples = world * 2 * n * args.steps
    value = total_samples / elapsed / 1e6

    # dominant kernel + its roofline (algorithmic bytes / mean launch duration)
    dom = max(prof, key=lambda k: prof[k][0])
    ms, launches, alg_bytes = prof[dom]
    avg_ms = ms / max(launches, 1)
    achieved = (alg_bytes / max(launches, 1)) / (avg_ms * 1e-3) / 1e9
    kernels = {k: {"avg_us": v[0] / max(v[1], 1) * 1e3, "launches": v[1],
                   "alg_GBps": (v[2] / max(v[1], 1)) / (v[0] / max(v[1], 1) * 1e-3) / 1e9 if v[0] else None,
                   "share": v[0] / max(sum(p[0] for p in prof.values()), 1e-12)} for k, v in prof.items()}

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(ir, args.cpu_sample)
        traffic = None
        tfile = ROOT / "profiles" / "pmc_traffic.json"
        if tfile.exists():
            try:
                traffic = json.loads(tfile.read_text()).get(dom, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        line = {
            "metric": "Msamples/sec, overlap-save conv 131072-tap IR @48kHz; achieved HBM GB/s",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: SplitMix64 white noise (seed 0x5EED+channel) x Large Church IR from web/irs.irlib "
                    "(f16, reference decodeF16), zero padded 95432->131072 taps",
            "config": {
                "workload": "OverlapSave partitioned conv, stereo, 131072-tap IR, full linear convolution "
                            f"(2 ch x {n} samples per GPU per step)",
                "channels_per_gpu": 2,
                "samples_per_channel": n,
                "kernel_taps": K,
                "hop": args.hop,
                "partitions": (K + args.hop - 1) // args.hop,
                "parallelism": f"channel-group per GPU x{world}" + (" + RCCL reduce mixdown" if mixdown else ""),
            },
            "roofline": {
                "kernel": dom,
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "avg_launch_us": round(avg_ms * 1e3, 2),
                "timing": "HIP events on the launch stream, " + ("inside the timed region" if live else
                                                                 "separate pass after the timed region"),
            },
            "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in kernels.items()},
            "cpu_baseline": cpu,
        }
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
