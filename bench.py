#!/usr/bin/env python3
"""Benchmark: overlap-save partitioned convolution, stereo x 131072-tap IR
(BASELINE.json configs[2] / metric), one step = one pass of the hot path over
2 channels x 2^24 samples of synthetic 48 kHz white noise resident in HBM.

  python bench.py --gpus N --steps K --warmup W

N > 1 (torchrun, one rank per GPU): config 4's shard (BASELINE.json
configs[3]): every rank convolves its own group of 8 channels x 2^24 samples
(ch c with IR[c mod 2]), so per-GPU work is fixed (weak scaling) and N = 8 is
the 64-channel job, and the per-rank stereo partial mixes are summed to rank 0
with one RCCL reduce over xGMI (the north star's stereo mixdown), inside the
timed step.  The channels are as long as the N = 1 stereo config's, so the
convolution tail and the launch ramps weigh the same per sample at every N.
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
FX_CLOCK_HZ = 2.4e9     # MI355X engine clock (MI355X_MICROARCH.md)
FX_CHAIN_CLK = 24.5     # config 5's serial chain per sample, clocks: the compressor's envelope
                        # follower (tools/chain_latency.hip).  The EQ sections and the Freeverb
                        # combs run time-parallel in the default engine,
                        # so the envelope is the one recurrence left serial per channel


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--samples", type=int, default=None,
                   help="samples per channel per step (default 2^24)")
    p.add_argument("--hop", type=int, default=8192)
    p.add_argument("--chunk", type=int, default=0, help="blocks per channel per engine chunk (0 = auto)")
    p.add_argument("--schedule", choices=["serial", "pipelined", "chunked"], default="serial",
                   help="conv: the engine's offline schedule (ad_conv_multi_set_schedule): serial chunks on the "
                        "caller's stream, or Infinity-Cache-sized chunks with K1 / K2 / K3 of consecutive chunks "
                        "overlapped on three streams")
    p.add_argument("--pipe-chunk", type=int, default=0, help="pipelined schedule: blocks per channel per chunk (0 = auto)")
    p.add_argument("--pipe-run", type=int, default=0, help="pipelined schedule: K2 run length in blocks (0 = auto)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=1 << 24, help="samples per channel (per host thread) for the CPU leg")
    p.add_argument("--mixdown", choices=["auto", "on", "off"], default="auto")
    p.add_argument("--host-io", choices=["on", "off"], default="on",
                   help="N = 1: also time the same step host buffer -> host buffer (PCIe included)")
    p.add_argument("--shard-sub", choices=["on", "off"], default="on",
                   help="N = 1 conv: also measure config 4's per-GPU shard (8 ch x 2^24 + the stereo mixdown "
                        "through the ABI at world 1), the like-for-like base of the N > 1 curve")
    p.add_argument("--fx-leg", choices=["on", "off"], default="on",
                   help="N = 1 conv: also time config 5 (256 ch x 2^20 effect chain, AUTO engine, 5 steps, "
                        "with its parity and CPU baseline) as the line's config5 key")
    p.add_argument("--stream-leg", choices=["on", "off"], default="on",
                   help="N = 1 conv: also time config 2 (StreamingOverlapSave, 4096-sample host blocks, "
                        "1024 blocks: p50 / p99 per block) as the line's config2_stream key")
    p.add_argument("--corr-leg", choices=["on", "off"], default="on",
                   help="N = 1 conv: also time CorrelateFFT of two 2^23-sample signals (SURVEY 8(f)3, device "
                        "buffers, 40 calls, parity + CPU leg) as the line's correlate key")
    p.add_argument("--pipeline", choices=["on", "off"], default="on",
                   help="N > 1: overlap step i's mixdown reduce with step i+1's convolution (two output buffers)")
    p.add_argument("--mix-fused", choices=["on", "off"], default="on",
                   help="shard with mixdown: the stereo mix fused into the inverse transform "
                        "(ad_conv_multi_process_device_mix, no per-channel outputs) or per-channel outputs + "
                        "k_mixdown inside ad_mixdown_reduce")
    p.add_argument("--segments", type=int, default=1,
                   help="output segments per step (ad_conv_multi_process_device_segment); each segment's "
                        "mixdown reduce starts as soon as it is computed")
    p.add_argument("--step-events", choices=["on", "off"], default="on",
                   help="N = 1: an event between the timed steps (the line's step_ms)")
    p.add_argument("--clock-settle", type=int, default=60,
                   help="untimed steps before the W warm-up steps: the board's clock dips for ~10 ms once the load "
                        "turns sustained and recovers after ~30-45 steps (profiles/r05_step_curve.json, DESIGN.md "
                        "section 2), so the timed region measures the steady state (the line's clock_settle_steps)")
    p.add_argument("--settle-steps", type=int, default=0,
                   help="N = 1: after the timed region, this many more steps event-timed one by one (the line's "
                        "`settled` key: the step once the board's clock has recovered from its load-onset dip)")
    p.add_argument("--kernel-timing", choices=["dominant", "on", "off"], default="dominant",
                   help="HIP events inside the timed region around the dominant kernel's launches only "
                        "(dominant: picked by a profiled warm-up pass, the other kernels timed in a pass "
                        "after the timed region), around every launch (on), or none (off: all kernels "
                        "timed after)")
    p.add_argument("--channels", type=int, default=None,
                   help="conv: channels per GPU (IR[c %% 2]); default 2 (the stereo config) at N = 1, "
                        "8 (config 4's shard) at N > 1")
    p.add_argument("--graph", choices=["config5", "branched"], default=None,
                   help="fx workload: run an effectchain graph through the batched graph runtime")
    p.add_argument("--workload", choices=["conv", "shard", "fx", "stream", "corr"], default="conv",
                   help="conv: BASELINE metric (overlap-save conv; config 3 at N = 1, config 4's shard at N > 1); "
                        "shard: config 4's shard (8 ch x 2^24 per GPU + RCCL stereo mixdown) at any N; "
                        "fx: config 5 effect chain (256 ch); "
                        "stream: config 2 streaming OLS (mono, 16384 taps, 4096-sample host blocks); "
                        "corr: CorrelateFFT of two 2^23-sample signals (SURVEY 8(f)3, device buffers)")
    return p.parse_args(argv)


class GpuRuntime:
    """What run_conv needs from the machine: torch.cuda streams and events, the
    HIP engine (conv.MultiChannelConvolver) and the library's RCCL communicator
    (shard.Comm, ad_comm_* / ad_mixdown_reduce).  The product path.  The N > 1
    orchestration around it (bootstrap, two-buffer reduce pipeline, conv-only
    pass, max over ranks, rank 0's parity) is plain Python over this interface,
    so tests/test_bench_orchestration.py runs the same code at world 2 over gloo
    with CPU stand-ins for these members."""

    dist_backend = "nccl"  # RCCL on ROCm

    def __init__(self, local: int):
        import torch

        self.torch = torch
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        self.local = local

    def init_dist(self):
        import torch.distributed as dist

        dist.init_process_group(self.dist_backend, device_id=self.dev)

    def current_stream(self):
        return self.torch.cuda.current_stream(self.dev)

    def new_stream(self):
        return self.torch.cuda.Stream(self.dev)

    def event(self, timing: bool = False):
        return self.torch.cuda.Event(enable_timing=timing)

    def synchronize(self):
        self.torch.cuda.synchronize(self.dev)

    def engine(self, ir, hop, channels, ir_index, chunk_blocks):
        from algodsp import conv

        return conv.MultiChannelConvolver(ir, hop=hop, channels=channels, ir_index=ir_index,
                                          chunk_blocks=chunk_blocks, device=self.local)

    def comm(self, rank, world, bootstrap):
        from algodsp import shard

        return shard.Comm(rank, world, self.local, bootstrap)

    def empty_cache(self):
        self.torch.cuda.empty_cache()


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` outside a launcher: start N ranks (one process per GPU) with
    torch.distributed.run and return its exit status.  Runs before anything
    touches the GPU; the children see WORLD_SIZE = N."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "bench.py")] + sys.argv[1:]
    return subprocess.call(cmd, stdout=sys.stdout)  # the JSON channel, not the fd-1 banner sink


def affinity_cores() -> int:
    """Cores this process's CPU affinity allows (os.cpu_count() on the GPU box
    reports the whole machine)."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        return os.cpu_count() or 1


def host_cores() -> int:
    """Host cores this process may use, capped at the GPU box's per-GPU CPU
    share (16)."""
    return max(1, min(16, affinity_cores()))


def cpu_baseline(ir, sample_len):
    """Times the oracle (C restatement of the reference's batch OverlapSave.Process,
    dsp/conv/overlap_save.go:126-254, N = 262144, step 131073) over a bounded
    sample of the same workload: one channel on one core, then one channel per
    host core (ctypes releases the GIL, so T threads run T oracle instances in
    parallel).  `value` is the all-cores rate."""
    sys.path.insert(0, str(ROOT / "tests"))
    from concurrent.futures import ThreadPoolExecutor

    import oracle_lib as O
    from algodsp import signals

    T = host_cores()
    xs = [signals.white_noise(sample_len, 0x5EED + c) for c in range(T)]
    ols = O.OverlapSave(ir[0], 0)
    t0 = time.perf_counter()
    ols.process(xs[0])
    dt1 = time.perf_counter() - t0
    del ols

    def one(c):
        return O.OverlapSave(ir[c % 2], 0).process(xs[c]).size

    with ThreadPoolExecutor(T) as ex:
        t0 = time.perf_counter()
        list(ex.map(one, range(T)))
        dtT = time.perf_counter() - t0
    fast = cpu_fast_fft(ir, xs, T)
    del xs
    # every core the affinity mask allows (capped at 64 threads, a shorter
    # channel each): the box's whole-machine figure beside the per-GPU share
    A = affinity_cores()
    wide = None
    if A > T:
        TA = min(A, 64)
        la = max(1 << 20, sample_len // 8)
        xa = [signals.white_noise(la, 0x7000 + c) for c in range(TA)]
        with ThreadPoolExecutor(TA) as ex:
            t0 = time.perf_counter()
            list(ex.map(lambda c: O.OverlapSave(ir[c % 2], 0).process(xa[c]).size, range(TA)))
            dtA = time.perf_counter() - t0
        del xa
        wide = {"value": round(TA * la / dtA / 1e6, 3), "unit": "Msamples/s", "threads": TA, "affinity_cores": A,
                "sample": f"one channel of {la} samples per thread on {TA} threads ({dtA:.1f} s)"}
    return {
        "value": T * sample_len / dtT / 1e6,
        "unit": "Msamples/s",
        "cores": T,
        "kind": "port",
        "per_gpu_share_cores": T,
        "affinity_cores": A,
        "affinity_wide": wide,
        "single_core": sample_len / dt1 / 1e6,
        "optimized_fft": fast,
        "sample": f"oracle OverlapSave.Process (N=262144, Large Church 131072 taps) on {T} host threads, one "
                  f"channel of {sample_len} white-noise samples each ({dtT:.1f} s; host cpu_count "
                  f"{os.cpu_count()}, affinity {A}; `value` uses the per-GPU share of 16 cores, affinity_wide every "
                  f"allowed core up to 64); single_core: 1 channel on 1 thread ({dt1:.1f} s)",
    }


def cpu_fast_fft(ir, xs, T):
    """The reference's OverlapSave.Process block structure (overlap_save.go:126-254:
    N = nextPow2(2K) = 262144 complex points per block, step N - K + 1, history
    of K - 1 samples, a complex forward FFT, the product with the kernel
    spectrum, a complex inverse, the valid part kept) with an optimised FFT
    library in place of the oracle's radix-2 restatement: scipy.fft (pocketfft),
    the T channels' blocks in one batched call on T workers.  Context for the
    oracle's figure (algo-fft's FastPlan is not runnable here); not the oracle,
    not the baseline the contract names."""
    import numpy as np
    import scipy.fft as sf

    K = ir.shape[1]
    N = 1
    while N < 2 * K:
        N *= 2
    step = N - K + 1
    n = xs[0].size
    H = np.stack([sf.fft(np.concatenate([ir[c % 2], np.zeros(N - K)])) for c in range(T)])
    X = np.stack(xs)
    out = np.empty((T, n + K - 1))
    hist = np.zeros((T, K - 1))
    buf = np.zeros((T, N), dtype=np.complex128)
    t0 = time.perf_counter()
    pos = 0
    while pos < n + K - 1:
        ns = min(step, max(0, n - pos))
        buf[:] = 0
        buf[:, :K - 1] = hist
        if ns:
            buf[:, K - 1:K - 1 + ns] = X[:, pos:pos + ns]
        y = sf.ifft(sf.fft(buf, axis=1, workers=T) * H, axis=1, workers=T)
        take = min(step, n + K - 1 - pos)
        out[:, pos:pos + take] = y[:, K - 1:K - 1 + take].real
        seg = np.concatenate([hist, X[:, pos:pos + ns]], axis=1)
        hist = seg[:, seg.shape[1] - (K - 1):]
        pos += step if ns else take
    dt = time.perf_counter() - t0
    ref = exact_window(xs[0], ir[0], n // 2, 8)
    err = float(np.max(np.abs(out[0, n // 2:n // 2 + 8] - ref)))
    return {"value": round(T * n / dt / 1e6, 3), "unit": "Msamples/s", "cores": T,
            "sample": f"{T} channels x {n} samples, N = {N}, step {step}, scipy.fft {sf.__name__} workers={T} "
                      f"({dt:.1f} s)", "max_abs_err_vs_exact": err}


def exact_window(x, h, t0, w):
    """y[t0 .. t0+w) of the full linear convolution x * h by direct float64
    dot products (numpy; independent of the engine and of the oracle)."""
    import numpy as np

    K = h.size
    lo = t0 - K + 1
    seg = x[max(lo, 0):t0 + w]
    if lo < 0:
        seg = np.concatenate([np.zeros(-lo), seg])
    if seg.size < w + K - 1:
        seg = np.concatenate([seg, np.zeros(w + K - 1 - seg.size)])
    return np.convolve(seg, h, mode="valid")


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus)
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    if args.workload == "fx":
        return main_fx(args)
    if args.workload == "corr":
        return main_corr(args)
    if args.workload == "stream":
        return main_stream(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rt = GpuRuntime(local)
    if world > 1:
        rt.init_dist()
    return conv_main(args, rt, world, rank, local)


def conv_main(args, rt, world, rank, local):
    """The conv / shard workload on this rank (the BASELINE metric): measure
    with run_conv, then rank 0 assembles and prints the JSON line.  `rt` is a
    GpuRuntime (or a test's CPU stand-in with the same members); a world > 1
    process group is already initialised."""
    import numpy as np
    import torch.distributed as dist

    from algodsp import irlib

    dev = rt.dev
    # config 4's shard (8 ch x 2^24 per GPU + the stereo mixdown) at N > 1, or
    # at any N with --workload shard; config 3 (stereo x 2^24) at N = 1
    shard_cfg = world > 1 or args.workload == "shard"
    mixdown = shard_cfg if args.mixdown == "auto" else args.mixdown == "on"

    if args.channels is None:
        args.channels = 8 if shard_cfg else 2
    if args.samples is None:
        args.samples = 1 << 24
    ir = irlib.large_church()                       # [2][131072], Large Church zero padded
    r = run_conv(args, world, rank, rt, ir, args.channels, shard_cfg, mixdown, args.steps, args.warmup,
                 args.kernel_timing, args.settle_steps, args.clock_settle)
    C, n, K, out_len = args.channels, args.samples, ir.shape[1], r["out_len"]
    elapsed, prof, prof_live, mode = r["elapsed"], r["prof"], r["prof_live"], args.kernel_timing
    ids, x_host, eng, ys, mixes, last = r["ids"], r["x_host"], r["eng"], r["ys"], r["mixes"], r["last"]
    comm = r["comm"]

    total_samples = world * C * n * args.steps
    value = total_samples / elapsed / 1e6

    # dominant kernel + its roofline (algorithmic bytes / mean launch duration)
    dom = max(prof, key=lambda k: prof[k][0])
    if mode == "dominant":
        dom = next(k for k, v in prof_live.items() if v[1] > 0)
    ms, launches, alg_bytes = prof[dom]
    avg_ms = ms / max(launches, 1)
    achieved = (alg_bytes / max(launches, 1)) / (avg_ms * 1e-3) / 1e9
    kernels = {k: {"avg_us": v[0] / max(v[1], 1) * 1e3, "launches": v[1],
                   "alg_GBps": (v[2] / max(v[1], 1)) / (v[0] / max(v[1], 1) * 1e-3) / 1e9 if v[0] else None,
                   "share": v[0] / max(sum(p[0] for p in prof.values()), 1e-12)} for k, v in prof.items()}

    if rank == 0:
        # Parity of the measured output itself: windows of the last step's
        # result (the whole-job stereo mix on rank 0 when the mixdown runs)
        # against exact float64 dot products -- the signal start, a K2 run
        # boundary (auto run length: multiples of 16 blocks), the middle and
        # the tail of the output.
        parity = output_parity(args, r, ir, C * world, mixdown)
        host_io = None
        if world == 1 and args.host_io == "on":
            # the same step from HOST buffers to HOST buffers through the C ABI
            # (ad_conv_ols_process_multi: chunked pinned staging, H2D || UPOLS ||
            # D2H on three streams) -- PCIe included, not the metric
            yh = eng.process_host(x_host)  # warm-up (pinned buffers, device scratch, output pages)
            reps = 3
            split = [0.0, 0.0, 0.0]
            th = time.perf_counter()
            for _ in range(reps):
                eng.process_host(x_host, out=yh)  # ProcessTo into the caller's buffer
                split = [a + b for a, b in zip(split, eng.host_io_profile())]
            dth = (time.perf_counter() - th) / reps
            split = [v / reps for v in split]
            hd = ys[last].cpu().numpy() if not mixdown else None
            pcie_bytes = C * (n + out_len) * 8
            # the same call through the staged path (host memcpy into pinned chunks)
            eng.set_host_io(eng.HOST_IO_STAGE)
            eng.process_host(x_host, out=yh)
            ts = time.perf_counter()
            for _ in range(2):
                eng.process_host(x_host, out=yh)
            dts = (time.perf_counter() - ts) / 2
            eng.set_host_io(eng.HOST_IO_AUTO)
            host_io = {"value": round(C * n / dth / 1e6, 3), "unit": "Msamples/s", "ms_per_call": round(dth * 1e3, 3),
                       "bytes_per_sample_pcie": 8 + 8 * out_len / n,
                       "split_ms": {"hipHostRegister": round(split[0], 3), "transfers_and_compute": round(split[1], 3),
                                    "hipHostUnregister": round(split[2], 3)},
                       "pcie_GBps_in_transfer_phase": round(pcie_bytes / (split[1] * 1e-3) / 1e9, 2) if split[1] else None,
                       "staged_path": {"value": round(C * n / dts / 1e6, 3), "ms_per_call": round(dts * 1e3, 3)},
                       "equals_device_result": bool(hd is not None and np.array_equal(yh, hd)),
                       "note": "host buffer in -> host buffer out per call (ad_conv_ols_process_multi), "
                               "PCIe + host copies included; wall time.  Default path: the caller's pages are "
                               "registered for the call (split_ms); staged_path: memcpy through pinned chunks"}
            del yh, hd
        shard_sub = None
        if world == 1 and args.workload == "conv" and args.shard_sub == "on" and not shard_cfg:
            ys.clear(), mixes.clear()
            r8 = run_conv(args, 1, 0, rt, ir, 8, True, True, min(args.steps, 5), 2, "off")
            fused = args.mix_fused == "on"
            shard_sub = {"value": round(8 * n * min(args.steps, 5) / r8["elapsed"] / 1e6, 3), "unit": "Msamples/s",
                         "ms_per_step": round(r8["elapsed"] / min(args.steps, 5) * 1e3, 4),
                         "workload": f"config 4 shard at N = 1: 8 ch x {n} samples (IR[c mod 2]), device-resident, " +
                                     ("stereo mixdown fused into the inverse transform "
                                      "(ad_conv_multi_process_device_mix) + " if fused else "k_mixdown + ") +
                                     "RCCL reduce through ad_mixdown_reduce (world 1), the per-GPU work of every "
                                     "rank at N > 1",
                         "kernels_avg_us": {k: round(v[0] / max(v[1], 1) * 1e3, 1) for k, v in r8["prof"].items()},
                         "mixdown_reduce": r8["reduce_diag"],
                         "parity": output_parity(args, r8, ir, 8, True)}
            r8["comm"].close()
            del r8
        legs_on = world == 1 and args.workload == "conv" and not shard_cfg
        if legs_on:
            # the legs get the process to themselves: the conv handle's stream
            # would share the device's 4 hardware queues with the effect chain's
            # three, and the low-latency streaming path pre-enqueues only while
            # the library owns at most 3 streams (include/algodsp.h)
            import gc

            r["eng"] = eng = None
            gc.collect()
        config5 = None
        if legs_on and args.fx_leg == "on":
            ys.clear(), mixes.clear()
            config5 = fx_measure(args, 1, 0, local, dev, 5, 2, not args.no_cpu_baseline, n=1 << 20)
            rt.empty_cache()
        config2 = None
        if legs_on and args.stream_leg == "on":
            config2 = stream_measure(1024, 32, not args.no_cpu_baseline)
        correlate = None
        if legs_on and args.corr_leg == "on":
            correlate = corr_measure(40, 3, not args.no_cpu_baseline)
            rt.empty_cache()
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(ir, args.cpu_sample)
        traffic = None
        step_pmc = None
        tfile = ROOT / "profiles" / "pmc_traffic.json"
        if tfile.exists():
            try:
                tab = json.loads(tfile.read_text())
                # only for the per-GPU workload the PMC passes ran
                same = tab.get("_config") == {"channels": C, "samples": n, "hop": args.hop}
                key = next((k for k in tab if k == dom or k.startswith(dom)), None)
                traffic = tab[key]["hbm_bytes_per_launch"] if key and same else None
                if same and world == 1 and not shard_cfg:
                    # the whole step: K1 + K2 + K3's PMC bytes (one launch each per step at N = 1)
                    ks = [k for k in tab if k.startswith(("k_window_rfft", "k_fdl_mac", "k_irfft_store"))]
                    step_pmc = sum(tab[k]["hbm_bytes_per_launch"] for k in ks) if len(ks) == 3 else None
            except Exception:
                traffic = None
        workload = ("OverlapSave partitioned conv, stereo, 131072-tap IR, full linear convolution, "
                    "input and output device-resident (PCIe excluded; host_io is the host-buffer rate) "
                    if not shard_cfg else
                    f"{C * world}-channel x 131072-tap IR convolution reverb (IR[c mod 2]), channels "
                    f"sharded {C}-per-GPU, device-resident (PCIe excluded)" +
                    ((", stereo mixdown fused into the inverse transform" if args.mix_fused == "on" else
                      ", k_mixdown") + " + RCCL reduce (ad_mixdown_reduce) " if mixdown else " "))
        line = {
            "metric": "Msamples/sec, overlap-save conv 131072-tap IR @48kHz; achieved HBM GB/s",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "clock_settle_steps": args.clock_settle,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: SplitMix64 white noise (seed 0x5EED+channel) x Large Church IR from web/irs.irlib "
                    "(f16, reference decodeF16), zero padded 95432->131072 taps",
            "config": {
                "workload": workload + f"({C} ch x {n} samples per GPU per step)",
                "baseline_config": "configs[3] shard" if shard_cfg else "configs[2]",
                "channels_per_gpu": C,
                "samples_per_channel": n,
                "kernel_taps": K,
                "hop": args.hop,
                "partitions": (K + args.hop - 1) // args.hop,
                "schedule": {"mode": ["serial", "pipelined", "chunked"][r["schedule"][0]], "chunk_blocks": r["schedule"][1]},
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
                "timing": "HIP events on the launch stream, " + (
                    "inside the timed region (that kernel's launches only; the other kernels' table "
                    "entries from a pass after it)" if mode == "dominant" else
                    "inside the timed region" if mode == "on" else "separate pass after the timed region"),
            },
            "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in kernels.items()},
            "parity": parity,
            "host_io": host_io,
            "shard_per_gpu": shard_sub,
            "cpu_baseline": cpu,
        }
        if step_pmc:
            alg = 80 * C * n  # x in, y out, X and Z written and read: 8 + 8 + 32 + 32 B per sample
            sec = elapsed / args.steps
            line["step_hbm"] = {"pmc_bytes": step_pmc, "alg_bytes": alg,
                                "frac_pmc": round(step_pmc / sec / 1e9 / HBM_PEAK_GBS, 4),
                                "frac_alg": round(alg / sec / 1e9 / HBM_PEAK_GBS, 4),
                                "note": "whole step at ms_per_step against 8 TB/s: PMC bytes of K1 + K2 + K3 "
                                        "(profiles/pmc_traffic.json, FETCH_SIZE x 2 + WRITE_SIZE) and the 80 B/sample "
                                        "algorithmic figure"}
        if r["step_ms"]:
            line["step_ms"] = r["step_ms"]  # each timed step, event-timed on the launch stream
        if r["settled"]:
            line["settled"] = dict(r["settled"], value=round(C * n / (r["settled"]["median_ms_last_half"] * 1e-3) / 1e6, 3),
                                   note="the same step after the timed region once the board's clock has recovered "
                                        "from its load-onset dip (median of the last half of the settle steps); "
                                        "not `value`")
        if config5 is not None:
            line["config5"] = config5
        if config2 is not None:
            line["config2_stream"] = config2
        if correlate is not None:
            line["correlate"] = correlate
        if r["reduce_diag"] is not None:
            line["mixdown_reduce"] = dict(r["reduce_diag"], note=(
                "max over ranks; conv_ms_per_step: the same step with the reduce off; reduce_ms: RCCL reduce "
                "of the stereo partial mix (ad_mixdown_reduce) event-timed on the side stream; overlap: the share "
                "of reduce_ms the step did not pay; hide_GBps: the reduce rate that fits under the convolution"))
        if world > 1:
            line["like_for_like_base"] = ("shard_per_gpu of the N = 1 line: the same 8 ch x 2^24 per GPU with "
                                          "the mixdown fused into K3, at world 1")
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


def output_parity(args, r, ir, C_total, mixdown):
    """Parity of a measured step's output itself: 64-sample windows of the last
    step's result (the whole-job stereo mix when the mixdown runs, else every
    channel) against exact float64 dot products -- the signal start, K2 run
    boundaries of the stereo (R = 176-192) and the shard (R = 688) geometries,
    the middle and the tail of the output."""
    import numpy as np

    from algodsp import signals

    K, n, out_len, L = ir.shape[1], args.samples, r["out_len"], args.hop
    wins = sorted({t for t in (K - 32, 192 * L - 32, 16 * L - 7, 688 * L - 32, out_len // 2, out_len - 64)
                   if 0 <= t <= out_len - 64})
    errs = []
    if mixdown:
        got = r["mixes"][r["last"]].cpu().numpy()
        for s_ in range(2):
            for t0w in wins:
                ref = np.zeros(64)
                a0 = t0w - K + 1
                lo, hi = max(0, a0), min(n, t0w + 64)
                for c in range(C_total):
                    if c % 2 == s_ and hi > lo:
                        # the input span this window reads, regenerated (counter-based noise)
                        seg = np.zeros(64 + K - 1)
                        seg[lo - a0:hi - a0] = signals.white_noise(hi - lo, 0x5EED + c, start=lo)
                        ref += np.convolve(seg, ir[c % 2], mode="valid")
                errs.append(got[s_, t0w:t0w + 64] - ref)
    else:
        got = r["ys"][r["last"]].cpu().numpy()
        for ci, c in enumerate(r["ids"]):
            for t0w in wins:
                errs.append(got[ci, t0w:t0w + 64] - exact_window(r["x_host"][ci], ir[c % 2], t0w, 64))
    err = np.concatenate(errs)
    parity = {"rms": float(np.sqrt(np.mean(err ** 2))), "max_abs": float(np.max(np.abs(err))),
              "outputs_checked": int(err.size),
              "against": "exact float64 dot products (numpy) over windows at " + ", ".join(map(str, wins)) +
                         (f" of the whole-job stereo mix ({C_total} channels)" if mixdown else " of every channel"),
              "tolerance_rms": 1e-7}
    if parity["rms"] > 1e-7:
        print(f"bench.py: PARITY FAILURE {parity}", file=sys.stderr)
    return parity


def run_conv(args, world, rank, rt, ir, C, shard_cfg, mixdown, steps, warmup, mode, settle_steps=0, pre_steps=0):
    """One conv measurement: C channels x args.samples per GPU per step (IR[c mod 2]),
    optionally with the RCCL stereo mixdown; `steps` timed steps after `warmup`,
    bracketed by barrier + synchronize, max over ranks.  Returns the timing, the
    per-kernel event profile and the buffers for the parity check.  `rt`
    supplies the device, streams, events, the engine and the communicator
    (GpuRuntime; a CPU stand-in in tests/test_bench_orchestration.py)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from algodsp import shard, signals

    dev = rt.dev

    K = ir.shape[1]
    n = args.samples
    comm = None
    out_len = n + K - 1                             # full linear convolution (OverlapSave.Process)
    if mixdown and C % 2 and world > 1:
        raise SystemExit("--channels must be even for the multi-GPU stereo mixdown")
    ids = list(shard.channel_group(rank, world, C * world))  # this rank's global channel ids
    x_host = np.stack([signals.white_noise(n, 0x5EED + c) for c in ids])
    x = torch.from_numpy(x_host).to(dev)
    # Mixdown through the library's own RCCL communicator (ad_mixdown_reduce),
    # the path a cgo caller takes: k_mixdown of this rank's group + one
    # in-place sum-reduce to rank 0, on a side stream.  Two output buffers:
    # step i's mixdown/reduce overlaps step i+1's convolution into the other
    # buffer; a buffer is rewritten only after its reduce (event wait on the
    # device, no host block).  The last step's reduce completes inside the
    # timed region.
    if mixdown:
        def bootstrap(uid: bytes) -> bytes:
            if world == 1:
                return uid
            obj = [uid]
            dist.broadcast_object_list(obj, src=0)
            return obj[0]

        comm = rt.comm(rank, world, bootstrap)
    nbuf = 2 if (mixdown and args.pipeline == "on") else 1
    # fused: the engine writes the stereo mix directly (no per-channel rows)
    fused = mixdown and C != 2 and args.mix_fused == "on"
    ys = [torch.empty((2 if fused else C, out_len), dtype=torch.float64, device=dev) for _ in range(nbuf)]
    mixes = [y if (C == 2 or fused) else torch.empty((2, out_len), dtype=torch.float64, device=dev) for y in ys]

    eng = rt.engine(ir, args.hop, C, shard.ir_index(ids), args.chunk)
    if args.schedule != "serial":
        eng.set_schedule(["serial", "pipelined", "chunked"].index(args.schedule), args.pipe_chunk, args.pipe_run)
    stream = rt.current_stream()
    sptr = stream.cuda_stream
    side = rt.new_stream() if mixdown else None  # mixdown + reduce
    blocks = -(-out_len // args.hop)
    cuts = [min(out_len, args.hop * (blocks * i // args.segments)) for i in range(args.segments + 1)]
    segs = [(b, e) for b, e in zip(cuts[:-1], cuts[1:]) if e > b]
    red_done = [None] * nbuf
    it = [0]
    reduce_on = [True]   # off: the conv-only steps after the timed region (N > 1 diagnostics)
    red_ev = []          # (start, end) timing events around each reduce on the side stream

    def step():
        i = it[0] % nbuf
        it[0] += 1
        if red_done[i] is not None:  # the reduce that last read this buffer
            stream.wait_event(red_done[i])
        yb, mb = ys[i], mixes[i]
        for b, e in segs:
            if fused:
                eng.process_device_mix(x.data_ptr(), n, n, mb.data_ptr(), out_len, out_len, ids[0] % 2, b, e, sptr)
            elif len(segs) == 1:
                eng.process_device(x.data_ptr(), n, n, yb.data_ptr(), out_len, out_len, sptr)
            else:
                eng.process_device_segment(x.data_ptr(), n, n, yb.data_ptr(), out_len, out_len, b, e, sptr)
            if mixdown and reduce_on[0]:
                done = rt.event()
                done.record(stream)
                side.wait_event(done)
                r0, r1 = rt.event(True), rt.event(True)
                r0.record(side)
                # stereo group or fused mix: mb already holds the partial mix (no k_mixdown)
                comm.mixdown_reduce(yb.data_ptr() + 8 * b, 0 if (C == 2 or fused) else C, out_len, e - b,
                                    mb.data_ptr() + 8 * b, out_len, ids[0] % 2, 0, side.cuda_stream)
                r1.record(side)
                red_ev.append((r0, r1))
        if mixdown and reduce_on[0]:
            ev = rt.event()
            ev.record(side)
            red_done[i] = ev

    def drain():
        if mixdown:
            side.synchronize()

    for _ in range(pre_steps + warmup):  # pre_steps: the clock settle (--clock-settle)
        step()
    drain()
    rt.synchronize()
    eng.profile_read()  # clear

    dom_mask = 7
    if mode == "dominant":  # one profiled warm-up pass names the dominant kernel
        eng.profile_enable(True)
        for _ in range(2):
            step()
        drain()
        rt.synchronize()
        pw = eng.profile_read()
        dom_mask = 1 << list(pw).index(max(pw, key=lambda k: pw[k][0]))
    eng.profile_enable(mode != "off", kernels=dom_mask if mode == "dominant" else 7)
    if world > 1:
        dist.barrier()
    rt.synchronize()
    red_ev.clear()
    # per-step events on the launch stream (record only: no host wait inside the loop)
    sev = ([rt.event(True) for _ in range(steps + 1)]
           if world == 1 and args.step_events == "on" else None)
    t0 = time.perf_counter()
    if sev:
        sev[0].record(stream)
    for i in range(steps):
        step()
        if sev:
            sev[i + 1].record(stream)
    drain()
    rt.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = [round(sev[i].elapsed_time(sev[i + 1]), 4) for i in range(steps)] if sev else None
    last = (it[0] - 1) % nbuf
    # the reduces of the timed steps, event-timed on the side stream
    reduce_ms = sum(a.elapsed_time(b) for a, b in red_ev) / steps if red_ev else 0.0
    red_ev.clear()
    prof_live = eng.profile_read() if mode != "off" else {}
    if mode != "on":  # the kernels not timed live: a separate event-timed pass
        eng.profile_enable(True)
        for _ in range(max(2, steps // 2)):
            step()
        drain()
        rt.synchronize()
        last = (it[0] - 1) % nbuf
        prof = eng.profile_read()
        for k, v in prof_live.items():  # live (timed-region) numbers win
            if v[1] > 0:
                prof[k] = v
    else:
        prof = prof_live
    eng.profile_enable(False)

    conv_elapsed = None
    if mixdown:
        # the same step with the reduce off: what the convolution alone takes
        # (N > 1 diagnostics: does the reduce hide?)
        reduce_on[0] = False
        ksteps = min(steps, 5)
        step()
        rt.synchronize()
        if world > 1:
            dist.barrier()
        tc = time.perf_counter()
        for _ in range(ksteps):
            step()
        rt.synchronize()
        if world > 1:
            dist.barrier()
        conv_elapsed = (time.perf_counter() - tc) / ksteps * steps
        reduce_on[0] = True
        red_done[:] = [None] * nbuf
        # one full step again, so the buffers the parity check reads hold a
        # reduced (whole-job) mix
        step()
        drain()
        rt.synchronize()
        last = (it[0] - 1) % nbuf
    conv_elapsed = conv_elapsed if conv_elapsed is not None else 0.0
    if world > 1:
        t = torch.tensor([elapsed, conv_elapsed, reduce_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, conv_elapsed, reduce_ms = (float(v) for v in t.tolist())
    diag = None
    if mixdown:
        diag = shard.scaling_diagnostics(elapsed / steps * 1e3, conv_elapsed / steps * 1e3, reduce_ms,
                                         2 * out_len * 8)

    settled = None
    if world == 1 and not mixdown and settle_steps > 0:
        # The board's clock dips for a few ms once the load turns sustained and then
        # recovers (tools/step_curve.py): the same step after
        # the timed region, event-timed per step, median of the last half.  Reported
        # beside `value`, never as it.
        ev = [rt.event(True) for _ in range(settle_steps + 1)]
        ev[0].record(stream)
        for i in range(settle_steps):
            step()
            ev[i + 1].record(stream)
        rt.synchronize()
        per = [ev[i].elapsed_time(ev[i + 1]) for i in range(settle_steps)]
        tail = sorted(per[settle_steps // 2:])
        settled = {"steps": settle_steps, "median_ms_last_half": round(tail[len(tail) // 2], 4),
                   "max_ms": round(max(per), 4), "min_ms": round(min(per), 4)}
        last = (it[0] - 1) % nbuf

    return {"elapsed": elapsed, "prof": prof, "prof_live": prof_live, "ids": ids, "x_host": x_host, "eng": eng,
            "ys": ys, "mixes": mixes, "last": last, "comm": comm, "out_len": out_len, "schedule": eng.schedule(),
            "reduce_diag": diag, "step_ms": step_ms, "settled": settled}


def stream_measure(nblk: int, warmup_blocks: int, cpu_leg: bool) -> dict:
    """BASELINE config 2: StreamingOverlapSave(K=16384, B=4096) driven block by
    block through the host-buffer ABI, as a Go caller would (ProcessBlockTo per
    block: PCIe in, UPOLS on the GPU, PCIe out, synchronous; reference
    streaming_overlap_save.go:100-164).  Per-block wall times give p50 / p99;
    parity: the measured output's first blocks against exact float64 products."""
    import numpy as np

    from algodsp import conv, irlib, signals

    ir = irlib.large_church()[0, :16384]
    B = 4096
    x = signals.white_noise(nblk * B, 0x5EED)
    y = np.empty_like(x)
    s = conv.NewStreamingOverlapSave(ir, B)
    for i in range(min(warmup_blocks, nblk)):
        s.ProcessBlockTo(y[i * B:(i + 1) * B], x[i * B:(i + 1) * B])
    s.Reset()
    lat = np.empty(nblk)
    t0 = time.perf_counter()
    for i in range(nblk):
        tb = time.perf_counter()
        s.ProcessBlockTo(y[i * B:(i + 1) * B], x[i * B:(i + 1) * B])
        lat[i] = time.perf_counter() - tb
    dt = time.perf_counter() - t0
    hits, timeouts = s.LowLatencyStats()
    nchk = min(nblk, 4) * B
    ref = np.convolve(x[:nchk], ir)[:nchk]
    err = y[:nchk] - ref
    parity = {"rms": float(np.sqrt(np.mean(err ** 2))), "max_abs": float(np.max(np.abs(err))),
              "outputs_checked": int(nchk), "against": "exact float64 convolution (numpy) of the first blocks",
              "tolerance_rms": 1e-7}
    if parity["rms"] > 1e-7:
        print(f"bench.py: PARITY FAILURE (config 2) {parity}", file=sys.stderr)
    cpu = None
    if cpu_leg:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_lib as O

        o = O.Streaming(ir, B)
        m = min(nblk, 256)
        tc = time.perf_counter()
        for i in range(m):
            o.process_block(x[i * B:(i + 1) * B])
        dtc = time.perf_counter() - tc
        cpu = {"value": m * B / dtc / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port",
               "sample": f"{m} blocks of {B}, oracle StreamingOverlapSave (N=32768); {dtc:.1f} s"}
    us = lat * 1e6
    return {"value": round(nblk * B / dt / 1e6, 3), "unit": "Msamples/s", "blocks": nblk, "block": B,
            "kernel_taps": 16384, "ms_per_block": round(dt / nblk * 1e3, 4),
            "p50_us": round(float(np.percentile(us, 50)), 1), "p99_us": round(float(np.percentile(us, 99)), 1),
            "mean_us": round(float(us.mean()), 1), "max_us": round(float(us.max()), 1),
            "pre_enqueued_blocks": hits, "timed_out_blocks": timeouts,
            "workload": "config 2: StreamingOverlapSave mono K=16384 B=4096, host buffers in and out, one "
                        "synchronous ProcessBlockTo per block (PCIe + 3 kernels + completion wait per block)",
            "parity": parity, "cpu_baseline": cpu}


def main_stream(args):
    """BASELINE config 2 as its own line (replicas only)."""
    nblk = max(1, args.samples // 4096) if args.samples else 2048
    r = stream_measure(nblk, args.warmup * 8, not args.no_cpu_baseline)
    line = {
        "metric": "Msamples/sec, streaming overlap-save 16384-tap IR, 4096-sample blocks (config 2)",
        "value": r["value"], "unit": "Msamples/s", "n_gpus": 1, "steps": nblk,
        "warmup": args.warmup, "ms_per_step": r["ms_per_block"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: SplitMix64 white noise x Large Church L (first 16384 taps)",
        "config": {"workload": "StreamingOverlapSave mono K=16384 B=4096, host buffers, one block per step",
                   "block": 4096, "kernel_taps": 16384},
        "latency_us": {k: r[k] for k in ("p50_us", "p99_us", "mean_us", "max_us")},
        "note": "latency-bound: each block = H2D copy + 3 kernels + D2H copy + sync",
        "parity": r["parity"],
        "cpu_baseline": r["cpu_baseline"],
    }
    print(json.dumps(line), flush=True)


def _plan_radices(N):
    """Pass radices of the device FFT plan for size N (bigfft.hip BigFft::BigFft)."""
    k = max(0, N.bit_length() - 1)
    if k <= 3:
        return []
    if k <= 12:
        return [N]
    np_ = (k + 8) // 9
    base, extra = k // np_, k % np_
    return [1 << (base + (1 if p < extra else 0)) for p in range(np_)]


def corr_measure(steps: int, warmup: int, cpu_leg: bool, n: int | None = None, settle: int = 60) -> dict:
    """conv.CorrelateFFT (correlate.go:111-172) of two n-sample
    signals, one nextPow2(2n-1) = 2^24-point transform pair on the device
    (device-resident inputs/outputs; plans and work buffers cached), with the
    parity of the measured output and the CPU leg.  Replicas only."""
    import ctypes as C

    import numpy as np
    import torch

    from algodsp import _lib, signals

    dev = torch.device("cuda", 0)
    n = n or (1 << 23)
    ah, bh = signals.white_noise(n, 0x5EED), signals.white_noise(n, 0x5EEE)
    a = torch.from_numpy(ah).to(dev)
    b = torch.from_numpy(bh).to(dev)
    out = torch.full((2 * n - 1,), float("nan"), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    L = _lib.lib()

    def step():
        _lib.check(L.ad_correlate_fft_device(C.c_void_p(a.data_ptr()), n, C.c_void_p(b.data_ptr()), n,
                                             C.c_void_p(out.data_ptr()), 0, C.c_void_p(stream.cuda_stream)))

    for _ in range(settle + warmup):  # settle: the clock's load-onset dip
        step()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / steps
    # parity of the measured output: 16-lag windows (result[j] = sum_i a[i + j - (n-1)] b[i],
    # correlate.go:176-185) at the most negative lags, around lag 0, two middles and the
    # most positive lags, against exact float64 dot products (numpy)
    got = out.cpu().numpy()
    wins = [0, n // 3, n - 1 - 8, n - 1 + n // 2, 2 * n - 2 - 15]
    errs, refs = [], []
    for j0 in wins:
        for j in range(j0, j0 + 16):
            lag = j - (n - 1)
            ref = float(np.dot(ah[lag:], bh[:n - lag])) if lag >= 0 else float(np.dot(ah[:n + lag], bh[-lag:]))
            errs.append(got[j] - ref)
            refs.append(ref)
    errs, refs = np.array(errs), np.array(refs)
    scale = max(1.0, float(np.max(np.abs(refs))))
    parity = {"max_abs": float(np.max(np.abs(errs))), "rms": float(np.sqrt(np.mean(errs ** 2))),
              "max_rel": float(np.max(np.abs(errs)) / scale), "outputs_checked": int(errs.size),
              "no_nan": bool(not np.isnan(got).any()),
              "against": "exact float64 dot products (numpy) at lags " + ", ".join(str(j - (n - 1)) for j in wins) +
                         " (+0..15)",
              "tolerance": "max |err| <= 1e-10 max(1, max |ref|) (tests/test_spectral_gpu.py)"}
    if not (parity["max_rel"] <= 1e-10 and parity["no_nan"]):
        print(f"bench.py: CORRELATE PARITY FAILURE {parity}", file=sys.stderr)
    N = 1 << (2 * n - 2).bit_length()
    # algorithmic bytes per call (DESIGN.md "spectral row") of the passes the
    # call runs: the forward transform of a + i b (its first pass reads the
    # n + m real samples, zero padding is not read, and writes 16 B per bin;
    # each middle pass reads and writes 16 B per bin), the inverse at half
    # length (its middle passes 16 + 16 B per half bin, its last pass reading
    # 16 B per half bin and writing the n + m - 1 kept lags).  With the fused
    # forward-last / inverse-first pass (plans of 256 x 256 x ... both sides:
    # k_corr_fwd_last_inv_first) the packed spectrum Z is never stored: that
    # pass reads 16 B per bin and writes 16 B per half bin.  The max-abs
    # pre-pass (another read of a and b) is counted where it still runs.
    rad = _plan_radices(N)
    rad_h = _plan_radices(N // 2)
    P, Ph = len(rad), len(rad_h)
    fused = P >= 2 and Ph >= 2 and rad[-1] == 256 and rad_h[0] == 256 and N // 256 >= 16
    split = fused and rad == [256, 256, 256]
    fwd = 2 * n * 8 + N * 16 + N * 32 * (P - 2 if fused else P - 1)
    if fused:
        mid = N * 16 + (N // 2) * 16
        inv = (N // 2) * 32 * (Ph - 2) + (N // 2) * 16 + (2 * n - 1) * 8
    else:
        mid = 0
        inv = N * 16 + (N // 2) * 16 + (N // 2) * 32 * max(0, Ph - 2) + (N // 2) * 16 + (2 * n - 1) * 8
    alg = fwd + mid + inv + (0 if split else 2 * n * 8)
    gbs = alg / (ms * 1e-3) / 1e9
    cpu = None
    if cpu_leg:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_lib as O

        m = 1 << 20
        xa, xb = signals.white_noise(m, 1), signals.white_noise(m, 2)
        tc = time.perf_counter()
        O.correlate_fft(xa, xb)
        dtc = time.perf_counter() - tc
        cpu = {"value": 2 * m / dtc / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port",
               "sample": f"oracle CorrelateFFT of two 2^20-sample signals (N = 2^21 radix-2); {dtc:.2f} s"}
    # HBM bytes per call from the committed PMC passes of this same workload
    # (tools/gpu_corr_prof.sh -> tools/pmc_call_traffic.py), max-abs included
    traffic = None
    tfile = ROOT / "profiles" / "corr_pmc_traffic.json"
    if tfile.exists():
        try:
            tab = json.loads(tfile.read_text())
            if tab.get("_config") == {"workload": "corr", "n": n}:
                traffic = tab["hbm_bytes_per_call"]
        except Exception:
            traffic = None
    return {
        "value": round(2 * n / (ms * 1e-3) / 1e6, 3), "unit": "Msamples/s", "steps": steps, "warmup": warmup,
        "clock_settle_calls": settle,
        "ms_per_call": round(ms, 4),
        "workload": f"conv.CorrelateFFT n = m = {n}, FFT size {N} (forward: {P} device passes over a + i b; "
                    f"inverse: {Ph} passes at N/2{'; forward last + inverse first fused' if fused else ''}"
                    f"{'; max-abs in the first pass' if split else ''}), device-resident (PCIe excluded), "
                    f"event-timed over {steps} back-to-back calls",
        "fft_size": N,
        "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "note": "whole call: algorithmic bytes of the passes it runs (pointwise op, lag order and "
                             "the Z round trip fused away) / event time; traffic = HBM bytes per call from PMC "
                             "(FETCH_SIZE x2 + WRITE_SIZE, every kernel of the call)"},
        "parity": parity,
        "cpu_baseline": cpu,
        "wall_ms_per_call": round(dt / steps * 1e3, 4),
    }


def main_corr(args):
    r = corr_measure(args.steps, args.warmup, not args.no_cpu_baseline, args.samples, args.clock_settle)
    line = {
        "metric": "Msamples/sec, CorrelateFFT of two 2^23-sample signals (input samples per second)",
        "value": r["value"], "unit": "Msamples/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "clock_settle_calls": r["clock_settle_calls"], "ms_per_step": r["ms_per_call"],
        "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic: SplitMix64 white noise",
        "config": {"workload": r["workload"], "fft_size": r["fft_size"]},
        "roofline": r["roofline"], "parity": r["parity"], "cpu_baseline": r["cpu_baseline"],
        "wall_ms_per_step": r["wall_ms_per_call"],
    }
    print(json.dumps(line), flush=True)


def fx_chain_oracle(eq, comp_cfg, verb, fs, v):
    """One channel through the oracle chain (chain_process.go:11-33: biquad
    chains with the avx2 registry kernel's 4x-unrolled DF-II-T, Compressor,
    Freeverb); ctypes releases the GIL."""
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np

    import oracle_lib as O

    for co, g in eq:
        v, _ = O.biquad_chain_block(np.ravel(co), np.zeros(2 * len(co)), g, v)
    v = O.Compressor(fs, **comp_cfg).process_in_place(v)
    o = O.Freeverb()
    o.set(*verb)
    return o.process_in_place(v)


def fx_cpu_baseline(eq, comp_cfg, verb, fs, m):
    """The oracle chain on the host cores (one channel per thread, m/4 samples
    each), on one core (m samples), and the EQ alone on one core: five
    sections of the avx2 registry kernel's 4x-unrolled DF-II-T
    (internal/arch/amd64/avx2/register.go:23-66, oracle/or_filters.c), north
    star's "AVX2 biquad"."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    from algodsp import signals

    T = host_cores()
    vs = [0.5 * signals.white_noise(m // 4, 0x5EED + c) for c in range(T)]
    x1 = 0.5 * signals.white_noise(m, 0x5EED)
    tc = time.perf_counter()
    fx_chain_oracle(eq, comp_cfg, verb, fs, x1)
    dt = time.perf_counter() - tc
    with ThreadPoolExecutor(T) as ex:
        tc = time.perf_counter()
        list(ex.map(lambda v: fx_chain_oracle(eq, comp_cfg, verb, fs, v).size, vs))
        dtT = time.perf_counter() - tc
    coeffs = np.concatenate([np.ravel(co) for co, _ in eq])
    tq = time.perf_counter()
    O.biquad_chain_block(coeffs, np.zeros(2 * (coeffs.size // 5)), 1.0, x1)
    dtq = time.perf_counter() - tq
    return {"value": T * (m // 4) / dtT / 1e6, "unit": "Msamples/s", "cores": T, "kind": "port",
            "single_core": m / dt / 1e6,
            "eq_avx2_biquad_single_core": {"value": round(m / dtq / 1e6, 3), "unit": "Msamples/s",
                                           "sections": coeffs.size // 5,
                                           "sample": f"{m} samples through the config-5 EQ's 5 sections, "
                                                     f"oracle avx2 registry kernel (4x-unrolled DF-II-T), "
                                                     f"{dtq:.2f} s"},
            "sample": f"oracle biquad chains + Compressor + Freeverb, one channel of {m // 4} samples per "
                      f"host thread on {T} threads ({dtT:.2f} s); single_core: 1 channel x {m} samples "
                      f"({dt:.2f} s)"}


def fx_measure(args, world, rank, local, dev, steps, warmup, cpu_leg, graph=None, n=None, parity_on=True) -> dict:
    """BASELINE config 5: effectchain filter(x5 RBJ) -> dyn-compressor ->
    reverb-freeverb on 256 channels x 2^20 samples (device buffers, the
    engine AUTO picks), `steps` timed calls after `warmup`; barrier +
    synchronize around them, max over ranks.  Parity: a fresh chain over the
    same input against the oracle chain on channels 0 and 255 (a 2^17-sample
    prefix: the chain is causal)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from algodsp import design, processors, signals

    fs = 48000.0
    C = 256
    n = n or (1 << 20)
    eq = design.config5_eq(fs)
    comp_cfg = {"auto_makeup": 0, "makeup_db": 0.0}  # runtime_dynamics.go:46-54
    verb = (0.22, 1.0, 0.72, 0.45, 0.015)
    x_host = np.stack([0.5 * signals.white_noise(n, 0x5EED + c) for c in range(C)])
    x = torch.from_numpy(x_host).to(dev)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    if graph:  # the batched effectchain graph runtime
        from algodsp import effectchain

        fx = effectchain.Chain(fs, C, designer=design.RBJDesigner(), device=local)
        fx.LoadGraph(effectchain.EXAMPLE_GRAPHS[graph])
    else:
        fx = processors.EffectChain(C, eq, comp_cfg, verb, fs, device=local)

    def step():
        fx.process_device(x.data_ptr(), n, n, sptr)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    value = world * C * n * steps / elapsed / 1e6
    engine = None
    if not graph:
        eng_id, noise = fx.LastEngine()
        engine = {"id": eng_id, "name": {1: "fused", 2: "staged_nosplit", 3: "staged", 4: "time_parallel"}.get(
            eng_id, str(eng_id)), "eq_noise_estimate": noise}
    parity = None
    if parity_on and not graph and rank == 0:
        fx.Reset()
        x.copy_(torch.from_numpy(x_host))
        step()
        torch.cuda.synchronize(dev)
        m0 = min(n, 1 << 17)
        errs = []
        for c in (0, C - 1):
            got = x[c, :m0].cpu().numpy()
            want = fx_chain_oracle(eq, comp_cfg, verb, fs, x_host[c, :m0].copy())
            errs.append(got - want)
        err = np.concatenate(errs)
        ref_rms = float(np.sqrt(np.mean(np.concatenate([x_host[0, :m0], x_host[-1, :m0]]) ** 2)))
        parity = {"rms": float(np.sqrt(np.mean(err ** 2))), "max_abs": float(np.max(np.abs(err))),
                  "outputs_checked": int(err.size),
                  "against": f"oracle chain (biquad chains -> Compressor -> Freeverb) on channels 0 and {C - 1}, "
                             f"first {m0} samples, fresh chain state",
                  "tolerance_rms": 1e-12, "input_rms": ref_rms}
        if parity["rms"] > 1e-12:
            print(f"bench.py: PARITY FAILURE (config 5) {parity}", file=sys.stderr)
    cpu = fx_cpu_baseline(eq, comp_cfg, verb, fs, 1 << 25) if cpu_leg and world == 1 and rank == 0 else None
    # The bound is the one serial recurrence left, not HBM (16 B/sample of
    # input and output moves 0.5 % of peak): the time-parallel engine cuts the
    # EQ sections and the Freeverb combs into time segments, but the envelope
    # follower (attack or release by the sign of src - env) is serial per
    # channel, 24.5 clocks per sample (tools/chain_latency.hip).
    # Ceiling = clock x channels / 24.5.
    ceiling = FX_CLOCK_HZ * C / FX_CHAIN_CLK / 1e6
    return {
        "value": round(value, 3), "unit": "Msamples/s", "steps": steps, "warmup": warmup,
        "ms_per_step": round(elapsed / steps * 1e3, 3), "channels_per_gpu": C, "samples_per_channel": n,
        "workload": (f"effectchain graph '{graph}' through the batched graph runtime ({fx.op_count()[0]} device "
                     f"ops per call), {C} ch x {n} samples per GPU per step" if graph else
                     f"effectchain filter x5 (RBJ) -> dyn-compressor -> reverb-freeverb, {C} ch x {n} samples "
                     f"per GPU per step, device buffers, engine AUTO"),
        "engine": engine,
        "roofline": {"bound": "serial-recurrence latency (compressor envelope)", "achieved": round(value, 3),
                     "peak": round(ceiling, 1), "unit": "Msamples/s", "frac": round(value / ceiling, 4),
                     "traffic": None, "hbm_GBps": round(value * 16e6 / 1e9, 3),
                     "note": f"ceiling = {FX_CLOCK_HZ / 1e9} GHz x {C} channels / {FX_CHAIN_CLK} clk per sample "
                             f"(the envelope follower's dependency chain, each channel's own); HBM carries "
                             f"16 B/sample of input and output"},
        "parity": parity, "cpu_baseline": cpu,
    }


def main_fx(args):
    """BASELINE config 5 as its own line.  Replicas only for N > 1."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    r = fx_measure(args, world, rank, local, dev, args.steps, args.warmup, not args.no_cpu_baseline,
                   graph=args.graph, n=args.samples)
    if rank == 0:
        line = {
            "metric": "Msamples/sec, effectchain biquad EQ + Compressor + Freeverb (config 5)",
            "value": r["value"], "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": r["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: 0.5 x SplitMix64 white noise, 48 kHz",
            "config": {"workload": r["workload"], "channels_per_gpu": r["channels_per_gpu"],
                       "samples_per_channel": r["samples_per_channel"],
                       "parallelism": "replicas" if world > 1 else "single GPU"},
            "engine": r["engine"],
            "roofline": r["roofline"],
            "parity": r["parity"],
            "cpu_baseline": r["cpu_baseline"],
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    # stdout carries exactly one JSON line: native libraries that print to
    # fd 1 (RCCL's version banner at comm init) are sent to stderr, and
    # Python's stdout keeps a private duplicate of the original fd 1.
    sys.stdout.flush()
    sys.stdout = os.fdopen(os.dup(1), "w", buffering=1)
    os.dup2(2, 1)
    sys.exit(main() or 0)
