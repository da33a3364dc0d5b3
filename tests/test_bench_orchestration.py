"""bench.py's N > 1 orchestration, executed at world 2 over gloo on the CPU.

bench.conv_main / bench.run_conv are the code the driver's 8-GPU run executes:
the unique-id bootstrap through broadcast_object_list, the two-buffer reduce
pipeline (step i's mixdown reduce on a side stream beside step i+1's
convolution, a buffer rewritten only after its reduce's event), the output
segments, the conv-only pass after the timed region, the max-over-ranks
timing and rank 0's parity of the whole-job stereo mix and its JSON line.
Here the same functions run with CPU stand-ins for what GpuRuntime supplies:
streams and events that order nothing (the CPU runs in program order), the
engine as a numpy FFT convolution per channel written through the same raw
pointers, and the communicator as k_mixdown in numpy plus a gloo sum-reduce of
the caller's mix buffer in place.  The per-rank operation is OverlapSave.Process
(dsp/conv/overlap_save.go:126-254) per channel; the GPU side of each call is
covered by the -m gpu tests (test_config4_shard, test_schedule_gpu).
"""
import contextlib
import ctypes
import io
import json
import os
import pathlib
import subprocess
import sys
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _view(ptr: int, count: int) -> np.ndarray:
    return np.ctypeslib.as_array((ctypes.c_double * count).from_address(ptr))


class _Event:
    def __init__(self, timing=False):
        self.t = None

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3

    def synchronize(self):
        pass


class _Stream:
    cuda_stream = 0

    def wait_event(self, ev):
        assert ev.t is not None, "waiting on an event that was never recorded"

    def synchronize(self):
        pass


class _Engine:
    """conv.MultiChannelConvolver's device calls as a numpy FFT convolution."""

    KERNELS = ("k_window_rfft", "k_fdl_mac", "k_irfft_store")

    def __init__(self, ir, hop, channels, ir_index):
        from scipy.signal import fftconvolve

        self.fftconvolve = fftconvolve
        self.ir, self.hop, self.C, self.ids = ir, hop, channels, list(ir_index)
        self.prof_on, self.mask = False, 7
        self.prof = {k: [0.0, 0, 0.0] for k in self.KERNELS}
        self.cache = {}
        self.calls = []

    def _y(self, d_in, in_stride, n):
        key = (d_in, in_stride, n)
        if key not in self.cache:
            x = _view(d_in, self.C * in_stride).reshape(self.C, in_stride)[:, :n]
            self.cache[key] = np.stack([self.fftconvolve(x[c], self.ir[self.ids[c]]) for c in range(self.C)])
        return self.cache[key]

    def _count(self):
        if self.prof_on:
            for i, k in enumerate(self.KERNELS):
                if self.mask >> i & 1:
                    self.prof[k][0] += 0.1 * (i + 1)
                    self.prof[k][1] += 1
                    self.prof[k][2] += 1e6

    def process_device(self, d_in, in_stride, in_len, d_out, out_stride, out_len, stream=0):
        self.process_device_segment(d_in, in_stride, in_len, d_out, out_stride, out_len, 0, out_len, stream)

    def process_device_segment(self, d_in, in_stride, in_len, d_out, out_stride, out_len, b, e, stream=0):
        y = self._y(d_in, in_stride, in_len)
        out = _view(d_out, self.C * out_stride).reshape(self.C, out_stride)
        out[:, b:e] = y[:, b:e]
        self.calls.append(("segment", b, e))
        self._count()

    def process_device_mix(self, d_in, in_stride, in_len, d_mix, mix_stride, out_len, first_parity=0, b=0, e=0,
                           stream=0):
        e = e or out_len
        y = self._y(d_in, in_stride, in_len)
        mix = _view(d_mix, 2 * mix_stride).reshape(2, mix_stride)
        for s in range(2):
            mix[s, b:e] = sum(y[c, b:e] for c in range(self.C) if (first_parity + c) % 2 == s)
        self.calls.append(("mix", b, e))
        self._count()

    def profile_enable(self, on=True, kernels=7):
        self.prof_on, self.mask = on, kernels

    def profile_read(self):
        out = {k: tuple(v) for k, v in self.prof.items()}
        self.prof = {k: [0.0, 0, 0.0] for k in self.KERNELS}
        return out

    def set_schedule(self, mode, chunk_blocks=0, run_blocks=0):
        pass

    def schedule(self):
        return 0, 0


class _Comm:
    """ad_comm_* / ad_mixdown_reduce: k_mixdown + an in-place sum-reduce to root."""

    def __init__(self, rank, world, bootstrap):
        uid = bytes([0xA5]) * 128 if rank == 0 else bytes(128)
        got = bootstrap(uid)
        assert got == bytes([0xA5]) * 128, "bootstrap did not move rank 0's unique id"
        self.reduces = 0

    def mixdown_reduce(self, d_chan, channels, stride, length, d_mix, mix_stride, first_parity=0, root=0, stream=0):
        for s in range(2):
            row = _view(d_mix + 8 * s * mix_stride, length)
            if channels:
                row[:] = sum(_view(d_chan + 8 * c * stride, length) for c in range(channels)
                             if (first_parity + c) % 2 == s)
            dist.reduce(torch.from_numpy(row), dst=root)
        self.reduces += 1

    def close(self):
        pass


class CpuRuntime:
    dist_backend = "gloo"

    def __init__(self):
        self.dev = torch.device("cpu")
        self.s0, self.engines, self.comms = _Stream(), [], []

    def current_stream(self):
        return self.s0

    def new_stream(self):
        return _Stream()

    def event(self, timing=False):
        return _Event(timing)

    def synchronize(self):
        pass

    def engine(self, ir, hop, channels, ir_index, chunk_blocks):
        e = _Engine(ir, hop, channels, ir_index)
        self.engines.append(e)
        return e

    def comm(self, rank, world, bootstrap):
        c = _Comm(rank, world, bootstrap)
        self.comms.append(c)
        return c

    def empty_cache(self):
        pass


def _worker(rank, world, port, argv, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, str(ROOT))
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        args = bench.parse(argv)
        rt = CpuRuntime()
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            rc = bench.conv_main(args, rt, world, rank, 0)
        eng, comm = rt.engines[0], rt.comms[0]
        q.put((rank, rc, buf.getvalue(), eng.calls, comm.reduces))
    except BaseException as e:  # report, do not hang the other rank's queue read
        q.put((rank, -1, repr(e), [], 0))
        raise


def _run_world(argv, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, world, port, argv, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, rc, out, calls, reduces = q.get(timeout=240)
        res[rank] = (rc, out, calls, reduces)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


BASE = ["--gpus", "2", "--steps", "3", "--warmup", "1", "--clock-settle", "2", "--samples", "8192", "--no-cpu-baseline",
        "--host-io", "off", "--shard-sub", "off", "--fx-leg", "off", "--stream-leg", "off"]


@pytest.mark.parametrize("extra", [
    [],                                  # the driver's default: fused mix + two-buffer pipeline
    ["--mix-fused", "off"],              # per-channel outputs + k_mixdown inside the reduce
    ["--segments", "3"],                 # each segment's reduce starts as soon as it is computed
    ["--pipeline", "off"],               # one buffer, each reduce waited on before the next step
], ids=["fused", "kmixdown", "segments", "no-pipeline"])
def test_conv_main_world2_over_gloo(extra):
    res = _run_world(BASE + extra)
    assert {r: v[0] for r, v in res.items()} == {0: 0, 1: 0}
    assert res[1][1] == "", "only rank 0 prints"
    line = json.loads(res[0][1].strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["channels_per_gpu"] == 8 and "RCCL reduce" in line["config"]["parallelism"]
    # whole-job aggregate: 2 ranks x 8 channels x 8192 samples x 3 steps
    assert line["value"] == pytest.approx(2 * 8 * 8192 * 3 / (line["ms_per_step"] * 3e-3) / 1e6, rel=1e-3)
    # rank 0's parity: the reduced whole-job stereo mix (16 channels) against exact dot products
    par = line["parity"]
    assert "16 channels" in par["against"] and par["outputs_checked"] > 0
    assert par["rms"] < 1e-9, par
    diag = line["mixdown_reduce"]
    assert diag["conv_ms_per_step"] > 0 and diag["reduce_ms"] > 0 and diag["step_over_conv"] > 0
    assert line["roofline"]["kernel"] in _Engine.KERNELS
    segs = 3 if "--segments" in extra else 1
    for rank in (0, 1):
        calls, reduces = res[rank][2], res[rank][3]
        kind = "segment" if "--mix-fused" in extra else "mix"
        assert all(c[0] == kind for c in calls)
        # every step with the reduce on reduces each segment once; the conv-only pass does not
        steps_total = len(calls) // segs
        conv_only = 1 + min(3, 5)
        assert reduces == (steps_total - conv_only) * segs


def test_rank_mismatch_exits_before_any_gpu_call():
    """WORLD_SIZE disagreeing with --gpus exits with status 2 before bench.py
    imports torch (so before any HIP call)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    code = ("import sys, runpy; sys.argv = ['bench.py', '--gpus', '4']\n"
            "try:\n    runpy.run_path('bench.py', run_name='__main__')\n"
            "except SystemExit as e:\n    assert 'torch' not in sys.modules, 'torch imported'\n    raise\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, (p.returncode, p.stderr)
    assert "WORLD_SIZE=2 but --gpus 4" in p.stderr
