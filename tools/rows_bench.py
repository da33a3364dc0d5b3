#!/usr/bin/env python3
"""Per-row measurement of SURVEY 8(a)'s hot-path functions on one MI355X.

For every row: the device entry point on HBM-resident buffers, timed with HIP
events on the stream the work is enqueued on (torch's current stream, passed
through the C ABI), its algorithmic bytes or flops -> roofline fraction, and
the oracle (CPU restatement of the reference, 1 core) timed on a bounded
sample of the same workload beside it.  Host-buffer rows (streaming and
partitioned convolution, batch OverlapSave / OverlapAdd) are wall-clock per
call through the same ABI a Go caller would use (PCIe included).

  python tools/rows_bench.py [--out gpurun_out/rows.json] [--quick]

Peaks: HBM 8.0 TB/s (MI355X_MICROARCH.md); FP64 vector 78.6 TFLOP/s (MI355X
spec sheet, FMA counted as 2 flops).  Rows bound by serial per-channel
recurrences (biquad, compressor, Freeverb) are reported against HBM with
their 16 B/sample, and the note says they are latency-bound, not HBM-bound.
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
sys.path.insert(0, str(ROOT / "tests"))

HBM = 8000.0     # GB/s
FP64 = 78.6      # TFLOP/s, FMA = 2 flops


def dev_time(fn, reps: int, warm: int = 2):
    """Mean ms per call of fn(stream_ptr) between HIP events on torch's current stream."""
    import torch

    s = torch.cuda.current_stream()
    for _ in range(warm):
        fn(s.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn(s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def cpu_time(fn, budget_s: float = 1.5, max_reps: int = 1000):
    t0 = time.perf_counter()
    fn()
    reps, dt = 1, time.perf_counter() - t0
    while dt < budget_s and reps < max_reps:
        fn()
        reps += 1
        dt = time.perf_counter() - t0
    return dt / reps


def row(name, ref, workload, units, unit_name, ms, cpu_s, cpu_units, cpu_sample, bound, alg, note=""):
    """alg: algorithmic bytes (bound 'hbm') or flops (bound 'fp64') of one call."""
    r = {"row": name, "reference": ref, "workload": workload,
         "value": round(units / (ms * 1e-3) / 1e6, 3), "unit": f"M{unit_name}/s", "ms_per_call": round(ms, 5)}
    if bound == "hbm":
        ach = alg / (ms * 1e-3) / 1e9
        r["roofline"] = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM, "unit": "GB/s",
                         "frac": round(ach / HBM, 5), "alg_bytes": alg}
    elif bound == "fp64":
        ach = alg / (ms * 1e-3) / 1e12
        r["roofline"] = {"bound": "fp64-valu", "achieved": round(ach, 3), "peak": FP64, "unit": "TFLOP/s",
                         "frac": round(ach / FP64, 5), "alg_flops": alg}
    else:
        r["roofline"] = None
    if cpu_s is not None:
        cv = cpu_units / cpu_s / 1e6
        r["cpu_baseline"] = {"value": round(cv, 4), "unit": f"M{unit_name}/s", "cores": 1, "kind": "port",
                             "sample": cpu_sample}
        r["speedup_vs_cpu"] = round(r["value"] / cv, 1)
    if note:
        r["note"] = note
    print(json.dumps(r), flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "rows.json"))
    ap.add_argument("--quick", action="store_true", help="smaller sizes (CPU-side smoke of the script)")
    args = ap.parse_args()

    import numpy as np
    import torch

    import oracle_lib as O
    from algodsp import conv, design, irlib, processors, signals
    from algodsp._lib import lib

    import ctypes as C

    torch.cuda.set_device(0)
    cuda = torch.device("cuda", 0)
    rows = []
    q = args.quick

    # ---- 8(f)3 Deconvolve / InverseFilter (host buffers, one call each), in a
    # child process without torch, like the Go caller: in this process the same
    # calls took 3-5x longer (16-32 ms vs 3.5-7 ms, tools/spectral_host_probe.py,
    # tools/spec_diag.py), a host-side effect of this process's state
    import subprocess

    out = subprocess.run([sys.executable, str(ROOT / "tools" / "spectral_rows.py")] + (["--quick"] if q else []),
                         check=True, capture_output=True, text=True).stdout
    for line in out.splitlines():
        if line.startswith("{"):
            r = json.loads(line)
            print(json.dumps(r), flush=True)
            rows.append(r)

    # ---- a1 conv.Direct: config 1 (48000 x 256) and a chip-filling size --------
    m = 256
    b = signals.make_test_kernel(m)
    for n, tag in ((48000, "config 1: 1 s mono 48 kHz"), (1 << (18 if q else 22), "2^22 samples")):
        a = signals.white_noise(n, 0x5EED)
        da, db = torch.from_numpy(a).to(cuda), torch.from_numpy(b).to(cuda)
        dd = torch.empty(n + m - 1, dtype=torch.float64, device=cuda)
        ms = dev_time(lambda s: conv.direct_device(da.data_ptr(), n, db.data_ptr(), m, dd.data_ptr(), s),
                      reps=50 if n < 100000 else 10)
        assert np.array_equal(dd.cpu().numpy(), O.direct(a, b)), "Direct parity"
        nc = 48000
        ac = signals.white_noise(nc, 0x5EED)
        cs = cpu_time(lambda: O.direct(ac, b))
        rows.append(row("a1", "conv.Direct / DirectTo conv.go:76-154", f"{tag} x {m}-tap makeTestKernel",
                        n, "samples", ms, cs, nc, f"oracle Direct, 1 x {nc} samples x {m} taps",
                        "fp64", 2.0 * n * m,
                        "no FMA (reference order: rounded product, rounded add), so the VALU ceiling of "
                        "this form is half the FMA peak"))

    # ---- a11 fir.Filter: 256 taps, 64 channels ---------------------------------
    taps = 256
    ch, n = 64, 1 << (16 if q else 20)
    h = signals.make_test_kernel(taps)
    f = processors.Filter(h, channels=ch)
    x = torch.from_numpy(np.stack([signals.white_noise(n, 0x5EED + c) for c in range(ch)])).to(cuda)
    y = torch.empty_like(x)

    def fir(s):
        f.process_device(x.data_ptr(), n, y.data_ptr(), n, n, s)
    ms = dev_time(fir, reps=5)
    f.Reset()
    fir(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    nc = 1 << 18
    xc = signals.white_noise(nc, 0x5EED)
    fo = O.Fir(h)
    want = fo.process_block(x[0, :4096].cpu().numpy())
    assert np.sqrt(np.mean((y[0, :4096].cpu().numpy() - want) ** 2)) <= 1e-12, "FIR parity"
    cs = cpu_time(lambda: O.Fir(h).process_block(xc), budget_s=1.0)
    rows.append(row("a11", "fir.Filter.ProcessBlockTo filter.go:119-159", f"{taps} taps, {ch} ch x {n} samples",
                    ch * n, "samples", ms, cs, nc, f"oracle Fir.ProcessBlock, 1 x {nc} samples",
                    "fp64", 2.0 * ch * n * taps))

    # ---- a12-a17 per-sample processors (config 5 shapes: 256 ch x 2^20) --------
    fs = 48000.0
    eq = design.config5_eq(fs)
    comp_cfg = {"auto_makeup": 0, "makeup_db": 0.0}
    verb = (0.22, 1.0, 0.72, 0.45, 0.015)
    nc = 1 << 21
    vc = 0.5 * signals.white_noise(nc, 0x5EED)

    def cpu_eq():
        v = vc
        for co, g in eq:
            v, _ = O.biquad_chain_block(np.ravel(co), np.zeros(2 * len(co)), g, v)

    def cpu_comp():
        O.Compressor(fs, **comp_cfg).process_in_place(vc)

    def cpu_verb():
        o = O.Freeverb()
        o.set(*verb)
        o.process_in_place(vc)

    procs = [
        ("a12-a14", "biquad.Chain.ProcessBlock chain.go:59-70 (section.go:56-138), config-5 EQ: 5 RBJ sections",
         dict(eq=eq), cpu_eq, "oracle biquad chains (avx2-registered 4x unroll)"),
        ("a15-a16", "dynamics.Compressor.ProcessInPlace compressor.go:362-366 (core.go:274-540)",
         dict(compressor=comp_cfg), cpu_comp, "oracle Compressor (libm log2/pow)"),
        ("a17", "reverb.Reverb.ProcessInPlace reverb.go:185-189 (Freeverb)",
         dict(freeverb=verb), cpu_verb, "oracle Freeverb"),
    ]
    for chn, n in ((256, 1 << (16 if q else 20)), (16384, 1 << (12 if q else 15))):
        xb = torch.from_numpy(np.stack([0.5 * signals.white_noise(n, 0x5EED + c) for c in range(min(chn, 256))]))
        xb = xb.repeat(chn // xb.shape[0], 1).contiguous().to(cuda)
        for name, ref, kw, cfn, cdesc in procs:
            fx = processors.EffectChain(chn, sample_rate=fs, **kw)
            ms = dev_time(lambda s: fx.process_device(xb.data_ptr(), n, n, s), reps=3, warm=1)
            cs = cpu_time(cfn, budget_s=1.0) if chn == 256 else None
            rows.append(row(name, ref, f"{chn} ch x {n} samples (effect-chain engine)", chn * n, "samples",
                            ms, cs, nc, f"{cdesc}, 1 x {nc} samples", "hbm", 16.0 * chn * n,
                            "serial per-channel recurrence: bound by dependent-op latency x channels in flight, "
                            "not by HBM; 16 B/sample is the in+out stream"))
            fx.close()
        # the time-parallel engine on request (AD_FX_ENGINE_TIME_PARALLEL): the
        # EQ-only and Freeverb-only chains within 1e-12 of the serial recurrences
        # instead of bit-exact
        if chn == 256:
            for pi, note in ((0, "two passes over the chunk plus a per-channel scan"),
                             (2, "one channel per CU, its delay lines in LDS")):
                name, ref, kw, cfn, cdesc = procs[pi]
                fx = processors.EffectChain(chn, sample_rate=fs, **kw)
                fx.SetEngine(processors.EffectChain.ENGINE_TIME_PARALLEL)
                ms = dev_time(lambda s: fx.process_device(xb.data_ptr(), n, n, s), reps=3, warm=1)
                cs = cpu_time(cfn, budget_s=1.0)
                rows.append(row(f"{name} (time-parallel)", ref, f"{chn} ch x {n} samples (time-parallel engine, "
                                "<= 1e-12 relative of the serial recurrence)", chn * n, "samples", ms, cs, nc,
                                f"{cdesc}, 1 x {nc} samples", "hbm", 16.0 * chn * n,
                                f"{note}; 16 B/sample is the in+out stream"))
                fx.close()
        del xb

    # ---- config 5: the fused effect chain ------------------------------------
    chn, n = 256, 1 << (16 if q else 20)
    xb = torch.from_numpy(np.stack([0.5 * signals.white_noise(n, 0x5EED + c) for c in range(chn)])).to(cuda)
    fx = processors.EffectChain(chn, eq, comp_cfg, verb, fs)
    ms = dev_time(lambda s: fx.process_device(xb.data_ptr(), n, n, s), reps=3, warm=1)
    cs = cpu_time(lambda: (cpu_eq(), cpu_comp(), cpu_verb()), budget_s=1.0)
    rows.append(row("a18 (config 5)", "effectchain.Chain.Process chain_process.go:11-319",
                    f"filter x5 -> dyn-compressor -> reverb-freeverb, {chn} ch x {n} samples", chn * n, "samples",
                    ms, cs, nc, f"oracle EQ + Compressor + Freeverb, 1 x {nc} samples", "hbm", 16.0 * chn * n,
                    "latency-bound serial recurrences (see a12-a17)"))
    fx.close()
    del xb

    # ---- 8(f)2 IRLB decodeF16 --------------------------------------------------
    frames, chn = 1 << (20 if q else 24), 2
    raw = torch.randint(0, 65536, (frames * chn,), dtype=torch.int32).to(torch.int16).to(cuda)
    out = torch.empty((chn, frames), dtype=torch.float64, device=cuda)
    ms = dev_time(lambda s: lib().ad_decode_f16_device(C.c_void_p(raw.data_ptr()), frames, chn,
                                                       C.c_void_p(out.data_ptr()), C.c_void_p(s)), reps=10)
    rr = raw[:8192].cpu().numpy().view(np.uint16)
    assert np.array_equal(out[:, :4096].cpu().numpy().T.ravel(), np.array([O.decode_f16(int(v)) for v in rr]), equal_nan=True), \
        "decodeF16 parity"
    img = (ROOT / "data" / "irs.irlib").read_bytes()
    nc = sum(v[2].size for v in O.irlib_read(img))
    cs = cpu_time(lambda: O.irlib_read(img), budget_s=1.0)
    rows.append(row("8(f)2", "webdemo decodeF16 irlib.go:136-170", f"{chn} ch x {frames} frames interleaved f16",
                    chn * frames, "samples", ms, cs, nc, f"oracle IRLB read of data/irs.irlib ({nc} samples)",
                    "hbm", 10.0 * chn * frames))

    # ---- host-buffer rows: streaming, partitioned, batch ----------------------
    ir = irlib.large_church()
    k16 = ir[0, :16384]
    B = 4096
    nblk = 128 if q else 1024
    xs = signals.white_noise(nblk * B, 0x5EED)
    ys = np.empty_like(xs)
    for ctor, name, ref in ((conv.NewStreamingOverlapSave, "a5", "StreamingOverlapSaveT.ProcessBlockTo "
                             "streaming_overlap_save.go:152-164"),
                            (conv.NewStreamingOverlapAdd, "a6", "StreamingOverlapAddT.ProcessBlockTo "
                             "streaming_overlap_add.go")):
        s = ctor(k16, B)
        for i in range(16):
            s.ProcessBlockTo(ys[i * B:(i + 1) * B], xs[i * B:(i + 1) * B])
        s.Reset()
        t0 = time.perf_counter()
        for i in range(nblk):
            s.ProcessBlockTo(ys[i * B:(i + 1) * B], xs[i * B:(i + 1) * B])
        ms = (time.perf_counter() - t0) / nblk * 1e3
        o = O.Streaming(k16, B, ola=(name == "a6"))
        cs = cpu_time(lambda: o.process_block(xs[:B]), budget_s=1.0)
        rows.append(row(name, ref, f"config 2: mono, K=16384, B={B}, host buffers, one block per call", B,
                        "samples", ms, cs, B, "oracle streaming block (N=32768 complex FFT)", None, 0,
                        "latency-bound: per-block wall time incl. PCIe in/out and 3 kernel launches"))

    lam = 128
    kpc = ir[0, :95432]
    pc = conv.NewPartitionedConvolution(kpc, 7, 13)
    op = O.Partitioned(kpc, 7, 13)
    ncb = 512
    xp = signals.white_noise(96 * 4096, 1)
    cs = cpu_time(lambda: [op.process_block(xp[i * lam:(i + 1) * lam]) for i in range(ncb)], budget_s=1.0,
                  max_reps=4)
    # one latency-sized block per call, then 4096-sample calls (a stage's whole blocks in one launch)
    for cb, nb in ((lam, 256 if q else 2048), (4096, 16 if q else 64)):
        yp = np.empty(cb)
        pc.Reset()
        for i in range(16):
            pc.ProcessBlock(xp[i * cb:(i + 1) * cb], yp)
        t0 = time.perf_counter()
        for i in range(nb):
            pc.ProcessBlock(xp[i * cb:(i + 1) * cb], yp)
        ms = (time.perf_counter() - t0) / nb * 1e3
        rows.append(row("a9/a10", "PartitionedConvolution.ProcessBlock partitioned.go:348-396",
                        f"Large Church L (95432 taps), minOrder 7 / maxOrder 13 (latency {lam}), "
                        f"{cb}-sample calls, host buffers", cb,
                        "samples", ms, cs, ncb * lam, f"oracle PartitionedConvolution, {ncb} blocks", None, 0,
                        "latency-bound: mean per-call wall time incl. PCIe"))

    # float32 instantiations (streaming_overlap_save.go:94, streaming_overlap_add.go:93, partitioned.go:340)
    xs32, ys32 = xs.astype(np.float32), np.empty(nblk * B, dtype=np.float32)
    k32 = k16.astype(np.float32)
    for ctor, name, ref in ((conv.NewStreamingOverlapSave32, "a5 (f32)", "NewStreamingOverlapSave32 "
                             "streaming_overlap_save.go:94"),
                            (conv.NewStreamingOverlapAdd32, "a6 (f32)", "NewStreamingOverlapAdd32 "
                             "streaming_overlap_add.go:93")):
        s = ctor(k32, B)
        for i in range(16):
            s.ProcessBlockTo(ys32[i * B:(i + 1) * B], xs32[i * B:(i + 1) * B])
        t0 = time.perf_counter()
        for i in range(nblk):
            s.ProcessBlockTo(ys32[i * B:(i + 1) * B], xs32[i * B:(i + 1) * B])
        ms = (time.perf_counter() - t0) / nblk * 1e3
        o = O.Streaming32(k32, B, ola=(name.startswith("a6")))
        cs = cpu_time(lambda: o.process_block(xs32[:B]), budget_s=1.0)
        rows.append(row(name, ref, f"config 2 in float32: mono, K=16384, B={B}, host buffers, one block per call",
                        B, "samples", ms, cs, B, "float32 oracle streaming block (N=32768 complex64 FFT)", None, 0,
                        "latency-bound; float32 boundary, float64 engine"))
    pc32 = conv.NewPartitionedConvolution32(kpc.astype(np.float32), 7, 13)
    xp32 = xp.astype(np.float32)
    yp32 = np.empty(lam, dtype=np.float32)
    for i in range(16):
        pc32.ProcessBlock(xp32[i * lam:(i + 1) * lam], yp32)
    nb = 256 if q else 2048
    t0 = time.perf_counter()
    for i in range(nb):
        pc32.ProcessBlock(xp32[i * lam:(i + 1) * lam], yp32)
    ms = (time.perf_counter() - t0) / nb * 1e3
    op32 = O.Partitioned32(kpc.astype(np.float32), 7, 13)
    cs = cpu_time(lambda: [op32.process_block(xp32[i * lam:(i + 1) * lam]) for i in range(ncb)], budget_s=1.0,
                  max_reps=4)
    rows.append(row("a9 (f32)", "NewPartitionedConvolution32 partitioned.go:340",
                    f"Large Church L (95432 taps) in float32, latency {lam}, {lam}-sample calls, host buffers", lam,
                    "samples", ms, cs, ncb * lam, f"float32 oracle PartitionedConvolution, {ncb} blocks", None, 0,
                    "latency-bound: mean per-call wall time incl. PCIe"))

    # many-channel forms: config 4 block by block (64 reverb channels, IR[c mod 2]),
    # and the reverb-conv node's engine (64 channels sharing one IR, latency 128)
    import torch

    C4, B4 = 64, 4096
    ms4 = conv.MultiChannelStreamingConvolver(ir, B4, C4, ir_index=[c % 2 for c in range(C4)])
    dx4 = torch.from_numpy(np.stack([signals.white_noise(B4, 0x5EED + c) for c in range(C4)])).cuda()
    dy4 = torch.empty_like(dx4)
    ms = dev_time(lambda sp: ms4.process_block_device(dx4.data_ptr(), B4, dy4.data_ptr(), B4, sp), 8 if q else 64)
    rows.append(row("a5 x64 (config 4 streaming)", "StreamingOverlapSave.ProcessBlockTo x 64 channels "
                    "streaming_overlap_save.go:152-164", f"64 ch x {B4}-sample blocks, 131072-tap Large Church "
                    "IR[c mod 2], device buffers, one handle", C4 * B4, "samples", ms, None, 0, "", None, 0,
                    "one launch per engine kernel per block for all 64 channels (hop 4096, P = 32)"))
    for Bx in (480, 960, 4800):  # block sizes that are not a whole number of hops (partial-block carry)
        msx = conv.MultiChannelStreamingConvolver(ir, Bx, C4, ir_index=[c % 2 for c in range(C4)])
        dxx = torch.from_numpy(np.stack([signals.white_noise(Bx, 0x5EED + c) for c in range(C4)])).cuda()
        dyx = torch.empty_like(dxx)
        ms = dev_time(lambda sp: msx.process_block_device(dxx.data_ptr(), Bx, dyx.data_ptr(), Bx, sp),
                      8 if q else 128)
        hop = max(1 << (Bx - 1).bit_length(), 2048)
        rows.append(row(f"a5 x64 B={Bx}", "StreamingOverlapSave.ProcessBlockTo x 64 channels "
                        "streaming_overlap_save.go:45-58,152-164", f"64 ch x {Bx}-sample blocks, 131072-tap Large "
                        "Church IR[c mod 2], device buffers, one handle", C4 * Bx, "samples", ms, None, 0, "", None,
                        0, f"hop {hop} with the unfinished block carried between calls (<= "
                        f"{(hop - 1 + Bx + hop - 1) // hop} FFT blocks per channel per call)"))
        del msx, dxx, dyx
    pcm = conv.PartitionedConvolutionMulti(kpc, 7, 13, C4)
    dxp = torch.from_numpy(np.stack([signals.white_noise(lam * 64, c) for c in range(C4)])).cuda()
    dyp = torch.empty_like(dxp)
    cnt = [0]

    def pc_call(sp):
        o = (cnt[0] % 64) * lam
        cnt[0] += 1
        pcm.process_device(dxp.data_ptr() + 8 * o, lam * 64, dyp.data_ptr() + 8 * o, lam * 64, lam, sp)

    ms = dev_time(pc_call, 128 if q else 1024, warm=64)
    rows.append(row("a9/f1 x64 (reverb-conv engine)", "PartitionedConvolution.ProcessBlock x 64 channels "
                    "partitioned.go:348-396", f"64 ch sharing Large Church L (95432 taps), latency {lam}, "
                    f"{lam}-sample device calls", C4 * lam, "samples", ms, None, 0, "", None, 0,
                    "device-resident many-channel engine (ad_conv_pc_multi): mean per-call time, all stages"))

    nbt = 1 << (18 if q else 22)
    xbt = signals.white_noise(nbt, 3)
    for ctor, name, ref, ocls in ((conv.NewOverlapSave, "a4", "OverlapSave.ProcessTo overlap_save.go:258-272",
                                   O.OverlapSave),
                                  (conv.NewOverlapAdd, "a3", "OverlapAdd.ProcessTo overlap_add.go:168-182",
                                   O.OverlapAdd)):
        e = ctor(k16)
        e.Process(xbt[:1 << 16])
        t0 = time.perf_counter()
        for _ in range(3):
            e.Process(xbt)
        ms_fresh = (time.perf_counter() - t0) / 3 * 1e3
        # ProcessTo into a reused output (overlap_save.go:258-272): the engine's
        # rate; Process above also pays the OS for a fresh 34 MB output per call
        yb = np.empty(nbt + k16.size - 1)
        e.ProcessTo(yb, xbt)
        t0 = time.perf_counter()
        for _ in range(6):
            e.ProcessTo(yb, xbt)
        ms = (time.perf_counter() - t0) / 6 * 1e3
        oc = ocls(k16)
        ncs = 1 << 18
        cs = cpu_time(lambda: oc.process(xbt[:ncs]), budget_s=1.0, max_reps=3)
        rows.append(row(name, ref,
                        f"mono {nbt} samples x 16384 taps, host buffers (PCIe in + out), ProcessTo", nbt,
                        "samples", ms, cs, ncs, f"oracle {ocls.__name__}.Process, {ncs} samples", None, 0,
                        "host-buffer call: PCIe-bound (16 B/sample over ~50 GB/s); Process with a fresh output "
                        f"array per call: {nbt / ms_fresh / 1e3:.0f} Msamples/s (first-touch page faults)"))

    pathlib.Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    pathlib.Path(args.out).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
