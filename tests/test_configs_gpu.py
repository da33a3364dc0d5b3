"""One named GPU parity test per BASELINE.json config, collected first.

Each test runs its config's reference operation through the HIP C ABI at the
shape bench.py (or the named row) measures, and checks it against the CPU
oracle (oracle/, the C restatement of the Go reference):

  config 1  conv.Direct, 256-tap kernel, 1 s mono 48 kHz white noise     bit-exact
  config 2  StreamingOverlapSave, 16384-tap IR, 4096-sample blocks       <= 1e-7 RMS
  config 3  OverlapSave, stereo x 2^24, 131072-tap Large Church (bench)  <= 1e-7 RMS
  config 4  8-channel shard of the 64-channel job, mixdown fused (2^24)  <= 4e-7 RMS
  config 5  effectchain EQ -> Compressor -> Freeverb, 256 channels        <= 1e-12 RMS

Tolerances are north_star's (<= 1e-12 RMS direct/per-sample, <= 1e-7 RMS FFT
conv); the config-4 mix sums 4 channels per side, so its bar is 4x.
"""
import numpy as np
import pytest

import oracle_lib as O
from algodsp import conv, design, irlib, processors as P, signals
from test_conv_gpu import FFT_RMS_TOL, _exact_window, _multi_run, rms

pytestmark = pytest.mark.gpu


def test_config1_direct(gpu):
    """configs[0]: dsp/conv.Direct (conv.go:76-154) of 48000 white-noise samples
    with a 256-tap makeTestKernel (conv_bench_test.go:296-312): bit-exact with
    the reference's scatter-add order (no FMA)."""
    x = signals.white_noise(48000, 0x5EED)
    h = signals.make_test_kernel(256)
    got = conv.Direct(x, h)
    want = O.direct(x, h)
    assert got.size == 48000 + 256 - 1
    assert np.array_equal(got, want), float(np.max(np.abs(got - want)))


def test_config2_stream(gpu):
    """configs[1]: NewStreamingOverlapSave(kernel, 4096) with the first 16384
    taps of Large Church L, block by block through
    ProcessBlockTo (streaming_overlap_save.go:100-164) against the oracle's
    streaming restatement, including FFTSize = nextPow2(4096 + 16383)."""
    h = irlib.large_church()[0, :16384].copy()
    B, nb = 4096, 8
    x = signals.white_noise(B * nb, 0x5EED)
    g = conv.NewStreamingOverlapSave(h, B)
    o = O.Streaming(h, B)
    assert g.FFTSize() == o.fft_size() == 32768
    got, want = [], []
    for i in range(nb):
        blk = x[i * B:(i + 1) * B]
        out = np.empty(B)
        g.ProcessBlockTo(out, blk)
        got.append(out)
        want.append(o.process_block(blk))
    got, want = np.concatenate(got), np.concatenate(want)
    assert rms(got, want) < FFT_RMS_TOL
    assert np.max(np.abs(got - want)) < 1e-9


def test_config3_bench_instance(gpu):
    """configs[2] exactly as bench.py runs it (hop 8192, auto chunk, auto run
    length -> P = 16, stereo x 2^24 samples, one chunk): the whole output of
    both channels against the oracle's batch OverlapSave.Process
    (overlap_save.go:126-254), plus exact dot products on windows across the
    K2 run boundaries and the signal ends."""
    ir = irlib.large_church()
    K = ir.shape[1]
    n = 1 << 24
    x = np.stack([signals.white_noise(n, 0x5EED + c) for c in range(2)])
    y, eng = _multi_run(ir, x, hop=8192)
    assert eng.FFTSize() == 16384
    out_len = n + K - 1
    for c in range(2):
        want = O.OverlapSave(ir[c], 0).process(x[c])
        assert want.size == out_len
        assert rms(y[c], want) < FFT_RMS_TOL
        assert np.max(np.abs(y[c] - want)) < 1e-9
        del want
    # run boundaries of the auto run length (multiples of 16 blocks around
    # 176-192 blocks) and the chunk's first/last blocks
    L = 8192
    for c in range(2):
        for t0 in [0, K - 64, 16 * L - 32, 176 * L - 32, 192 * L - 32, 352 * L - 32, 384 * L - 32, 193 * L - 7,
                   n - 40, out_len - 64]:
            got = y[c][t0:t0 + 64]
            ref = _exact_window(x[c], ir[c], t0, got.size)
            assert np.max(np.abs(got - ref)) < 1e-9, (c, t0)


def test_config4_shard(gpu):
    """configs[3]'s per-GPU shard exactly as bench.py --workload shard runs it
    (8 of the 64 channels, channel c with IR[c mod 2], 131072 taps, hop 8192,
    auto chunk and run length, 2^24 samples per channel -- the measured
    geometry, K2 runs of R = 688), with the stereo mixdown fused into K3
    (ad_conv_multi_process_device_mix: L = even channels, R = odd).  The mix
    against the oracle's per-channel OverlapSave outputs summed by parity
    (8 oracle channels on host threads), plus exact dot-product windows at the
    signal start, K2 run boundaries and the tail."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    ir = irlib.large_church()
    K = ir.shape[1]
    C_, n = 8, 1 << 24
    out_len = n + K - 1
    x = np.stack([signals.white_noise(n, 0x5EED + c) for c in range(C_)])
    eng = conv.MultiChannelConvolver(ir, hop=8192, channels=C_, ir_index=[c % 2 for c in range(C_)])
    dx = torch.from_numpy(x).cuda()
    mix = torch.empty((2, out_len), dtype=torch.float64, device="cuda")
    eng.process_device_mix(dx.data_ptr(), n, n, mix.data_ptr(), out_len, out_len, 0)
    torch.cuda.synchronize()
    del dx
    m = mix.cpu().numpy()
    del mix
    with ThreadPoolExecutor(8) as ex:  # ctypes releases the GIL
        per = list(ex.map(lambda c: O.OverlapSave(ir[c % 2], 0).process(x[c]), range(C_)))
    for s in range(2):
        want = per[s] + per[s + 2] + per[s + 4] + per[s + 6]
        assert rms(m[s], want) < FFT_RMS_TOL * 4
        assert np.max(np.abs(m[s] - want)) < 4e-9
    del per
    L = 8192
    for s in range(2):
        for t0 in [0, K - 64, 688 * L - 32, 1376 * L - 7, n - 40, out_len - 64]:
            ref = sum(_exact_window(x[c], ir[c % 2], t0, 64) for c in range(s, C_, 2))
            assert np.max(np.abs(m[s][t0:t0 + 64] - ref)) < 4e-9, (s, t0)


def test_config5_chain(gpu):
    """configs[4] at the shape bench.py --workload fx times: 256 channels,
    device buffers, the engine AUTO picks for a chain with a compressor -- the
    time-parallel engine (fx_tp.hip; the EQ's noise estimate, 3.6e-13 at
    48 kHz, is under its 4.5e-13 gate) -- 2^19 samples = 10 2/3 of its
    49152-sample chunks (each chunk's gain runs on the caller's stream behind
    the next chunk's EQ, and the second call reuses the four chunk slots
    twice), in two calls (the second starts mid-chunk); channels 0, 63, 64
    (the first of the second 64-channel group) and 255 against the oracle
    chain (chain_process.go:11-33: biquad chains -> Compressor -> Freeverb)."""
    import torch

    fs = 48000.0
    eq = design.config5_eq(fs)
    comp_cfg = {"auto_makeup": 0, "makeup_db": 0.0}
    verb = (0.22, 1.0, 0.72, 0.45, 0.015)
    C, n = 256, 1 << 19
    x = np.stack([0.5 * signals.white_noise(n, 0x5EED + c) for c in range(C)])
    fx = P.EffectChain(C, eq, comp_cfg, verb, fs)
    dx = torch.from_numpy(x).cuda()
    s = torch.cuda.current_stream()
    cut = 5 * 16384 + 1000
    fx.process_device(dx.data_ptr(), n, cut, s.cuda_stream)
    fx.process_device(dx.data_ptr() + 8 * cut, n, n - cut, s.cuda_stream)
    s.synchronize()
    engine, noise = fx.LastEngine()
    assert engine == P.EffectChain.ENGINE_TIME_PARALLEL, engine
    assert 3e-13 < noise < 4.5e-13, noise
    y = dx.cpu().numpy()
    for c in (0, 63, 64, 255):
        v = x[c].copy()
        for co, g in eq:
            v, _ = O.biquad_chain_block(np.ravel(co), np.zeros(2 * len(co)), g, v)
        v = O.Compressor(fs, **comp_cfg).process_in_place(v)
        o = O.Freeverb()
        o.set(*verb)
        v = o.process_in_place(v)
        assert rms(y[c], v) <= 1e-12, (c, rms(y[c], v))
