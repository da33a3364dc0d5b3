"""The pipelined offline schedule of the multi-channel UPOLS engine
(ad_conv_multi_set_schedule): chunks whose block spectra
and Z rows stay in the Infinity Cache, K1 on the caller's stream and K2 / K3 on
internal streams.  The reference operation is the batch OverlapSave.Process
(dsp/conv/overlap_save.go:126-254) per channel; the schedule must not change a
bit of it, so every case compares the pipelined result with the serial one
exactly, and one case also with the oracle."""
import numpy as np
import pytest

import oracle_lib as O
from algodsp import conv, irlib, signals
from test_conv_gpu import FFT_RMS_TOL, rms

pytestmark = pytest.mark.gpu


def _run(eng, x, out_len, stream=None):
    import torch

    C_, n = x.shape
    dx = torch.from_numpy(x).cuda()
    dy = torch.full((C_, out_len), np.nan, dtype=torch.float64, device="cuda")
    s = stream or torch.cuda.current_stream()
    eng.process_device(dx.data_ptr(), n, n, dy.data_ptr(), out_len, out_len, s.cuda_stream)
    return dy, s


@pytest.mark.parametrize("hop,C_,n,chunk,run", [
    (8192, 2, 1 << 21, 32, 0),      # config 3's geometry, 8 chunks + the tail
    (8192, 2, 1 << 21, 0, 0),       # auto chunk
    (8192, 2, 1 << 21, 40, 16),     # chunks that are not run multiples
    (4096, 3, 700001, 17, 16),      # ragged signal, odd channels, P = 32 (two K2 partition launches)
    (2048, 1, 123457, 5, 0),        # chunks shorter than the partition count (P = 64)
])
def test_pipelined_bit_identical_to_serial(gpu, hop, C_, n, chunk, run):
    import torch

    ir = irlib.large_church()
    x = np.stack([signals.white_noise(n, 0x5EED + 7 * c) for c in range(C_)])
    K = ir.shape[1]
    out_len = n + K - 1
    ids = [c % 2 for c in range(C_)]
    ser = conv.MultiChannelConvolver(ir, hop=hop, channels=C_, ir_index=ids)
    pip = conv.MultiChannelConvolver(ir, hop=hop, channels=C_, ir_index=ids)
    pip.set_schedule(pip.SCHED_PIPELINED, chunk, run)
    mode, got_chunk = pip.schedule()
    assert mode == pip.SCHED_PIPELINED and got_chunk > 0
    ys, _ = _run(ser, x, out_len)
    yp, s = _run(pip, x, out_len)
    # the caller's stream alone orders the call: read the output right after it
    out = torch.empty_like(yp)
    out.copy_(yp)
    s.synchronize()
    a, b = ys.cpu().numpy(), out.cpu().numpy()
    assert not np.isnan(b).any()
    assert np.array_equal(a, b), float(np.max(np.abs(a - b)))
    # a second signal on the same handle (rings reused, logical blocks restart)
    yp2, _ = _run(pip, x[::-1].copy(), out_len)
    ys2, _ = _run(ser, x[::-1].copy(), out_len)
    torch.cuda.synchronize()
    assert torch.equal(yp2, ys2)


def test_pipelined_vs_oracle(gpu):
    """Stereo Large Church through the pipelined schedule against the oracle's
    OverlapSave.Process at an oracle-sized length."""
    import torch

    ir = irlib.large_church()
    n = 1 << 18
    x = np.stack([signals.white_noise(n, 0x5EED + c) for c in range(2)])
    out_len = n + ir.shape[1] - 1
    eng = conv.MultiChannelConvolver(ir, hop=8192, channels=2)
    eng.set_schedule(eng.SCHED_PIPELINED, 8, 0)
    y, _ = _run(eng, x, out_len)
    torch.cuda.synchronize()
    y = y.cpu().numpy()
    for c in range(2):
        want = O.OverlapSave(ir[c], 0).process(x[c])
        assert rms(y[c], want) < FFT_RMS_TOL
        assert np.max(np.abs(y[c] - want)) < 1e-9


def test_pipelined_mix_and_segments(gpu):
    """The fused-mixdown entry point and output segments under the pipelined
    schedule equal the serial schedule bit for bit."""
    import torch

    ir = irlib.large_church()
    C_, n, hop = 8, 1 << 20, 8192
    K = ir.shape[1]
    out_len = n + K - 1
    x = np.stack([signals.white_noise(n, 0x5EED + c) for c in range(C_)])
    dx = torch.from_numpy(x).cuda()
    ids = [c % 2 for c in range(C_)]
    res = []
    for mode in (0, 1):
        eng = conv.MultiChannelConvolver(ir, hop=hop, channels=C_, ir_index=ids)
        eng.set_schedule(mode, 12, 0)
        mix = torch.zeros((2, out_len), dtype=torch.float64, device="cuda")
        eng.process_device_mix(dx.data_ptr(), n, n, mix.data_ptr(), out_len, out_len, 1)
        y = torch.zeros((C_, out_len), dtype=torch.float64, device="cuda")
        blocks = -(-out_len // hop)
        cuts = [min(out_len, hop * (blocks * i // 3)) for i in range(4)]
        for b, e in zip(cuts[:-1], cuts[1:]):
            eng.process_device_segment(dx.data_ptr(), n, n, y.data_ptr(), out_len, out_len, b, e)
        torch.cuda.synchronize()
        res.append((mix.cpu().numpy(), y.cpu().numpy()))
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])


def test_schedule_rejects_bad_arguments(gpu):
    ir = irlib.large_church()
    eng = conv.MultiChannelConvolver(ir, hop=8192, channels=2)
    with pytest.raises(Exception):
        eng.set_schedule(7)
    with pytest.raises(Exception):
        eng.set_schedule(1, -1)
    # hop < 2048 stays serial
    small = conv.MultiChannelConvolver(ir[:, :4096], hop=1024, channels=1)
    small.set_schedule(small.SCHED_PIPELINED)
    assert small.schedule() == (small.SCHED_SERIAL, 0)


@pytest.mark.parametrize("first,second", [
    ((1, 12, 0), (0, 0, 0)),     # pipelined signal, serial requested mid-signal
    ((1, 12, 0), (1, 64, 0)),    # a larger chunk requested mid-signal
    ((0, 0, 0), (1, 12, 0)),     # serial signal, pipelined requested mid-signal
])
def test_schedule_change_between_segments(gpu, first, second):
    """A set_schedule between two segments of one signal applies from the next
    signal start (begin_offline): the signal in flight keeps the rings it began
    with, so its output equals the serial schedule bit for bit, and the next
    signal runs the new schedule, also bit for bit."""
    import torch

    ir = irlib.large_church()
    C_, n, hop = 4, 1 << 20, 8192
    out_len = n + ir.shape[1] - 1
    x = np.stack([signals.white_noise(n, 0xC4A7 + c) for c in range(C_)])
    dx = torch.from_numpy(x).cuda()
    ids = [c % 2 for c in range(C_)]
    ref = conv.MultiChannelConvolver(ir, hop=hop, channels=C_, ir_index=ids)
    want, _ = _run(ref, x, out_len)
    eng = conv.MultiChannelConvolver(ir, hop=hop, channels=C_, ir_index=ids)
    eng.set_schedule(*first)
    blocks = -(-out_len // hop)
    cuts = [min(out_len, hop * (blocks * i // 3)) for i in range(4)]
    y = torch.full((C_, out_len), np.nan, dtype=torch.float64, device="cuda")
    for i, (b, e) in enumerate(zip(cuts[:-1], cuts[1:])):
        if i == 1:
            eng.set_schedule(*second)
            assert eng.schedule()[0] == (second[0] if second[0] == 0 else eng.SCHED_PIPELINED)
        eng.process_device_segment(dx.data_ptr(), n, n, y.data_ptr(), out_len, out_len, b, e)
    torch.cuda.synchronize()
    assert torch.equal(y, want)
    y2, _ = _run(eng, x, out_len)
    torch.cuda.synchronize()
    assert torch.equal(y2, want)
