"""The reference's own dsp/conv unit tests, restated against the HIP engine.

Each test names the reference test it follows (file:line under
github.com/cwbudde/algo-dsp/dsp/conv) and keeps its inputs, thresholds and
expected errors, so a reader can hold the two side by side.  Where the
reference compares two of its own paths (streaming against batch, OLA
against OLS, FFT against direct), both paths here are the GPU's.
"""
import math

import numpy as np
import pytest

from algodsp import conv


def _next_pow2(n: int) -> int:
    p = 1
    while p < n:
        p <<= 1
    return p


# ------------------------------------------------------------------ getters
@pytest.mark.gpu
@pytest.mark.parametrize("ctor", ["ols", "ola"])
def test_streaming_getters(ctor):
    """TestStreamingOverlapSaveGetters (streaming_overlap_save_test.go:279-303),
    TestStreamingOverlapAddGetters (streaming_overlap_add_test.go:286-308)."""
    kernel = [1.0, 0.5, 0.25, 0.1]
    block = 8
    new = conv.NewStreamingOverlapSave if ctor == "ols" else conv.NewStreamingOverlapAdd
    s = new(kernel, block)
    assert s.BlockSize() == block
    assert s.KernelLen() == len(kernel)
    assert s.FFTSize() == _next_pow2(block + len(kernel) - 1)


# ------------------------------------------------------------ dirac / long
@pytest.mark.gpu
@pytest.mark.parametrize("ctor", ["ols", "ola"])
def test_streaming_dirac_delta(ctor):
    """TestStreamingOverlapSaveDiracDelta (streaming_overlap_save_test.go:306-329),
    TestStreamingOverlapAddDiracDelta (streaming_overlap_add_test.go:311-334)."""
    new = conv.NewStreamingOverlapSave if ctor == "ols" else conv.NewStreamingOverlapAdd
    s = new([1.0], 8)
    x = [1, 2, 3, 4, 5, 6, 7, 8]
    y = s.ProcessBlock(x)
    assert np.max(np.abs(y - np.asarray(x, dtype=np.float64))) <= 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("ctor", ["ols", "ola"])
def test_streaming_long_kernel(ctor):
    """TestStreamingOverlapSaveLongKernel (streaming_overlap_save_test.go:331-383),
    TestStreamingOverlapAddLongKernel (streaming_overlap_add_test.go:336-388):
    a 256-tap 0.95^k kernel at block 64; the impulse's first output is k[0]
    and the next three all-zero blocks still carry the tail (max > 1e-6).
    Beyond the reference: every output equals the kernel itself."""
    kernel = np.empty(256)
    kernel[0] = 1.0
    for i in range(1, 256):
        kernel[i] = 0.95 * kernel[i - 1]
    block = 64
    new = conv.NewStreamingOverlapSave if ctor == "ols" else conv.NewStreamingOverlapAdd
    s = new(kernel, block)
    b1 = np.zeros(block)
    b1[0] = 1.0
    outs = [s.ProcessBlock(b1)]
    assert abs(outs[0][0] - kernel[0]) <= 1e-10
    for _ in range(3):
        out = s.ProcessBlock(np.zeros(block))
        assert np.max(np.abs(out)) >= 1e-6
        outs.append(out)
    assert np.max(np.abs(np.concatenate(outs) - kernel)) <= 1e-12


# ------------------------------------------------------ streaming vs batch
@pytest.mark.gpu
def test_streaming_ols_vs_batch():
    """TestStreamingOverlapSaveVsBatch (streaming_overlap_save_test.go:51-100)."""
    kernel = [0.5, 1.0, 0.5, 0.2]
    block, nblk = 8, 4
    sig = np.sin(np.arange(block * nblk) * 0.1)
    batch = conv.NewOverlapSave(kernel, 0).Process(sig)
    s = conv.NewStreamingOverlapSave(kernel, block)
    stream = np.concatenate([s.ProcessBlock(sig[i * block:(i + 1) * block]) for i in range(nblk)])
    assert np.max(np.abs(batch[:sig.size] - stream)) <= 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("ctor", ["ols", "ola"])
def test_streaming_continuity(ctor):
    """TestStreamingOverlapSaveContinuity (streaming_overlap_save_test.go:385-440),
    TestStreamingOverlapAddContinuity (streaming_overlap_add_test.go:390-433):
    8 blocks of 16 of sin(0.2 i) through a 5-tap kernel against the batch
    convolver (OverlapSave fft 0 / OverlapAdd block 16), 1e-9."""
    kernel = [0.25, 0.5, 1.0, 0.5, 0.25]
    block, nblk = 16, 8
    sig = np.sin(np.arange(block * nblk) * 0.2)
    if ctor == "ols":
        s = conv.NewStreamingOverlapSave(kernel, block)
        batch = conv.NewOverlapSave(kernel, 0).Process(sig)
    else:
        s = conv.NewStreamingOverlapAdd(kernel, block)
        batch = conv.NewOverlapAdd(kernel, block).Process(sig)
    stream = np.concatenate([s.ProcessBlock(sig[i * block:(i + 1) * block]) for i in range(nblk)])
    assert np.max(np.abs(batch[:sig.size] - stream)) <= 1e-9


@pytest.mark.gpu
def test_streaming_algorithm_equivalence():
    """TestStreamingAlgorithmEquivalence (streaming_test.go:122-177): OLA and
    OLS give the same stream, 1e-9."""
    kernel = [0.5, 1.0, 0.5, 0.2, 0.1]
    block, nblk = 16, 8
    i = np.arange(block * nblk)
    sig = np.sin(i * 0.1) + 0.5 * np.cos(i * 0.05)
    ola = conv.NewStreamingOverlapAdd(kernel, block)
    ols = conv.NewStreamingOverlapSave(kernel, block)
    a = np.concatenate([ola.ProcessBlock(sig[k * block:(k + 1) * block]) for k in range(nblk)])
    b = np.concatenate([ols.ProcessBlock(sig[k * block:(k + 1) * block]) for k in range(nblk)])
    assert a.size == b.size
    assert np.max(np.abs(a - b)) <= 1e-9


@pytest.mark.gpu
def test_streaming_process_block_to_equivalence():
    """TestStreamingAlgorithmProcessBlockToEquivalence (streaming_test.go:271-305)."""
    kernel = [0.25, 0.5, 1.0, 0.5, 0.25]
    block = 8
    x = np.arange(block, dtype=np.float64)
    ola = conv.NewStreamingOverlapAdd(kernel, block)
    ols = conv.NewStreamingOverlapSave(kernel, block)
    oa, os_ = np.zeros(block), np.zeros(block)
    ola.ProcessBlockTo(oa, x)
    ols.ProcessBlockTo(os_, x)
    assert np.max(np.abs(oa - os_)) <= 1e-9


# ------------------------------------------------------------------ errors
@pytest.mark.gpu
def test_streaming_ols_errors():
    """TestStreamingOverlapSaveErrors (streaming_overlap_save_test.go:225-277)."""
    with pytest.raises(conv.ErrEmptyKernel):
        conv.NewStreamingOverlapSave([], 128)
    with pytest.raises(conv.ADError):
        conv.NewStreamingOverlapSave([1.0], 0)
    with pytest.raises(conv.ADError):
        conv.NewStreamingOverlapSave([1.0], -1)
    s = conv.NewStreamingOverlapSave([1.0, 0.5], 4)
    with pytest.raises(conv.ADError):
        s.ProcessBlock([1, 2, 3])
    with pytest.raises(conv.ADError):
        s.ProcessBlockTo(np.zeros(3), [1, 2, 3, 4])


@pytest.mark.gpu
def test_overlap_save_invalid_fft_size():
    """TestOverlapSaveInvalidFFTSize (conv_test.go:675-682)."""
    with pytest.raises(conv.ADError):
        conv.NewOverlapSave([0.25, 0.5, 0.25], 100)


@pytest.mark.gpu
def test_overlap_save_process_to():
    """TestOverlapSaveProcessTo (conv_test.go:423-449): the right output
    length succeeds (and matches Direct here), a wrong one errors."""
    kernel = [0.25, 0.5, 0.25]
    sig = np.asarray([i % 10 for i in range(100)], dtype=np.float64)
    o = conv.NewOverlapSave(kernel, 0)
    out = np.zeros(sig.size + o.KernelLen() - 1)
    o.ProcessTo(out, sig)
    assert np.max(np.abs(out - conv.Direct(sig, kernel))) <= 1e-12
    with pytest.raises(conv.ADError):
        o.ProcessTo(np.zeros(5), sig)


@pytest.mark.gpu
@pytest.mark.parametrize("ctor", ["ols", "ola"])
def test_batch_reset(ctor):
    """TestOverlapSaveReset / TestOverlapAddReset (conv_test.go:451-461), and
    a Process after Reset gives the same result as before it."""
    o = conv.NewOverlapSave([1.0, 0.0], 0) if ctor == "ols" else conv.NewOverlapAdd([1.0, 0.0], 8)
    x = np.arange(20, dtype=np.float64)
    y0 = o.Process(x)
    o.Reset()
    assert np.array_equal(o.Process(x), y0)


# ------------------------------------------------------------ dispatch etc
@pytest.mark.gpu
def test_convolve_auto_selection():
    """TestConvolveAutoSelection (conv_test.go:171-215): a 3-tap kernel (direct
    path) and a 100-tap one (FFT path) both match Direct to 1e-10."""
    sig = np.asarray([i % 10 for i in range(1000)], dtype=np.float64)
    short = [1.0, 2.0, 1.0]
    r1 = conv.Convolve(sig, short)
    assert np.array_equal(r1, conv.Direct(sig, short))  # the direct kernel itself: same bits
    long_k = np.exp(-np.arange(100) / 20.0)
    r2 = conv.Convolve(sig, long_k)
    d2 = conv.Direct(sig, long_k)
    assert r2.size == d2.size
    assert np.max(np.abs(r2 - d2)) <= 1e-10


@pytest.mark.gpu
def test_correlate_fft_matches_correlate():
    """TestCorrelateFFT (conv_test.go:463-485) and TestCorrelateFFTErrors
    (conv_test.go:487-492)."""
    a, b = [1, 2, 3, 4, 5], [1, 2, 3]
    r = conv.CorrelateFFT(a, b)
    d = conv.Correlate(a, b)
    assert r.size == d.size
    assert np.max(np.abs(r - d)) <= 1e-8
    with pytest.raises(conv.ErrEmptyInput):
        conv.CorrelateFFT([], [1, 2])


def test_find_peak_empty():
    """TestFindPeakEmpty (conv_test.go:668-673); host helper, no device call."""
    assert conv.FindPeak([]) == (-1, 0.0)
    assert conv.FindPeak([0.5, 3.0, 3.0, -7.0]) == (1, 3.0)
    assert conv.LagFromIndex(conv.IndexFromLag(-4, 9), 9) == -4
    assert not math.isnan(conv.SNR([1.0, 2.0], [1.0, 2.5]))


# ------------------------------------------------ PartitionedConvolution
def _impulse_kernel(n):
    """makeImpulseKernel (partitioned_test.go:11-20): 0.99^k."""
    k = np.empty(n)
    k[0] = 1.0
    for i in range(1, n):
        k[i] = k[i - 1] * 0.99
    return k


def _test_signal(n):
    """Stands in for makePartitionedTestSignal (partitioned_test.go:23-32, Go's
    PCG(42, 0) uniforms in [-1, 1)): seeded uniforms of the same range; the
    tests compare two paths on the same input, so the generator is free."""
    return np.random.default_rng(42).uniform(-1.0, 1.0, n)


def _partitioned_out(kernel, sig, lo, hi):
    """convolveWithPartitioned (partitioned_test.go:78-101)."""
    pc = conv.NewPartitionedConvolution(kernel, lo, hi)
    lat = pc.Latency()
    padded = np.concatenate([sig, np.zeros(lat)])
    out = np.zeros(padded.size)
    pc.ProcessBlock(padded, out)
    return out[lat:]


def _soa_out(kernel, sig, block):
    """convolveWithSOA (partitioned_test.go:36-76): the last block zero padded."""
    s = conv.NewStreamingOverlapAdd(kernel, block)
    outs = []
    for i in range(0, sig.size, block):
        b = np.zeros(block)
        b[:min(block, sig.size - i)] = sig[i:i + block]
        outs.append(s.ProcessBlock(b))
    return np.concatenate(outs)


@pytest.mark.gpu
@pytest.mark.parametrize("order", [4, 5, 6, 7])
def test_partitioned_latency(order):
    """TestPartitionedConvolutionLatency (partitioned_test.go:103-119)."""
    assert conv.NewPartitionedConvolution(_impulse_kernel(64), order, order + 4).Latency() == 1 << order


@pytest.mark.gpu
@pytest.mark.parametrize("klen, slen, lo, hi", [(64, 512, 4, 10), (256, 1024, 5, 12), (1024, 4096, 6, 13),
                                                (8192, 16384, 6, 13)])
def test_partitioned_matches_soa(klen, slen, lo, hi):
    """TestPartitionedConvolutionMatchesSOA (partitioned_test.go:121-165), 1e-7."""
    k, sig = _impulse_kernel(klen), _test_signal(slen)
    pc = _partitioned_out(k, sig, lo, hi)
    soa = _soa_out(k, sig, 1 << lo)
    n = min(sig.size, pc.size, soa.size)
    assert np.max(np.abs(pc[:n] - soa[:n])) <= 1e-7


@pytest.mark.gpu
def test_partitioned_reset():
    """TestPartitionedConvolutionReset (partitioned_test.go:167-197); equal
    bits here."""
    sig = _test_signal(512)
    pc = conv.NewPartitionedConvolution(_impulse_kernel(128), 6, 12)
    o1, o2 = np.zeros(512), np.zeros(512)
    pc.ProcessBlock(sig, o1)
    pc.Reset()
    pc.ProcessBlock(sig, o2)
    assert np.array_equal(o1, o2)


@pytest.mark.gpu
def test_partitioned_errors():
    """TestPartitionedConvolutionErrors (partitioned_test.go:199-235)."""
    with pytest.raises(conv.ErrEmptyImpulseResponse):
        conv.NewPartitionedConvolution([], 6, 12)
    with pytest.raises(conv.ErrInvalidBlockOrder):
        conv.NewPartitionedConvolution([1, 2, 3], 0, 12)
    with pytest.raises(conv.ErrInvalidBlockOrder):
        conv.NewPartitionedConvolution([1, 2, 3], 8, 5)
    pc = conv.NewPartitionedConvolution([1, 2, 3, 4], 2, 10)
    with pytest.raises(conv.ErrLengthMismatch):
        pc.ProcessBlock(np.zeros(10), np.zeros(8))


@pytest.mark.gpu
def test_partitioned_stage_info_and_kernel_len():
    """TestPartitionedConvolutionStageInfo (partitioned_test.go:237-277) and
    TestPartitionedConvolutionKernelLen (:279-290)."""
    pc = conv.NewPartitionedConvolution(_impulse_kernel(1024), 6, 13)
    count = pc.StageCount()
    assert count > 0
    for bad in (-1, count):
        with pytest.raises(conv.ErrStageIndexOutOfRange):
            pc.StageInfo(bad)
    for i in range(count):
        part, blocks = pc.StageInfo(i)
        assert part > 0 and blocks > 0
    assert conv.NewPartitionedConvolution(_impulse_kernel(300), 6, 13).KernelLen() == 300


@pytest.mark.gpu
def test_partitioned_dirac_delta_reference_form():
    """TestPartitionedConvolutionDiracDelta (partitioned_test.go:292-322): a
    one-tap kernel delays the input by 2^minBlockOrder, 1e-9."""
    sig = _test_signal(256)
    lat = 1 << 4
    pc = conv.NewPartitionedConvolution([1.0], 4, 12)
    padded = np.concatenate([sig, np.zeros(lat)])
    out = np.zeros(padded.size)
    pc.ProcessBlock(padded, out)
    assert np.max(np.abs(out[lat:lat + sig.size] - sig)) <= 1e-9
