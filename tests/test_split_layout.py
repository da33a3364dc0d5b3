"""CPU check of the index algebra of CorrelateFFT's split first pass
(bigfft.hip k_corr_split0 and k_fft_pass_pf's PACKIN form):
the first pass stores the real transforms A_j = DFT(a_j), B_j = DFT(b_j) of
each 256-sample column in 256 slots, and the second pass's tiles (8
butterflies k = kb..kb+7 and their mirrors 256 - k) rebuild the packed
first-pass output sa A + i sb B from two slots per element.  numpy restates
both sides at a small N; the kernels themselves are checked on the GPU
(test_spectral_gpu.py::test_correlate_fft_2p24)."""
import numpy as np

K0 = 256


def _slots(A, B):
    Y = np.empty_like(A)
    for k in range(K0):
        if k in (0, K0 // 2):
            Y[:, k] = A[:, k].real + 1j * B[:, k].real
        elif k < K0 // 2:
            Y[:, k] = A[:, k]
        else:
            Y[:, k] = B[:, K0 - k]
    return Y.reshape(-1)


def test_split_slots_rebuild_packed_pass():
    N = 1 << 17
    nb = N // K0
    rng = np.random.default_rng(7)
    a, b = rng.standard_normal(N), 1e-6 * rng.standard_normal(N)
    sa, sb = 2.0**-2, 2.0**18
    ca, cb = a.reshape(K0, nb).T, b.reshape(K0, nb).T  # ca[j, r] = a[j + r nb]
    packed = np.fft.fft(sa * ca + 1j * sb * cb, axis=1).reshape(-1)  # Y[j 256 + k]
    Y = _slots(np.fft.fft(ca, axis=1), np.fft.fft(cb, axis=1))
    kmir = lambda k: K0 // 2 if k == 0 else K0 - k  # noqa: E731
    scale = np.abs(packed).max()
    covered = set()
    for t in range(nb // 16):
        cg, kb = t // (K0 // 16), 8 * (t % (K0 // 16))
        for jj in range(8):
            k = kb + jj
            rows = cg * K0 + np.arange(K0) * nb
            A, B = Y[rows + k], Y[rows + kmir(k)]
            if k == 0:
                zA, zB = sa * A.real + 1j * sb * A.imag, sa * B.real + 1j * sb * B.imag
            else:
                zA = (sa * A.real - sb * B.imag) + 1j * (sa * A.imag + sb * B.real)
                zB = (sa * A.real + sb * B.imag) + 1j * (sb * B.real - sa * A.imag)
            assert np.max(np.abs(zA - packed[rows + k])) <= 1e-14 * scale
            assert np.max(np.abs(zB - packed[rows + kmir(k)])) <= 1e-14 * scale
            covered |= {(cg, k), (cg, kmir(k))}
    assert len(covered) == nb  # every second-pass butterfly exactly once per tile set
