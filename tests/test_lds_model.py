"""The LDS swizzle of the FFT kernels (fft_device.hpp lds_slot) against the
bank model of tools/lds_conflicts.py (MI355X_MICROARCH.md's lane groups):
the constant in the header is the one the model checks, it permutes each
aligned 16-element block, and every Stockham store and load of the V = 4 and
8 plans the kernels instantiate is conflict-free under it (the round-1
swizzle is not).  CPU only."""
import re
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import lds_conflicts as L  # noqa: E402


def header_constant():
    src = (ROOT / "algo-dsp_amd" / "csrc" / "fft_device.hpp").read_text()
    m = re.search(r"\(0x([0-9a-f]+)ull >> \(4 \* t\)\)", src)
    assert m, "lds_slot's packed table not found in fft_device.hpp"
    return int(m.group(1), 16)


def test_header_matches_model():
    K = header_constant()
    for i in range(4096):
        t = (i >> 3) & 15
        assert i ^ ((K >> (4 * t)) & 15) == L.swz1(i)


def test_swizzle_permutes_each_16_block():
    for base in range(0, 8192, 16):
        assert sorted(L.swz1(i) for i in range(base, base + 16)) == list(range(base, base + 16))


@pytest.mark.parametrize("M,V", [(256, 8), (256, 4), (1024, 8), (2048, 8), (4096, 8)])
def test_plans_conflict_free(M, V):
    pats = L.patterns(M, V)
    for rowoff in (M, M + 1):
        assert L.extra_cycles(pats, rowoff, L.swz1) == 0
    # the round-1 swizzle left the stride-8 / stride-4 stores 2-way
    assert L.extra_cycles(pats, M, L.swz0) > 0
