"""Deterministic synthetic inputs shared by tests and the benchmark.

White noise: SplitMix64(seed) mapped to uniform [-1, 1); the
reference's own generators (Go math/rand, math/rand/v2 PCG) are not
reproducible here, so identical inputs means identical buffers fed to the
oracle and to the GPU.  Helper kernels restate the reference test helpers.
"""
from __future__ import annotations

import math

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """Outputs start .. start+n-1 of SplitMix64 started at `seed` (vectorised;
    the generator is counter-based, so any slice is computed directly)."""
    with np.errstate(over="ignore"):
        idx = np.arange(start + 1, start + n + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def white_noise(n: int, seed: int = 0x5EED, start: int = 0) -> np.ndarray:
    """Uniform [-1, 1) float64 white noise (seed 0x5EED + channel);
    `start` returns samples start .. start+n-1 of the same sequence."""
    z = splitmix64(seed, n, start)
    u = (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return u * 2.0 - 1.0


def make_test_kernel(n: int) -> np.ndarray:
    """Hann-windowed sinc (dsp/conv/conv_bench_test.go:296-312)."""
    k = np.empty(n)
    center = (n - 1) / 2.0
    for i in range(n):
        x = i - center
        k[i] = 1.0 if x == 0 else math.sin(math.pi * x / 4) / (math.pi * x / 4)
        k[i] *= 0.5 * (1 - math.cos(2 * math.pi * i / (n - 1))) if n > 1 else 1.0
    return k


def make_test_signal(n: int) -> np.ndarray:
    """dsp/conv/conv_bench_test.go:286-293"""
    i = np.arange(n, dtype=np.float64)
    return np.sin(2 * math.pi * i / 100) + 0.5 * np.cos(2 * math.pi * i / 30)


def make_impulse_kernel(n: int) -> np.ndarray:
    """0.99^i decay (dsp/conv/partitioned_test.go:11-20), built by repeated multiply."""
    k = np.empty(n)
    if n:
        k[0] = 1.0
    for i in range(1, n):
        k[i] = k[i - 1] * 0.99
    return k
