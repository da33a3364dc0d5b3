"""Channel-group sharding across GPUs.

The path shards by channel: each rank (one process per GPU) convolves its own
contiguous group of channels with no data-path collective; the only exchange
is one sum-reduce of the per-rank stereo partial mixes to rank 0 (the north
star's stereo mixdown; the reference defines no mixdown, so it is
build-defined: L = sum of even global channels, R = sum of odd ones).
"""
from __future__ import annotations

import numpy as np


def channel_group(rank: int, world: int, total: int) -> range:
    """Contiguous channel ids owned by `rank` (earlier ranks take the remainder)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return range(lo, lo + base + (1 if rank < rem else 0))


def ir_index(channel_ids, n_ir: int = 2) -> np.ndarray:
    """IR of each channel: c mod n_ir (config 4: ch c uses IR[c mod 2])."""
    return np.asarray([c % n_ir for c in channel_ids], dtype=np.int32)


def stereo_partial_mix(y: np.ndarray, channel_ids) -> np.ndarray:
    """[2][n] partial mix of this rank's channels by global channel parity
    (what k_mixdown computes on the device when the group starts at an even id)."""
    mix = np.zeros((2, y.shape[1]))
    for row, c in zip(y, channel_ids):
        mix[c % 2] += row
    return mix


def reduce_mix(mix_tensor, dist, async_op: bool = False):
    """Sum the per-rank partial mixes into rank 0's tensor (RCCL over xGMI on
    the GPU path, gloo in the CPU tests).  async_op: returns the work handle;
    on RCCL the reduce runs on the process group's stream after the work
    already queued on the current stream, overlapping what is queued next."""
    return dist.reduce(mix_tensor, dst=0, op=dist.ReduceOp.SUM, async_op=async_op)
