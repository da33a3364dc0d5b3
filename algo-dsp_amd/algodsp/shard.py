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


def scaling_diagnostics(step_ms: float, conv_ms: float, reduce_ms: float, reduce_bytes: float) -> dict:
    """What an N > 1 bench line needs to tell whether the mixdown reduce hides
    under the convolution (every input already the max over ranks):
    step_ms   the timed step (convolution + reduce on the side stream, pipelined);
    conv_ms   the same step with the reduce off;
    reduce_ms the reduce alone (events around it on the side stream);
    reduce_bytes the partial mix each rank contributes (2 rows x out_len x 8 B).
    overlap = the share of the reduce that the step did not pay for,
    (conv + reduce - step) / reduce, clipped to [0, 1]; hide_GBps = the rate the
    reduce needs to fit under the convolution."""
    hidden = conv_ms + reduce_ms - step_ms
    return {
        "conv_ms_per_step": round(conv_ms, 4),
        "reduce_ms": round(reduce_ms, 4),
        "reduce_bytes_per_rank": int(reduce_bytes),
        "reduce_GBps": round(reduce_bytes / (reduce_ms * 1e-3) / 1e9, 2) if reduce_ms > 0 else None,
        "hide_GBps": round(reduce_bytes / (conv_ms * 1e-3) / 1e9, 2) if conv_ms > 0 else None,
        "overlap": round(min(1.0, max(0.0, hidden / reduce_ms)), 3) if reduce_ms > 0 else None,
        "step_over_conv": round(step_ms / conv_ms, 4) if conv_ms > 0 else None,
    }


class Comm:
    """The library's own RCCL communicator (include/algodsp.h ad_comm_*): the
    path a cgo caller takes to shard without torch.distributed.  `bootstrap`
    moves rank 0's 128-byte unique id to every rank (here: a torch.distributed
    broadcast of the bytes; any transport works)."""

    def __init__(self, rank: int, world: int, device: int, bootstrap=None):
        import ctypes as C

        from ._lib import check, lib

        if world > 1 and bootstrap is None:
            # without it, ranks != 0 would hand RCCL an all-zero id and block in
            # ncclCommInitRank
            raise ValueError("Comm: world > 1 needs a bootstrap to share rank 0's unique id")
        L = lib()
        uid = (C.c_uint8 * 128)()
        if rank == 0:
            check(L.ad_comm_get_unique_id(uid))
        if bootstrap is not None:
            data = bootstrap(bytes(uid))
            C.memmove(uid, data, 128)
        h = C.c_void_p()
        check(L.ad_comm_create(uid, int(world), int(rank), int(device), C.byref(h)))
        self._h = h
        self.rank, self.world = rank, world

    def mixdown_reduce(self, d_chan: int, channels: int, stride: int, length: int, d_mix: int, mix_stride: int,
                       first_parity: int = 0, root: int = 0, stream: int = 0) -> None:
        """k_mixdown of this rank's channel group, then one in-place RCCL
        sum-reduce of the [2][mix_stride] mix to `root`, both on `stream`."""
        import ctypes as C

        from ._lib import check, lib

        check(lib().ad_mixdown_reduce(self._h, C.c_void_p(d_chan), int(channels), int(stride), int(length),
                                      int(first_parity), C.c_void_p(d_mix), int(mix_stride), int(root),
                                      C.c_void_p(stream)))

    def close(self) -> None:
        from ._lib import lib

        if getattr(self, "_h", None):
            lib().ad_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
