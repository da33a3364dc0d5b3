"""World-size-2 `gloo` rehearsal of the multi-GPU path on the CPU (no GPU).

Each rank convolves its own channel group (the oracle stands in for the GPU
convolution here; the GPU side of the same step is covered by the -m gpu
tests), builds its stereo partial mix and the ranks sum-reduce to rank 0,
exactly as bench.py does over RCCL.  Rank 0 compares against the
single-process mix of all channels.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
from algodsp import shard, signals

TOTAL_CH, N, K = 6, 3000, 700


def _kernels():
    return [signals.make_test_kernel(K), signals.make_impulse_kernel(K)]


def _channel_output(c):
    x = signals.white_noise(N, 0x5EED + c)
    return O.OverlapSave(_kernels()[c % 2], 0).process(x)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = list(shard.channel_group(rank, world, TOTAL_CH))
        y = np.stack([_channel_output(c) for c in ids])
        mix = torch.from_numpy(shard.stereo_partial_mix(y, ids))
        base = mix.clone()
        shard.reduce_mix(mix, dist)
        if rank == 0:
            q.put(mix.numpy())
        # bench.py's pipelined form: two steps in flight on two buffers, each
        # reduced asynchronously per (row, output segment), waited on later
        bufs = [base * (s + 1) for s in range(2)]
        cuts = [0, 1024, 2048, base.shape[1]]
        works = [shard.reduce_mix(b[r, lo:hi], dist, async_op=True)
                 for b in bufs for lo, hi in zip(cuts[:-1], cuts[1:]) for r in range(2)]
        for w in works:
            w.wait()
        if rank == 0:
            q.put([b.numpy() for b in bufs])
        # bench.py's N > 1 diagnostics: per-rank step / conv-only / reduce
        # times, max over ranks, then the assembled fields on rank 0
        t = torch.tensor([2.30 + 0.05 * rank, 2.10 + 0.10 * rank, 1.00 - 0.20 * rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        step_ms, conv_ms, reduce_ms = t.tolist()
        if rank == 0:
            q.put(shard.scaling_diagnostics(step_ms, conv_ms, reduce_ms, 2 * (N + K - 1) * 8))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_channel_shard_reduce_world2():
    O.build()
    port = 29500 + os.getpid() % 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    piped = q.get(timeout=240)
    diag = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = shard.stereo_partial_mix(np.stack([_channel_output(c) for c in range(TOTAL_CH)]), range(TOTAL_CH))
    np.testing.assert_allclose(got, full, rtol=0, atol=1e-12 * np.max(np.abs(full)))
    for s, b in enumerate(piped):
        np.testing.assert_allclose(b, full * (s + 1), rtol=0, atol=1e-12 * np.max(np.abs(full)) * (s + 1))
    # max over ranks: step 2.35, conv 2.20, reduce 1.00 ms -> 0.85 of the reduce hidden
    assert diag["conv_ms_per_step"] == 2.2 and diag["reduce_ms"] == 1.0
    assert diag["overlap"] == 0.85
    nbytes = 2 * (N + K - 1) * 8
    assert diag["reduce_bytes_per_rank"] == nbytes
    assert diag["reduce_GBps"] == round(nbytes / 1e-3 / 1e9, 2)
    assert diag["hide_GBps"] == round(nbytes / 2.2e-3 / 1e9, 2)


def test_channel_groups_partition():
    for world in (1, 2, 3, 8):
        for total in (1, 2, 7, 64):
            if total < world:
                continue
            ids = [c for r in range(world) for c in shard.channel_group(r, world, total)]
            assert ids == list(range(total))
    assert list(shard.ir_index(range(5))) == [0, 1, 0, 1, 0]
