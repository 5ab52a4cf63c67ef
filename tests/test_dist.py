"""Multi-rank path of bench.py on CPU (gloo, world_size 2): stream sharding
covers every stream exactly once and the only collective (timing / sample
counters) reduces max / sum."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = bench.shard_streams(1024, rank, world)
    elapsed, samples = bench.reduce_stats(0.5 + rank, (hi - lo) * 2 * 441000, device=torch.device("cpu"))
    q.put((rank, lo, hi, elapsed, samples))
    dist.destroy_process_group()


def test_gloo_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, lo0, hi0, e0, s0), (r1, lo1, hi1, e1, s1) = res
    assert (lo0, hi0, lo1, hi1) == (0, 512, 512, 1024)
    assert e0 == e1 == 1.5                     # max over ranks
    assert s0 == s1 == 1024 * 2 * 441000       # summed samples


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shards_partition_streams(world):
    import bench
    seen = []
    for r in range(world):
        lo, hi = bench.shard_streams(1024, r, world)
        seen.extend(range(lo, hi))
    assert seen == list(range(1024))


def _worker_resample(rank, world, port, q):
    """Each rank resamples its contiguous shard of config 4's streams (dry-run handle: the host
    state machine, exact reference counts, no GPU) in 4096-frame ProcessMulti calls + FlushMulti,
    then the counters go through bench.reduce_stats (the only collective)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    import gar
    from helpers import chunk_sizes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    streams, frames = 64, 44_100  # config 4's shape at 1/16 of the streams and 1/10 of the length
    lo, hi = bench.shard_streams(streams, rank, world)
    r = gar.NewBatch(gar.Config(44100, 48000, 2, gar.QualityHigh, DryRun=True), hi - lo)
    out = 0
    for n in chunk_sizes(frames, 4096):
        xs = [np.zeros(n)] * (2 * (hi - lo))
        out += sum(len(y) for y in r.ProcessMulti(xs))
    out += sum(len(y) for y in r.FlushMulti())
    _, total = bench.reduce_stats(1.0, out, device=torch.device("cpu"))
    q.put((rank, hi - lo, out, total))
    dist.destroy_process_group()


def test_gloo_two_ranks_resample_shards(O):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_resample, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the reference's own count for one stream, every stream identical
    ref = O.NewResampler(44100, 48000, 1, O.P_HIGH)
    per_channel = sum(len(ref.process(__import__("numpy").zeros(n), 0)) for n in [4096] * 10 + [44_100 - 40_960])
    per_channel += len(ref.flush(0))
    (_, n0, out0, t0), (_, n1, out1, t1) = res
    assert (n0, n1) == (32, 32)
    assert out0 == out1 == 32 * 2 * per_channel
    assert t0 == t1 == 64 * 2 * per_channel
