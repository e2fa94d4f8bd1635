"""Multi-process layout on CPU (gloo, world size 2): contiguous batch shards, one broadcast of the
key material from rank 0, optional all-gather of the shard results."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tfhe-rs-odd_amd"))
    from tfhe_mi355.distributed import broadcast_u64, gather_u64, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        key = np.arange(1000, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) if rank == 0 else None
        t = broadcast_u64(key, 1000, 0, torch.device("cpu"))
        got = t.numpy().view(np.uint64)
        ok_key = bool(np.array_equal(got, np.arange(1000, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)))
        total = 11
        lo, hi = shard_range(total, rank, world)
        local = np.stack([np.full(3, i, dtype=np.uint64) for i in range(lo, hi)])
        full = gather_u64(local, total, torch.device("cpu"))
        ok_gather = bool(np.array_equal(full[:, 0], np.arange(total, dtype=np.uint64)))
        q.put((rank, ok_key, ok_gather, lo, hi))
    finally:
        dist.destroy_process_group()


def test_shard_range_partitions_batch():
    from tfhe_mi355.distributed import shard_range

    for total in [0, 1, 7, 4096, 4099]:
        for world in [1, 2, 3, 8]:
            ranges = [shard_range(total, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.timeout(120)
def test_gloo_world2_broadcast_and_gather():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=90) for _ in range(2)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    res.sort()
    assert all(r[1] and r[2] for r in res), res
    assert res[0][3:] == (0, 6) and res[1][3:] == (6, 11)
