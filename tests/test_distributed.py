"""Sharding and the statistics all-reduce, world_size 2 over gloo on CPU."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from flipcomplexityempirical_amd import distributed as D


def test_shard_covers_all_chains():
    for n in (1, 7, 4096, 65536):
        for w in (1, 2, 3, 8):
            got = [D.shard(n, w, r) for r in range(w)]
            assert got[0][0] == 0 and sum(c for _, c in got) == n
            for (o1, c1), (o2, _) in zip(got, got[1:]):
                assert o1 + c1 == o2
            for g in range(0, n, max(1, n // 97)):
                r = D.owner(g, n, w)
                o, c = got[r]
                assert o <= g < o + c


def test_group_aggregate():
    stats = {f: np.arange(10, dtype=np.int64) * (i + 1) for i, f in enumerate(D.AGG_FIELDS)}
    groups = np.arange(10) % 3
    agg = D.group_aggregate(stats, groups, 3)
    assert agg.shape == (3, len(D.AGG_FIELDS))
    assert agg[:, 0].tolist() == [0 + 3 + 6 + 9, 1 + 4 + 7, 2 + 5 + 8]
    assert agg.sum(0).tolist() == [stats[f].sum() for f in D.AGG_FIELDS]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_total = 40
    off, cnt = D.shard(n_total, world, rank)
    gids = np.arange(off, off + cnt)
    # synthetic per-chain statistics that depend only on the global chain id
    stats = {f: (gids * (j + 2) + 1).astype(np.int64) for j, f in enumerate(D.AGG_FIELDS)}
    agg = D.group_aggregate(stats, gids % 10, 10)
    tot = D.allreduce_sum(agg, dist)
    mx = D.allreduce_max(float(rank + 1), dist)
    q.put((rank, tot, mx))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gids = np.arange(40)
    stats = {f: (gids * (j + 2) + 1).astype(np.int64) for j, f in enumerate(D.AGG_FIELDS)}
    expect = D.group_aggregate(stats, gids % 10, 10)
    for _, tot, mx in res:
        assert np.array_equal(tot, expect)
        assert mx == 2.0
