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


# ---- every §8(e) statistic, from real chains of the CPU oracle -------------------------
N_REAL = 12          # chains of the C1 lattice (10x10 grid), bases cycling over BASES_REAL
BASES_REAL = (0.5, 1.0, 2.63815853, 4.0)
STEPS_REAL = 3000


def _real_chain(g):
    """Chain g of the C1 workload on the C oracle with every driver tally on."""
    from flipcomplexityempirical_amd import graphs as G
    from oracle.flipref import CRef
    spec = G.grid_graph(10, 10)
    a0 = spec.assignment_array(G.threshold_plan(spec.nodes, 0, 5), [-1, 1])
    _, (lo, hi) = G.population_bounds(spec.n, 2, 0.1)
    r = CRef().run(spec, a0, base=BASES_REAL[g % len(BASES_REAL)], pop_lo=lo, pop_hi=hi, seed=77, chain_id=g,
                   n_steps=STEPS_REAL, log1mp=G.log1mp_table(spec.n, 2), want_hist=True, want_edges=True,
                   want_flips=True)
    return r


def _real_local(gids):
    rs = [_real_chain(int(g)) for g in gids]
    stats = {f: np.asarray([r["stats"][f] for r in rs], dtype=np.int64) for f in D.AGG_FIELDS}
    arrays = {name: np.stack([r[name] for r in rs]) for name in D.SUM_ARRAYS + D.MAX_ARRAYS}
    return D.local_statistics(stats, np.asarray(gids) % len(BASES_REAL), len(BASES_REAL), arrays)


def _real_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = D.shard(N_REAL, world, rank)
    red = D.allreduce_statistics(_real_local(np.arange(off, off + cnt)), dist)
    q.put((rank, red, D.checksums(red)))
    dist.barrier()
    dist.destroy_process_group()


def test_allreduce_all_statistics_world2_gloo():
    """SURVEY §8(e), per configuration: the one reduction carries the |cut| / |B| histograms,
    per-edge cut_times, per-node num_flips / part_sum (sums) and last_flipped (max) besides the
    grouped scalars, each as one row per group (here the base: chain g runs base g % 4, so every
    group has chains on both ranks).  Real per-chain arrays from the C oracle (C1 lattice, 12
    chains) sharded over a gloo world of 2 must reduce to the host-side combination of each
    group's chains -- the reference's per-configuration outputs (grid_chain_sec11.py:383-384,
    396-400,416-419), not their sum over configurations."""
    from oracle import flipref
    flipref.build_lib()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_real_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = _real_local(np.arange(N_REAL))   # every chain on one host, no collective
    assert set(expect) == {"scalars"} | set(D.SUM_ARRAYS) | set(D.MAX_ARRAYS)
    rs = [_real_chain(g) for g in range(N_REAL)]
    ng = len(BASES_REAL)
    for grp in range(ng):
        members = [r for g, r in enumerate(rs) if g % ng == grp]
        for name in D.SUM_ARRAYS:
            assert np.array_equal(expect[name][grp], sum(r[name] for r in members)), (name, grp)
        assert np.array_equal(expect["last_flipped"][grp], np.max([r["last_flipped"] for r in members], axis=0))
        # every yield of the group's chains (the initial state + one per step) lands in one |cut| bin
        assert int(expect["cut_hist"][grp].sum()) == len(members) * (STEPS_REAL + 1)
    for _, red, cs in res:
        for name, arr in expect.items():
            assert np.array_equal(red[name], arr), name
        assert cs == D.checksums(expect)


def test_group_arrays_edge_cases():
    a = np.arange(12, dtype=np.int64).reshape(4, 3)
    g = np.array([2, 0, 2, 0])
    s = D.group_arrays(a, g, 4, "sum")
    assert s.tolist() == [[12, 14, 16], [0, 0, 0], [6, 8, 10], [0, 0, 0]]
    m = D.group_arrays(a, g, 4, "max")
    assert m.tolist() == [[9, 10, 11], [0, 0, 0], [6, 7, 8], [0, 0, 0]]
    with pytest.raises(ValueError):
        D.group_arrays(a, np.array([0, 1, 2, 4]), 4)
    with pytest.raises(ValueError):
        D.group_arrays(a, np.array([0, 1]), 4)
    assert D.sweep_groups(10, 3, offset=4, count=4).tolist() == [1, 2, 0, 1]
    cs = D.group_checksums({"x": s})
    assert cs["x"][1] == 0 and cs["x"][0] == D.checksums({"x": s[0]})["x"]


def test_forced_collective_world1_gloo():
    """``force=True`` runs the collectives at world size 1 (the path tests/test_rccl_gpu.py takes
    over RCCL on the GPU box): identity results, through the real gloo all-reduce calls."""
    import socket
    import torch.distributed as dist
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        calls = []
        real = dist.all_reduce
        dist.all_reduce = lambda t, op=None: (calls.append(op), real(t, op=op))[1]
        try:
            rng = np.random.default_rng(2)
            st = {f: rng.integers(0, 1000, 10) for f in D.AGG_FIELDS}
            loc = D.local_statistics(st, np.arange(10) % 3, 3, {"last_flipped": rng.integers(0, 99, (10, 4))})
            red = D.allreduce_statistics(loc, dist, force=True)
            assert np.array_equal(red["scalars"], loc["scalars"])
            assert np.array_equal(red["last_flipped"], loc["last_flipped"])
            assert D.allreduce_max(2.5, dist, force=True) == 2.5
            assert len(calls) == 3
            D.allreduce_statistics(loc, dist)  # no force: no collective at one rank
            assert len(calls) == 3
        finally:
            dist.all_reduce = real
    finally:
        dist.destroy_process_group()
