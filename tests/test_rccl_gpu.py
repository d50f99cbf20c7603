"""The RCCL branch of the one statistics reduction on real hardware.

Multi-rank runs on the CPU use gloo (tests/test_distributed.py); the 8-GPU bench uses backend
"nccl" (RCCL on ROCm) with device tensors.  A world-size-1 process group on the box's GPU runs
that branch here: ``force=True`` makes ``distributed.allreduce_*`` and ``Sweep.grouped`` call the
collectives instead of short-circuiting at one rank, on int64 SUM, int64 MAX and float64 MAX
device tensors.  At one rank a reduction is the identity, so every result must equal the
host-side numpy reduction of the same per-chain data bit for bit."""
import socket

import numpy as np
import pytest

from flipcomplexityempirical_amd import distributed as D

pytestmark = pytest.mark.gpu


def _port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return int(so.getsockname()[1])


@pytest.fixture(scope="module")
def rccl(gpu):
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group(backend="nccl", init_method=f"tcp://127.0.0.1:{_port()}", world_size=1, rank=0)
    assert dist.get_backend() == "nccl"
    yield dist, torch.device("cuda", 0)
    dist.destroy_process_group()


def test_rccl_statistics_sum_and_max(rccl):
    dist, dev = rccl
    rng = np.random.default_rng(5)
    n_chains, n_groups, E, n = 96, 7, 300, 160
    stats = {f: rng.integers(0, 1 << 40, n_chains, dtype=np.int64) for f in D.AGG_FIELDS}
    groups = rng.integers(0, n_groups, n_chains)
    arrays = {"cut_hist": rng.integers(0, 1000, (n_chains, E + 1)), "nb_hist": rng.integers(0, 1000, (n_chains, n + 1)),
              "cut_times": rng.integers(0, 1 << 33, (n_chains, E)), "num_flips": rng.integers(0, 1 << 20, (n_chains, n)),
              "part_sum": rng.integers(-(1 << 45), 1 << 45, (n_chains, n)),
              "last_flipped": rng.integers(0, 1 << 50, (n_chains, n))}
    local = D.local_statistics(stats, groups, n_groups, arrays)
    red = D.allreduce_statistics(local, dist, dev, force=True)
    # the host-side reduction of the same data
    assert np.array_equal(red["scalars"], D.group_aggregate(stats, groups, n_groups))
    for name in D.SUM_ARRAYS:
        exp = np.zeros((n_groups, arrays[name].shape[1]), dtype=np.int64)
        np.add.at(exp, groups, arrays[name])
        assert np.array_equal(red[name], exp), name
    exp = np.zeros((n_groups, n), dtype=np.int64)
    for g in range(n_groups):
        if (groups == g).any():
            exp[g] = arrays["last_flipped"][groups == g].max(axis=0)
    assert np.array_equal(red["last_flipped"], exp)
    # the bench's scalar collectives: int64 SUM of a packed buffer, float64 MAX
    flat = rng.integers(-(1 << 62), 1 << 62, 1000, dtype=np.int64)
    assert np.array_equal(D.allreduce_sum(flat, dist, dev, force=True), flat)
    assert D.allreduce_max(123.456789, dist, dev, force=True) == 123.456789
    # without force a one-rank group short-circuits (no collective), with the same result
    assert D.allreduce_statistics(local, dist, dev)["scalars"] is not None


def test_rccl_sweep_grouped(rccl):
    """``Sweep.grouped`` (the reference sweep's per-configuration sums, :383-419) through the RCCL
    collectives equals the host-side reduction of the same chains."""
    from flipcomplexityempirical_amd import sweep as SW
    dist, dev = rccl
    cfgs = SW.sweep_configs("sec11")[:6]
    kw = dict(replicas=3, total_steps=2000, seed=9, configs=cfgs, series=False, corrected=False)
    sw = SW.Sweep("sec11", dist=dist, dist_device=dev, force_collective=True, **kw).run()
    assert sw.world == 1
    red = sw.grouped()
    host = SW.Sweep("sec11", **kw).run()
    exp = host.grouped()
    for name in exp:
        assert np.array_equal(red[name], exp[name]), name
    st = host._run.stats()
    assert np.array_equal(red["chain_sum_wait"].reshape(-1), st["sum_wait"])
    assert int(red["scalars"][:, D.AGG_FIELDS.index("steps")].sum()) == int(st["steps"].sum())
    sw.close()
    host.close()
