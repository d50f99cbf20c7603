"""Chains -> GPUs sharding and the one statistics reduction.

Chains are independent: global chain id g = offset(rank) + c, and the Philox counter holds
g, so every chain's trajectory is independent of how many GPUs run it.  There is no
data-path collective; at the end one all-reduce (RCCL over xGMI with backend "nccl", gloo on
CPU) sums every statistic the reference's driver accumulates (grid_chain_sec11.py:350-419),
**per configuration**: every chain carries a group id -- its (pop, base, alignment)
configuration of the sweep at :182-184, or any caller-given key -- and each statistic is kept
as one row per group, because the reference writes and plots them per configuration
(:383-384,396-400,416-419 accumulated, :410-528 written):

* per-group scalars (AGG_FIELDS: proposals, steps, accepted, invalid counts, the per-yield
  sums behind rce / rbn / wait.txt);
* the |cut| and |B| histograms over yields (E + 1 and N + 1 bins), ``[n_groups, bins]``;
* per-edge ``cut_times`` (:383-384), ``[n_groups, E]``;
* per-node ``num_flips`` and ``part_sum`` (:396-400), ``[n_groups, N]`` each;
* per-node ``last_flipped`` (:398), ``[n_groups, N]``, reduced by MAX (the one non-additive
  field; a second all-reduce with op MAX).

The sum fields travel as one packed int64 buffer (C2's 30 configurations: ~3 MB), so the
collective is latency-bound whatever the link: xGMI bandwidth is irrelevant here.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Tuple

import numpy as np

AGG_FIELDS = ("proposals", "steps", "accepted", "inv_contig", "inv_pop", "sum_cut", "sum_nb", "sum_wait",
              "sum_cut2", "sum_nb2", "draws")


def shard(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous blocks: chain g -> rank floor(g * world / n_total).  Returns (offset, count)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    lo = -(-rank * n_total // world)          # ceil(rank * n / world)
    hi = -(-(rank + 1) * n_total // world)
    return lo, hi - lo


def owner(g: int, n_total: int, world: int) -> int:
    return g * world // n_total


def group_aggregate(stats: Dict[str, np.ndarray], groups: np.ndarray, n_groups: int) -> np.ndarray:
    """[n_groups, len(AGG_FIELDS)] int64 sums of the per-chain statistics by group id."""
    out = np.zeros((n_groups, len(AGG_FIELDS)), dtype=np.int64)
    for j, f in enumerate(AGG_FIELDS):
        vals = np.asarray(stats[f], dtype=np.int64)
        np.add.at(out[:, j], groups, vals)
    return out


def _collective(dist, force: bool) -> bool:
    """Whether to call the collective: a process group of more than one rank, or any process
    group when ``force`` (a world-size-1 group still runs the RCCL / gloo call, so the device
    tensor path is exercised on one GPU)."""
    if not (dist is not None and dist.is_initialized() and (force or dist.get_world_size() > 1)):
        return False
    if dist.get_backend() == "nccl":
        import torch
        if not torch.cuda.is_available():
            # the flip-chain library was loaded before torch started its HIP runtime: the process
            # then holds two runtimes and torch's finds no GPU.  Start torch.cuda first (bench.py
            # _dist, sweep.main) so the library binds to the same runtime.
            raise RuntimeError("RCCL collective requested but torch.cuda is unavailable in this process: initialise "
                               "torch.cuda (and the process group) before loading libflipchain.so")
    return True


def allreduce_sum(arr: np.ndarray, dist=None, device=None, force: bool = False) -> np.ndarray:
    """Sum ``arr`` over ranks (identity without a process group)."""
    if not _collective(dist, force):
        return arr
    import torch
    t = torch.as_tensor(np.ascontiguousarray(arr), device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def allreduce_max(x: float, dist=None, device=None, force: bool = False) -> float:
    if not _collective(dist, force):
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# per-run arrays of the full diagnostics (FlipRun.hist / cut_times / flips), reduced over
# chains on each rank and then over ranks
SUM_ARRAYS = ("cut_hist", "nb_hist", "cut_times", "num_flips", "part_sum")
MAX_ARRAYS = ("last_flipped",)


def group_arrays(arr: np.ndarray, groups: np.ndarray, n_groups: int, op: str = "sum") -> np.ndarray:
    """``[n_groups, len]``: the rows of a per-chain array ``[chains, len]`` summed (or maxed)
    by group id; groups without chains give zero rows."""
    a = np.asarray(arr, dtype=np.int64)
    if a.ndim == 1:
        a = a[None, :]
    g = np.asarray(groups, dtype=np.int64).reshape(-1)
    if g.size != a.shape[0]:
        raise ValueError("one group id per chain")
    if g.size and (g.min() < 0 or g.max() >= n_groups):
        raise ValueError("group id out of range")
    out = np.zeros((n_groups, a.shape[1]), dtype=np.int64)
    if op == "sum":
        np.add.at(out, g, a)
    else:
        for grp in np.unique(g):
            out[grp] = a[g == grp].max(axis=0)
    return out


def local_statistics(stats: Dict[str, np.ndarray], groups: np.ndarray, n_groups: int,
                     arrays: Optional[Dict[str, np.ndarray]] = None) -> Dict[str, np.ndarray]:
    """One rank's contribution, per group (configuration): grouped scalar sums and, for every
    per-chain array present in ``arrays`` (``[chains, len]``), its ``[n_groups, len]`` sum (or
    max, ``last_flipped``) over the rank's chains of each group."""
    out = {"scalars": group_aggregate(stats, groups, n_groups)}
    for name, arr in (arrays or {}).items():
        if name in SUM_ARRAYS:
            out[name] = group_arrays(arr, groups, n_groups, "sum")
        elif name in MAX_ARRAYS:
            out[name] = group_arrays(arr, groups, n_groups, "max")
        else:
            raise KeyError(f"unknown statistic {name!r}")
    return out


def sweep_groups(n_chains_total: int, n_configs: int, offset: int = 0, count: Optional[int] = None) -> np.ndarray:
    """Group id of global chains offset .. offset + count - 1 when chain g runs configuration
    g % n_configs (the bench's and the sweep drivers' dealing of configurations to chains)."""
    count = n_chains_total - offset if count is None else count
    return (np.arange(offset, offset + count) % n_configs).astype(np.int64)


def _pack(d: Dict[str, np.ndarray], names) -> Tuple[np.ndarray, list]:
    layout, parts = [], []
    for name in names:
        if name in d:
            a = np.ascontiguousarray(d[name], dtype=np.int64)
            layout.append((name, a.shape))
            parts.append(a.reshape(-1))
    flat = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64)
    return flat, layout


def _unpack(flat: np.ndarray, layout) -> Dict[str, np.ndarray]:
    out, pos = {}, 0
    for name, shape in layout:
        size = int(np.prod(shape))
        out[name] = flat[pos:pos + size].reshape(shape)
        pos += size
    return out


def allreduce_statistics(local: Dict[str, np.ndarray], dist=None, device=None,
                         force: bool = False) -> Dict[str, np.ndarray]:
    """Every rank's ``local_statistics`` combined: one SUM all-reduce of the packed additive
    fields (scalars, histograms, cut_times, num_flips, part_sum; all ``[n_groups, ...]``) and
    one MAX all-reduce of last_flipped.  Every rank must pass the same set of fields with the
    same shapes (the same n_groups, even where it runs no chain of a group)."""
    flat_s, lay_s = _pack(local, ("scalars",) + SUM_ARRAYS)
    flat_m, lay_m = _pack(local, MAX_ARRAYS)
    if _collective(dist, force):
        import torch
        t = torch.as_tensor(flat_s, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        flat_s = t.cpu().numpy()
        if flat_m.size:
            t = torch.as_tensor(flat_m, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            flat_m = t.cpu().numpy()
    out = _unpack(flat_s, lay_s)
    out.update(_unpack(flat_m, lay_m))
    return out


def _checksum(a) -> int:
    x = np.asarray(a, dtype=np.int64).reshape(-1)
    w = np.arange(1, x.size + 1, dtype=np.int64)
    return int((x * w).sum() & ((1 << 63) - 1))


def checksums(red: Dict[str, np.ndarray]) -> Dict[str, int]:
    """Order-sensitive int64 checksums of the reduced fields (the N > 1 bench line's record of
    what the collective produced): sum_i (i + 1) * x_i mod 2^63 per field."""
    return {name: _checksum(a) for name, a in red.items()}


def group_checksums(red: Dict[str, np.ndarray]) -> Dict[str, list]:
    """Per-group checksums of every reduced field (row g of each ``[n_groups, ...]`` array):
    what each configuration's outputs came to after the collective."""
    return {name: [_checksum(row) for row in np.asarray(a)] for name, a in red.items()}
