"""Chains -> GPUs sharding and the one statistics reduction.

Chains are independent: global chain id g = offset(rank) + c, and the Philox counter holds
g, so every chain's trajectory is independent of how many GPUs run it.  There is no
data-path collective; at the end one all-reduce (RCCL over xGMI with backend "nccl", gloo on
CPU) sums the per-group statistics.
"""
from __future__ import annotations

from typing import Dict, Sequence, Tuple

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


def allreduce_sum(arr: np.ndarray, dist=None, device=None) -> np.ndarray:
    """Sum ``arr`` over ranks (identity without a process group)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return arr
    import torch
    t = torch.as_tensor(np.ascontiguousarray(arr), device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def allreduce_max(x: float, dist=None, device=None) -> float:
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
