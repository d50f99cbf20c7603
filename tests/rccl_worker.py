"""Subprocess body of tests/test_rccl_gpu.py: one rank of backend "nccl" (RCCL) at world size 1 on
the box's GPU, in the order bench.py's N > 1 path takes -- torch and its HIP runtime first
(``torch.cuda`` initialised, the process group up), then the flip-chain library, which then
binds to the same runtime (one HIP runtime per process).  Prints one JSON line of checks."""
import json
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    assert torch.cuda.is_available(), "torch sees no GPU"
    torch.cuda.set_device(0)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group(backend="nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0)
    dev = torch.device("cuda", 0)
    from flipcomplexityempirical_amd import _lib
    from flipcomplexityempirical_amd import distributed as D
    from flipcomplexityempirical_amd import sweep as SW
    _lib.load()
    out = {"backend": dist.get_backend(), "hip_runtime": _lib.hip_runtime_path(), "checks": {}}
    chk = out["checks"]

    rng = np.random.default_rng(5)
    n_chains, n_groups, E, n = 96, 7, 300, 160
    stats = {f: rng.integers(0, 1 << 40, n_chains, dtype=np.int64) for f in D.AGG_FIELDS}
    groups = rng.integers(0, n_groups, n_chains)
    arrays = {"cut_hist": rng.integers(0, 1000, (n_chains, E + 1)), "nb_hist": rng.integers(0, 1000, (n_chains, n + 1)),
              "cut_times": rng.integers(0, 1 << 33, (n_chains, E)), "num_flips": rng.integers(0, 1 << 20, (n_chains, n)),
              "part_sum": rng.integers(-(1 << 45), 1 << 45, (n_chains, n)),
              "last_flipped": rng.integers(0, 1 << 50, (n_chains, n))}
    local = D.local_statistics(stats, groups, n_groups, arrays)
    calls = []
    real = dist.all_reduce

    def counting(t, op=None):
        calls.append((str(op), str(t.dtype), str(t.device)))
        return real(t, op=op)
    dist.all_reduce = counting
    red = D.allreduce_statistics(local, dist, dev, force=True)
    chk["scalars"] = bool(np.array_equal(red["scalars"], D.group_aggregate(stats, groups, n_groups)))
    for name in D.SUM_ARRAYS:
        exp = np.zeros((n_groups, arrays[name].shape[1]), dtype=np.int64)
        np.add.at(exp, groups, arrays[name])
        chk[name] = bool(np.array_equal(red[name], exp))
    exp = np.zeros((n_groups, n), dtype=np.int64)
    for g in range(n_groups):
        if (groups == g).any():
            exp[g] = arrays["last_flipped"][groups == g].max(axis=0)
    chk["last_flipped_max"] = bool(np.array_equal(red["last_flipped"], exp))
    flat = rng.integers(-(1 << 62), 1 << 62, 1000, dtype=np.int64)
    chk["int64_sum"] = bool(np.array_equal(D.allreduce_sum(flat, dist, dev, force=True), flat))
    chk["f64_max"] = D.allreduce_max(123.456789, dist, dev, force=True) == 123.456789

    # the reference sweep's per-configuration sums through the collectives vs the host reduction
    cfgs = SW.sweep_configs("sec11")[:6]
    kw = dict(replicas=3, total_steps=2000, seed=9, configs=cfgs, series=False, corrected=False)
    sw = SW.Sweep("sec11", dist=dist, dist_device=dev, force_collective=True, **kw).run()
    red = sw.grouped()
    dist.all_reduce = real
    host = SW.Sweep("sec11", **kw).run()
    ref = host.grouped()
    chk["sweep_grouped"] = all(bool(np.array_equal(red[k], ref[k])) for k in ref)
    st = host._run.stats()
    chk["sweep_chain_sum_wait"] = bool(np.array_equal(red["chain_sum_wait"].reshape(-1), st["sum_wait"]))
    chk["sweep_steps"] = int(red["scalars"][:, D.AGG_FIELDS.index("steps")].sum()) == int(st["steps"].sum())
    sw.close()
    host.close()
    out["collective_calls"] = calls
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
