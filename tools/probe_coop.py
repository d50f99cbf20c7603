"""Workgroup-cooperative search against the one-wave search (BASELINE config 5's "workgroup-per-
chain BFS contiguity"), by district size: the Delaunay dual of 10^4 points without positions
(every multi-run contiguity case goes to the device search) at k = 18 (C5, ~555 nodes per
district), k = 8 and k = 4 (~2,500 nodes per district).  One launch of one wave of resident
chains per mode; per chain, the search time is approximated by the launch time over its searches.

    python tools/probe_coop.py [steps]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from flipcomplexityempirical_amd import _lib, graphs as G  # noqa: E402
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig  # noqa: E402
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
spec = G.delaunay_graph(10000, seed=0)
fg = FlipGraph(spec, use_positions=False)
out = []
for k in (18, 8, 4):
    a0 = spec.assignment_array(G.bisection_plan(spec, k), list(range(k)))
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, 0.1)
    for sw in (1, 4):
        tune = {"search_waves": sw}
        cfg = RunConfig(k=k, labels=tuple(range(k)), proposal=_lib.FC_PROPOSE_PAIR, seed=0x5EED0005, pop_lo=lo,
                        pop_hi=hi, flags=_lib.FC_FLAG_FORCE_BFS, tune=tune)
        probe = FlipRun(fg, a0[None, :], cfg)
        lds = probe.chain_lds_bytes()
        probe.close()
        lds_g = -(-lds // bench.LDS_GRANULE) * bench.LDS_GRANULE
        per_cu = max(1, min(160 * 1024 // lds_g, 16 if sw == 1 else 4))
        C = 256 * per_cu if sw == 1 else 256 * 2  # coop: two 256-thread workgroups per CU (VGPR-bound)
        run = FlipRun(fg, np.broadcast_to(a0, (C, spec.n)), cfg, bases=np.full(C, 1.0))
        run.steps(200)
        run.sync()
        s0 = run.stats()
        run.timings()
        t0 = time.perf_counter()
        run.steps(steps)
        run.sync()
        dt = time.perf_counter() - t0
        ms = float(run.timings().mean())
        s1 = run.stats()
        props = float((s1["proposals"] - s0["proposals"]).sum())
        calls = float((s1["bfs_calls"] - s0["bfs_calls"]).sum())
        levels = float((s1["bfs_levels"] - s0["bfs_levels"]).sum())
        per_chain_searches = calls / C
        rec = {"k": k, "search_waves": sw, "chains": C, "chain_lds_bytes": lds, "kernel": run.kernel_name(),
               "kernel_ms": ms, "proposals_per_s": props / dt, "searches_per_proposal": calls / props if props else None,
               "levels_per_search": levels / calls if calls else None,
               "us_per_search_upper": ms * 1e3 / per_chain_searches if per_chain_searches else None,
               "cycles_per_level_upper": (ms * 1e-3 * 2.4e9 / per_chain_searches / (levels / calls))
               if calls and per_chain_searches else None}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        run.close()
