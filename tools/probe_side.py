"""Side-config probe: python tools/probe_side.py WORKLOAD [chains] [steps/launch] [iters]
Prints kernel ms, proposals/s, BFS calls / proposal and BFS levels / call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import bench
from flipcomplexityempirical_amd import graphs as G
from flipcomplexityempirical_amd import _lib  # noqa: E402
_lib.load(allow_variant=True)  # A/B and profiling tool: FC_LIB_PATH / FC_LIB_VARIANT libraries allowed
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig, parse_tune

W = bench.Workload(sys.argv[1])
S = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
IT = int(sys.argv[4]) if len(sys.argv) > 4 else 2
# FC_PROBE_NOPOS=1: build the graph without positions (no planar rings); FC_PROBE_FLAGS: fc_params.flags
fg = FlipGraph(W.spec, use_positions=os.environ.get("FC_PROBE_NOPOS", "0") != "1")
C = (int(sys.argv[2]) if len(sys.argv) > 2 else 0) or (bench.resident_chains(fg, W) if W.name in ("c4", "c5")
                                                         else W.chains)
inits = np.stack([W.init_of(g) for g in range(C)])
bases = np.asarray([W.base_of(g) for g in range(C)])
_, (lo, hi) = G.population_bounds(int(W.spec.pop.sum()), W.k, W.pct)
run = FlipRun(fg, inits, RunConfig(tune=parse_tune(os.environ.get('FC_TUNE', '')), flags=int(os.environ.get("FC_PROBE_FLAGS", "0")), k=W.k, labels=tuple(W.labels), proposal=W.proposal, seed=W.seed, pop_lo=lo,
                                   pop_hi=hi), bases=bases)
for it in range(IT):
    s0 = run.stats()
    t = time.time(); run.steps(S); run.sync(); dt = time.time() - t
    s1 = run.stats()
    d = {k: float((s1[k] - s0[k]).sum()) for k in ("proposals", "draws", "bfs_calls", "bfs_levels", "accepted")}
    print(f"{sys.argv[1]} C={C} it {it}: kernel {run.last_ms():9.2f} ms  prop/s {d['proposals']/dt:.3e}  "
          f"draws/prop {d['draws']/d['proposals']:.2f}  bfs/prop {d['bfs_calls']/d['proposals']:.4f}  "
          f"levels/bfs {d['bfs_levels']/max(d['bfs_calls'],1):.1f}  {run.kernel_name()}", flush=True)
