"""Multi-flip pass coverage of the k > 2 instance (FC_PHASE_PROF build): how many passes ran, how
many fell back to one flip at a time in the district tables.  Run with
FC_LIB_PATH=.../libflipchain_prof.so FC_PROF_OUT=<file>:  python tools/mf_cover.py <file>"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flipcomplexityempirical_amd import _lib  # noqa: E402
_lib.load(allow_variant=True)  # A/B and profiling tool: FC_LIB_PATH / FC_LIB_VARIANT libraries allowed
from flipcomplexityempirical_amd import graphs as G  # noqa: E402
from flipcomplexityempirical_amd.engine import FlipGraph, FlipRun, RunConfig  # noqa: E402

cases = {
    "grid_small": (G.grid_graph(12, 12), 9, 0.9, "strip"),
    "c4": (G.triangular_graph(40, 78), 8, 0.1, "strip"),
}
out = sys.argv[1]
for name, (spec, k, pct, plan) in cases.items():
    if os.path.exists(out):
        os.remove(out)
    a0 = spec.assignment_array(G.strip_plan(spec, k), list(range(k)))
    inits = np.stack([a0] * 12)
    _, (lo, hi) = G.population_bounds(int(spec.pop.sum()), k, pct)
    cfg = RunConfig(k=k, labels=tuple(range(k)), proposal=_lib.FC_PROPOSE_PAIR, seed=21, pop_lo=lo, pop_hi=hi,
                    tune={"multi_flip": 1})
    r = FlipRun(FlipGraph(spec), inits, cfg, bases=np.asarray([1.0, 0.5, 2.0, 1.0] * 3))
    r.steps(3000)
    print(name, r.kernel_name())
    raw = np.fromfile(out, dtype=np.int64)
    S = next(s for s in (32, 28, 24) if (raw.size // 12) % s == 0)
    x = raw.reshape(-1, 12, S)[-1].sum(axis=0)
    print(f"  passes {x[21]}  not taken {x[27]}  one-by-one tables {x[20]}  flips in passes {x[22]}  flips {x[7]}")
